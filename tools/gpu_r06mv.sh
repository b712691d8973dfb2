# Round 6: k_gauss_bwd_multi with SH coefficients 9-15 from global memory, dL/dSH in
# registers, 4 waves/SIMD (GSR_MV_SPLIT) -- parity of the multi-view tests with that library, then an
# alternated A/B (headline + solo gauss_bwd) against the same tree without it, and its SQ counters.
set -o pipefail
O=gpurun_out/r06mv; mkdir -p $O
GSR_LIB=tools/ab/libgsr_mvsplit.so timeout -k 10 600 python -u -m pytest tests/test_headline_parity.py tests/test_multiview.py tests/test_view_order.py tests/test_repeatability.py -m gpu -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -le 1 ] || exit $rc
bash tools/lib_ab.sh $O 3 mvsplit mvbase || exit 1
bash tools/pmc_lib.sh $O mvsplit sq && bash tools/pmc_lib.sh $O mvbase sq
exit $rc
