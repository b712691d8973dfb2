set -o pipefail
O=gpurun_out/r05d; mkdir -p $O
timeout -k 10 200 python -u tools/bwd_determinism.py C3 3 > $O/det.log 2>&1; rc=$?; grep -v amdgpu.ids $O/det.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_headline_parity.py tests/test_multiview.py tests/test_repeatability.py tests/test_inference.py tests/test_dp_gpu.py -m gpu -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; cp gpurun_out/parity_stats.json $O/ 2>/dev/null
[ $rc -le 1 ] || exit $rc
bash tools/lib_ab.sh $O 2 r04tree def w5 mvold sh4 || exit 1
bash tools/pmc_lib.sh $O def sq
