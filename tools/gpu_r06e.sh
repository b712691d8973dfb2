# Round 6: the pipelined saturation re-walk -- parity tests, then an alternated A/B against the library
# before the re-walk (tools/ab/libgsr_base.so).   usage: bash tools/gpu_r06e.sh
set -o pipefail
O=gpurun_out/r06e; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -6 $O/pytest.log; cp gpurun_out/parity_stats.json $O/ 2>/dev/null
[ $rc -le 1 ] || exit $rc
bash tools/lib_ab.sh $O 3 base def || exit 1
exit $rc
