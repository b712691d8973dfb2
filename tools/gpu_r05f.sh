set -o pipefail
O=gpurun_out/r05g; mkdir -p $O
timeout -k 10 800 python -u -m pytest tests/test_gpu_parity.py tests/test_inference.py tests/test_headline_parity.py -m gpu -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
cp gpurun_out/parity_stats.json $O/ 2>/dev/null
[ $rc -le 1 ] || exit $rc
bash tools/lib_ab.sh $O 2 def fast || exit 1
