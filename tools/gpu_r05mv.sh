set -o pipefail
O=gpurun_out/r05mv; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_multiview.py tests/test_headline_parity.py tests/test_train_iteration.py tests/test_dp_gpu.py tests/test_native_bind.py tests/test_gpu_parity.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
cp gpurun_out/parity_stats.json $O/ 2>/dev/null
[ $rc -eq 0 ] || exit $rc
bash tools/lib_ab.sh $O 2 def cur || exit 1
