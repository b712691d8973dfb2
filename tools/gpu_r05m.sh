set -o pipefail
O=gpurun_out/r05v; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_repeatability.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
bash tools/lib_ab.sh $O 2 def cur fast cur_fast || exit 1
