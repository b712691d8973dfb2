set -o pipefail
O=gpurun_out/r05e; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_inference.py tests/test_gpu_parity.py -m gpu -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -le 1 ] || exit $rc
bash tools/lib_ab.sh $O 2 def noany qms nq || exit 1
