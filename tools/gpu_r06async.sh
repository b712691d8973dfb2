# Round 6: the asynchronous-forward tests (stream lookup, held-back and speculative halves).
set -o pipefail
O=gpurun_out/r06async; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_async_forward.py -m gpu -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
exit $rc
