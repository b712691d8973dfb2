# Round 6: the C3M (clustered, long lists) full-view parity test.
set -o pipefail
O=gpurun_out/r06c3m; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_headline_parity.py -m gpu -q --timeout 500 --timeout-method thread -k c3m > $O/pytest.log 2>&1; rc=$?
tail -30 $O/pytest.log | cut -c1-300
exit $rc
