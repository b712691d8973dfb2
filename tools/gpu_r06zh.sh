# Round 6: async-forward race fix (default stream handle 0 -> torch.cuda.default_stream): the repro
# (held back and speculative halves, 5 and 1 views), the async tests, then the whole suite.
set -o pipefail
O=gpurun_out/r06zh; mkdir -p $O
timeout -k 10 200 python -u tools/spec_half_repro.py --reps 4 > $O/repro5.log 2>&1 || { tail -5 $O/repro5.log; exit 1; }
grep -E '^(async|blocking)' $O/repro5.log | cut -c1-170
timeout -k 10 200 python -u tools/spec_half_repro.py --reps 3 --views 1 > $O/repro1.log 2>&1 || { tail -5 $O/repro1.log; exit 1; }
grep -E '^(async)' $O/repro1.log | cut -c1-170
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; cp gpurun_out/parity_stats.json $O/ 2>/dev/null
exit $rc
