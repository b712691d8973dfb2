# Round 6: pipelined 128-thread re-walk blocks -- suite, probes, headline A/B vs the pre-re-walk library.
set -o pipefail
O=gpurun_out/r06m; mkdir -p $O
R=$(pwd)
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; cp gpurun_out/parity_stats.json $O/ 2>/dev/null
[ $rc -le 1 ] || exit $rc
for c in C3 C3M; do
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/probe_$c -- python3 $R/tools/tsat_probe.py $c 3 > $R/$O/probe_$c.log 2>&1) || { echo "probe $c failed"; tail -5 $O/probe_$c.log; exit 1; }
  grep -v "amdgpu\|^W20\|^E20" $O/probe_$c.log | tail -1
  python3 tools/rocprof_summary.py trace $O/probe_$c | grep -E "render|tsat" | head -4
done
bash tools/lib_ab.sh $O 3 base def || exit 1
exit $rc
