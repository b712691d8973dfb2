# full GPU suite + smoke (round-end shape): bash tools/gpu_suite.sh OUTDIR
set -o pipefail
O=${1:-gpurun_out/suite}; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -5 $O/pytest.log
cp gpurun_out/parity_stats.json $O/ 2>/dev/null
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rs=$?
tail -2 $O/smoke.log
exit $(( rc | rs ))
