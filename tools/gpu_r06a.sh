# Round 6, first GPU call: reproduce the round-5 C4 mismatch with the DPP-hazard build,
# then the fixed tree's GPU suite, smoke and bench.   usage: bash tools/gpu_r06a.sh
set -o pipefail
O=gpurun_out/r06a; mkdir -p $O
HZ=tools/ab/libgsr_dpphaz.so
ok() { [ "$1" -le 1 ] || { echo "step failed rc=$1"; exit "$1"; }; }
for cfg in C4 C3; do
  GSR_LIB=$HZ timeout -k 10 240 python -u tools/bwd_determinism.py $cfg 6 > $O/det_haz_$cfg.log 2>&1; ok $?
  grep -v amdgpu.ids $O/det_haz_$cfg.log | tail -4
done
timeout -k 10 240 python -u tools/bwd_determinism.py C4 6 > $O/det_def_C4.log 2>&1; ok $?
grep -v amdgpu.ids $O/det_def_C4.log | tail -2
GSR_LIB=$HZ timeout -k 10 400 python -u -m pytest tests/test_dp_gpu.py -k "one_rank_c4" -x -q --timeout 300 --timeout-method thread > $O/dp_haz.log 2>&1; ok $?
grep -E "off, worst|passed|failed" $O/dp_haz.log | tail -3
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -4 $O/pytest.log; cp gpurun_out/parity_stats.json $O/ 2>/dev/null; ok $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; ok $?
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err; ok $?
tail -1 $O/bench.json | cut -c1-400
exit $rc
