# Round 6: the `nonop` DPP-hazard form (the shipped asm minus its s_nop) on the round-5 failure's test,
# then the round-6 profile passes of the current tree.   usage: bash tools/gpu_r06b.sh
set -o pipefail
O=gpurun_out/r06b; mkdir -p $O
HZ=tools/ab/libgsr_dppnonop.so
ok() { [ "$1" -le 1 ] || { echo "step failed rc=$1"; exit "$1"; }; }
GSR_LIB=$HZ timeout -k 10 240 python -u tools/bwd_determinism.py C4 8 > $O/det_nonop_C4.log 2>&1; ok $?
grep -v amdgpu.ids $O/det_nonop_C4.log | tail -6
for r in 1 2 3; do
  GSR_LIB=$HZ timeout -k 10 400 python -u -m pytest tests/test_dp_gpu.py -k "one_rank_c4" -x -q --timeout 300 --timeout-method thread > $O/dp_nonop$r.log 2>&1; ok $?
  grep -E "off, worst|passed|failed" $O/dp_nonop$r.log | tail -2
done
bash tools/profile_round.sh r06 || exit 1
