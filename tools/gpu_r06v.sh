# Round 6: repro of the intermittent test_speculative_render_half_bitwise[True] mismatch.
set -o pipefail
O=gpurun_out/r06v; mkdir -p $O
timeout -k 10 300 python -u tools/spec_half_repro.py --reps 4 > $O/repro.log 2>&1; rc=$?
grep -v amdgpu $O/repro.log | tail -14
exit $rc
