# Round 6: async-forward gradient mismatch, one view, held back, busy GPU: probe the render half.
set -o pipefail
O=gpurun_out/r06za; mkdir -p $O
timeout -k 10 200 python -u tools/spec_half_repro.py --reps 2 --views 1 --halves 0 --stash > $O/probe.log 2>&1; rc=$?
grep -v amdgpu $O/probe.log | cut -c1-200 | tail -40
exit $rc
