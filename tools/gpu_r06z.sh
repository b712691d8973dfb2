# Round 6: async-forward gradient mismatch, one view (a stood speculation with capacity > K):
# held-back vs speculative render half, async vs blocking speculative forwards.
set -o pipefail
O=gpurun_out/r06z; mkdir -p $O
run() { name=$1; shift; timeout -k 10 200 python -u tools/spec_half_repro.py --reps 3 --views 1 "$@" > $O/$name.log 2>&1; echo "== $name: $(grep -E '^(async|blocking) spec' $O/$name.log | grep -c 'means3D: max 0 n 0') of $(grep -cE '^(async|blocking) spec' $O/$name.log) equal"; grep -E '^(async|blocking) spec' $O/$name.log | cut -c1-150; }
run async_held --halves 0
run async_spec --halves 1
run blocking_spec --halves 0 --blocking
run async_held_nobusy --halves 0 --no-busy
