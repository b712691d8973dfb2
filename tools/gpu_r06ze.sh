# Round 6: async-forward gradient mismatch: visible vs invisible Gaussians; zero-filled targets.
set -o pipefail
O=gpurun_out/r06ze; mkdir -p $O
run() { name=$1; shift; timeout -k 10 200 python -u tools/spec_half_repro.py --reps 3 --views 1 --halves 0 --stash "$@" > $O/$name.log 2>&1; echo "== $name"; grep -E '^(async|  rep|visible)' $O/$name.log | cut -c1-230; }
run def
run nofresh --nofresh
timeout -k 10 60 python -u tools/stream0_threads.py 2>&1 | grep -v amdgpu | tail -3
