# Round 6: async-forward gradient mismatch: does holding the forwards' / render halves' results fix it?
set -o pipefail
O=gpurun_out/r06zd; mkdir -p $O
run() { name=$1; shift; timeout -k 10 200 python -u tools/spec_half_repro.py --reps 2 --views 1 --halves 0 --stash "$@" > $O/$name.log 2>&1; echo "== $name"; grep -E '^(async|  rep)' $O/$name.log | cut -c1-160; }
run holdfwd --hold fwd
run holdhalf --hold half
