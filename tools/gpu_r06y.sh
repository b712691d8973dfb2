# Round 6: async-forward gradient mismatch -- does it need a redone forward, several views, a busy GPU?
set -o pipefail
O=gpurun_out/r06y; mkdir -p $O
run() { name=$1; shift; timeout -k 10 200 python -u tools/spec_half_repro.py --reps 4 --halves 0 "$@" > $O/$name.log 2>&1; echo "== $name: $(grep '^async' $O/$name.log | grep -c 'means3D: max 0 n 0') of $(grep -c '^async' $O/$name.log) equal"; grep '^async' $O/$name.log | cut -c1-150; }
run stood --history-scale 3.0
run redo1view --views 1
run redo2views --views 2
run notbusy --no-busy
