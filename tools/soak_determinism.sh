#!/bin/bash
# Soak + determinism check (GPU box, repo root): two separate processes run the headline step for
# STEPS steps on 3 streams / 3 submitting threads, then one more step whose summed gradients are saved;
# the two buckets must be bitwise equal.  usage: bash tools/soak_determinism.sh [STEPS]
set -u
S=${1:-1500}
O=gpurun_out/soak; mkdir -p $O
L="--no-cpu-baseline --call-site-steps 0 --inference-steps 0 --train-steps 0 --loss-steps 0 --densify-steps 0 --io-timesteps 0 --unchanged-steps 0 --c2-steps 0 --probe-steps 0"
for r in a b; do
  timeout -k 10 400 python -u bench.py $L --steps $S --warmup 5 --grad-checksum $O/g_$r > $O/bench_$r.json 2> $O/bench_$r.err \
    || { echo "run $r failed"; tail -5 $O/bench_$r.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bench_$r.json').read().strip().splitlines()[-1]); print('$r', d['value'], d['median_ms_per_step'], d['step_ms_quartiles'])"
done
python3 - <<PY
import torch
a = torch.load("$O/g_a.rank0.pt", weights_only=True); b = torch.load("$O/g_b.rank0.pt", weights_only=True)
assert a["views"] == b["views"], (a["views"], b["views"])
eq = torch.equal(a["bucket"], b["bucket"])
d = (a["bucket"] - b["bucket"]).abs().max().item()
print("views", a["views"], "bitwise equal:", eq, "max abs diff", d, "finite:", bool(torch.isfinite(a["bucket"]).all()))
PY
