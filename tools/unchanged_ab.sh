#!/bin/bash
# A/B library builds on the unchanged train.py step (bench.py's unchanged_call_site leg), alternated.
# usage (GPU box, repo root): bash tools/unchanged_ab.sh OUTDIR REPS NAME...  (NAME -> tools/ab/libgsr_NAME.so)
set -u
O=$1; N=$2; shift 2
mkdir -p "$O"
LEGS="--steps 1 --warmup 1 --probe-steps 0 --call-site-steps 0 --inference-steps 0 --train-steps 0 --loss-steps 0 --densify-steps 0 --io-timesteps 0 --c2-steps 0 --no-cpu-baseline --unchanged-steps 60"
for r in $(seq "$N"); do
  for v in "$@"; do
    GSR_LIB=tools/ab/libgsr_$v.so timeout -k 10 300 python -u bench.py $LEGS > "$O/u_$v$r.json" 2> "$O/u_$v$r.err" \
      || { echo "bench $v failed"; tail -5 "$O/u_$v$r.err"; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/u_$v$r.json').read().strip().splitlines()[-1]); u=d['unchanged_call_site']
print('$v', u['Msplats_per_s'], u['median_ms_per_step'], u['step_ms_quartiles'])"
  done
done
