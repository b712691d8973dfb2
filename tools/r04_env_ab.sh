#!/bin/bash
# A/B an environment switch on the bench (headline + unchanged + c2), alternated
# usage: bash tools/r04_env_ab.sh "VAR=value ..." [reps]
set -u
mkdir -p gpurun_out/r04
E=$1; N=${2:-2}
LEGS="--call-site-steps 0 --train-steps 0 --loss-steps 0 --densify-steps 0 --io-timesteps 0 --no-cpu-baseline"
for r in $(seq $N); do
  for v in def env; do
    if [ $v = def ]; then env timeout -k 10 300 python -u bench.py $LEGS > gpurun_out/r04/eab_$v$r.json 2>/dev/null || exit 1
    else env $E timeout -k 10 300 python -u bench.py $LEGS > gpurun_out/r04/eab_$v$r.json 2>/dev/null || exit 1; fi
    python3 -c "
import json; d=json.loads(open('gpurun_out/r04/eab_$v$r.json').read().strip().splitlines()[-1])
u=d['unchanged_call_site']; c=d['c2']
print('$v' if '$v'=='def' else '$E', d['value'], d['median_ms_per_step'], 'unchanged', u['Msplats_per_s'], 'c2', c['Msplats_per_s'])"
  done
done
