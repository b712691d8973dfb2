#!/bin/bash
# A/B a library build variant against the default on the bench (headline + solo phases), alternated
# usage: bash tools/r04_lib_ab.sh NAME [reps]   (tools/ab/libgsr_NAME.so)
set -u
mkdir -p gpurun_out/r04
V=$1; N=${2:-2}
LEGS="--call-site-steps 0 --train-steps 0 --loss-steps 0 --densify-steps 0 --io-timesteps 0 --c2-steps 0 --no-cpu-baseline"
for r in $(seq $N); do
  for v in def $V; do
    if [ $v = def ]; then L=animating-gaussian-splats_amd/diff_gaussian_rasterization/libgsr.so; else L=tools/ab/libgsr_$v.so; fi
    GSR_LIB=$L timeout -k 10 300 python -u bench.py $LEGS > gpurun_out/r04/lab_$v$r.json 2>/dev/null || exit 1
    python3 -c "
import json; d=json.loads(open('gpurun_out/r04/lab_$v$r.json').read().strip().splitlines()[-1])
s=d['phase_ms_per_launch_solo']; u=d['unchanged_call_site']
print('$v', d['value'], d['median_ms_per_step'], 'unchanged', u['Msplats_per_s'], 'solo fwd/bwd', s['render_fwd'], s['render_bwd'], 'step bwd', d['phase_ms_per_launch']['render_bwd'])"
  done
done
