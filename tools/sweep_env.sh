#!/bin/bash
# Rasterizer-only bench of the in-tree libgsr.so once per value of an environment variable.
# usage: bash tools/sweep_env.sh VAR v1 v2 ...
set -u
var=$1; shift
for v in "$@"; do
  env $var=$v timeout -k 10 200 python -u bench.py --no-cpu-baseline --loss-steps 0 --densify-steps 0 --call-site-steps 0 --io-timesteps 0 > gpurun_out/sw_$v.log 2>&1 || { echo "run $v failed"; tail -3 gpurun_out/sw_$v.log; exit 1; }
  grep '^{' gpurun_out/sw_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['phase_ms_per_launch']; print('$var=$v', d['value'], d['ms_per_step'], ' '.join(f'{k}={v*1e3:.1f}' for k,v in p.items()))"
done
