#!/bin/bash
# A/B/C... over builds of libgsr.so (paths as arguments): rasterizer-only bench per build, twice,
# printing Msplats/s, ms per step and every phase's per-launch time.
set -u
for r in 1 2; do
  for lib in "$@"; do
    tag=$(basename $lib .so)
    GSR_LIB=$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline --loss-steps 0 --densify-steps 0 --call-site-steps 0 --io-timesteps 0 > gpurun_out/abp_$tag$r.log 2>&1 || { echo "run $tag$r failed"; tail -3 gpurun_out/abp_$tag$r.log; exit 1; }
    grep '^{' gpurun_out/abp_$tag$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['phase_ms_per_launch']; print('$tag$r', d['value'], d['ms_per_step'], ' '.join(f'{k}={v*1e3:.1f}' for k,v in p.items()))"
  done
done
