#!/bin/bash
# Short rasterizer-only bench (no side legs) for kernel iteration; prints value, ms/step, phase times.
timeout -k 10 300 python -u bench.py --no-cpu-baseline --loss-steps 0 --densify-steps 0 --call-site-steps 0 --io-timesteps 0 "$@" > gpurun_out/qb.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/qb.log; exit 1; }
grep '^{' gpurun_out/qb.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config']['mean_num_rendered']); print(d['phase_ms_per_launch'])"
