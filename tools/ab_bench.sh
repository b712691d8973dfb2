#!/bin/bash
# A/B the rasterizer on the same box: alternates runs of bench.py over two builds of libgsr.so
# (paths as arguments), rasterizer-only, and prints value / ms per step / render phase times.
set -u
A=$1; B=$2; shift 2
for r in 1 2; do
  for v in A B; do
    lib=$A; [ $v = B ] && lib=$B
    GSR_LIB=$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline --loss-steps 0 --densify-steps 0 --call-site-steps 0 --io-timesteps 0 "$@" > gpurun_out/ab_$v$r.log 2>&1 || { echo "run $v$r failed"; tail -3 gpurun_out/ab_$v$r.log; exit 1; }
    grep '^{' gpurun_out/ab_$v$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['phase_ms_per_launch']; print('$v$r', d['value'], d['ms_per_step'], 'fwd', p['render_fwd'], 'bwd', p['render_bwd'], 'bwd_timed', d['roofline']['avg_kernel_ms'])"
  done
done
