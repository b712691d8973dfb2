#!/bin/bash
# A/B two libgsr.so builds at a given stream count, alternating, N rounds: bash tools/ab_streams.sh A B STREAMS ROUNDS
set -u
A=$1; B=$2; S=$3; N=$4
for r in $(seq $N); do
  for lib in $A $B; do
    GSR_LIB=$lib timeout -k 10 200 python -u bench.py --streams $S --no-cpu-baseline --loss-steps 0 --densify-steps 0 --call-site-steps 0 --io-timesteps 0 > gpurun_out/abs.log 2>&1 || { echo "run failed"; tail -3 gpurun_out/abs.log; exit 1; }
    grep '^{' gpurun_out/abs.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$(basename $lib .so) s$S', d['value'])"
  done
done
