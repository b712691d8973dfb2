#!/bin/bash
# headline step traced with the asynchronous forward on vs off: per-stream gaps (forward -> backward bubble)
set -u
mkdir -p gpurun_out/r04
R=$(pwd)
LEGS="--call-site-steps 0 --train-steps 0 --loss-steps 0 --densify-steps 0 --io-timesteps 0 --unchanged-steps 0 --c2-steps 0 --no-cpu-baseline --steps 20 --warmup 5"
cd /tmp && export TMPDIR=/tmp
for a in 0 1; do
  GSR_ASYNC_FORWARD=$a timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r04/atr$a -- python3 $R/bench.py $LEGS > $R/gpurun_out/r04/atr$a.log 2>&1 || exit 1
done
cd $R
for a in 0 1; do
  echo "== async $a"; grep -o '"value": [0-9.]*\|"median_ms_per_step": [0-9.]*' gpurun_out/r04/atr$a.log | head -2
  python3 tools/stream_paths.py gpurun_out/r04/atr$a --steps 10:30 --gaps 100 | head -16
done
