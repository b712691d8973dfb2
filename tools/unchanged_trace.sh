#!/bin/bash
# Kernel trace of the unchanged train.py step alone (bench.py's unchanged_call_site leg), then the
# per-kernel time and the idle gaps of its last 20 % (timeline_gaps.py).
# usage (GPU box, repo root): bash tools/unchanged_trace.sh <tag>
set -u
tag=${1:-u}
R=$(pwd)
O=$R/gpurun_out/utrace_$tag
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$O/trace" -- \
    python3 "$R/bench.py" --no-cpu-baseline --steps 1 --warmup 1 --probe-steps 0 --call-site-steps 0 --inference-steps 0 \
    --train-steps 0 --loss-steps 0 --densify-steps 0 --io-timesteps 0 --c2-steps 0 --unchanged-steps 40 > "$O/trace.log" 2>&1 \
    || { echo "trace failed rc=$?"; exit 1; }
cd "$R"
python3 tools/timeline_gaps.py "$O/trace" > "$O/gaps.txt" && cat "$O/gaps.txt"
