#!/bin/bash
# SQ counters for the render kernels (one PMC pass, kernel-trace only).
set -u
R=$(pwd); O=$R/gpurun_out/pmc_${1:-x}; mkdir -p "$O"; shift || true
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY \
   --kernel-include-regex "render|gauss_bwd|tile_sort|preprocess" --kernel-trace --output-format csv -d "$O" -- \
   python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline "$@" > "$O/run.log" 2>&1 || { echo "pmc pass failed rc=$?"; exit 1; }
echo "pmc ok"
