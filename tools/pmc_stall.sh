#!/bin/bash
# Stall breakdown of the render kernels: two PMC passes (kernel-trace only), same short bench.
set -u
R=$(pwd); O=$R/gpurun_out/pmc_stall_${1:-x}; mkdir -p "$O"; shift || true
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --loss-steps 0 --densify-steps 0 --call-site-steps 0 --io-timesteps 0"
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT \
   --kernel-include-regex "render" --kernel-trace --output-format csv -d "$O/p1" -- \
   python3 "$R/bench.py" $ARGS "$@" > "$O/p1.log" 2>&1 || { echo "pass1 failed rc=$?"; tail -3 "$O/p1.log"; exit 1; }
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_WAIT_ANY SQ_INSTS_VALU_TRANS_F32 \
   --kernel-include-regex "render" --kernel-trace --output-format csv -d "$O/p2" -- \
   python3 "$R/bench.py" $ARGS "$@" > "$O/p2.log" 2>&1 || { echo "pass2 failed rc=$?"; tail -3 "$O/p2.log"; exit 2; }
echo "pmc ok"
