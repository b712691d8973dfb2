#!/bin/bash
# Profile bench.py with rocprofv3 on the GPU box: kernel trace + stats, then the HBM counters in
# two separate PMC passes (FETCH_SIZE and WRITE_SIZE do not fit one pass on gfx950), then two
# passes of SQ counters (VALU / LDS / SALU activity) for the compute-bound kernels.  Same bench
# arguments in every pass, so the per-launch averages describe the command bench.py reports on.
# usage (on the box, from the repo root): bash tools/profile_round.sh <tag> [bench args...]
# TIMED_RANGE (default 40:140 = (warmup 5 + probe 3) x 5 views .. + 20 steps x 5 views; BENCH_LEGS pins those counts)
# outputs: gpurun_out/prof_<tag>/{trace,fetch,write,sq1,sq2}/ raw CSV, trace_summary.txt, hbm_pmc.json, sq_pmc.json
set -u
tag=${1:-r01}; shift || true
BENCH_LEGS="--call-site-steps 0 --inference-steps 0 --train-steps 0 --loss-steps 0 --densify-steps 0 --io-timesteps 0 --unchanged-steps 0 --c2-steps 0 --steps 20 --warmup 5"
R=$(pwd)
O=$R/gpurun_out/prof_$tag
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -- \
    python3 "$R/bench.py" --no-cpu-baseline $BENCH_LEGS "$@" > "$O/trace.log" 2>&1 || { echo "trace pass failed rc=$?"; exit 1; }
echo "trace ok"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$O/fetch" -- \
    python3 "$R/bench.py" --no-cpu-baseline $BENCH_LEGS "$@" > "$O/fetch.log" 2>&1 || { echo "fetch pass failed rc=$?"; exit 2; }
echo "fetch ok"
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$O/write" -- \
    python3 "$R/bench.py" --no-cpu-baseline $BENCH_LEGS "$@" > "$O/write.log" 2>&1 || { echo "write pass failed rc=$?"; exit 3; }
echo "write ok"
for pass in 1 2; do
  if [ $pass = 1 ]; then CTR="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE";
  else CTR="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_WAIT_ANY SQ_INSTS_VALU_TRANS_F32"; fi
  timeout -k 10 400 rocprofv3 --pmc $CTR --kernel-include-regex "gsr::" --kernel-trace --output-format csv -d "$O/sq$pass" -- \
      python3 "$R/bench.py" --no-cpu-baseline $BENCH_LEGS "$@" > "$O/sq$pass.log" 2>&1 || { echo "sq pass $pass failed rc=$?"; exit 4; }
done
echo "sq ok"
cd "$R"
python3 tools/rocprof_summary.py trace "$O/trace" --last 20 --range ${TIMED_RANGE:-40:140} --out "$O/trace_summary.json" > "$O/trace_summary.txt"
python3 tools/rocprof_summary.py pmc "$O/fetch" "$O/write" --out "$O/hbm_pmc.json" > "$O/hbm_pmc.txt"
python3 tools/rocprof_summary.py sq "$O/sq1" "$O/sq2" --out "$O/sq_pmc.json" > "$O/sq_pmc.txt"
cp "$O"/trace/*/*_kernel_stats.csv "$O/kernel_stats.csv" 2>/dev/null || true
echo "summaries ok"
