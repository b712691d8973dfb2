#!/bin/bash
# Stall breakdown of the render kernels, three PMC passes of 8 SQ counters (kernel trace only), 1-stream
# short bench.  usage (GPU box): bash tools/pmc_stall2.sh OUTDIR [NAME]   (NAME: def or tools/ab/libgsr_NAME.so)
set -u
O=$1; v=${2:-def}
R=$(pwd); mkdir -p "$O/stall_$v"; OO=$(cd "$O/stall_$v" && pwd)
case "$v" in
  def) export GSR_LIB=$R/animating-gaussian-splats_amd/diff_gaussian_rasterization/libgsr.so ;;
  *) export GSR_LIB=$R/tools/ab/libgsr_$v.so ;;
esac
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD"
P2="SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_INST_LEVEL_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS"
P3="SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_IFETCH SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_MISC SQ_LDS_DATA_FIFO_FULL SQ_INSTS_SMEM"
i=0
for CT in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $CT --kernel-include-regex "render|preprocess|gauss_bwd_multi" --kernel-trace --output-format csv -d "$OO/p$i" -- \
    python3 "$R/bench.py" --no-cpu-baseline --streams 1 --steps 4 --warmup 2 --probe-steps 1 --call-site-steps 0 --train-steps 0 --c2-steps 0 --unchanged-steps 0 --inference-steps 0 --loss-steps 0 --densify-steps 0 --io-timesteps 0 > "$OO/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OO/p$i.log"; exit 1; }
done
cd "$R"
python3 - "$OO" "$v" <<'PY'
import csv, glob, sys, collections
O, v = sys.argv[1], sys.argv[2]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); disp = collections.defaultdict(set)
for f in glob.glob(O + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].split("<")[0].replace("void gsr::", "").replace("gsr::", "")
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"]); disp[(k, r["Counter_Name"])].add(r["Dispatch_Id"])
out = {}
for k, c in acc.items():
    per = {m: x / len(disp[(k, m)]) for m, x in c.items()}
    out[k] = per
    wc = per.get("SQ_WAVE_CYCLES", 1)
    line = {m: round(x / 1e6, 3) for m, x in sorted(per.items())}
    print(v, k, line)
    if "SQ_INSTS_VMEM_RD" in per and per["SQ_INSTS_VMEM_RD"]:
        print("   avg VMEM level/insts (cycles in flight per VMEM instr):", round(per["SQ_INST_LEVEL_VMEM"] / per["SQ_INSTS_VMEM_RD"], 1))
    if "SQ_INSTS_LDS" in per and per["SQ_INSTS_LDS"]:
        print("   avg LDS level/insts:", round(per["SQ_INST_LEVEL_LDS"] / per["SQ_INSTS_LDS"], 1))
    print("   fractions of wave cycles: wait_any %.3f wait_inst_any %.3f active_any %.3f" % (
        per.get("SQ_WAIT_ANY", 0) / wc, per.get("SQ_WAIT_INST_ANY", 0) / wc, per.get("SQ_ACTIVE_INST_ANY", 0) / wc))
import json; json.dump(out, open(O + "/summary.json", "w"), indent=1)
PY
