#!/bin/bash
# SQ counters of the render kernels for one library build (one pass of 8 SQ counters, short 1-stream bench).
# usage (GPU box): bash tools/pmc_lib.sh OUTDIR NAME [sq|lds]   (NAME = def or tools/ab/libgsr_NAME.so)
set -u
O=$1; v=$2; set_=${3:-sq}
if [ "$set_" = lds ]; then
  CTRS="SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU"
else
  CTRS="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAIT_ANY"
fi
R=$(pwd); mkdir -p "$O/pmc_${v}_$set_"; OO=$(cd "$O/pmc_${v}_$set_" && pwd)
B=$R/bench.py; EXTRA="--inference-steps 0"
case "$v" in
  def) export GSR_LIB=$R/animating-gaussian-splats_amd/diff_gaussian_rasterization/libgsr.so ;;
  *tree) B=$R/tools/ab/$v/bench.py; EXTRA="" ;;
  *) export GSR_LIB=$R/tools/ab/libgsr_$v.so ;;
esac
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc $CTRS \
  --kernel-include-regex "render|sort" --kernel-trace --output-format csv -d "$OO/sq" -- \
  python3 "$B" --no-cpu-baseline --streams 1 --steps 6 --warmup 2 --probe-steps 1 --call-site-steps 0 --train-steps 0 --c2-steps 0 --unchanged-steps 0 $EXTRA --loss-steps 0 --densify-steps 0 --io-timesteps 0 > "$OO/log" 2>&1 || { echo "pmc failed"; tail -5 "$OO/log"; exit 1; }
cd "$R"
python3 - "$OO" "$v" <<'PY'
import csv, glob, sys, collections
O, v = sys.argv[1], sys.argv[2]
f = glob.glob(O + "/sq/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); disp = set()
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].split("(")[0].split("<")[0]
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"]); disp.add((k, r["Dispatch_Id"]))
n = collections.Counter(k for k, _ in disp)
for k, c in acc.items():
    print(v, k, {m: round(x / n[k] / 1e6, 2) for m, x in sorted(c.items())}, "(M per launch)")
PY
