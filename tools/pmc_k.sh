# One PMC pass (counters in $PMC, default: the SQ stall breakdown + GRBM_GUI_ACTIVE) over the render
# kernels of a short one-stream C3 bench; prints per-launch means.  usage (GPU box):
#   PMC="..." bash tools/pmc_k.sh <tag> [variant]      (variant: tools/ab/libgsr_<variant>.so)
set -u
tag=${1:-k}; v=${2:-}
PMC=${PMC:-SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VALU GRBM_GUI_ACTIVE}
R=$(pwd); O=$R/gpurun_out/pmck_$tag; mkdir -p "$O"
if [ -n "$v" ]; then export GSR_LIB=$R/tools/ab/libgsr_$v.so; fi
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc $PMC --kernel-include-regex "render|gauss_bwd" --kernel-trace --output-format csv -d "$O/d" -- \
  python3 "$R/bench.py" --no-cpu-baseline --streams 1 --steps 4 --warmup 2 --probe-steps 1 --call-site-steps 0 --loss-steps 0 --densify-steps 0 --io-timesteps 0 > "$O/log" 2>&1 || { echo "pmc failed"; tail -5 "$O/log"; exit 1; }
cd "$R"
python3 - "$O" <<'PY'
import csv, glob, sys, collections, re
O = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); disp = collections.defaultdict(set)
for f in glob.glob(O + "/d/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = re.search(r"(k_\w+)", r["Kernel_Name"]).group(1)
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"]); disp[k].add(r["Dispatch_Id"])
dur = collections.defaultdict(list)
for f in glob.glob(O + "/d/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        m = re.search(r"(k_\w+)", r["Kernel_Name"])
        if m: dur[m.group(1)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, c in acc.items():
    n = len(disp[k]); d = sorted(dur[k]); us = d[len(d) // 2] if d else 0
    row = {m: v / n for m, v in c.items()}
    print(f"{k} n={n} us={us:.1f} " + " ".join(f"{m}={v/1e6:.2f}M" for m, v in sorted(row.items())))
    if "SQ_WAVE_CYCLES" in row:
        w = row["SQ_WAVE_CYCLES"]
        print("   fractions of wave cycles: " + " ".join(f"{m[3:]}={row[m]/w:.3f}" for m in sorted(row) if m.startswith(("SQ_WAIT", "SQ_ACTIVE"))))
    if "GRBM_GUI_ACTIVE" in row and us:
        print(f"   clock ~ {row['GRBM_GUI_ACTIVE']/8/(us*1e-6)/1e9:.2f} GHz")
PY
