# Per-kernel instruction counts (one SQ pass) and one-stream durations (kernel trace) of the C3 bench
# step, round-1 tree vs the current tree (optionally a tools/ab variant).
# usage (GPU box): bash tools/pmc_ab.sh [variant ...]
set -u
R=$(pwd); O=$R/gpurun_out/pmcab; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
ARGS="--no-cpu-baseline --streams 1 --steps 6 --warmup 2 --probe-steps 1 --call-site-steps 0 --loss-steps 0 --densify-steps 0 --io-timesteps 0"
for v in r01 cur "$@"; do
  B=$R/bench.py; E=""
  [ $v = r01 ] && B=$R/tools/ab/r01/bench.py
  [ $v != r01 ] && [ $v != cur ] && E="$R/tools/ab/libgsr_$v.so"
  if [ -n "$E" ]; then export GSR_LIB=$E; else unset GSR_LIB; fi
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
    --kernel-trace --output-format csv -d "$O/$v" -- python3 "$B" $ARGS > "$O/$v.log" 2>&1 || { echo "$v pmc failed"; tail -5 "$O/$v.log"; exit 1; }
done
cd "$R"
python3 - "$O" r01 cur "$@" <<'PY'
import csv, glob, sys, collections, re
O = sys.argv[1]
def short(n):
    m = re.search(r"gsr::(\w+?)(?:<|\(|$)", n) or re.search(r"(k_\w+)", n)
    return m.group(1) if m else n.split("(")[0][:40]
for v in sys.argv[2:]:
    f = glob.glob(f"{O}/{v}/**/*counter_collection.csv", recursive=True)[0]
    acc = collections.defaultdict(lambda: collections.defaultdict(float)); disp = collections.defaultdict(set)
    dur = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        k = short(r["Kernel_Name"])
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    for t in glob.glob(f"{O}/{v}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(t)):
            dur[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print("==", v)
    for k in sorted(acc, key=lambda k: -acc[k]["SQ_INSTS_VALU"]):
        n = len(disp[k])
        row = {m.replace("SQ_INSTS_", ""): acc[k][m] / n / 1e6 for m in acc[k]}
        d = sorted(dur[k]); med = d[len(d) // 2] if d else 0.0
        print(f"  {k:<22} n={n:4d} us={med:7.1f} " + " ".join(f"{m}={x:8.2f}" for m, x in sorted(row.items())))
PY
