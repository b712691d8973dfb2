# Kernel trace (rocprofv3 --kernel-trace --stats) of a short one-stream bench: true per-kernel
# durations without event gaps.  usage (GPU box): bash tools/ktrace.sh <tag> [bench args]
set -u
tag=${1:-kt}; shift || true
R=$(pwd); O=$R/gpurun_out/kt_$tag; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -- \
    python3 "$R/bench.py" --no-cpu-baseline --call-site-steps 0 --loss-steps 0 --densify-steps 0 --io-timesteps 0 "$@" > "$O/trace.log" 2>&1 || { echo "trace failed"; tail -5 "$O/trace.log"; exit 1; }
cd "$R"
python3 - "$O" <<'PY'
import csv, glob, sys, collections
O = sys.argv[1]
f = glob.glob(O + "/trace/**/*kernel_trace.csv", recursive=True)[0]
d = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    d[r["Kernel_Name"].split("(")[0][:60]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    if k.startswith("_ZN3gsr") or "k_" in k:
        v2 = v[len(v) // 3:]
        print(f"{k[:60]:60s} n={len(v):5d} avg_us={sum(v2)/len(v2):8.1f} min={min(v2):8.1f}")
PY
