# SQ counters of the render kernels (one pass, 8 SQ counters) on a short one-stream bench.
# usage (GPU box): bash tools/pmc_bwd.sh <tag> [bench args]
set -u
tag=${1:-pmc}; shift || true
R=$(pwd); O=$R/gpurun_out/pmc_$tag; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAIT_ANY \
  --kernel-include-regex "render" --kernel-trace --output-format csv -d "$O/sq" -- \
  python3 "$R/bench.py" --no-cpu-baseline --streams 1 --steps 6 --warmup 2 --probe-steps 1 --call-site-steps 0 --loss-steps 0 --densify-steps 0 --io-timesteps 0 "$@" > "$O/log" 2>&1 || { echo "pmc failed"; tail -5 "$O/log"; exit 1; }
cd "$R"
python3 - "$O" <<'PY'
import csv, glob, sys, collections
O = sys.argv[1]
f = glob.glob(O + "/sq/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
disp = set()
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].split("(")[0]
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    disp.add((k, r["Dispatch_Id"]))
for k, _ in disp: n[k] += 1
for k, c in acc.items():
    print(k, {m: round(v / n[k] / 1e6, 2) for m, v in sorted(c.items())}, "(M per launch)")
PY
