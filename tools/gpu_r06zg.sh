# Round 6: async-forward gradient mismatch: kernel trace of the failing run (1 view, held back, busy GPU).
set -o pipefail
O=gpurun_out/r06zg; mkdir -p $O
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/$O/trace -- python3 -u $R/tools/spec_half_repro.py --reps 2 --views 1 --halves 0 --stash --nofresh > $R/$O/run.log 2>&1; rc=$?
cd $R
grep -E '^(async|  rep)' $O/run.log | cut -c1-200
f=$(find $O/trace -name "*kernel_trace.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
print(list(rows[0].keys()))
keep = [r for r in rows if any(k in r["Kernel_Name"] for k in ("gsr::", "sleep"))]
keep.sort(key=lambda r: int(r["Start_Timestamp"]))
t0 = int(keep[0]["Start_Timestamp"])
# the last async step: from the last sleep kernel on
last_sleep = max(i for i, r in enumerate(keep) if "sleep" in r["Kernel_Name"])
for r in keep[last_sleep:last_sleep + 40]:
    name = r["Kernel_Name"].split("(")[0][:40]
    print(f"{(int(r['Start_Timestamp']) - t0) / 1e3:12.1f} {(int(r['End_Timestamp']) - t0) / 1e3:12.1f}  q {r.get('Queue_Id', '?'):>3} s {r.get('Stream_Id', '?'):>3} t {r.get('Thread_Id', '?'):>8}  {name}")
PY
exit $rc
