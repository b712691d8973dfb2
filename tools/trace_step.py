"""Per-step breakdown of a one-stream rocprofv3 kernel trace: kernel time by name, idle gaps (total and
the largest ones, with the kernels around them).  usage: python tools/trace_step.py TRACE.csv [views/step]"""
import csv
import re
import sys
from collections import defaultdict


def short(n):
    m = re.search(r"gsr::(\w+?)(?:<|\(|$)", n) or re.search(r"(k_\w+)", n)
    if m:
        return m.group(1)
    m = re.search(r"at::native::(?:\w+::)*(\w+)", n)
    return ("torch:" + m.group(1)) if m else n.split("(")[0][:40]


rows = []
for r in csv.DictReader(open(sys.argv[1])):
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), r["Kernel_Name"]))
rows.sort()
vps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
rows = rows[len(rows) // 3:]  # skip warm-up
steps = sum(1 for r in rows if r[2] == "k_render_fwd") / vps
span = rows[-1][1] - rows[0][0]
tot = defaultdict(float)
cnt = defaultdict(int)
gaps = []
prev = rows[0]
for r in rows:
    tot[r[2]] += r[1] - r[0]
    cnt[r[2]] += 1
for a, b in zip(rows, rows[1:]):
    gaps.append((max(0, b[0] - a[1]), a[2], b[2]))
busy = sum(tot.values())
idle = sum(g for g, _, _ in gaps)
print(f"steps {steps:.1f}: span/step {span / steps / 1e3:.1f} us, kernel time/step {busy / steps / 1e3:.1f} us, "
      f"idle/step {idle / steps / 1e3:.1f} us, kernels/step {len(rows) / steps:.0f}")
for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
    print(f"  {k:44s} {v / steps / 1e3:8.1f} us/step  {cnt[k] / steps:5.1f}/step  {v / cnt[k] / 1e3:7.1f} us avg")
pair = defaultdict(float)
for g, a, b in gaps:
    pair[(a, b)] += g
print("idle before/after (us/step):")
for (a, b), g in sorted(pair.items(), key=lambda kv: -kv[1])[:15]:
    print(f"  {a:30s} -> {b:30s} {g / steps / 1e3:8.1f}")
