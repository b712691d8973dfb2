"""Idle time between consecutive kernels in a rocprofv3 kernel trace (one GPU, one stream).

Usage: python tools/timeline_gaps.py <trace_dir> [--from-kernel NAME] [--last-ms X]
Prints, over the window (default: the last 20% of the trace), the span, the summed kernel time,
the summed idle gaps, and the idle gap before each kernel name (total and mean), largest first.
"""
import argparse
import csv
import glob
import os
import re
from collections import defaultdict


def _short(name):
    m = re.search(r"gsr::(\w+?)(?:<|\(|$)", name) or re.search(r"(k_\w+)", name)
    return m.group(1) if m else name.split("(")[0][:50]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("--frac", type=float, default=0.2, help="analyse the last FRAC of the trace")
    a = ap.parse_args()
    rows = []
    for f in glob.glob(os.path.join(a.trace_dir, "**", "*kernel_trace.csv"), recursive=True):
        with open(f, newline="") as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), _short(r["Kernel_Name"])))
    rows.sort()
    t0 = rows[0][0] + (1 - a.frac) * (rows[-1][1] - rows[0][0])
    rows = [r for r in rows if r[0] >= t0]
    busy = sum(e - s for s, e, _ in rows)
    span = rows[-1][1] - rows[0][0]
    gaps = defaultdict(list)
    prev_end = rows[0][1]
    for s, e, n in rows[1:]:
        gaps[n].append(max(0, s - prev_end))
        prev_end = max(prev_end, e)
    idle = sum(sum(v) for v in gaps.values())
    print(f"window {span / 1e3:.1f} us, kernels {len(rows)}, busy {busy / 1e3:.1f} us, idle {idle / 1e3:.1f} us "
          f"({100 * idle / span:.1f}%)")
    for n, v in sorted(gaps.items(), key=lambda kv: -sum(kv[1])):
        print(f"  before {n:40s} n={len(v):4d} total {sum(v) / 1e3:9.1f} us  mean {sum(v) / len(v) / 1e3:7.2f} us")


if __name__ == "__main__":
    main()
