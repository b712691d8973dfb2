"""Per-stream occupancy over a rocprofv3 kernel trace window (several streams, one GPU).

usage: python tools/stream_paths.py <trace_dir> [--frac F]
Over the last FRAC of the trace: for every HIP stream (Stream_Id), the share of the window it has a
kernel in flight ("busy": its serial chain of kernels) and its idle gaps, and per kernel name on it the
summed duration -- whether the step is bound by one stream's serial chain (busy ~ 1.0) or by the
chip (every stream partly idle)."""
import argparse
import csv
import glob
import os
import re
from collections import defaultdict


def _short(name):
    m = re.search(r"gsr::(\w+?)(?:<|\(|$)", name) or re.search(r"(k_\w+)", name)
    return m.group(1) if m else name.split("(")[0][:40]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("--frac", type=float, default=0.2)
    ap.add_argument("--steps", default=None,
                    help="A:B -- the window from the end of the A-th to the end of the B-th k_gauss_bwd_multi "
                         "launch (one per step; bench.py's timed region at warmup 5 + probe 3 + solo 3: 10:30)")
    ap.add_argument("--gaps", type=float, default=0.0,
                    help="also list each stream's idle gaps longer than this many us by (previous kernel -> "
                         "next kernel): where the serial chain waits (host submission, cross-stream events)")
    a = ap.parse_args()
    rows = []
    for f in glob.glob(os.path.join(a.trace_dir, "**", "*kernel_trace.csv"), recursive=True):
        with open(f, newline="") as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"], _short(r["Kernel_Name"])))
    rows.sort()
    t0, t1 = rows[0][0], max(r[1] for r in rows)
    if a.steps:
        A, B = (int(x) for x in a.steps.split(":"))
        ends = [r[1] for r in rows if r[3] == "k_gauss_bwd_multi"]
        w0, w1 = ends[A], ends[B]
        win = [r for r in rows if r[0] >= w0 and r[1] <= w1]
    else:
        w0 = t1 - (t1 - t0) * a.frac
        win = [r for r in rows if r[0] >= w0]
    span = max(r[1] for r in win) - min(r[0] for r in win)
    by = defaultdict(list)
    for r in win:
        by[r[2]].append(r)
    print(f"window {span / 1e6:.3f} ms, {len(win)} kernels, {len(by)} streams")
    for sid, rs in sorted(by.items(), key=lambda kv: -len(kv[1])):
        busy, last, gaps = 0, None, []
        for s, e, _, _ in rs:
            if last is not None and s > last:
                gaps.append(s - last)
            busy += e - max(s, last or s) if last is None or e > last else 0
            last = max(last or e, e)
        per = defaultdict(float)
        for s, e, _, n in rs:
            per[n] += (e - s) / 1e3
        top = sorted(per.items(), key=lambda kv: -kv[1])[:8]
        print(f"stream {sid}: {len(rs)} kernels, busy {busy / span:.3f} of the window, idle gaps {sum(gaps) / 1e3:.0f} us "
              f"(mean {sum(gaps) / max(len(gaps), 1) / 1e3:.1f} us)")
        print("   " + ", ".join(f"{n} {v:.0f}" for n, v in top))
        if a.gaps > 0:
            where = defaultdict(list)
            last, prev = None, None
            for s, e, _, n in rs:
                if last is not None and s - last > a.gaps * 1e3:
                    where[(prev, n)].append((s - last) / 1e3)
                if last is None or e > last:
                    last, prev = e, n
            for (p0, p1), v in sorted(where.items(), key=lambda kv: -sum(kv[1]))[:8]:
                print(f"     gap {p0} -> {p1}: n={len(v)} total {sum(v):.0f} us mean {sum(v) / len(v):.1f} us")


if __name__ == "__main__":
    main()
