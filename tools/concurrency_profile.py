"""Kernel concurrency over a rocprofv3 kernel trace window (several streams, one GPU).

usage: python tools/concurrency_profile.py <trace_dir> [--frac F] [--window K0:A:K1:B]
Over the last FRAC of the trace (or from the start of launch A of kernel K0 to the end of launch B of
kernel K1, e.g. k_preprocess:40:k_gauss_bwd_multi:27 = bench.py's timed region at warmup 5, probe 3,
20 steps): the share of wall time with 0, 1, 2, 3, 4+ kernels in flight, and
per kernel name its summed duration, its duration while running alone, and the mean number of
other kernels in flight beside it -- which kernels share the chip and which run exposed."""
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
    ap.add_argument("--window", default=None)
    a = ap.parse_args()
    rows = []
    for f in glob.glob(os.path.join(a.trace_dir, "**", "*kernel_trace.csv"), recursive=True):
        with open(f, newline="") as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), _short(r["Kernel_Name"])))
    rows.sort()
    if a.window:
        k0, i0, k1, i1 = a.window.split(":")
        t0 = [r for r in rows if r[2] == k0][int(i0)][0]
        tend = [r for r in rows if r[2] == k1][int(i1)][1]
        rows = [r for r in rows if r[0] >= t0 and r[1] <= tend]
    else:
        t0 = rows[0][0] + (1 - a.frac) * (rows[-1][1] - rows[0][0])
        rows = [r for r in rows if r[0] >= t0]
    t1 = max(e for _, e, _ in rows)
    ev = []
    for i, (s, e, n) in enumerate(rows):
        ev.append((s, 1, i))
        ev.append((e, -1, i))
    ev.sort()
    live = set()
    last = ev[0][0]
    share = defaultdict(float)
    alone = defaultdict(float)
    beside = defaultdict(float)
    for t, d, i in ev:
        dt = t - last
        if dt > 0:
            share[min(len(live), 4)] += dt
            for k in live:
                if len(live) == 1:
                    alone[rows[k][2]] += dt
                beside[rows[k][2]] += dt * (len(live) - 1)
        last = t
        if d > 0:
            live.add(i)
        else:
            live.discard(i)
    span = t1 - rows[0][0]
    print(f"window {span / 1e6:.3f} ms, {len(rows)} kernels")
    print("kernels in flight: " + ", ".join(f"{k}{'+' if k == 4 else ''}: {v / span:.3f}" for k, v in sorted(share.items())))
    tot = defaultdict(float)
    cnt = defaultdict(int)
    for s, e, n in rows:
        tot[n] += e - s
        cnt[n] += 1
    print(f"{'kernel':<22}{'launches':>9}{'sum ms':>9}{'alone ms':>10}{'mean others':>12}")
    for n in sorted(tot, key=lambda k: -tot[k]):
        print(f"{n:<22}{cnt[n]:>9}{tot[n] / 1e6:>9.3f}{alone[n] / 1e6:>10.3f}{beside[n] / max(tot[n], 1):>12.2f}")


if __name__ == "__main__":
    main()
