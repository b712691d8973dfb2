"""Kernel concurrency in a rocprofv3 kernel trace window (multi-stream runs).

Usage: python tools/concurrency.py <trace_dir> [--from-launch KERNEL A B]
Takes the window spanned by launches [A, B) of KERNEL (default k_render_bwd 40 140 = bench.py's timed
region at its defaults) and prints the time with 0 / 1 / 2+ kernels in flight and, per kernel, its
total time and the part of it during which it ran alone.
"""
import csv, glob, os, re, sys
from collections import defaultdict


def short(n):
    m = re.search(r"gsr::(\w+?)(?:<|\(|$)", n) or re.search(r"(k_\w+)", n)
    return m.group(1) if m else n.split("(")[0][:40]


def main():
    d = sys.argv[1]
    kern, a, b = "k_render_bwd", 40, 140
    if "--from-launch" in sys.argv:
        i = sys.argv.index("--from-launch")
        kern, a, b = sys.argv[i + 1], int(sys.argv[i + 2]), int(sys.argv[i + 3])
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    ks = [r for r in rows if r[2] == kern]
    t0, t1 = ks[a][0], ks[b - 1][1]
    rows = [r for r in rows if r[1] > t0 and r[0] < t1]
    ev = []
    for s, e, n in rows:
        ev.append((max(s, t0), 1, n)); ev.append((min(e, t1), -1, n))
    ev.sort()
    active = defaultdict(int); nact = 0; last = t0
    hist = defaultdict(float); alone = defaultdict(float); tot = defaultdict(float)
    for t, dlt, n in ev:
        dt = t - last
        if dt > 0:
            hist[min(nact, 2)] += dt
            for k, c in active.items():
                if c:
                    tot[k] += dt
                    if nact == 1:
                        alone[k] += dt
        active[n] += dlt; nact += dlt; last = t
    span = t1 - t0
    print(f"window {span/1e3:.1f} us: idle {100*hist[0]/span:.1f}%  one kernel {100*hist[1]/span:.1f}%  "
          f"two+ {100*hist[2]/span:.1f}%")
    for k in sorted(tot, key=lambda k: -tot[k]):
        print(f"  {k:<28} in flight {tot[k]/1e3:9.1f} us   alone {alone[k]/1e3:9.1f} us")


if __name__ == "__main__":
    main()
