"""Summarise rocprofv3 CSV output into per-kernel tables (profiles/ evidence for bench.py).

Usage:
  python tools/rocprof_summary.py trace  <dir> [--last N] [--range A:B] [--out x.json]
        -> per-kernel calls / avg / total us (+ average of the last N launches; + average of launches
           [A, B) of each once-per-view kernel = bench.py's timed region, (W+probe)V : (W+probe+K)V)
  python tools/rocprof_summary.py pmc    <fetch_dir> <write_dir> [--out profiles/x.json]
        -> per-kernel avg FETCH_SIZE / WRITE_SIZE per launch and corrected HBM bytes
  python tools/rocprof_summary.py sq     <dir> [<dir> ...] [--out profiles/x.json]
        -> per-kernel avg of every SQ counter per launch (tools/pmc_stall.sh passes), the launches'
           avg duration in those passes, and the VALU instruction-issue fraction
           SQ_INSTS_VALU / (duration x 1024 SIMDs x 2.4 GHz / 2 cycles)

gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE (KiB) reports exactly half the
bytes of a wide coalesced streaming read, so HBM read bytes = 2 x FETCH_SIZE x 1024; WRITE_SIZE is
exact for 16-B-per-lane streaming stores.  Other access widths are uncalibrated; the corrected
figure is an estimate and ratios between kernels/variants are what it is trusted for.
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


PER_STEP = {"k_gauss_bwd_multi"}  # kernels launched once per bench step (summed step shape)
VIEWS = 5                         # views per step (bench.py --views-per-rank)


def _short(name):
    if "k_render_bwd<true>" in name:  # the near-record overflow tiles' launch (a few us, usually empty)
        return "k_render_bwd_near"
    m = re.search(r"gsr::(\w+?)(?:<|\(|$)", name) or re.search(r"(k_\w+)", name)
    return m.group(1) if m else name.split("(")[0][:60]


def _rows(d, pattern):
    files = glob.glob(os.path.join(d, "**", pattern), recursive=True)
    for f in files:
        with open(f, newline="") as fh:
            yield from csv.DictReader(fh)


def trace(d, last=0, rng=None):
    acc = defaultdict(list)
    rows = sorted(_rows(d, "*kernel_trace.csv"), key=lambda r: int(r["Start_Timestamp"]))
    for r in rows:
        acc[_short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    out = {k: {"calls": len(v), "avg_us": sum(v) / len(v), "total_us": sum(v)} for k, v in acc.items()}
    if last:  # the last `last` calls of each kernel
        for k, v in acc.items():
            out[k]["last_avg_us"] = sum(v[-last:]) / len(v[-last:])
    if rng:  # launches [a, b) of each once-per-view kernel: bench.py's timed region
        a, b = rng
        for k, v in acc.items():
            if k in PER_STEP:  # once per step (the multi-view per-Gaussian pass): [a/V, b/V)
                a2, b2 = a // VIEWS, b // VIEWS
                if len(v) >= b2:
                    out[k]["timed_avg_us"] = sum(v[a2:b2]) / (b2 - a2)
                    out[k]["timed_launches"] = [a2, b2]
            elif len(v) >= b:
                out[k]["timed_avg_us"] = sum(v[a:b]) / (b - a)
                out[k]["timed_launches"] = [a, b]
    return dict(sorted(out.items(), key=lambda kv: -kv[1]["total_us"]))


def pmc(fetch_dir, write_dir):
    res = defaultdict(dict)
    for d, ctr in ((fetch_dir, "FETCH_SIZE"), (write_dir, "WRITE_SIZE")):
        acc = defaultdict(list)
        for r in _rows(d, "*counter_collection.csv"):
            if r.get("Counter_Name") != ctr:
                continue
            acc[_short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
        for k, v in acc.items():
            res[k][ctr + "_KiB_avg"] = sum(v) / len(v)
            res[k]["launches_" + ctr] = len(v)
    for k, v in res.items():
        f = v.get("FETCH_SIZE_KiB_avg", 0.0)
        w = v.get("WRITE_SIZE_KiB_avg", 0.0)
        v["hbm_bytes_per_launch_corrected"] = 2 * f * 1024 + w * 1024
    return dict(res)


def sq(dirs):
    acc = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    for d in dirs:
        for r in _rows(d, "*counter_collection.csv"):
            acc[_short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for r in _rows(d, "*kernel_trace.csv"):
            dur[_short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    out = {}
    for k, v in acc.items():
        o = {c: sum(x) / len(x) for c, x in v.items()}
        if "SQ_INSTS_VALU" in v:  # dispatches profiled (bench.py: launches per view -> VALU per step)
            o["launches"] = len(v["SQ_INSTS_VALU"])
        if dur.get(k):
            o["avg_us_in_pass"] = sum(dur[k]) / len(dur[k])
            if "GRBM_GUI_ACTIVE" in o:  # summed over the 8 XCDs (MI355X_MICROARCH.md, DVFS give-back)
                o["clock_ghz"] = o["GRBM_GUI_ACTIVE"] / 8 / (o["avg_us_in_pass"] * 1e-6) / 1e9
            if "SQ_INSTS_VALU" in o:
                o["valu_issue_frac"] = o["SQ_INSTS_VALU"] * 2 / (1024 * o["avg_us_in_pass"] * 1e-6 * 2.4e9)
                if "clock_ghz" in o:  # the same at the clock the chip held during the launch
                    o["valu_issue_frac_at_clock"] = o["SQ_INSTS_VALU"] * 2 / (1024 * o["avg_us_in_pass"] * 1e-6 * o["clock_ghz"] * 1e9)
        out[k] = o
    return out


def main():
    mode = sys.argv[1]
    if mode == "trace":
        last = int(sys.argv[sys.argv.index("--last") + 1]) if "--last" in sys.argv else 0
        rng = tuple(int(x) for x in sys.argv[sys.argv.index("--range") + 1].split(":")) if "--range" in sys.argv else None
        t = trace(sys.argv[2], last, rng)
        print(f"{'kernel':<28}{'calls':>8}{'avg_us':>12}{'total_us':>14}" + (f"{'last%d_avg_us' % last:>16}" if last else "")
              + (f"{'timed_avg_us':>14}" if rng else ""))
        for k, v in t.items():
            print(f"{k:<28}{v['calls']:>8}{v['avg_us']:>12.2f}{v['total_us']:>14.1f}"
                  + (f"{v['last_avg_us']:>16.2f}" if last else "")
                  + (f"{v['timed_avg_us']:>14.2f}" if rng and 'timed_avg_us' in v else ""))
        if "--out" in sys.argv:
            json.dump(t, open(sys.argv[sys.argv.index("--out") + 1], "w"), indent=1)
    elif mode == "sq":
        dirs = [a for a in sys.argv[2:] if not a.startswith("--") and a != (sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else None)]
        q = sq(dirs)
        for k, v in q.items():
            print(k, {c: (round(x, 3) if isinstance(x, float) and x < 100 else int(x)) for c, x in v.items()})
        if "--out" in sys.argv:
            json.dump(q, open(sys.argv[sys.argv.index("--out") + 1], "w"), indent=1)
    elif mode == "pmc":
        p = pmc(sys.argv[2], sys.argv[3])
        print(f"{'kernel':<28}{'FETCH KiB':>14}{'WRITE KiB':>14}{'HBM MB (corr)':>16}")
        for k, v in sorted(p.items(), key=lambda kv: -kv[1]["hbm_bytes_per_launch_corrected"]):
            print(f"{k:<28}{v.get('FETCH_SIZE_KiB_avg', 0):>14.1f}{v.get('WRITE_SIZE_KiB_avg', 0):>14.1f}"
                  f"{v['hbm_bytes_per_launch_corrected'] / 1e6:>16.2f}")
        if "--out" in sys.argv:
            json.dump(p, open(sys.argv[sys.argv.index("--out") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
