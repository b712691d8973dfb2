"""Per-kernel SQ counter table from a tools/pmc_render.sh output directory."""
import collections, csv, glob, re, sys
rows = []
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    m = re.search(r"gsr::(\w+)", r["Kernel_Name"])
    acc[m.group(1) if m else r["Kernel_Name"][:30]][r["Counter_Name"]].append(float(r["Counter_Value"]))
print(f"{'kernel':<18}{'waves':>8}{'valu/w':>9}{'lds/w':>8}{'salu/w':>8}{'cyc/w(q)':>10}{'wait%':>7}{'act%':>6}{'VALU Ginst':>11}")
for k, v in acc.items():
    d = {c: sum(x) / len(x) for c, x in v.items()}
    w = d.get("SQ_WAVES", 1)
    print(f"{k:<18}{w:>8.0f}{d['SQ_INSTS_VALU']/w:>9.0f}{d['SQ_INSTS_LDS']/w:>8.0f}{d['SQ_INSTS_SALU']/w:>8.0f}"
          f"{d['SQ_WAVE_CYCLES']/w:>10.0f}{100*d['SQ_WAIT_ANY']/d['SQ_WAVE_CYCLES']:>7.0f}"
          f"{100*d['SQ_ACTIVE_INST_ANY']/d['SQ_WAVE_CYCLES']:>6.0f}{d['SQ_INSTS_VALU']/1e9:>11.3f}")
