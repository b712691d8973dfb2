"""Mean per-dispatch value of every PMC counter, per kernel, from rocprofv3 counter_collection CSVs."""
import collections, csv, glob, re, sys
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        m = re.search(r"gsr::(\w+)", r["Kernel_Name"])
        acc[m.group(1) if m else r["Kernel_Name"][:30]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in acc.items():
    print(k)
    for c, x in sorted(v.items()):
        print(f"   {c:<28}{sum(x) / len(x):>18.0f}")
