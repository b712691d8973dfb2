"""CPU placement facts of the GPU box: allowed CPUs, their NUMA nodes, the GPU's NUMA node."""
import glob
import os

aff = sorted(os.sched_getaffinity(0))
print("allowed cpus", len(aff), aff[:8], "...", aff[-4:])
node_of = {}
for d in glob.glob("/sys/devices/system/node/node*"):
    n = int(d.rsplit("node", 1)[1])
    try:
        txt = open(os.path.join(d, "cpulist")).read().strip()
    except OSError:
        continue
    for part in txt.split(","):
        a, _, b = part.partition("-")
        for c in range(int(a), int(b or a) + 1):
            node_of[c] = n
print("nodes of allowed cpus", sorted({node_of.get(c) for c in aff}))
for p in glob.glob("/sys/class/drm/card*/device/numa_node"):
    try:
        print(p, open(p).read().strip())
    except OSError:
        pass
print("HIP_VISIBLE_DEVICES", os.environ.get("HIP_VISIBLE_DEVICES"), "ROCR_VISIBLE_DEVICES", os.environ.get("ROCR_VISIBLE_DEVICES"))
