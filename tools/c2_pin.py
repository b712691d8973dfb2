"""C2 leg (bench.c2_leg) with the process pinned to a CPU set: none | node0 | node1 | gpu (the GPU's NUMA
node) | first8 (8 CPUs of the GPU's node).  usage (GPU box): python tools/c2_pin.py MODE [reps]"""
import glob
import json
import os
import sys

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(REPO, "animating-gaussian-splats_amd"), REPO]


def node_cpus(n):
    txt = open(f"/sys/devices/system/node/node{n}/cpulist").read().strip()
    out = []
    for part in txt.split(","):
        a, _, b = part.partition("-")
        out += list(range(int(a), int(b or a) + 1))
    return [c for c in out if c in os.sched_getaffinity(0)]


mode = sys.argv[1]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
gnode = 0
try:
    gnode = int(open("/sys/class/drm/card0/device/numa_node").read())
except OSError:
    pass
if mode == "node0":
    os.sched_setaffinity(0, node_cpus(0))
elif mode == "node1":
    os.sched_setaffinity(0, node_cpus(1))
elif mode == "gpu":
    os.sched_setaffinity(0, node_cpus(max(gnode, 0)))
elif mode.startswith("first"):
    os.sched_setaffinity(0, node_cpus(max(gnode, 0))[:int(mode[5:])])
if mode == "early":  # bench.py's placement, before the GPU runtime starts
    import splat_affinity
    print("early", splat_affinity.pin_host_threads(0, 0, 1, 8), flush=True)
import torch  # noqa: E402

import bench  # noqa: E402
from diff_gaussian_rasterization import _C  # noqa: E402

dev = torch.device("cuda", 0)
_C.load_library()
if mode == "late":  # pinned after the runtime started
    torch.zeros(1, device=dev)
    import splat_affinity
    print("late", splat_affinity.pin_host_threads(0, 0, 1, 8), flush=True)
if mode == "none":
    pr = torch.cuda.get_device_properties(0)
    print({k: getattr(pr, k) for k in dir(pr) if "pci" in k.lower() or "uuid" in k.lower()}, flush=True)
for r in range(reps):
    c = bench.c2_leg(60, 10, dev)
    print(json.dumps({"mode": mode, "rep": r, **{k: c[k] for k in ("Msplats_per_s", "step_ms_quartiles", "host_ms_per_step_median")}}), flush=True)
