"""Run only bench.c2_leg (C2: 4 x 800x800 views, 100k Gaussians, one thread, 3 streams), pinned before
the GPU runtime starts as bench.py does -- a short program for rocprofv3 kernel traces of the C2 step.
usage (GPU box): python tools/c2_only.py [steps]"""
import os
import sys

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(REPO, "animating-gaussian-splats_amd"), REPO]
import splat_affinity  # noqa: E402

print("pinned", splat_affinity.pin_host_threads(0, 0, 1, 8))
import torch  # noqa: E402

import bench  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 100
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
r = bench.c2_leg(steps, 10, dev)
print({k: r[k] for k in ("Msplats_per_s", "median_ms_per_step", "host_ms_per_step_median")})
