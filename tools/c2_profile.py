"""cProfile of bench.c2_leg (C2: 4 views of 800x800, 100k Gaussians, one host thread, 3 streams) and
the wrapped wall time of the library's entry points per step.  usage (GPU box): python tools/c2_profile.py"""
import cProfile
import os
import pstats
import sys

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(REPO, "animating-gaussian-splats_amd"), REPO]
import torch  # noqa: E402

import bench  # noqa: E402
from diff_gaussian_rasterization import _C  # noqa: E402

dev = torch.device("cuda", 0)
_C.load_library()
torch.zeros(1, device=dev)
import splat_affinity  # noqa: E402
print("pinned", splat_affinity.pin_host_threads(0, 0, 1, 8))
r = bench.c2_leg(100, 10, dev)
print({k: r[k] for k in ("Msplats_per_s", "median_ms_per_step", "host_ms_per_step_median")})
pr = cProfile.Profile()
pr.enable()
r = bench.c2_leg(200, 10, dev)
pr.disable()
print({k: r[k] for k in ("Msplats_per_s", "median_ms_per_step", "host_ms_per_step_median")})
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(45)
st.sort_stats("cumulative").print_stats(45)
