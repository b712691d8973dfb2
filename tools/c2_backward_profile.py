"""cProfile of the C2 leg with the autograd engine's device threads off (torch.autograd
set_multithreading_enabled(False)), so that the rasterizer's Python backward -- which the engine
otherwise runs on its own thread, out of cProfile's sight -- is counted.  usage (GPU box):
python tools/c2_backward_profile.py"""
import cProfile
import os
import pstats
import sys

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(REPO, "animating-gaussian-splats_amd"), REPO]
import splat_affinity  # noqa: E402

print("pinned", splat_affinity.pin_host_threads(0, 0, 1, 8))
import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
with torch.autograd.set_multithreading_enabled(False):
    r = bench.c2_leg(60, 10, dev)
    print({k: r[k] for k in ("Msplats_per_s", "median_ms_per_step", "host_ms_per_step_median")})
    pr = cProfile.Profile()
    pr.enable()
    r = bench.c2_leg(200, 0, dev)
    pr.disable()
print({k: r[k] for k in ("Msplats_per_s", "median_ms_per_step", "host_ms_per_step_median")})
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(50)
