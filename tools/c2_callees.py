"""cProfile of the C2 leg: the library binding's Python functions and what they call (diagnostic).
usage (GPU box): python tools/c2_callees.py"""
import cProfile
import io
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
bench.c2_leg(50, 10, dev)
pr = cProfile.Profile()
pr.enable()
r = bench.c2_leg(200, 0, dev)
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(60)
s = io.StringIO()
st2 = pstats.Stats(pr, stream=s)
st2.sort_stats("tottime").print_callees("_forward|rasterize_gaussians_backward_render|rasterize_gaussians_backward_views|_try_defer|_run_group|__init__.py:.*\\(forward\\)|__init__.py:.*\\(backward\\)")
print(s.getvalue()[:20000])
