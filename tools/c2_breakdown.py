"""Wall time of the library's entry points inside the C2 leg (bench.c2_leg: 4 x 800x800 views, 100k
Gaussians, one thread, 3 streams), per step; the engine thread's calls included.
usage (GPU box): python tools/c2_breakdown.py"""
import collections
import functools
import os
import sys
import time

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(REPO, "animating-gaussian-splats_amd"), REPO]
import torch  # noqa: E402

import bench  # noqa: E402
import diff_gaussian_rasterization as dgr  # noqa: E402
from diff_gaussian_rasterization import _C  # noqa: E402

T = collections.defaultdict(float)
N = collections.defaultdict(int)


def wrap(mod, name, tag):
    f = getattr(mod, name)

    @functools.wraps(f)
    def g(*a, **k):
        t = time.perf_counter()
        try:
            return f(*a, **k)
        finally:
            T[tag] += time.perf_counter() - t
            N[tag] += 1
    setattr(mod, name, g)


for n in ("_forward", "rasterize_gaussians_backward_render", "rasterize_gaussians_backward_views", "_gaussians",
          "_camera"):
    wrap(_C, n, "_C." + n)
for n in ("_try_defer", "_flush_pending", "_run_group", "_accumulation_target", "_fresh_target", "_input_nodes"):
    wrap(dgr, n, "dgr." + n)
bw = dgr._RasterizeGaussians.backward


def bwrap(ctx, *g):
    t = time.perf_counter()
    try:
        return bw(ctx, *g)
    finally:
        T["Function.backward"] += time.perf_counter() - t
        N["Function.backward"] += 1


dgr._RasterizeGaussians.backward = staticmethod(bwrap)
fw = dgr._RasterizeGaussians.forward


def fwrap(ctx, *a):
    t = time.perf_counter()
    try:
        return fw(ctx, *a)
    finally:
        T["Function.forward"] += time.perf_counter() - t
        N["Function.forward"] += 1


dgr._RasterizeGaussians.forward = staticmethod(fwrap)
dev = torch.device("cuda", 0)
L = _C.load_library()
for n in ("gsr_forward_async", "gsr_forward_info_call", "gsr_backward_render", "gsr_backward_gaussians",
          "gsr_forward_resolve"):  # the C calls themselves (kernel launches + host logic)
    wrap(L, n, "C." + n)
torch.zeros(1, device=dev)
import splat_affinity  # noqa: E402
print("pinned", splat_affinity.pin_host_threads(0, 0, 1, 8))
bench.c2_leg(30, 10, dev)
T.clear(); N.clear()
steps = 200
t0 = time.perf_counter()
r = bench.c2_leg(steps, 0, dev)
print({k: r[k] for k in ("Msplats_per_s", "median_ms_per_step", "host_ms_per_step_median")})
for k in sorted(T, key=lambda k: -T[k]):
    print(f"  {k:45s} {T[k] / steps * 1e3:8.3f} ms/step  ({N[k] / steps:.1f}/step, {T[k] / max(N[k], 1) * 1e6:7.1f} us/call)")
