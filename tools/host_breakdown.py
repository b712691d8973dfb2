"""Host time breakdown of the unchanged train.py step (one thread, current stream, non-leaf RGB, 5 views):
wall time of each library entry point (wrapped here, no library change) and of the whole forward /
backward, with the GPU idle at the start of each step (a device synchronisation first) so that host time
is not confused with waiting for the device, and again with the GPU busy (steady state).
usage (GPU box): python tools/host_breakdown.py [--no-async] [--no-view-streams]"""
import argparse
import collections
import functools
import os
import sys
import time

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(REPO, "animating-gaussian-splats_amd"), REPO]
import torch  # noqa: E402

import splat_scenes as S  # noqa: E402
import diff_gaussian_rasterization as dgr  # noqa: E402
from diff_gaussian_rasterization import GaussianRasterizer, _C  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--no-async", action="store_true")
ap.add_argument("--no-view-streams", action="store_true")
ap.add_argument("--steps", type=int, default=20)
args = ap.parse_args()
dgr.set_async_forward(not args.no_async)
# (library view streams removed in round 5)
T = collections.defaultdict(float)
N = collections.defaultdict(int)


def wrap(mod, name, tag=None):
    f = getattr(mod, name)

    @functools.wraps(f)
    def g(*a, **k):
        t = time.perf_counter()
        try:
            return f(*a, **k)
        finally:
            T[tag or name] += time.perf_counter() - t
            N[tag or name] += 1
    setattr(mod, name, g)


for n in ("_forward", "rasterize_gaussians_backward", "rasterize_gaussians_backward_render", "_camera", "_gaussians",
          "_grad_outputs"):
    wrap(_C, n)
_orig_resolve = _C.AsyncForward.resolve


def _res(self):
    t = time.perf_counter()
    try:
        return _orig_resolve(self)
    finally:
        T["AsyncForward.resolve"] += time.perf_counter() - t
        N["AsyncForward.resolve"] += 1


_C.AsyncForward.resolve = _res
for n in ("_on_view_stream", "rasterize_gaussians"):
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
dev = torch.device("cuda", 0)
_C.load_library()
base_cfg = S.CONFIGS["C3"]
cfg = S.SceneConfig("C3", base_cfg.P, base_cfg.width, base_cfg.height, base_cfg.focal, base_cfg.s0, views=S.RIG27)
cams = S.scene_cameras(cfg, device=dev)
dl = S.upstream_grad(cfg.height, cfg.width, device=dev)
base = S.synthetic_cloud(cfg.P, cfg.s0, sh_degree=-1, seed=0, device=dev)
delta = torch.zeros(cfg.P, 7, device=dev, requires_grad=True)
phase = collections.defaultdict(list)


def step(it, idle):
    if idle:
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    p = {k: v.clone() for k, v in base.items()}
    p["means"] = p["means"].detach()
    p["means"] += delta[:, :3] * 0.01
    p["rotation_quaternions"] = p["rotation_quaternions"].detach()
    p["rotation_quaternions"] += delta[:, 3:] * 0.01
    t1 = time.perf_counter()
    losses = []
    for k in range(5):
        ci = (it * 5 + k) % len(cams)
        a = S.render_arguments(p)
        t2 = time.perf_counter()
        img = GaussianRasterizer(raster_settings=cams[ci])(**a)[0]
        t3 = time.perf_counter()
        losses.append((img * dl).sum())
        phase["render_arguments"].append(t2 - (t1 if k == 0 else t_prev))
        phase["rasterizer_call"].append(t3 - t2)
        t_prev = time.perf_counter()
    loss = torch.stack(losses).sum(dim=0)
    t4 = time.perf_counter()
    loss.backward()
    t5 = time.perf_counter()
    delta.grad = None
    phase["step_setup"].append(t1 - t0)
    phase["forward_total"].append(t4 - t1)
    phase["backward_total"].append(t5 - t4)
    phase["step"].append(t5 - t0)


for it in range(5):
    step(it, False)
for mode in ("idle", "busy"):
    T.clear(); N.clear(); phase.clear()
    torch.cuda.synchronize()
    for it in range(args.steps):
        step(10 + it, mode == "idle")
    torch.cuda.synchronize()
    print(f"== {mode} GPU at step start (async={not args.no_async}); "
          f"ms per step (median of phases, totals per step)")
    for k, v in phase.items():
        v = sorted(v)
        per = len(v) // args.steps
        print(f"  {k:22s} median {v[len(v) // 2] * 1e3:8.3f} ms x {per}/step")
    for k in sorted(T, key=lambda k: -T[k]):
        print(f"  {k:38s} {T[k] / args.steps * 1e3:8.3f} ms/step  ({N[k] // args.steps}/step, "
              f"{T[k] / max(N[k], 1) * 1e6:7.1f} us/call)")
