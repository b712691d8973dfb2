"""cProfile of the host side of the unchanged train.py step (bench.unchanged_call_site's step body: one
thread, torch's current stream, non-leaf RGB inputs, 5 views, summed losses, one backward).

usage (GPU box): python tools/unchanged_profile.py [--no-async] [--no-view-streams] [--steps N]"""
import argparse
import cProfile
import os
import pstats
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
ap.add_argument("--P", type=int, default=1_000_000)
args = ap.parse_args()
dgr.set_async_forward(not args.no_async)
# (library view streams removed in round 5)
dev = torch.device("cuda", 0)
_C.load_library()
base_cfg = S.CONFIGS["C3"]
cfg = S.SceneConfig("C3", args.P, base_cfg.width, base_cfg.height, base_cfg.focal, base_cfg.s0, views=S.RIG27)
cams = S.scene_cameras(cfg, device=dev)
dl = S.upstream_grad(cfg.height, cfg.width, device=dev)
base = S.synthetic_cloud(cfg.P, cfg.s0, sh_degree=-1, seed=0, device=dev)
delta = torch.zeros(cfg.P, 7, device=dev, requires_grad=True)


def step(it):
    p = {k: v.clone() for k, v in base.items()}
    p["means"] = p["means"].detach()
    p["means"] += delta[:, :3] * 0.01
    p["rotation_quaternions"] = p["rotation_quaternions"].detach()
    p["rotation_quaternions"] += delta[:, 3:] * 0.01
    views = [(it * 5 + k) % len(cams) for k in range(5)]
    losses = torch.stack([(GaussianRasterizer(raster_settings=cams[ci])(**S.render_arguments(p))[0] * dl).sum()
                          for ci in views])
    losses.sum(dim=0).backward()
    delta.grad = None


for it in range(5):
    step(it)
torch.cuda.synchronize()
t = time.perf_counter()
for it in range(args.steps):
    step(5 + it)
host = (time.perf_counter() - t) / args.steps * 1e3
torch.cuda.synchronize()
wall = (time.perf_counter() - t) / args.steps * 1e3
# GPU-free host cost: the same step with the GPU idle (synchronise before each step, time the host part)
hs = []
for it in range(args.steps):
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    step(100 + it)
    hs.append((time.perf_counter() - t1) * 1e3)
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
for it in range(args.steps):
    step(200 + it)
torch.cuda.synchronize()
pr.disable()
print(f"async={not args.no_async}: wall {wall:.3f} ms/step, submission "
      f"{host:.3f} ms/step, host from an idle GPU {sorted(hs)[len(hs) // 2]:.3f} ms/step (median)")
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(30)
st.sort_stats("cumulative").print_stats(35)
