"""Host time of train.py's call site (GPU box): one thread, 5 views per step, RGB, frozen Gaussians,
means / rotations = detach + 0.01 delta, per-view create_render_arguments, summed backward (as
bench.train_call_site, without the stream threads).  Splits each step's host time into the
rasterizer Functions' forward / backward (Python + native) and everything else (torch ops of the
caller and the autograd engine)."""
import os
import sys
import time

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "animating-gaussian-splats_amd")]
import torch  # noqa: E402

import splat_scenes as S  # noqa: E402
import diff_gaussian_rasterization as D  # noqa: E402
from diff_gaussian_rasterization import GaussianRasterizer, _C  # noqa: E402

dev = torch.device("cuda", 0)
_C.load_library()
cfg = S.CONFIGS["C3"]
cfg = S.SceneConfig("C3", cfg.P, cfg.width, cfg.height, cfg.focal, cfg.s0, sh_degree=cfg.sh_degree, views=S.RIG27)
cams = S.scene_cameras(cfg, device=dev)
dl = S.upstream_grad(cfg.height, cfg.width, device=dev)
base = S.synthetic_cloud(cfg.P, cfg.s0, sh_degree=-1, seed=0, device=dev)
delta = torch.zeros(cfg.P, 7, device=dev, requires_grad=True)
acc = {"fwd": 0.0, "bwd": 0.0, "bwd_c": 0.0}
of, ob, oc = D._RasterizeGaussians.forward, D._RasterizeGaussians.backward, D._C.rasterize_gaussians_backward


def tf(ctx, *a):
    t = time.perf_counter(); r = of(ctx, *a); acc["fwd"] += time.perf_counter() - t; return r


def tb(ctx, *g):
    t = time.perf_counter(); r = ob(ctx, *g); acc["bwd"] += time.perf_counter() - t; return r


def tc(*a, **k):
    t = time.perf_counter(); r = oc(*a, **k); acc["bwd_c"] += time.perf_counter() - t; return r


D._RasterizeGaussians.forward = staticmethod(tf)
D._RasterizeGaussians.backward = staticmethod(tb)
D._C.rasterize_gaussians_backward = tc


def step(it):
    p = dict(base)
    p["means"] = base["means"].clone()
    p["means"] += delta[:, :3] * 0.01
    p["rotation_quaternions"] = base["rotation_quaternions"].clone()
    p["rotation_quaternions"] += delta[:, 3:] * 0.01
    imgs = [GaussianRasterizer(raster_settings=cams[(it * 5 + k) % 27])(**S.render_arguments(p))[0] for k in range(5)]
    torch.autograd.backward(imgs, [dl] * 5)
    delta.grad = None


for it in range(5):
    step(it)
torch.cuda.synchronize()
for k in acc:
    acc[k] = 0.0
_C.profile_reset()
_C.profile_enable(True)
_C.profile_select(["none"])
n = 30
t = time.perf_counter()
for it in range(n):
    step(5 + it)
host = (time.perf_counter() - t) / n
torch.cuda.synchronize()
wall = (time.perf_counter() - t) / n
_C.profile_enable(False)
ph = {k: _C.profile_read(k) for k in ("host_forward", "host_wait_K", "host_backward")}
print(f"per step: wall {wall * 1e3:.3f} ms, host submission {host * 1e3:.3f} ms "
      f"({5 * cfg.P / wall / 1e6:.0f} Msplats/s)")
print(f"  rasterizer forward {acc['fwd'] / n * 1e3:.3f} ms (native {ph['host_forward'][0] / n:.3f}, of it waiting for K "
      f"{ph['host_wait_K'][0] / n:.3f}), backward {acc['bwd'] / n * 1e3:.3f} ms (the _C call {acc['bwd_c'] / n * 1e3:.3f}, "
      f"native {ph['host_backward'][0] / n:.3f}); the rest {(host - (acc['fwd'] + acc['bwd']) / n) * 1e3:.3f} ms")
