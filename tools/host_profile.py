"""cProfile of the host side of one summed multi-view step (GPU box, one thread, one stream): where
the Python / ctypes time of the drop-in module goes when the GPU work per view is small (C2: 100k
Gaussians, 4 x 800x800).  usage: python tools/host_profile.py [C2|C3] [steps]"""
import cProfile
import os
import pstats
import sys
import time

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "animating-gaussian-splats_amd")]
import torch  # noqa: E402

import splat_scenes as S  # noqa: E402
from diff_gaussian_rasterization import GaussianRasterizer, _C  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "C2"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
dev = torch.device("cuda", 0)
_C.load_library()
cfg = S.CONFIGS[name]
cams = S.scene_cameras(cfg, device=dev)
p = S.synthetic_cloud(cfg.P, cfg.s0, sh_degree=cfg.sh_degree, seed=0, device=dev)
with torch.no_grad():
    act = S.activated_inputs(p, cfg.sh_degree)
if cfg.sh_degree >= 0:
    act.pop("colors_precomp")
leaves = {k: v.detach().clone().requires_grad_(True) for k, v in act.items() if k != "means2D"}
dl = S.upstream_grad(cfg.height, cfg.width, device=dev)
views = list(range(min(len(cams), 5 if name != "C2" else 4)))


def step():
    imgs = []
    for ci in views:
        m2 = torch.zeros_like(leaves["means3D"], requires_grad=True)
        imgs.append(GaussianRasterizer(raster_settings=cams[ci])(**leaves, means2D=m2)[0])
    torch.autograd.backward(imgs, [dl] * len(imgs))
    for v in leaves.values():
        v.grad = None


for _ in range(5):
    step()
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(steps):
    step()
torch.cuda.synchronize()
wall = (time.perf_counter() - t) / steps * 1e3
pr = cProfile.Profile()
pr.enable()
for _ in range(steps):
    step()
torch.cuda.synchronize()
pr.disable()
print(f"{name}: {len(views)} views per step, wall {wall:.3f} ms per step ({wall / len(views):.3f} ms per view), one thread")
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(25)
st.sort_stats("cumulative").print_stats(30)
