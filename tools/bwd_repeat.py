"""One C3 view forward, then its backward repeated N times (retain_graph) -- a short program for
per-kernel counters / PC sampling of k_render_bwd.  usage (GPU box): python tools/bwd_repeat.py [N]"""
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "animating-gaussian-splats_amd")]
import torch  # noqa: E402

import splat_scenes as S  # noqa: E402
from diff_gaussian_rasterization import GaussianRasterizer, _C  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dev = torch.device("cuda", 0)
_C.load_library()
cfg = S.CONFIGS["C3"]
cfg = S.SceneConfig("C3", cfg.P, cfg.width, cfg.height, cfg.focal, cfg.s0, views=S.RIG27)
cams = S.scene_cameras(cfg, device=dev)
p = S.synthetic_cloud(cfg.P, cfg.s0, sh_degree=-1, seed=0, device=dev)
with torch.no_grad():
    a = S.activated_inputs(p, -1)
leaves = {k: v.detach().clone().requires_grad_(True) for k, v in a.items() if v is not None}
dl = S.upstream_grad(cfg.height, cfg.width, device=dev)
img = GaussianRasterizer(raster_settings=cams[0])(**leaves)[0]
ins = list(leaves.values())
for _ in range(n):
    torch.autograd.grad(img, ins, dl, retain_graph=True, allow_unused=True)
torch.cuda.synchronize()
print("done", n)
