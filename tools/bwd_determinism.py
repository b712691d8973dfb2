"""One view forward, its backward repeated N times: every repeat must be bitwise equal (a race in the
backward kernels shows as run-to-run differences).  usage (GPU box): python tools/bwd_determinism.py [C3|C4|C2] [N]"""
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "animating-gaussian-splats_amd")]
import torch  # noqa: E402

import splat_scenes as S  # noqa: E402
from diff_gaussian_rasterization import GaussianRasterizer, _C  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "C3"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 5
dev = torch.device("cuda", 0)
_C.load_library()
cfg = S.CONFIGS[name]
cams = S.scene_cameras(cfg, device=dev)
p = S.synthetic_cloud(cfg.P, cfg.s0, sh_degree=-1, seed=0, device=dev)
with torch.no_grad():
    a = S.activated_inputs(p, -1)
leaves = {k: v.detach().clone().requires_grad_(True) for k, v in a.items() if v is not None}
dl = S.upstream_grad(cfg.height, cfg.width, device=dev)
for ci in range(min(3, len(cams))):
    img = GaussianRasterizer(raster_settings=cams[ci])(**leaves)[0]
    ins = [v for k, v in leaves.items()]
    ref = None
    for r in range(n):
        g = torch.autograd.grad(img, ins, dl, retain_graph=True, allow_unused=True)
        g = [x.clone() if x is not None else None for x in g]
        if ref is None:
            ref = g
            continue
        for k, x, y in zip(leaves, ref, g):
            if x is None:
                continue
            d = (x != y).sum().item()
            if d:
                print(f"{name} cam {ci} repeat {r}: {k} {d} values differ, max {(x - y).abs().max().item():.3g}")
torch.cuda.synchronize()
print("done", name, n)
