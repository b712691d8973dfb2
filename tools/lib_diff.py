"""Dump one summed multi-view step's outputs (images, every leaf gradient) for a bitwise comparison of
two libgsr builds (GSR_LIB).  usage (GPU box): python tools/lib_diff.py OUT.pt [C3|C4] [views] [streams]"""
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "animating-gaussian-splats_amd")]
import torch  # noqa: E402

import splat_scenes as S  # noqa: E402
import splat_step  # noqa: E402
from diff_gaussian_rasterization import _C  # noqa: E402

out, name = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "C4"
nv = int(sys.argv[3]) if len(sys.argv) > 3 else 27
ns = int(sys.argv[4]) if len(sys.argv) > 4 else 3
dev = torch.device("cuda", 0)
_C.load_library()
cfg = S.CONFIGS[name]
cfg = S.SceneConfig(name, cfg.P, cfg.width, cfg.height, cfg.focal, cfg.s0, sh_degree=cfg.sh_degree, views=S.RIG27)
p = S.synthetic_cloud(cfg.P, cfg.s0, sh_degree=cfg.sh_degree, seed=0, device=dev)
with torch.no_grad():
    act = S.activated_inputs(p, cfg.sh_degree)
if cfg.sh_degree >= 0:
    act.pop("colors_precomp")
leaves = {k: v.detach().clone().requires_grad_(True) for k, v in act.items()}
cams = S.scene_cameras(cfg, device=dev)
streams = [torch.cuda.Stream() for _ in range(ns)]
for s in streams:
    s.wait_stream(torch.cuda.current_stream())
step = splat_step.RenderStep(dev, cams, lambda ci: leaves, S.upstream_grad(cfg.height, cfg.width, device=dev),
                             streams, threads=ns > 1)
imgs = step(list(range(nv)))
step.close()
torch.cuda.synchronize()
torch.save({"imgs": [i.cpu() for i in imgs], "grads": {k: v.grad.cpu() for k, v in leaves.items()}}, out)
print("saved", out)
