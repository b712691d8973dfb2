"""The exact saturation re-walk on one view: how many pixels k_render_fwd flagged (the
IMAGE counter), how many final T lie near 1e-4, and the re-walk's kernel time (run under rocprofv3
--kernel-trace).  usage (GPU box): python tools/tsat_probe.py [C3|C4|C2|C3M] [reps]"""
import os
import sys

import numpy as np
import torch

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(REPO, "animating-gaussian-splats_amd"), REPO, os.path.join(REPO, "tests")]
import splat_scenes as S  # noqa: E402
from test_gpu_parity import _gpu_forward, _np  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "C3"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
cfg = S.CONFIGS["C3" if name == "C3M" else name]
dev = torch.device("cuda", 0)
p = (S.clustered_cloud if name == "C3M" else S.synthetic_cloud)(cfg.P, cfg.s0, sh_degree=cfg.sh_degree, seed=0,
                                                              device="cpu")
a = {k: (v.detach() if isinstance(v, torch.Tensor) else v) for k, v in S.activated_inputs(p, cfg.sh_degree).items()}
if cfg.sh_degree >= 0:
    a.pop("colors_precomp")
rs = S.scene_cameras(cfg, device="cpu")[0]
for r in range(reps):
    fw = _gpu_forward(a, rs, dev)
    torch.cuda.synchronize()
    T = _np(fw["dec"]["pix_end"])[..., 3]
    nc = _np(fw["dec"]["n_contrib"])
    print(f"{name} rep {r}: flagged {int(_np(fw['dec']['tsat_count'])[0])}, final T in [0.99e-4, 1.01e-4): "
          f"{int(((T >= 0.99e-4) & (T < 1.01e-4)).sum())}, T < 1e-4: {int((T < 1e-4).sum())}, "
          f"n_contrib max {int(nc.max())}, K {fw['K']}")
