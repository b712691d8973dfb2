"""How far the fast forward's transmittance drifts from the oracle's (the T >= 1e-4
saturation test): per view, over pixels with the same n_contrib, |T_gpu / T_oracle - 1|, and the share of
pixels a relative window w around 1e-4 would send to an exact re-walk (T_gpu < 1e-4 (1 + w)).
usage (GPU box): python tools/t_drift.py [C3|C4|C2] [views]"""
import os
import sys

import numpy as np
import torch

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(REPO, "animating-gaussian-splats_amd"), REPO, os.path.join(REPO, "tests")]
import splat_scenes as S  # noqa: E402
from test_gpu_parity import _gpu_forward, _ora_forward, _np  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "C3"
nviews = int(sys.argv[2]) if len(sys.argv) > 2 else 2
cfg = S.CONFIGS[name]
dev = torch.device("cuda", 0)
p = S.synthetic_cloud(cfg.P, cfg.s0, sh_degree=cfg.sh_degree, seed=0, device="cpu")
a = {k: (v.detach() if isinstance(v, torch.Tensor) else v) for k, v in S.activated_inputs(p, cfg.sh_degree).items()}
if cfg.sh_degree >= 0:
    a.pop("colors_precomp")
cams = S.scene_cameras(cfg, device="cpu")
for ci in range(min(nviews, len(cams))):
    rs = cams[ci]
    fw = _gpu_forward(a, rs, dev)
    st = _ora_forward(a, rs)
    tg = _np(fw["dec"]["pix_end"])[..., 3].astype(np.float64)
    ng = _np(fw["dec"]["n_contrib"]).astype(np.int64)
    to = st["final_T"].astype(np.float64)
    no = st["n_contrib"].astype(np.int64)
    same = ng == no
    rel = np.abs(tg / np.maximum(to, 1e-30) - 1.0)[same]
    sat = to[same] < 1e-3
    print(f"{name} view {ci}: re-walked pixels {int(_np(fw['dec']['tsat_count'])[0])}, "
          f"nf max {int(ng.max())}")
    print(f"{name} view {ci}: pixels {tg.size}, n_contrib differ {int((~same).sum())}, "
          f"max rel T drift {rel.max():.3g} (T<1e-3: {rel[sat].max() if sat.any() else 0:.3g}), "
          f"p99.99 {np.quantile(rel, 0.9999):.3g}; T<1e-3 share {sat.mean():.3f}")
    for w in (1e-4, 3e-4, 1e-3, 3e-3):
        print(f"   w={w:g}: flagged share {(tg < 1e-4 * (1 + w)).mean():.2e} (T_gpu < 1e-4 (1 + w))")
    if (~same).any():
        i = np.nonzero(~same)
        print("   differing pixels: T_gpu", tg[i][:5], "T_ora", to[i][:5], "n", ng[i][:5], no[i][:5])
