"""gsr_bind against the ctypes path on the same forward calls (diagnostic): outputs and the three
workspaces' bytes must be identical.  usage (GPU box): python tools/native_vs_ctypes.py"""
import os
import sys

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(REPO, "animating-gaussian-splats_amd"), REPO]
import torch  # noqa: E402

import splat_scenes as S  # noqa: E402
from diff_gaussian_rasterization import _C  # noqa: E402

cuda = torch.device("cuda", 0)
cfg = S.CONFIGS["C2"]
p = S.synthetic_cloud(cfg.P, cfg.s0, sh_degree=-1, seed=0, device=cuda)
a = S.activated_inputs(p, -1)
cams = S.scene_cameras(cfg, device=cuda)
e = torch.empty(0, device=cuda)


def fwd(rs, mode, spec):
    _C._NATIVE_PARTS = 15 if mode == "nat" else 0
    info = {}
    out = _C.rasterize_gaussians(rs.bg, a["means3D"], a["colors_precomp"], a["opacities"], a["scales"], a["rotations"],
                                 1.0, e, rs.viewmatrix, rs.projmatrix, rs.tanfovx, rs.tanfovy, rs.image_height,
                                 rs.image_width, e, 0, rs.campos, False, prepare_backward=True, speculate=spec,
                                 info=info)
    torch.cuda.synchronize()
    return out, info


for it in range(3):
    for ci, rs in enumerate(cams):
        (o1, i1), (o2, i2) = fwd(rs, "py", True), fwd(rs, "nat", True)
        same = [o1[0] == o2[0], torch.equal(o1[1], o2[1]), torch.equal(o1[2], o2[2]), torch.equal(o1[6], o2[6])]
        bufs = []
        for k in (3, 4, 5):
            x, y = o1[k], o2[k]
            n = min(x.numel(), y.numel())
            bufs.append((x.numel(), y.numel(), int((x[:n] != y[:n]).sum())))
        print(it, ci, "K", o1[0], o2[0], "layout", i1["binning_layout"], i2["binning_layout"], "spec",
              i1["speculated"], i2["speculated"], "same", same, "geom/binning/image (n1, n2, differing bytes)", bufs,
              flush=True)
