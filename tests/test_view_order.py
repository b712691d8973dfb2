"""The deferred multi-view per-Gaussian pass sums a backward pass's views in an order fixed by their
cameras (gsr_backward.hip view_order), not in the order the pass queued them (a
caller whose threads finish their forwards in a varying order would otherwise get last-bit differences
in the summed gradients from run to run)."""
import pytest
import torch

import splat_scenes as S
from diff_gaussian_rasterization import GaussianRasterizer

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("sh_degree", [3, -1])
def test_summed_pass_independent_of_queue_order(sh_degree, cuda):
    P, W, H = 60_000, 320, 240
    p = S.synthetic_cloud(P, 0.01, sh_degree=max(sh_degree, 0), seed=7, device=cuda)
    a = S.activated_inputs(p, sh_degree)
    if sh_degree >= 0:
        a.pop("colors_precomp")
    cfg = [(0, -0.6), (50, 0.0), (100, 0.6), (150, -0.3), (200, 0.3)]
    cams = [S.render_settings(W, H, S.intrinsics(280.0, W, H), S.look_at(yaw, h, 4), device=cuda,
                              sh_degree=sh_degree) for yaw, h in cfg]
    dls = [S.upstream_grad(H, W, seed=10 + k, device=cuda) for k in range(len(cams))]

    def run(order):  # the summed losses of five views, one backward (train.py:753-767)
        leaves = {k: v.detach().clone().requires_grad_(True) for k, v in a.items()}
        imgs = [GaussianRasterizer(raster_settings=cams[k])(**leaves)[0] for k in order]
        torch.autograd.backward(imgs, [dls[k] for k in order])
        torch.cuda.synchronize()
        return {k: v.grad.clone() for k, v in leaves.items()}

    g1 = run([0, 1, 2, 3, 4])
    g2 = run([4, 2, 0, 3, 1])
    for k in g1:
        assert torch.isfinite(g1[k]).all(), k
        assert torch.equal(g1[k], g2[k]), (k, (g1[k] - g2[k]).abs().max().item())


def test_same_pose_other_intrinsics_independent_of_queue_order(cuda):
    """Views that share a pose but not their intrinsics or image size (the key now hashes the
    projection matrix and W, H too) are ordered by the camera as well.  The one remaining tie -- the
    same camera passed twice in one launch -- keeps queue order (include/gsr.h, gsr_backward_render)."""
    P = 60_000
    p = S.synthetic_cloud(P, 0.01, sh_degree=3, seed=8, device=cuda)
    a = S.activated_inputs(p, 3)
    a.pop("colors_precomp")
    pose = S.look_at(40, 0.2, 4)
    dims = [(320, 240, 280.0), (320, 240, 200.0), (256, 192, 280.0), (320, 240, 360.0)]
    cams = [S.render_settings(W, H, S.intrinsics(f, W, H), pose, device=cuda, sh_degree=3) for W, H, f in dims]
    dls = [S.upstream_grad(H, W, seed=20 + k, device=cuda) for k, (W, H, _) in enumerate(dims)]

    def run(order):
        leaves = {k: v.detach().clone().requires_grad_(True) for k, v in a.items()}
        imgs = [GaussianRasterizer(raster_settings=cams[k])(**leaves)[0] for k in order]
        torch.autograd.backward(imgs, [dls[k] for k in order])
        torch.cuda.synchronize()
        return {k: v.grad.clone() for k, v in leaves.items()}

    g1 = run([0, 1, 2, 3])
    g2 = run([3, 1, 0, 2])
    for k in g1:
        assert torch.isfinite(g1[k]).all(), k
        assert torch.equal(g1[k], g2[k]), (k, (g1[k] - g2[k]).abs().max().item())
