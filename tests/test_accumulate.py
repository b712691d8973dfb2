"""Gradient accumulation fused into the per-Gaussian backward kernel (gsr_grads.accumulate, ABI 6).

Summing several views' losses before one backward (train.py:413-418: 5 views per step; densify.py's
colour + segmentation renders of the same parameters) makes autograd accumulate each leaf's
gradient.  When a leaf already holds a gradient, the backward kernel adds into it in place and the
autograd Function returns None for it.  The result must be BITWISE what autograd's separate
AccumulateGrad add produces, for both the reference call-site Function and the fused-activation one;
a leaf with a hook is left to autograd (its hook must still run).
"""
import pytest
import torch

import splat_scenes as S
from diff_gaussian_rasterization import GaussianRasterizer, rasterize_parameters

pytestmark = pytest.mark.gpu


def _views(cuda, deg, W=128, H=96):
    cams = [S.render_settings(W, H, S.intrinsics(120.0, W, H), S.look_at(y, 0.2, 4.0), device=cuda,
                              sh_degree=deg) for y in (0.0, 35.0, 70.0)]
    return cams, [S.upstream_grad(H, W, seed=s, device=cuda) for s in (1, 2, 3)]


def _base(cuda, sh_degree=3, P=4000):
    p = S.synthetic_cloud(P, 0.03, sh_degree=sh_degree, seed=5, device="cpu")
    a = S.activated_inputs(p, sh_degree)
    if sh_degree >= 0:
        a.pop("colors_precomp")
    return p, {k: v.detach().to(cuda) for k, v in a.items()}


@pytest.mark.parametrize("sh_degree", [-1, 3])
def test_rasterizer_accumulates_bitwise(cuda, sh_degree):
    _, base = _base(cuda, sh_degree)
    cams, dls = _views(cuda, max(sh_degree, 0))
    sep = []
    for cam, dl in zip(cams, dls):  # each view alone (fresh leaves: no accumulation anywhere)
        lv = {k: v.clone().requires_grad_(True) for k, v in base.items()}
        GaussianRasterizer(raster_settings=cam)(**lv)[0].backward(dl)
        sep.append({k: v.grad for k, v in lv.items()})
    leaves = {k: v.clone().requires_grad_(True) for k, v in base.items()}
    calls = []
    leaves["opacities"].register_hook(lambda g: calls.append(1))  # hooked: stays on autograd's path
    for cam, dl in zip(cams, dls):
        GaussianRasterizer(raster_settings=cam)(**leaves)[0].backward(dl)
    assert len(calls) == 3
    for k, v in leaves.items():
        assert torch.equal(v.grad, (sep[0][k] + sep[1][k]) + sep[2][k]), k


def test_fused_parameters_accumulate_bitwise(cuda):
    p, _ = _base(cuda, -1)
    cams, dls = _views(cuda, 0)
    sep = []
    for cam, dl in zip(cams, dls):
        lv = {k: v.detach().to(cuda).requires_grad_(True) for k, v in p.items()}
        m2 = torch.zeros_like(lv["means"], requires_grad=True)
        rasterize_parameters(lv, cam, means2D=m2)[0].backward(dl)
        sep.append(({k: v.grad for k, v in lv.items()}, m2.grad))
    lv = {k: v.detach().to(cuda).requires_grad_(True) for k, v in p.items()}
    m2 = torch.zeros_like(lv["means"], requires_grad=True)
    for cam, dl in zip(cams, dls):
        rasterize_parameters(lv, cam, means2D=m2)[0].backward(dl)
    for k, v in lv.items():
        assert torch.equal(v.grad, (sep[0][0][k] + sep[1][0][k]) + sep[2][0][k]), k
    assert torch.equal(m2.grad, (sep[0][1] + sep[1][1]) + sep[2][1])


def test_autograd_grad_and_inputs_leave_grad_alone(cuda):
    """Stock autograd semantics: torch.autograd.grad returns the gradient and leaves .grad untouched;
    backward(inputs=[x]) writes only x.grad.  The in-place kernel accumulation must follow them."""
    _, base = _base(cuda, 3)
    cams, dls = _views(cuda, 3)
    ref = {k: v.clone().requires_grad_(True) for k, v in base.items()}
    GaussianRasterizer(raster_settings=cams[1])(**ref)[0].backward(dls[1])
    leaves = {k: v.clone().requires_grad_(True) for k, v in base.items()}
    GaussianRasterizer(raster_settings=cams[0])(**leaves)[0].backward(dls[0])
    before = {k: v.grad.clone() for k, v in leaves.items()}
    img = GaussianRasterizer(raster_settings=cams[1])(**leaves)[0]
    names = sorted(leaves)
    got = torch.autograd.grad(img, [leaves[k] for k in names], dls[1])
    for k, g in zip(names, got):
        assert torch.equal(leaves[k].grad, before[k]), k            # .grad untouched
        assert torch.equal(g, ref[k].grad), k                       # the gradient is returned
    img = GaussianRasterizer(raster_settings=cams[1])(**leaves)[0]
    img.backward(dls[1], inputs=[leaves["means3D"]])
    assert torch.equal(leaves["means3D"].grad, before["means3D"] + ref["means3D"].grad)
    for k in names:
        if k != "means3D":
            assert torch.equal(leaves[k].grad, before[k]), k
