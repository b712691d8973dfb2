"""Deferred multi-view per-Gaussian backward (ABI 12: gsr_backward_render + gsr_backward_gaussians).

A backward pass over several views of the same leaves (train.py:753-767: 5 view losses summed, one
backward) runs each view's per-pixel half in its node and ONE per-Gaussian pass over all views at
the end of the pass.  The gradients must equal the immediate per-view path's (the views' fp32
contributions are grouped differently: summed first, then added once) -- checked here against
``set_deferred_backward(False)`` and against the per-view C-ABI sums, for every SH coefficient count,
precomputed colours / covariances, fused activations, > 8 views (two launch groups), two streams,
existing and absent .grad, and the cases that must NOT defer (autograd.grad, non-leaf inputs)."""
import pytest
import torch

import splat_scenes as S
from diff_gaussian_rasterization import GaussianRasterizer, _C, rasterize_parameters, set_deferred_backward

pytestmark = pytest.mark.gpu

P, W, H = 30_000, 320, 240


def _close(name, got, ref, rtol=1e-4, atol_frac=1e-6):
    got, ref = got.double(), ref.double()
    tol = rtol * ref.abs() + atol_frac * float(ref.abs().max()) + 1e-12
    bad = ((got - ref).abs() > tol).sum().item()
    assert bad == 0, f"{name}: {bad} of {ref.numel()} values off (max err {(got - ref).abs().max().item():.3e})"


def _cams(dev, n, sh=3):
    cfg = [(yaw, h) for h in (-0.6, 0.0, 0.6) for yaw in (0, 45, 90, 135)][:n]
    return [S.render_settings(W, H, S.intrinsics(280.0, W, H), S.look_at(yaw, h, 4), device=dev, sh_degree=sh)
            for yaw, h in cfg]


def _inputs(dev, kind):
    deg = {"sh3": 3, "sh2": 2, "sh1": 1, "sh0": 0}.get(kind, -1)
    p = S.synthetic_cloud(P, 0.012, sh_degree=deg, seed=11, device=dev)
    a = S.activated_inputs(p, deg)
    if deg >= 0:
        a.pop("colors_precomp")
    if kind == "cov3d":
        s, q = a.pop("scales"), a.pop("rotations")
        qn = torch.nn.functional.normalize(q, dim=-1)
        w, x, y, z = qn.unbind(-1)
        R = torch.stack([1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y),
                         2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x),
                         2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)], -1).view(-1, 3, 3)
        M = R * s[:, None, :]
        cov = M @ M.transpose(1, 2)
        a["cov3D_precomp"] = torch.stack([cov[:, 0, 0], cov[:, 0, 1], cov[:, 0, 2], cov[:, 1, 1], cov[:, 1, 2],
                                          cov[:, 2, 2]], -1).contiguous()
    return a, max(deg, 0)


def _leaves(a):
    return {k: v.detach().clone().requires_grad_(True) for k, v in a.items() if v is not None}


def _views_loss(leaves, cams, dls, streams=None):
    imgs = []
    main = torch.cuda.current_stream()
    for k, cam in enumerate(cams):
        s = streams[k % len(streams)] if streams else main
        with torch.cuda.stream(s):
            img, _, _ = GaussianRasterizer(raster_settings=cam)(**leaves)
            imgs.append(img)
    if streams:
        for s in streams:
            main.wait_stream(s)
    return sum((img * dl).sum() for img, dl in zip(imgs, dls))


def _run(a, cams, dls, deferred, pre_grad=None, streams=None):
    leaves = _leaves(a)
    if pre_grad is not None:
        for k, v in leaves.items():
            v.grad = pre_grad[k].clone()
    prev = set_deferred_backward(deferred)
    try:
        _views_loss(leaves, cams, dls, streams).backward()
    finally:
        set_deferred_backward(prev)
    torch.cuda.synchronize()
    return {k: v.grad.clone() for k, v in leaves.items() if v.grad is not None}


@pytest.mark.parametrize("kind", ["sh3", "sh2", "sh1", "sh0", "rgb", "cov3d"])
def test_deferred_equals_immediate(kind, cuda):
    a, deg = _inputs(cuda, kind)
    cams = _cams(cuda, 5, deg)
    dls = [S.upstream_grad(H, W, seed=20 + k, device=cuda) for k in range(len(cams))]
    ref = _run(a, cams, dls, deferred=False)
    got = _run(a, cams, dls, deferred=True)
    assert set(ref) == set(got)
    for k in ref:
        _close(k, got[k], ref[k])


def test_deferred_accumulates_into_existing_grad_and_splits_groups(cuda):
    """Ten views (two launch groups of <= 8) into pre-existing gradients: old + sum of the views."""
    a, deg = _inputs(cuda, "sh3")
    cams = _cams(cuda, 10, deg)
    dls = [S.upstream_grad(H, W, seed=40 + k, device=cuda) for k in range(len(cams))]
    g = torch.Generator(device=cuda).manual_seed(3)
    pre = {k: torch.randn(v.shape, device=cuda, generator=g) * 1e-3 for k, v in _leaves(a).items()}
    ref = _run(a, cams, dls, deferred=False, pre_grad=pre)
    got = _run(a, cams, dls, deferred=True, pre_grad=pre)
    for k in ref:
        _close(k, got[k], ref[k])


def test_deferred_two_streams(cuda):
    a, deg = _inputs(cuda, "sh3")
    cams = _cams(cuda, 6, deg)
    dls = [S.upstream_grad(H, W, seed=60 + k, device=cuda) for k in range(len(cams))]
    ref = _run(a, cams, dls, deferred=True)
    streams = [torch.cuda.Stream() for _ in range(2)]
    for s in streams:
        s.wait_stream(torch.cuda.current_stream())
    got = _run(a, cams, dls, deferred=True, streams=streams)
    for k in ref:
        assert torch.equal(got[k], ref[k]), k  # same kernels, same order: bitwise


def test_deferred_rasterize_parameters(cuda):
    p = S.synthetic_cloud(P, 0.012, sh_degree=3, seed=12, device=cuda)
    cams = _cams(cuda, 5, 3)
    dls = [S.upstream_grad(H, W, seed=80 + k, device=cuda) for k in range(len(cams))]

    def run(deferred):
        params = {k: v.detach().clone().requires_grad_(True) for k, v in p.items()}
        m2 = torch.zeros_like(params["means"], requires_grad=True)
        prev = set_deferred_backward(deferred)
        try:
            loss = sum((rasterize_parameters(params, c, means2D=m2, shs=params["shs"])[0] * dl).sum()
                       for c, dl in zip(cams, dls))
            loss.backward()
        finally:
            set_deferred_backward(prev)
        torch.cuda.synchronize()
        out = {k: v.grad.clone() for k, v in params.items() if v.grad is not None}
        out["means2D"] = m2.grad.clone()
        return out

    ref, got = run(False), run(True)
    assert set(ref) == set(got)
    for k in ref:
        _close(k, got[k], ref[k])


def test_not_deferred_for_autograd_grad_and_non_leaves(cuda):
    """torch.autograd.grad returns the gradients and leaves .grad alone; non-leaf inputs (the
    reference's activated render arguments) get their gradients through autograd as usual."""
    a, deg = _inputs(cuda, "sh3")
    cams = _cams(cuda, 3, deg)
    dls = [S.upstream_grad(H, W, seed=90 + k, device=cuda) for k in range(len(cams))]
    ref = _run(a, cams, dls, deferred=False)
    leaves = _leaves(a)
    sentinel = torch.full_like(leaves["means3D"], 7.0)
    leaves["means3D"].grad = sentinel.clone()
    names = list(leaves)
    gs = torch.autograd.grad(_views_loss(leaves, cams, dls), [leaves[k] for k in names])
    torch.cuda.synchronize()
    assert torch.equal(leaves["means3D"].grad, sentinel)
    for k, g in zip(names, gs):
        _close(k, g, ref[k])
    # non-leaf inputs: every activated argument derived from one leaf set through autograd ops
    base = _leaves(a)
    nonleaf = {k: v * 1.0 for k, v in base.items()}
    _views_loss(nonleaf, cams, dls).backward()
    torch.cuda.synchronize()
    for k in ref:
        _close(k, base[k].grad, ref[k])


def test_views_abi_matches_per_view_sum(cuda):
    """C-ABI level: gsr_backward_gaussians over 3 views == the sum of gsr_backward per view, with
    each view's dL/dmeans2D in its own array."""
    a, deg = _inputs(cuda, "sh3")
    cams = _cams(cuda, 3, deg)
    dls = [S.upstream_grad(H, W, seed=100 + k, device=cuda) for k in range(len(cams))]
    e = torch.empty(0, device=cuda)
    fw = [_C.rasterize_gaussians(c.bg, a["means3D"], e, a["opacities"], a["scales"], a["rotations"], 1.0, e,
                                 c.viewmatrix, c.projmatrix, c.tanfovx, c.tanfovy, H, W, a["shs"], deg, c.campos,
                                 False) for c in cams]
    per = []
    for c, f, dl in zip(cams, fw, dls):
        per.append(_C.rasterize_gaussians_backward(c.bg, a["means3D"], f[2], e, a["scales"], a["rotations"], 1.0, e,
                                                   c.viewmatrix, c.projmatrix, c.tanfovx, c.tanfovy, dl, a["shs"],
                                                   deg, c.campos, f[3], f[0], f[4], f[5], skip_unused=True))
    views = []
    m2 = [torch.full((P, 3), 5.0, device=cuda) for _ in cams]
    for k, (c, f, dl) in enumerate(zip(cams, fw, dls)):
        scr = _C.rasterize_gaussians_backward_render(c.bg, a["means3D"], f[2], e, a["scales"], a["rotations"], 1.0,
                                                     e, c.viewmatrix, c.projmatrix, c.tanfovx, c.tanfovy, dl,
                                                     a["shs"], deg, c.campos, f[3], f[0], f[4], f[5])
        views.append({"viewmatrix": c.viewmatrix, "projmatrix": c.projmatrix, "tanfovx": c.tanfovx,
                      "tanfovy": c.tanfovy, "image_height": H, "image_width": W, "campos": c.campos, "bg": c.bg,
                      "radii": f[2], "geomBuffer": f[3], "scratch": scr, "num_rendered": f[0],
                      "means2D_grad": m2[k], "accumulate_means2D": k == 1})
    out = _C.rasterize_gaussians_backward_views(views, a["means3D"], e, a["scales"], a["rotations"], 1.0, e,
                                                a["shs"], deg)
    torch.cuda.synchronize()
    assert out[0] is None
    for k, name in enumerate(("means2D", "colors", "opacity", "means3D", "cov3D", "sh", "scales", "rot")):
        if k == 0 or out[k].numel() == 0:
            continue
        _close(name, out[k], sum(p[k] for p in per))
    for k in range(len(cams)):
        ref = per[k][0] + (5.0 if k == 1 else 0.0)
        assert torch.equal(m2[k], ref), k  # the screen-space gradient is the record sum itself: exact


def test_workspaces_freed_without_the_cyclic_collector(cuda):
    """Forward / backward workspaces (GEOM, BINNING, IMAGE, SCRATCH) are freed by reference counting
    as soon as the graph and the queued views are released: with the cyclic collector off, device
    memory returns to its starting level after every step (an allocator callback bound to its owner
    once kept every workspace alive until a gc run)."""
    import gc
    a, deg = _inputs(cuda, "sh3")
    cams = _cams(cuda, 3, deg)
    dls = [S.upstream_grad(H, W, seed=120 + k, device=cuda) for k in range(len(cams))]
    leaves = _leaves(a)
    torch.cuda.synchronize()
    base = torch.cuda.memory_allocated()
    gc.disable()
    try:
        for deferred in (True, False):
            prev = set_deferred_backward(deferred)
            try:
                for _ in range(3):
                    _views_loss(leaves, cams, dls).backward()
                    for v in leaves.values():
                        v.grad = None
                    torch.cuda.synchronize()
                    assert torch.cuda.memory_allocated() == base, deferred
            finally:
                set_deferred_backward(prev)
    finally:
        gc.enable()


def test_deferred_fresh_grad_with_a_second_path(cuda):
    """Leaves without a .grad get theirs allocated at the end of the pass and overwritten by the first
    launch (no zero fill): also when another term of the loss reaches the same leaves during the pass
    (autograd's AccumulateGrad sets .grad first, the deferred pass then adds into it) and over two
    launch groups (10 views)."""
    a, deg = _inputs(cuda, "sh3")
    cams = _cams(cuda, 10, deg)
    dls = [S.upstream_grad(H, W, seed=140 + k, device=cuda) for k in range(len(cams))]

    def run(deferred):
        leaves = _leaves(a)
        prev = set_deferred_backward(deferred)
        try:
            loss = _views_loss(leaves, cams, dls) + 0.5 * (leaves["means3D"] ** 2).sum() + leaves["opacities"].sum()
            loss.backward()
        finally:
            set_deferred_backward(prev)
        torch.cuda.synchronize()
        return {k: v.grad.clone() for k, v in leaves.items() if v.grad is not None}

    ref, got = run(False), run(True)
    assert set(ref) == set(got)
    for k in ref:
        assert torch.isfinite(got[k]).all(), k
        _close(k, got[k], ref[k])
