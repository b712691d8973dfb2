"""Library view streams for non-leaf inputs (diff_gaussian_rasterization._on_view_stream).

The unchanged train.py step (one host thread, torch's current stream, create_render_arguments' non-leaf
inputs, 5 views' losses summed, one backward: train.py:402-418 + shared.py:29-42) and densify.py's
two renders (densify.py:114-151, leaf means + non-leaf activations, ``means2D.retain_grad()``) run each
view on a library stream, with the non-leaf inputs bridged through a node made by a helper thread so
that the autograd engine runs every view's rasterizer backward before handing any view's gradients to
the caller's stream.

CPU: the engine-order property the design relies on (a node created by another thread has the lowest
priority among ready nodes: it runs after every later node of the caller's graph).
GPU: images and every gradient bitwise equal with the view streams on and off (and with the
asynchronous forward on and off).
"""
import pytest
import torch

import diff_gaussian_rasterization as dgr


class _Tag(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, log, name):
        ctx.log, ctx.name = log, name
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        ctx.log.append(ctx.name)
        return g, None, None


def test_helper_thread_nodes_run_after_the_callers_nodes():
    """train.py's graph: per view an activation, the rasterizer node (made by the helper thread), a loss;
    the losses stacked and summed.  The engine must run every view's loss backward before any rasterizer
    node, and the rasterizer nodes before their activations' backward."""
    log = []
    helper = dgr._HelperThread()
    p = torch.randn(8, requires_grad=True)
    # a training program's thread has made many autograd nodes before (train.py: the deformation
    # network, every earlier step); the helper makes one per view-stream render
    for _ in range(200):
        (p * 1.0).sum()
    losses = []
    for k in range(5):
        act = _Tag.apply(p * 2.0, log, f"act{k}")

        def make(act=act, k=k):
            with torch.enable_grad():
                return _Tag.apply(act, log, f"rast{k}")
        r = helper.call(make)
        losses.append(_Tag.apply(r.sum(), log, f"loss{k}"))
    torch.stack(losses).sum().backward()
    pos = {n: i for i, n in enumerate(log)}
    assert max(pos[f"loss{k}"] for k in range(5)) < min(pos[f"rast{k}"] for k in range(5)), log
    assert [n for n in log if n.startswith("rast")] == [f"rast{k}" for k in (4, 3, 2, 1, 0)], log
    assert all(pos[f"rast{k}"] < pos[f"act{k}"] for k in range(5)), log
    assert torch.equal(p.grad, torch.full_like(p, 10.0))


def _train_step(cams, base, dl, delta):
    import splat_scenes as S
    from diff_gaussian_rasterization import GaussianRasterizer
    p = {k: v.clone() for k, v in base.items()}
    p["means"] = p["means"].detach()
    p["means"] += delta[:, :3] * 0.01
    p["rotation_quaternions"] = p["rotation_quaternions"].detach()
    p["rotation_quaternions"] += delta[:, 3:] * 0.01
    imgs = [GaussianRasterizer(raster_settings=rs)(**S.render_arguments(p))[0] for rs in cams]
    torch.stack([(i * dl).sum() for i in imgs]).sum(dim=0).backward()
    torch.cuda.synchronize()
    g = delta.grad.clone()
    delta.grad = None
    return [i.detach() for i in imgs], g


def _densify_step(rs, params, dl):
    import splat_scenes as S
    from diff_gaussian_rasterization import GaussianRasterizer
    a = S.render_arguments(params)
    a["means2D"].retain_grad()
    img = GaussianRasterizer(raster_settings=rs)(**a)[0]
    b = S.render_arguments(params)
    b["colors_precomp"] = params["segmentation_masks"]
    seg = GaussianRasterizer(raster_settings=rs)(**b)[0]
    ((img * dl).sum() + 3 * (seg * dl).sum()).backward()
    torch.cuda.synchronize()
    out = {k: v.grad.clone() for k, v in params.items() if v.grad is not None}
    out["means2D"] = a["means2D"].grad.clone()
    for v in params.values():
        v.grad = None
    return [img.detach(), seg.detach()], out


@pytest.mark.gpu
@pytest.mark.parametrize("async_fwd,n_streams,helper", [(True, 3, True), (False, 3, True), (False, 1, False)])
def test_train_and_densify_shapes_bitwise(cuda, async_fwd, n_streams, helper):
    import splat_scenes as S
    P, W, H = 120_000, 640, 400
    base = S.synthetic_cloud(P, 0.008, seed=3, device=cuda)  # frozen (requires_grad False)
    cams = [S.render_settings(W, H, S.intrinsics(520.0, W, H), S.look_at(yaw, h, 8.0), device=cuda)
            for yaw, h in ((0, 0.0), (40, 0.8), (80, -0.8), (120, 0.0), (160, 0.8))]
    dl = S.upstream_grad(H, W, device=cuda)
    delta = torch.zeros(P, 7, device=cuda, requires_grad=True)
    with torch.no_grad():
        delta += 0.1 * torch.randn(P, 7, generator=torch.Generator().manual_seed(9)).to(cuda)
    params = {k: torch.nn.Parameter(v.clone()) for k, v in base.items()}
    g = torch.Generator().manual_seed(8)
    params["segmentation_masks"] = torch.nn.Parameter((torch.rand(P, 1, generator=g) > 0.5).float().repeat(1, 3).to(cuda))
    prev_async = dgr.set_async_forward(async_fwd)
    prev = dgr.set_view_streams(False)
    vs = dgr._VIEW_STREAMS
    prev_cfg = vs["n"], vs["helper"], vs["pool"], vs["next"]
    vs["n"], vs["helper"], vs["pool"], vs["next"] = n_streams, helper, {}, {}
    try:
        _train_step(cams, base, dl, delta)  # pair-count history for the asynchronous forwards
        _densify_step(cams[0], params, dl)
        ref_t = _train_step(cams, base, dl, delta)
        ref_d = _densify_step(cams[0], params, dl)
        dgr.set_view_streams(True)
        for _ in range(2):
            got_t = _train_step(cams, base, dl, delta)
            got_d = _densify_step(cams[0], params, dl)
            for x, y in zip(ref_t[0] + ref_d[0], got_t[0] + got_d[0]):
                assert torch.equal(x, y)
            assert torch.equal(ref_t[1], got_t[1])
            assert ref_d[1].keys() == got_d[1].keys()
            for k in ref_d[1]:
                assert torch.equal(ref_d[1][k], got_d[1][k]), k
    finally:
        dgr.set_view_streams(prev)
        dgr.set_async_forward(prev_async)
        vs["n"], vs["helper"], vs["pool"], vs["next"] = prev_cfg
