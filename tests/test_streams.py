"""Views rendered on several HIP streams (bench.py --streams): libgsr orders every per-Gaussian
backward that writes the same gradient buffers across streams (gsr_api.hip ordered_grad_write), so
the accumulated gradients are bitwise those of the single-stream loop."""
import pytest
import torch

import splat_scenes as S
from diff_gaussian_rasterization import GaussianRasterizer

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("nstreams", [2, 3])
def test_multistream_views_bitwise_equal(nstreams, cuda):
    P, W, H = 30_000, 320, 240
    p = S.synthetic_cloud(P, 0.01, sh_degree=3, seed=5, device=cuda)
    a = S.activated_inputs(p, 3)
    a.pop("colors_precomp")
    cfg = [(yaw, h) for h in (-0.8, 0.0, 0.8) for yaw in (0, 40, 80)]
    cams = [S.render_settings(W, H, S.intrinsics(300.0, W, H), S.look_at(yaw, h, 4), device=cuda, sh_degree=3)
            for yaw, h in cfg]
    dl = S.upstream_grad(H, W, device=cuda)

    def run(n):
        leaves = {k: v.detach().clone().requires_grad_(True) for k, v in a.items()}
        main = torch.cuda.current_stream()
        streams = [main] + [torch.cuda.Stream() for _ in range(n - 1)]
        for s in streams[1:]:
            s.wait_stream(main)
        imgs = []
        for k, cam in enumerate(cams):
            with torch.cuda.stream(streams[k % n]):
                img, _, _ = GaussianRasterizer(raster_settings=cam)(**leaves)
                img.backward(dl)
                imgs.append(img.detach())
        for s in streams[1:]:
            main.wait_stream(s)
        torch.cuda.synchronize()
        return imgs, {k: v.grad.clone() for k, v in leaves.items()}

    imgs1, g1 = run(1)
    imgsn, gn = run(nstreams)
    for x, y in zip(imgs1, imgsn):
        assert torch.equal(x, y)
    for k in g1:
        assert torch.equal(g1[k], gn[k]), k


def test_grad_fence_orders_a_reset_before_the_next_backward(cuda):
    """A reset of the gradients on another stream, declared with grad_fence, is ordered before the
    next backward's accumulation into them (the N > 1 bench: all-reduce + reset on the main stream
    while the next step's forwards already run on side streams)."""
    from diff_gaussian_rasterization import _C
    P, W, H = 200_000, 640, 480
    p = S.synthetic_cloud(P, 0.01, sh_degree=3, seed=6, device=cuda)
    a = S.activated_inputs(p, 3)
    a.pop("colors_precomp")
    cam = S.render_settings(W, H, S.intrinsics(600.0, W, H), S.look_at(20, 0.3, 4), device=cuda, sh_degree=3)
    dl = S.upstream_grad(H, W, device=cuda)
    leaves = {k: v.detach().clone().requires_grad_(True) for k, v in a.items()}
    main = torch.cuda.current_stream()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    for s in (s1, s2):
        s.wait_stream(main)
    with torch.cuda.stream(s1):  # first view: creates the gradients
        GaussianRasterizer(raster_settings=cam)(**leaves)[0].backward(dl)
    main.wait_stream(s1)
    for v in leaves.values():  # the "all-reduce + reset" on the main stream ...
        v.grad.mul_(3.0).zero_()
    _C.grad_fence(*[v.grad for v in leaves.values()])  # ... declared to the library
    with torch.cuda.stream(s2):  # second view, other stream: accumulates into the reset gradients
        GaussianRasterizer(raster_settings=cam)(**leaves)[0].backward(dl)
    torch.cuda.synchronize()
    ref = {k: v.detach().clone().requires_grad_(True) for k, v in a.items()}
    GaussianRasterizer(raster_settings=cam)(**ref)[0].backward(dl)
    torch.cuda.synchronize()
    for k in ref:
        assert torch.equal(leaves[k].grad, ref[k].grad), k


def test_multistream_without_means3d_grad_and_many_sets(cuda):
    """Ordering is per gradient array, not per set: with means3D frozen (a fresh, never-accumulated
    means3D gradient each call) the colour / opacity / scale / rotation accumulations across two
    streams must still be ordered, and 20 gradient sets in flight (more than any fixed table) must
    not drop a pending writer."""
    P, W, H = 20_000, 256, 192
    p = S.synthetic_cloud(P, 0.01, sh_degree=-1, seed=8, device=cuda)
    a = S.activated_inputs(p, -1)
    cams = [S.render_settings(W, H, S.intrinsics(240.0, W, H), S.look_at(yaw, 0.2, 4), device=cuda)
            for yaw in (0, 30, 60, 90)]
    dl = S.upstream_grad(H, W, device=cuda)
    nsets = 20

    def make():
        lv = [{k: v.detach().clone().requires_grad_(k != "means3D") for k, v in a.items()} for _ in range(nsets)]
        return lv

    def run(n):
        sets = make()
        main = torch.cuda.current_stream()
        streams = [main] + [torch.cuda.Stream() for _ in range(n - 1)]
        for s in streams[1:]:
            s.wait_stream(main)
        k = 0
        for cam in cams:
            for lv in sets:
                with torch.cuda.stream(streams[k % n]):
                    GaussianRasterizer(raster_settings=cam)(**lv)[0].backward(dl)
                k += 1
        for s in streams[1:]:
            main.wait_stream(s)
        torch.cuda.synchronize()
        return [{kk: v.grad.clone() for kk, v in lv.items() if v.grad is not None} for lv in sets]

    g1, g2 = run(1), run(2)
    for x, y in zip(g1, g2):
        assert set(x) == set(y) and "means3D" not in x
        for kk in x:
            assert torch.equal(x[kk], y[kk]), kk
