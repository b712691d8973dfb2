"""Is the backward's per-pixel half (gsr_backward_render) idempotent?  (diagnostic, GPU)

Captures the render-half closure the deferred backward builds (diff_gaussian_rasterization._try_defer) for
one view of the async-forward repro scene, and calls it several times after the pass, with the GPU idle:
every call must return the same SUMS.  Blocking and asynchronous forwards.

usage (GPU box): python tools/render_half_idem.py
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "animating-gaussian-splats_amd"), REPO]

import torch  # noqa: E402


def main():
    import splat_scenes as S
    import diff_gaussian_rasterization as dgr
    from diff_gaussian_rasterization import GaussianRasterizer, _C
    cuda = torch.device("cuda", 0)
    P, W, H = 80_000, 480, 320
    base = S.synthetic_cloud(P, 0.01, seed=7, device=cuda)
    rs = S.render_settings(W, H, S.intrinsics(400.0, W, H), S.look_at(0, 0.2, 8.0), device=cuda)
    dl = S.upstream_grad(H, W, device=cuda)
    with torch.no_grad():
        act = S.activated_inputs(base, -1)
    caught = []
    orig = dgr._try_defer

    def spy(ctx, gauss, radii, geomBuffer, leaf_inputs, nodes, need, render_fn, keep=()):
        caught.append((render_fn, ctx, keep))
        return orig(ctx, gauss, radii, geomBuffer, leaf_inputs, nodes, need, render_fn, keep)
    dgr._try_defer = spy

    def step(scale):
        leaves = {k: v.detach().clone().requires_grad_(True) for k, v in act.items()}
        with torch.no_grad():
            leaves["scales"].mul_(scale)
        img = GaussianRasterizer(raster_settings=rs)(**dict(leaves, means2D=torch.zeros_like(
            leaves["means3D"], requires_grad=True)))[0]
        (img * dl).sum().backward()
        torch.cuda.synchronize()

    for mode in ("blocking", "async"):
        for scale in (1.0, 3.0):
            dgr.set_async_forward(False)
            _C.speculation_stats(reset=True)
            step(1.0)
            dgr.set_async_forward(mode == "async")
            caught.clear()
            step(scale)
            fn, ctx, keep = caught[-1]
            outs = []
            for _ in range(4):
                sc, K = fn()
                torch.cuda.synchronize()
                outs.append(sc.clone())
                junk = torch.full((64 << 20,), float("nan"), device=cuda)  # dirty the allocator's free blocks
                del junk
            f = [o.view(torch.float32) if o.numel() % 4 == 0 else o.float() for o in outs]
            diffs = [(float((f[0] - x).abs().nan_to_num(1e30).max()), int(x.isnan().sum()), int((f[0] != x).sum()))
                     for x in f[1:]]
            print(f"{mode} scale {scale}: K {K}, SUMS {f[0].numel()} floats; vs the first call (max diff, NaNs, "
                  f"differing): {diffs}; first call NaNs {int(f[0].isnan().sum())}", flush=True)
    dgr.set_async_forward(False)


if __name__ == "__main__":
    main()
