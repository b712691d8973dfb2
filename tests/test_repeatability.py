"""Run-to-run bitwise repeatability of the pipelined summed step (-m gpu).

The kernels are deterministic by construction (no float atomics; every gradient record has one writer;
the deferred multi-view pass adds in a fixed order), so the same step run twice must give bitwise
identical images and leaf gradients.  A race shows up here as a run-to-run difference long before it
moves an oracle comparison out of tolerance: a missing LDS wait at k_render_fwd's blend-loop barrier
once let the waves of a block leave the loop at different batches, corrupting ~0.1 % of the
per-Gaussian gradients at random (the C4 rig step, 1M Gaussians x 27 views on 3 streams).  Covered:
that step, and a small cloud whose segment length is the shortest (seg_log2 = 6, C2 shape).
"""
import pytest
import torch

import splat_scenes as S
import splat_step

pytestmark = pytest.mark.gpu


def _step(cfg, views, cuda, sh_degree):
    p = S.synthetic_cloud(cfg.P, cfg.s0, sh_degree=sh_degree, seed=0, device=cuda)
    with torch.no_grad():
        act = S.activated_inputs(p, sh_degree)
    if sh_degree >= 0:
        act.pop("colors_precomp")
    leaves = {k: v.detach().clone().requires_grad_(True) for k, v in act.items()}
    cams = S.scene_cameras(cfg, device=cuda)
    streams = [torch.cuda.Stream() for _ in range(3)]
    for s in streams:
        s.wait_stream(torch.cuda.current_stream())
    step = splat_step.RenderStep(cuda, cams, lambda ci: leaves, S.upstream_grad(cfg.height, cfg.width, device=cuda),
                                 streams, threads=True)
    try:
        imgs = step(views)
    finally:
        step.close()
    torch.cuda.synchronize()
    return [i.cpu() for i in imgs], {k: v.grad.cpu() for k, v in leaves.items()}


@pytest.mark.parametrize("name", ["C4", "C2"])
def test_summed_step_bitwise_repeatable(name, cuda):
    cfg = S.CONFIGS[name]  # C4: the 27-camera rig; C2: its 4 cameras
    views = list(range(len(cfg.views)))
    a_imgs, a_grads = _step(cfg, views, cuda, cfg.sh_degree)
    b_imgs, b_grads = _step(cfg, views, cuda, cfg.sh_degree)
    for k, (x, y) in enumerate(zip(a_imgs, b_imgs)):
        assert torch.equal(x, y), f"{name} view {k}: image differs between two runs"
    for k in a_grads:
        d = (a_grads[k] != b_grads[k]).sum().item()
        assert d == 0, f"{name} {k}: {d} gradient values differ between two runs of the same step"
