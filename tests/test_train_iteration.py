"""One densify.py iteration on the native path (splat_train.densify_iteration) vs the reference's
composition of the same step (densify.py:110-162,218-247): torch activations (shared.py:29-42) +
GaussianRasterizer + 0.8 l1 + 0.2 (1 - calc_ssim) (restated with torch ops, the reference's
external.py:68-110) + torch statistics + torch.optim.Adam.

The comparison runs with every learning rate at 0, so after one step each Adam exp_avg equals
0.1 * grad bitwise and exposes the full parameter gradient of the iteration: native gradients must
match the composition within 1e-4 relative + 1e-5 of the largest magnitude on all but 1e-3 of the
values (the rasterizer tests' blend-threshold allowance), losses within 1e-5, statistics exactly.
"""
import os

import numpy as np
import pytest
import torch

from test_gpu_parity import STATS

ORDER = ["means", "colors", "segmentation_masks", "rotation_quaternions", "opacity_logits", "log_scales",
         "camera_matrices", "camera_center"]


def _torch_ssim(img1, img2):
    from math import exp
    g = torch.tensor([exp(-((x - 5) ** 2) / float(2 * 1.5 ** 2)) for x in range(11)])
    g = (g / g.sum()).unsqueeze(1)
    C = img1.size(-3)
    w = g.mm(g.t()).float()[None, None].expand(C, 1, 11, 11).contiguous().to(img1.device)
    conv = lambda t: torch.nn.functional.conv2d(t, w, padding=5, groups=C)  # noqa: E731
    mu1, mu2 = conv(img1), conv(img2)
    s1, s2, s12 = conv(img1 * img1) - mu1 ** 2, conv(img2 * img2) - mu2 ** 2, conv(img1 * img2) - mu1 * mu2
    c1, c2 = 0.01 ** 2, 0.03 ** 2
    return (((2 * mu1 * mu2 + c1) * (2 * s12 + c2)) / ((mu1 ** 2 + mu2 ** 2 + c1) * (s1 + s2 + c2))).mean()


@pytest.mark.gpu
@pytest.mark.parametrize("P,W,H,f,s0", [(20000, 320, 240, 300.0, 0.02),
                                        (1_000_000, 1920, 1080, 1600.0, 0.005)],  # C3 size
                         ids=["20k", "C3"])
def test_gpu_densify_iteration_matches_reference_composition(cuda, P, W, H, f, s0):
    import splat_adam
    import splat_scenes as S
    import splat_train
    from diff_gaussian_rasterization import GaussianRasterizer
    g = torch.Generator().manual_seed(2)
    base = S.synthetic_cloud(P, s0, seed=4, device="cpu")
    base["segmentation_masks"] = (torch.rand(P, 1, generator=g) > 0.5).float().repeat(1, 3)
    base["camera_matrices"] = torch.zeros(50, 3)
    base["camera_center"] = torch.zeros(50, 3)
    cam = S.render_settings(W, H, S.intrinsics(f, W, H), S.look_at(30.0, 0.3, 4.0), device=cuda)
    view = splat_train.View(0, cam, torch.rand(3, H, W, generator=g).to(cuda),
                            (torch.rand(1, H, W, generator=g) > 0.5).float().repeat(3, 1, 1).to(cuda))

    def fresh(cls):
        params = {k: torch.nn.Parameter(base[k].to(cuda).contiguous()) for k in ORDER}
        opt = cls([{"params": [params[k]], "name": k, "lr": 0.0} for k in ORDER], lr=0.0, eps=1e-15)
        return params, opt, splat_train.create_densification_variables(params)

    pn, on, dn = fresh(splat_adam.FusedAdam)
    (tot_n, img_n, seg_n), info = splat_train.densify_iteration(pn, view, dn, on, 4.0, 7)
    assert info is None

    pr, orf, dr = fresh(torch.optim.Adam)
    ra = S.render_arguments(pr)
    ra["means2D"].retain_grad()
    img, radii, _ = GaussianRasterizer(raster_settings=cam)(**ra)
    li = 0.8 * torch.nn.functional.l1_loss(img, view.image) + 0.2 * (1.0 - _torch_ssim(img, view.image))
    rs = S.render_arguments(pr)
    rs["colors_precomp"] = pr["segmentation_masks"]
    seg, _, _ = GaussianRasterizer(raster_settings=cam)(**rs)
    ls = 0.8 * torch.nn.functional.l1_loss(seg, view.segmentation_mask) + \
        0.2 * (1.0 - _torch_ssim(seg, view.segmentation_mask))
    pos = radii > 0
    dr.max_2d_radii[pos] = torch.max(radii[pos], dr.max_2d_radii[pos])
    (li + 3 * ls).backward()
    with torch.no_grad():
        dr.mean_2d_gradients_accumulated[pos] += torch.norm(ra["means2D"].grad[pos, :2], dim=-1)
        dr.visibility_count[pos] += 1
        orf.step()
    torch.cuda.synchronize()
    for a, b in ((img_n, li), (seg_n, ls)):
        assert abs(float(a) - float(b)) <= 1e-5 * abs(float(b)) + 1e-7
    np.testing.assert_array_equal(dn.max_2d_radii.cpu().numpy(), dr.max_2d_radii.cpu().numpy())
    np.testing.assert_array_equal(dn.visibility_count.cpu().numpy(), dr.visibility_count.cpu().numpy())
    # the native path activates on the GPU (fused) and the composition with torch ops: ulp-level input
    # differences can move a blend decision of a Gaussian with a tiny screen-space gradient (round 6: 2 of
    # 1M statistics at C3 outside 1e-3 relative, both below 2e-8 in magnitude)
    gn, gr = dn.mean_2d_gradients_accumulated.cpu().numpy(), dr.mean_2d_gradients_accumulated.cpu().numpy()
    off = np.abs(gn - gr) > 1e-3 * np.abs(gr) + 1e-9
    STATS.append((os.environ.get("PYTEST_CURRENT_TEST", "?").split(" ")[0], "mean_2d_gradients_accumulated",
                  float(off.mean()), float(np.abs(gn - gr).max()), float(np.abs(gr).max())))
    assert off.mean() <= 1e-5, f"{off.sum()} of {off.size} densify statistics off"
    for k in ORDER[:6]:
        got = on.state[pn[k]]["exp_avg"].cpu().numpy().astype(np.float64)
        ref = orf.state[pr[k]]["exp_avg"].cpu().numpy().astype(np.float64)
        assert np.abs(ref).max() > 0, k
        bad = np.abs(got - ref) > 1e-4 * np.abs(ref) + 1e-5 * np.abs(ref).max()
        STATS.append((os.environ.get("PYTEST_CURRENT_TEST", "?").split(" ")[0], k, float(bad.mean()),
                      float(np.abs(got - ref).max()), float(np.abs(ref).max())))
        assert bad.mean() <= 1e-3, f"{k}: {bad.mean():.2e} of gradients off"
        np.testing.assert_array_equal(pn[k].detach().cpu().numpy(), base[k].numpy())  # lr = 0
