"""GPU parity: the HIP rasterizer (through the C ABI) against the CPU oracle on identical inputs.

Bar (BASELINE.json north_star): tile/bin indices bit-exact -- radii, tiles touched, tile rects,
tile ranges, sorted Gaussian lists, sort keys, screen-space means/conics/depths; rendered colour,
depth and every gradient within 1e-4 relative (fp32).  Gradients are summed in a different order
than the oracle (per-tile wave reductions vs. a serial loop), so they are compared with
|gpu - oracle| <= 1e-4 |oracle| + 1e-5 max|oracle|.  The alpha >= 1/255 decisions are the
oracle's (the default exact-threshold mode re-evaluates weights within 1e-5 of the threshold in the
reference's expression order), and since round 6 so are the T >= 1e-4 saturation decisions (pixels whose
final T lies near 1e-4 are re-walked with the exact weights, k_render_tsat): n_contrib is bit-exact and
no case has an allowance (ALLOW is empty; the fast kernels alone keep theirs, ALLOW_FAST).  Rates are
reported in gpurun_out/parity_stats.json.
"""
import os

import numpy as np
import pytest
import torch

import splat_scenes as S
from diff_gaussian_rasterization import GaussianRasterizer, _C
from oracle import oracle as O

pytestmark = pytest.mark.gpu

RTOL = 1e-4
# Per-case allowances for values outside tolerance (pixels, gradient values).  Round 5 allowed the T >= 1e-4
# saturation flips (C3_yaw0 5.8e-6 / 1.33e-6, C4_yaw40_up 1.93e-6: 4x the measured rates); round 6 makes
# those decisions exact.  (Round 2-4, fast kernels alone: c1 1.5e-5 / 2.7e-4, C2_yaw180 3.1e-6 / 5e-5 -- ALLOW_FAST.)
ALLOW = {}  # round 6: none (the saturation test is exact too, k_render_tsat)


def allow(case):
    return ALLOW.get(case, (0.0, 0.0))
# (test, quantity, mismatch fraction, worst abs err, scale, fraction at a 1e-6 floor) -> gpurun_out/parity_stats.json
# (dumped by conftest.py at the end of the session; test_headline_parity.py appends to it too)
STATS = []


def _inputs(P, W, H, focal, s0, seed=0, sh_degree=-1, yaw=0.0, height=0.0, distance=4.0,
            bg=(0.0, 0.0, 0.0), active_degree=None, extra_coeffs=0, opacity_boost=0.0):
    p = S.synthetic_cloud(P, s0, sh_degree=sh_degree, seed=seed, device="cpu")
    a = {k: (v.detach() if isinstance(v, torch.Tensor) else v)
         for k, v in S.activated_inputs(p, sh_degree).items()}
    if opacity_boost:  # shift the opacity logits: many opacities above 0.99, where alpha is clamped
        a["opacities"] = torch.sigmoid(torch.logit(a["opacities"]) + opacity_boost)
    if extra_coeffs:  # more stored coefficients than the active degree uses (generic M path)
        g = torch.Generator().manual_seed(seed + 99)
        a["shs"] = torch.cat([a["shs"], 0.05 * torch.randn(P, extra_coeffs, 3, generator=g)], 1).contiguous()
    deg = max(sh_degree, 0) if active_degree is None else active_degree
    rs = S.render_settings(W, H, S.intrinsics(focal, W, H), S.look_at(yaw, height, distance),
                           device="cpu", sh_degree=deg)
    rs = rs._replace(bg=torch.tensor(bg, dtype=torch.float32))
    return a, rs


def _gpu_forward(a, rs, dev, cov3D=None):
    e = torch.empty(0, device=dev)
    g = lambda k: a[k].to(dev) if a.get(k) is not None else e  # noqa: E731
    out = _C.rasterize_gaussians(
        rs.bg.to(dev), a["means3D"].to(dev), g("colors_precomp"), a["opacities"].to(dev),
        e if cov3D is not None else g("scales"), e if cov3D is not None else g("rotations"),
        rs.scale_modifier, cov3D.to(dev) if cov3D is not None else e, rs.viewmatrix.to(dev),
        rs.projmatrix.to(dev), rs.tanfovx, rs.tanfovy, rs.image_height, rs.image_width, g("shs"),
        rs.sh_degree, rs.campos.to(dev), rs.prefiltered)
    K, color, radii, geom, binning, img, depth = out
    P = a["means3D"].shape[0]
    dec = _C.decode_buffers(P, rs.image_width, rs.image_height, K, geom, binning, img)
    return dict(K=K, color=color, radii=radii, geom=geom, binning=binning, img=img, depth=depth,
                dec=dec)


def _gpu_backward(a, rs, dev, fw, dl, cov3D=None):
    e = torch.empty(0, device=dev)
    g = lambda k: a[k].to(dev) if a.get(k) is not None else e  # noqa: E731
    return _C.rasterize_gaussians_backward(
        rs.bg.to(dev), a["means3D"].to(dev), fw["radii"], g("colors_precomp"),
        e if cov3D is not None else g("scales"), e if cov3D is not None else g("rotations"),
        rs.scale_modifier, cov3D.to(dev) if cov3D is not None else e, rs.viewmatrix.to(dev),
        rs.projmatrix.to(dev), rs.tanfovx, rs.tanfovy, dl.to(dev), g("shs"), rs.sh_degree,
        rs.campos.to(dev), fw["geom"], fw["K"], fw["binning"], fw["img"])


def _ora_forward(a, rs, cov3D=None):
    n = lambda k: a[k].numpy() if a.get(k) is not None else None  # noqa: E731
    return O.forward(rs.bg.numpy(), a["means3D"].numpy(), n("colors_precomp"), a["opacities"].numpy(),
                     None if cov3D is not None else n("scales"),
                     None if cov3D is not None else n("rotations"), rs.scale_modifier,
                     cov3D.numpy() if cov3D is not None else None, rs.viewmatrix, rs.projmatrix,
                     rs.tanfovx, rs.tanfovy, rs.image_height, rs.image_width, n("shs"),
                     rs.sh_degree, rs.campos.numpy())


def _np(t):
    return t.detach().cpu().numpy()


def _close(name, got, ref, rtol=RTOL, atol_frac=1e-5, max_bad_frac=0.0):
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    assert got.shape == ref.shape, (name, got.shape, ref.shape)
    if ref.size == 0:
        return
    scale = np.abs(ref).max() + 1e-30
    err = np.abs(got - ref)
    bad = err > rtol * np.abs(ref) + atol_frac * scale
    frac = bad.mean()
    tight = float((err > rtol * np.abs(ref) + 1e-6 * scale).mean())  # informational: a 10x lower floor
    STATS.append((os.environ.get("PYTEST_CURRENT_TEST", "?").split(" ")[0], name, float(frac),
                  float(err.max()), float(scale), tight))
    assert frac <= max_bad_frac, (f"{name}: {bad.sum()}/{bad.size} outside tolerance, worst "
                                  f"{np.abs(got - ref).max():.3g} (scale {scale:.3g})")


def check_forward(fw, st, pix_flip_frac=0.0):
    """Bit-exact integer state + tolerance on blended images."""
    d = fw["dec"]
    P = st["P"]
    assert fw["K"] == st["num_rendered"]
    np.testing.assert_array_equal(_np(fw["radii"]), st["radii"])
    np.testing.assert_array_equal(_np(d["tiles_touched"]).view(np.uint32), st["tiles_touched"])
    vis = st["radii"] > 0
    r = _np(d["rect"]).view(np.uint32)
    rect = np.stack([r[:, 0] & 0xFFFF, r[:, 0] >> 16, r[:, 1] & 0xFFFF, r[:, 1] >> 16], -1)
    np.testing.assert_array_equal(rect[vis], st["rects"][vis])
    np.testing.assert_array_equal(_np(d["depth"])[vis].view(np.uint32), st["depths"][vis].view(np.uint32))
    np.testing.assert_array_equal(_np(d["xy"])[vis].copy().view(np.uint32), st["xy"][vis].view(np.uint32))
    np.testing.assert_array_equal(_np(d["conic_opacity"])[vis].copy().view(np.uint32),
                                  st["conic_opacity"][vis].view(np.uint32))
    np.testing.assert_array_equal(_np(d["rgbd"])[vis, 3].copy().view(np.uint32), st["depths"][vis].view(np.uint32))
    np.testing.assert_array_equal(_np(d["ranges"]).view(np.uint32), st["ranges"])
    np.testing.assert_array_equal(_np(d["point_list"]).view(np.uint32), st["point_list"])
    if st["sh"] is not None:
        _close("rgb", _np(d["rgbd"])[vis, :3], st["rgb"][vis], atol_frac=1e-6)
    else:
        np.testing.assert_array_equal(_np(d["rgbd"])[vis, :3], st["colors_precomp"][vis])
    # goff: exclusive emission offsets; slot_emit maps sorted slots onto emissions (a permutation)
    goff = _np(d["goff"]).astype(np.int64)
    tt = st["tiles_touched"].astype(np.int64)
    np.testing.assert_array_equal(goff[:P], np.concatenate([[0], np.cumsum(tt)[:-1]]) if P else goff[:0])
    assert goff[P] == st["num_rendered"]
    se = _np(d["slot_emit"]).astype(np.int64)
    assert np.array_equal(np.sort(se), np.arange(st["num_rendered"]))
    # the emission at slot s belongs to the Gaussian at slot s
    owner = np.searchsorted(goff[:P], se, side="right") - 1
    np.testing.assert_array_equal(owner, st["point_list"].astype(np.int64))
    # blended outputs
    H, W = st["H"], st["W"]
    same_nc = (_np(d["n_contrib"]).view(np.uint32) == st["n_contrib"]).mean()
    STATS.append((os.environ.get("PYTEST_CURRENT_TEST", "?").split(" ")[0], "n_contrib", float(1 - same_nc), 0.0, 0.0))
    assert same_nc >= 1 - pix_flip_frac, f"n_contrib differs on {1 - same_nc:.2e} of pixels"
    _close("final_T", _np(d["final_T"]), st["final_T"], atol_frac=1e-6, max_bad_frac=pix_flip_frac)
    _close("color", _np(fw["color"]), st["color"], atol_frac=1e-6, max_bad_frac=pix_flip_frac)
    _close("depth", _np(fw["depth"]), st["depth"], atol_frac=1e-6, max_bad_frac=pix_flip_frac)
    assert fw["color"].shape == (3, H, W) and fw["depth"].shape == (1, H, W)


def check_backward(gb, gref, P, M, grad_flip_frac=0.0):
    (dm2, dcol, dop, dm3, dcov, dsh, dsc, drot) = [_np(t) for t in gb]
    _close("means2D", dm2, gref["means2D"], max_bad_frac=grad_flip_frac)
    _close("colors", dcol, gref["colors"], max_bad_frac=grad_flip_frac)
    _close("opacities", dop, gref["opacities"], max_bad_frac=grad_flip_frac)
    _close("means3D", dm3, gref["means3D"], max_bad_frac=grad_flip_frac)
    _close("cov3D", dcov, gref["cov3D"], max_bad_frac=grad_flip_frac)
    _close("scales", dsc, gref["scales"], max_bad_frac=grad_flip_frac)
    _close("rotations", drot, gref["rotations"], max_bad_frac=grad_flip_frac)
    assert dsh.shape == (P, M, 3)
    if M:
        _close("sh", dsh, gref["sh"], max_bad_frac=grad_flip_frac)


CASES = {
    # name: (P, W, H, focal, s0, sh_degree, extra)
    "c1": (10_000, 256, 256, 256.0, 0.02, -1, {}),
    "ragged_bg": (3_000, 200, 120, 150.0, 0.03, -1, dict(bg=(0.2, 0.5, 0.9))),
    "sh1_yaw": (5_000, 160, 96, 120.0, 0.03, 1, dict(yaw=90.0, height=0.8)),
    "sh3": (20_000, 480, 270, 400.0, 0.01, 3, {}),
    "dense_small": (4_000, 64, 48, 64.0, 0.08, -1, {}),
    "sh0": (3_000, 96, 80, 80.0, 0.03, 0, {}),
    "sh2": (3_000, 96, 80, 80.0, 0.03, 2, dict(yaw=200.0)),
    "sh3_active2": (3_000, 96, 80, 80.0, 0.03, 3, dict(active_degree=2)),
    "sh_m25_generic": (3_000, 96, 80, 80.0, 0.03, 3, dict(extra_coeffs=9)),
    # ~2/3 of the opacities above 0.99: the backward's clamping walk (alpha = min(0.99, o G)) beside
    # batches without such pairs
    "opaque": (10_000, 256, 256, 256.0, 0.02, -1, dict(opacity_boost=5.0)),
}


@pytest.mark.parametrize("case", list(CASES))
def test_forward_backward_parity(case, cuda):
    P, W, H, f, s0, shd, extra = CASES[case]
    a, rs = _inputs(P, W, H, f, s0, seed=3, sh_degree=shd, **extra)
    st = _ora_forward(a, rs)
    fw = _gpu_forward(a, rs, cuda)
    pix, grad = allow(case)
    check_forward(fw, st, pix)
    dl = S.upstream_grad(H, W, device="cpu")
    gref = O.backward(st, dl.numpy())
    gb = _gpu_backward(a, rs, cuda, fw, dl)
    check_backward(gb, gref, P, st["M"], grad)


def test_cov3d_precomp_parity(cuda):
    a, rs = _inputs(3_000, 128, 96, 96.0, 0.03, seed=5)
    from oracle import dense_torch as DT
    cov = DT.cov3d_from(a["scales"].double(), a["rotations"].double(), 1.0).float()
    st = _ora_forward(a, rs, cov3D=cov)
    fw = _gpu_forward(a, rs, cuda, cov3D=cov)
    check_forward(fw, st)
    dl = S.upstream_grad(96, 128, device="cpu")
    gref = O.backward(st, dl.numpy())
    check_backward(_gpu_backward(a, rs, cuda, fw, dl, cov3D=cov), gref, 3_000, 0)


def test_depth_ties_follow_index_order(cuda):
    """Cloned Gaussians (densify clone, external.py:234-239) share depth: order must be by index."""
    a, rs = _inputs(2_000, 128, 128, 128.0, 0.03, seed=11)
    for k in ("means3D", "colors_precomp", "opacities", "scales", "rotations"):
        a[k] = torch.cat([a[k], a[k][:700]], 0)  # 700 exact duplicates appended
    st = _ora_forward(a, rs)
    fw = _gpu_forward(a, rs, cuda)
    check_forward(fw, st)


@pytest.mark.parametrize("P", [800, 2_500, 12_000, 50_000, 200_000])
def test_long_tile_lists(P, cuda):
    """Clustered Gaussians: tile lists of ~P entries exercise every sort path (registers up to 512
    and 1024 pairs inside the render, one LDS block up to 4096, chunk sorts + merge passes beyond:
    50k pairs = 13 chunks, 4 passes; 200k = 49 chunks, 6 passes)."""
    g = torch.Generator().manual_seed(4)
    m = torch.zeros(P, 3)
    m[:, 0] = torch.rand(P, generator=g) * 0.02 - 0.01
    m[:, 1] = torch.rand(P, generator=g) * 0.02 - 0.01
    m[:, 2] = torch.rand(P, generator=g) * 2 - 1
    a = {"means3D": m, "colors_precomp": torch.rand(P, 3, generator=g),
         "opacities": torch.full((P, 1), 0.05), "scales": torch.full((P, 3), 0.004),
         "rotations": torch.tensor([[1.0, 0, 0, 0]]).repeat(P, 1)}
    rs = S.render_settings(64, 64, S.intrinsics(64.0, 64, 64), S.look_at(0, 0, 4), device="cpu")
    st = _ora_forward(a, rs)
    assert np.diff(st["ranges"].astype(np.int64), axis=1).max() > 0.5 * P
    fw = _gpu_forward(a, rs, cuda)
    check_forward(fw, st)
    dl = S.upstream_grad(64, 64, device="cpu")
    check_backward(_gpu_backward(a, rs, cuda, fw, dl), O.backward(st, dl.numpy()), P, 0)


@pytest.mark.parametrize("P,ks", [(150_000, 6), (300_000, 7), (600_000, 8)])
def test_segment_lengths(P, ks, cuda):
    """The backward's segment length follows the cloud size (seg_log2, gsr_common.h: 64 entries below
    262144 Gaussians, 128 below 524288, 256 above).  Faint clustered Gaussians (opacity 0.015, a
    few pixels wide) keep the ~32 centre pixels blending for thousands of list entries (oracle: up to
    ~18k), so their reverse walks cross many segment boundaries and restart from the blend states the
    forward saved there."""
    g = torch.Generator().manual_seed(6)
    m = torch.zeros(P, 3)
    m[:, 0] = torch.rand(P, generator=g) * 0.12 - 0.06
    m[:, 1] = torch.rand(P, generator=g) * 0.12 - 0.06
    m[:, 2] = torch.rand(P, generator=g) * 2 - 1
    a = {"means3D": m, "colors_precomp": torch.rand(P, 3, generator=g),
         "opacities": torch.full((P, 1), 0.015), "scales": torch.full((P, 3), 0.03),
         "rotations": torch.tensor([[1.0, 0, 0, 0]]).repeat(P, 1)}
    rs = S.render_settings(64, 64, S.intrinsics(64.0, 64, 64), S.look_at(0, 0, 4), device="cpu")
    st = _ora_forward(a, rs)
    assert int(st["n_contrib"].max()) > (4 << ks)  # the walks span more than 4 segments
    fw = _gpu_forward(a, rs, cuda)
    check_forward(fw, st)
    dl = S.upstream_grad(64, 64, device="cpu")
    check_backward(_gpu_backward(a, rs, cuda, fw, dl), O.backward(st, dl.numpy()), P, 0)


def test_wide_frame_global_binning(cuda):
    """A frame of more than kMaxLdsTiles = 16384 tiles (4224 x 1040: 264 x 65 = 17160 tiles) takes
    the binning path that counts and reserves with global atomics instead of the LDS histogram +
    (chunk, tile) column scan; its lists and ranges must be the same."""
    W, H = 4224, 1040
    a, rs = _inputs(30_000, W, H, 1100.0, 0.01, seed=8)
    assert -(-W // 16) * -(-H // 16) > 16384
    st = _ora_forward(a, rs)
    fw = _gpu_forward(a, rs, cuda)
    check_forward(fw, st)
    dl = S.upstream_grad(H, W, device="cpu")
    check_backward(_gpu_backward(a, rs, cuda, fw, dl), O.backward(st, dl.numpy()), 30_000, 0)


def test_empty_and_all_culled(cuda):
    rs = S.render_settings(48, 32, S.intrinsics(48.0, 48, 32), S.look_at(0, 0, 4), device="cpu")
    rs = rs._replace(bg=torch.tensor([0.25, 0.5, 0.75]))
    z3 = torch.zeros(0, 3)
    a = {"means3D": z3, "colors_precomp": z3, "opacities": torch.zeros(0, 1), "scales": z3,
         "rotations": torch.zeros(0, 4)}
    fw = _gpu_forward(a, rs, cuda)
    assert fw["K"] == 0 and not fw["color"].any() and not fw["depth"].any()  # P == 0: no background
    gb = _gpu_backward(a, rs, cuda, fw, torch.ones(3, 32, 48))
    assert all(t.shape[0] == 0 for t in gb)
    m = torch.tensor([[0.0, 0.0, -10.0]]).repeat(5, 1)
    a = {"means3D": m, "colors_precomp": torch.ones(5, 3), "opacities": torch.ones(5, 1),
         "scales": torch.full((5, 3), 0.1), "rotations": torch.tensor([[1.0, 0, 0, 0]]).repeat(5, 1)}
    fw = _gpu_forward(a, rs, cuda)
    assert fw["K"] == 0 and not fw["radii"].any()
    assert torch.equal(fw["color"].cpu(), rs.bg[:, None, None].expand(3, 32, 48))
    gb = _gpu_backward(a, rs, cuda, fw, torch.ones(3, 32, 48))
    assert all(not t.any() for t in gb)


def test_rasterizer_module_autograd(cuda):
    """The drop-in nn.Module + autograd.Function route, as train.py / densify.py call it."""
    P = 5_000
    p = S.synthetic_cloud(P, 0.02, seed=9, device=cuda)
    params = {k: torch.nn.Parameter(v) for k, v in p.items()}
    rs = S.render_settings(160, 128, S.intrinsics(160.0, 160, 128), S.look_at(30, 0.3, 4), device=cuda)
    args = S.render_arguments(params)
    args["means2D"].retain_grad()
    img, radii, depth = GaussianRasterizer(raster_settings=rs)(**args)
    assert img.shape == (3, 128, 160) and radii.dtype == torch.int32 and depth.shape == (1, 128, 160)
    dl = S.upstream_grad(128, 160, device=cuda)
    (img * dl).sum().backward()
    # oracle on the same activated inputs
    a = {k: v.detach().cpu() for k, v in args.items() if k != "means2D"}
    st = _ora_forward(a, rs._replace(bg=rs.bg.cpu(), viewmatrix=rs.viewmatrix.cpu(),
                                     projmatrix=rs.projmatrix.cpu(), campos=rs.campos.cpu()))
    np.testing.assert_array_equal(_np(radii), st["radii"])
    gref = O.backward(st, dl.cpu().numpy())
    _close("means2D.grad", _np(args["means2D"].grad), gref["means2D"], max_bad_frac=0.0)
    _close("colors.grad", _np(params["colors"].grad), gref["colors"], max_bad_frac=0.0)
    assert params["means"].grad is not None and params["log_scales"].grad is not None
    assert params["rotation_quaternions"].grad is not None and params["opacity_logits"].grad is not None
    with pytest.raises(Exception):
        GaussianRasterizer(raster_settings=rs)(means3D=args["means3D"], means2D=args["means2D"],
                                               opacities=args["opacities"], scales=args["scales"],
                                               rotations=args["rotations"])
    vis = GaussianRasterizer(raster_settings=rs).markVisible(params["means"].detach())
    np.testing.assert_array_equal(_np(vis), O.mark_visible(p["means"].cpu().numpy(), rs.viewmatrix.cpu(),
                                                           rs.projmatrix.cpu()))


@pytest.mark.parametrize("case", ["c1", "sh3", "ragged_bg"])
def test_fused_parameters_parity(case, cuda):
    """rasterize_parameters (normalize / sigmoid / exp of shared.py:33-41 inside the kernels) against
    the oracle fed with torch's own CPU activations, its gradients chained back to the raw
    parameters by torch autograd on the CPU (the reference's caller path, end to end)."""
    from diff_gaussian_rasterization import rasterize_parameters
    P, W, H, f, s0, shd, extra = CASES[case]
    p = S.synthetic_cloud(P, s0, sh_degree=shd, seed=3, device="cpu")
    g = torch.Generator().manual_seed(17)  # un-normalised raw quaternions: exercise normalize's chain rule
    p["rotation_quaternions"] = p["rotation_quaternions"] * (0.5 + 1.5 * torch.rand(P, 1, generator=g))
    raw = {k: v.clone().requires_grad_(True) for k, v in p.items()}
    act = S.activated_inputs(raw, shd)
    a = {k: v.detach() for k, v in act.items() if isinstance(v, torch.Tensor) and k != "means2D"}
    if shd >= 0:
        a.pop("colors_precomp", None)
    rs = S.render_settings(W, H, S.intrinsics(f, W, H), S.look_at(extra.get("yaw", 0.0), 0.0, 4.0),
                           device="cpu", sh_degree=max(shd, 0))
    rs = rs._replace(bg=torch.tensor(extra.get("bg", (0.0, 0.0, 0.0)), dtype=torch.float32))
    st = _ora_forward(a, rs)
    dl = S.upstream_grad(H, W, device="cpu")
    gref = O.backward(st, dl.numpy())
    t = lambda k: torch.from_numpy(np.ascontiguousarray(gref[k]))  # noqa: E731
    torch.autograd.backward([act["opacities"], act["scales"], act["rotations"]],
                            [t("opacities").view_as(act["opacities"]), t("scales"), t("rotations")])

    gp = {k: v.detach().to(cuda).requires_grad_(True) for k, v in p.items()}
    means2D = torch.zeros(P, 3, device=cuda, requires_grad=True)
    rsg = rs._replace(bg=rs.bg.to(cuda), viewmatrix=rs.viewmatrix.to(cuda),
                      projmatrix=rs.projmatrix.to(cuda), campos=rs.campos.to(cuda))
    color, radii, depth = rasterize_parameters(gp, rsg, means2D=means2D,
                                               shs=gp["shs"] if shd >= 0 else None)
    (color * dl.to(cuda)).sum().backward()
    same_r = (_np(radii) == st["radii"]).mean()
    STATS.append((f"test_fused_parameters_parity[{case}]", "radii", float(1 - same_r), 0.0, 0.0))
    assert same_r >= 1 - 1e-3, f"radii differ on {1 - same_r:.2e} of Gaussians"
    _close("fused.color", _np(color), st["color"], atol_frac=1e-6, max_bad_frac=0.0)
    _close("fused.depth", _np(depth), st["depth"], atol_frac=1e-6, max_bad_frac=0.0)
    _close("fused.means2D", _np(means2D.grad), gref["means2D"], max_bad_frac=0.0)
    _close("fused.means", _np(gp["means"].grad), gref["means3D"], max_bad_frac=0.0)
    if shd >= 0:
        _close("fused.shs", _np(gp["shs"].grad), gref["sh"], max_bad_frac=0.0)
        assert gp["colors"].grad is None
    else:
        _close("fused.colors", _np(gp["colors"].grad), gref["colors"], max_bad_frac=0.0)
    for k in ("opacity_logits", "log_scales", "rotation_quaternions"):
        assert gp[k].grad.shape == raw[k].shape
        _close("fused." + k, _np(gp[k].grad), raw[k].grad.numpy(), max_bad_frac=0.0)


def test_strided_camera_inputs_match_contiguous(cuda):
    """The reference hands the rasterizer a transposed viewmatrix view (shared.py:80) and a column
    slice of inv(w2c) as campos (shared.py:79); they are read in place through their strides
    (gsr_camera ABI 8), with results bitwise equal to contiguous copies of the same values."""
    P = 4_000
    p = S.synthetic_cloud(P, 0.02, sh_degree=3, seed=11, device=cuda)
    a = S.activated_inputs(p, 3)
    a.pop("colors_precomp")
    rs = S.render_settings(192, 144, S.intrinsics(180.0, 192, 144), S.look_at(70, 0.4, 4), device=cuda,
                           sh_degree=3)
    # the reference's layouts built on the device: w2c^T as a transposed view, campos as a column
    vm_t = rs.viewmatrix.transpose(1, 2).contiguous().transpose(1, 2)
    pm_t = rs.projmatrix.transpose(1, 2).contiguous().transpose(1, 2)
    cam4 = torch.zeros(4, 4, device=cuda)
    cam4[:3, 3] = rs.campos
    rs = rs._replace(viewmatrix=vm_t, projmatrix=pm_t, campos=cam4[:3, 3])
    assert not rs.viewmatrix.is_contiguous() and rs.campos.stride(0) == 4
    rc = rs._replace(viewmatrix=rs.viewmatrix.contiguous(), projmatrix=rs.projmatrix.contiguous(),
                     campos=rs.campos.contiguous())
    dl = S.upstream_grad(144, 192, device=cuda)
    outs = []
    for r in (rs, rc):
        leaves = {k: v.detach().clone().requires_grad_(True) for k, v in a.items()}
        img, radii, depth = GaussianRasterizer(raster_settings=r)(**leaves)
        img.backward(dl)
        outs.append([img.detach(), radii, depth.detach()] + [leaves[k].grad for k in sorted(leaves)])
    for x, y in zip(*outs):
        assert torch.equal(x, y)


# ---- BASELINE.json sizes: same bar, full-size inputs ----------
BASELINE_VIEWS = {
    # name: (config, yaw, height) -- C2: the 4 cameras of 800x800; C3: the 1080p SH3 view of the
    # bench (yaw 0); C4: rig views off the equator (heights -0.8 / +0.8 of the 27-camera rig)
    "C2_yaw0": ("C2", 0.0, 0.0), "C2_yaw90": ("C2", 90.0, 0.0), "C2_yaw180": ("C2", 180.0, 0.0),
    "C2_yaw270": ("C2", 270.0, 0.0),
    "C3_yaw0": ("C3", 0.0, 0.0),
    "C4_yaw40_up": ("C4", 40.0, 0.8), "C4_yaw200_down": ("C4", 200.0, -0.8),
}
_CLOUDS = {}


def _baseline_cloud(name):
    cfg = S.CONFIGS[name]
    if name not in _CLOUDS:
        p = S.synthetic_cloud(cfg.P, cfg.s0, sh_degree=cfg.sh_degree, seed=0, device="cpu")
        a = {k: (v.detach() if isinstance(v, torch.Tensor) else v)
             for k, v in S.activated_inputs(p, cfg.sh_degree).items()}
        _CLOUDS.clear()  # one 1M cloud resident at a time
        _CLOUDS[name] = a
    return cfg, _CLOUDS[name]


@pytest.mark.parametrize("view", list(BASELINE_VIEWS))
def test_baseline_size_parity(view, cuda):
    """C2 / C3 / C4 at the BASELINE.json sizes against the C oracle: bit-exact radii, rects, tiles,
    K, point lists, ranges, emission offsets; colour / depth / every gradient within 1e-4 rel with
    per-view blend-flip allowances of 4x the measured rates (ALLOW; rates in parity_stats.json)."""
    name, yaw, hgt = BASELINE_VIEWS[view]
    cfg, a = _baseline_cloud(name)
    rs = S.render_settings(cfg.width, cfg.height, S.intrinsics(cfg.focal, cfg.width, cfg.height),
                           S.look_at(yaw, hgt, cfg.distance), device="cpu", sh_degree=max(cfg.sh_degree, 0))
    st = _ora_forward(a, rs)
    fw = _gpu_forward(a, rs, cuda)
    pix, grad = allow(view)
    check_forward(fw, st, pix)
    dl = S.upstream_grad(cfg.height, cfg.width, device="cpu")
    gref = O.backward(st, dl.numpy())
    gb = _gpu_backward(a, rs, cuda, fw, dl)
    check_backward(gb, gref, cfg.P, st["M"], grad)
    STATS.append((view, "num_rendered", float(st["num_rendered"]), 0.0, 0.0))


# ---- exact-threshold mode (gsr_set_exact_thresholds; on by default since ABI 21) ------------------
# Every test above runs the default: tiles whose fast pass took a weight within 1e-5 of 1/255 are redone
# with such weights re-evaluated in the reference's expression order (IMAGE tile_flag / near_rec), so ALLOW only
# covers the T >= 1e-4 saturation test (T accumulates in a different rounding order than the oracle's).
# With the mode off, the fast kernels' decisions alone: the round-2 allowances (4x the measured rates,
# profiles/r02_parity_flips.json).
ALLOW_FAST = {"c1": (6.1e-5, 1.07e-3), "C2_yaw180": (1.25e-5, 2e-4)}


@pytest.fixture
def fast_mode():
    prev = _C.set_exact_thresholds(False)
    yield
    _C.set_exact_thresholds(prev)


def _case_inputs(case):
    if case in CASES:
        P, W, H, f, s0, shd, extra = CASES[case]
        a, rs = _inputs(P, W, H, f, s0, seed=3, sh_degree=shd, **extra)
        return a, rs, P, W, H
    name, yaw, hgt = BASELINE_VIEWS[case]
    cfg, a = _baseline_cloud(name)
    rs = S.render_settings(cfg.width, cfg.height, S.intrinsics(cfg.focal, cfg.width, cfg.height),
                           S.look_at(yaw, hgt, cfg.distance), device="cpu", sh_degree=max(cfg.sh_degree, 0))
    return a, rs, cfg.P, cfg.width, cfg.height


@pytest.mark.parametrize("case", list(ALLOW_FAST))
def test_fast_threshold_mode_parity(case, cuda, fast_mode):
    """Exact-threshold mode off: the fast kernels alone, no tile flagged, within ALLOW_FAST."""
    a, rs, P, W, H = _case_inputs(case)
    st = _ora_forward(a, rs)
    fw = _gpu_forward(a, rs, cuda)
    assert int(fw["dec"]["tile_flag"].sum()) == 0
    pix, grad = ALLOW_FAST[case]
    check_forward(fw, st, pix)
    dl = S.upstream_grad(H, W, device="cpu")
    gref = O.backward(st, dl.numpy())
    gb = _gpu_backward(a, rs, cuda, fw, dl)
    check_backward(gb, gref, P, st["M"], grad)


def test_exact_tiles_flagged_and_redone(cuda):
    """The default mode's near records (IMAGE tile_flag = re-evaluated weights per tile): on the densest
    case some tiles (not most) have some, their pixels are the oracle's in n_contrib, and the backward
    follows the records its forward wrote even when the setting changed in between (the setting applies
    to forwards only)."""
    a, rs, P, W, H = _case_inputs("c1")
    st = _ora_forward(a, rs)
    fw = _gpu_forward(a, rs, cuda)
    flag = _np(fw["dec"]["tile_flag"])
    T = flag.size
    STATS.append(("exact_tiles_c1", "flagged_tile_fraction", float((flag > 0).mean()), 0.0, 0.0, 0.0))
    assert 0 < (flag > 0).sum() < T // 4, f"{(flag > 0).sum()} of {T} tiles flagged"
    flag = flag > 0
    gx = (W + 15) // 16
    nc = _np(fw["dec"]["n_contrib"])
    bad = tot = 0
    for t in np.nonzero(flag)[0]:
        ty, tx = divmod(int(t), gx)
        sl = np.s_[16 * ty:16 * ty + 16, 16 * tx:16 * tx + 16]
        bad += int((nc[sl] != st["n_contrib"][sl]).sum())
        tot += nc[sl].size
    STATS.append(("exact_tiles_c1", "redone_tile_n_contrib_mismatch", bad / tot, 0.0, 0.0, 0.0))
    assert bad <= max(1, allow("c1")[0] * tot), f"{bad} of {tot} redone pixels differ from the oracle's n_contrib"
    dl = S.upstream_grad(H, W, device="cpu")
    gref = O.backward(st, dl.numpy())
    prev = _C.set_exact_thresholds(False)  # the backward still takes the exact items of flagged tiles
    try:
        gb = _gpu_backward(a, rs, cuda, fw, dl)
    finally:
        _C.set_exact_thresholds(prev)
    check_backward(gb, gref, P, st["M"], allow("c1")[1])


@pytest.mark.parametrize("where", ["band", "centre"])
def test_near_record_overflow(where, cuda):
    """40 copies of one Gaussian whose weight at one pixel sits on 1/255 (opacity solved from the
    oracle's power there): 40 near-threshold re-evaluations in one tile, more than the kNearCap = 16
    records the backward can look up, so that tile's items take the re-evaluating backward kernel.
    `band`: a pixel whose power is about -1.5; `centre`: the pixel nearest the Gaussian's
    centre, power near 0 and opacity near 1/255, where the fast power's sign test and the exact one
    meet.  Forward and gradients against the oracle with no allowance."""
    W, H = 64, 48
    base, rs = _inputs(300, W, H, 64.0, 0.05, seed=5)
    st0 = _ora_forward(base, rs)
    i = int(np.nonzero(st0["radii"] > 2)[0][0])
    a = {k: (v[i:i + 1].repeat(40, *([1] * (v.dim() - 1))).contiguous() if isinstance(v, torch.Tensor) and
             v.dim() > 0 and v.shape[0] == 300 else v) for k, v in base.items()}
    st = _ora_forward(a, rs)
    gx_, gy_ = st["xy"][0]
    A, B, C = (np.float32(v) for v in st["conic_opacity"][0, :3])
    best = None
    for py in range(max(0, int(gy_) - 6), min(H, int(gy_) + 7)):
        for px in range(max(0, int(gx_) - 6), min(W, int(gx_) + 7)):
            dx, dy = np.float32(gx_ - np.float32(px)), np.float32(gy_ - np.float32(py))
            pw = np.float32(np.float32(-0.5) * (A * dx * dx + C * dy * dy) - B * dx * dy)
            if where == "band":
                if -3.0 < pw < -0.5 and (best is None or abs(pw + 1.5) < abs(best[2] + 1.5)):
                    best = (px, py, pw)
            elif pw <= 0.0 and (best is None or abs(pw) < abs(best[2])):
                best = (px, py, pw)
    assert best is not None
    px, py, pw = best
    o = np.float32((1.0 / 255.0) / np.exp(np.float64(pw)))
    a["opacities"] = torch.full_like(a["opacities"], float(o))
    st = _ora_forward(a, rs)
    fw = _gpu_forward(a, rs, cuda)
    flag = _np(fw["dec"]["tile_flag"])
    t = (py // 16) * ((W + 15) // 16) + px // 16
    assert flag[t] > 16, f"tile {t}: {flag[t]} near records"
    check_forward(fw, st, 0.0)
    dl = S.upstream_grad(H, W, device="cpu")
    gref = O.backward(st, dl.numpy())
    gb = _gpu_backward(a, rs, cuda, fw, dl)
    check_backward(gb, gref, 40, st["M"], 0.0)
