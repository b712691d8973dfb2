"""CPU tests of the parity oracle (oracle/gsr_oracle.c): invariants and an autograd pin of its backward.

The rasterizer's reference source is absent, so the oracle is pinned by
(1) structural invariants of the binning it restates (stable (tile, depth) order, ranges),
(2) torch.autograd of an independent dense float64 restatement (oracle/dense_torch.py), and
(3) golden vectors of the reference's own Python callers (tests/test_golden.py).
"""
import numpy as np
import pytest
import torch

import splat_scenes as S
from oracle import dense_torch as DT
from oracle import oracle as O


def _scene(P, W, H, focal, s0, seed, sh_degree=-1, yaw=0.0, height=0.0, distance=4.0):
    p = S.synthetic_cloud(P, s0, sh_degree=sh_degree, seed=seed, device="cpu")
    a = S.activated_inputs(p, sh_degree)
    rs = S.render_settings(W, H, S.intrinsics(focal, W, H), S.look_at(yaw, height, distance),
                           device="cpu", sh_degree=max(sh_degree, 0))
    return p, {k: (v.detach() if isinstance(v, torch.Tensor) else v) for k, v in a.items()}, rs


def _fwd(a, rs, cov3D=None):
    return O.forward(rs.bg, a["means3D"], a.get("colors_precomp"), a["opacities"],
                     None if cov3D is not None else a["scales"],
                     None if cov3D is not None else a["rotations"], rs.scale_modifier, cov3D,
                     rs.viewmatrix, rs.projmatrix, rs.tanfovx, rs.tanfovy, rs.image_height,
                     rs.image_width, a.get("shs"), rs.sh_degree, rs.campos)


def test_binning_invariants_c1():
    cfg = S.CONFIGS["C1"]
    _, a, rs = _scene(cfg.P, cfg.width, cfg.height, cfg.focal, cfg.s0, seed=0)
    st = _fwd(a, rs)
    K = st["num_rendered"]
    assert K == int(st["tiles_touched"].sum()) and K > cfg.P
    r = st["ranges"].astype(np.int64)
    nonempty = r[:, 1] > r[:, 0]
    assert (r[~nonempty] == 0).all()  # empty tiles stay {0,0} (reference memsets ranges)
    assert (r[nonempty, 1] - r[nonempty, 0]).sum() == K
    order = np.argsort(r[nonempty, 0])
    starts, ends = r[nonempty, 0][order], r[nonempty, 1][order]
    assert starts[0] == 0 and ends[-1] == K and (starts[1:] == ends[:-1]).all()
    d = st["depths"].view(np.uint32).astype(np.uint64)
    for t in np.nonzero(nonempty)[0]:
        ids = st["point_list"][r[t, 0]:r[t, 1]].astype(np.int64)
        key = (d[ids] << np.uint64(32)) | ids.astype(np.uint64)
        assert (np.diff(key.astype(np.float64)) > 0).all() or (np.diff(key) > 0).all()
    # each visible Gaussian appears exactly tiles_touched times
    cnt = np.bincount(st["point_list"].astype(np.int64), minlength=cfg.P)
    assert (cnt == st["tiles_touched"]).all()
    assert (st["radii"][st["tiles_touched"] == 0] == 0).all()
    assert np.all(st["final_T"] > 0) and np.all(st["final_T"] <= 1)


def test_empty_and_culled():
    W = H = 40
    rs = S.render_settings(W, H, S.intrinsics(40.0, W, H), S.look_at(0, 0, 4), device="cpu")
    z = np.zeros((0, 3), np.float32)
    st = O.forward(rs.bg, z, z, np.zeros((0, 1), np.float32), z, np.zeros((0, 4), np.float32), 1.0,
                   None, rs.viewmatrix, rs.projmatrix, rs.tanfovx, rs.tanfovy, H, W, None, 0, rs.campos)
    assert st["num_rendered"] == 0 and not st["color"].any()
    # everything behind the near plane: T stays 1, colour = background
    bg = np.array([0.25, 0.5, 0.75], np.float32)
    m = np.tile(np.array([[0, 0, -10.0]], np.float32), (5, 1))
    st = O.forward(bg, m, np.ones((5, 3), np.float32), np.ones((5, 1), np.float32),
                   np.full((5, 3), 0.1, np.float32), np.tile(np.array([[1, 0, 0, 0]], np.float32), (5, 1)),
                   1.0, None, rs.viewmatrix, rs.projmatrix, rs.tanfovx, rs.tanfovy, H, W, None, 0,
                   rs.campos)
    assert st["num_rendered"] == 0 and (st["radii"] == 0).all()
    np.testing.assert_array_equal(st["color"], np.broadcast_to(bg[:, None, None], (3, H, W)))


def _autograd_case(seed, sh_degree=-1, use_cov3D=False, bg=(0.0, 0.0, 0.0), W=48, H=40, P=40):
    """Returns (oracle grads, autograd grads) on a scene whose decisions are well away from thresholds."""
    for s in range(seed, seed + 40):
        p, a, rs = _scene(P, W, H, 48.0, 0.06, seed=s, sh_degree=sh_degree)
        rs = rs._replace(bg=torch.tensor(bg, dtype=torch.float32))
        cov = None
        if use_cov3D:
            cov = DT.cov3d_from(a["scales"].double(), a["rotations"].double(), 1.0).float().numpy()
        st = _fwd(a, rs, cov3D=cov)
        dl = torch.randn(3, H, W, generator=torch.Generator().manual_seed(s + 1000))
        leaf = {k: a[k].double().clone().requires_grad_(True)
                for k in ("means3D", "opacities", "scales", "rotations")}
        kw = {}
        if sh_degree >= 0:
            kw["shs"] = a["shs"].double().clone().requires_grad_(True)
        else:
            kw["colors"] = a["colors_precomp"].double().clone().requires_grad_(True)
        if use_cov3D:
            kw["cov3D"] = torch.tensor(cov, dtype=torch.float64, requires_grad=True)
        else:
            kw["scales"], kw["rotations"] = leaf["scales"], leaf["rotations"]
        img, ex = DT.dense_forward(st, leaf["means3D"], leaf["opacities"], **kw)
        if ex["margin"] < 1e-3:
            continue  # a (pixel, Gaussian) pair sits on a threshold: f32/f64 could branch apart
        np.testing.assert_allclose(img.detach().numpy(), st["color"], rtol=1e-4, atol=2e-5)
        (img * dl.double()).sum().backward()
        g = O.backward(st, dl.numpy())
        ref = {"means3D": leaf["means3D"].grad, "opacities": leaf["opacities"].grad,
               "cov3D": ex["cov3D"].grad, "colors": ex["colors"].grad}
        W2, H2 = 0.5 * W, 0.5 * H
        ref["means2D"] = ex["xy"].grad * torch.tensor([W2, H2], dtype=torch.float64)
        if not use_cov3D:
            ref["scales"], ref["rotations"] = leaf["scales"].grad, leaf["rotations"].grad
        if sh_degree >= 0:
            ref["sh"] = kw["shs"].grad
        return g, {k: v.numpy() for k, v in ref.items()}, st
    pytest.skip("no threshold-free scene found")


def _close(name, got, ref, rel=2e-4):
    """|got - ref| <= rel * |ref| + 1e-5 * max|ref|: fp32 oracle (fp32 sums) vs fp64 autograd."""
    got, ref = np.asarray(got, np.float64), np.asarray(ref, np.float64)
    scale = np.abs(ref).max() + 1e-30
    bad = np.abs(got - ref) > rel * np.abs(ref) + 1e-5 * scale
    assert not bad.any(), f"{name}: {bad.sum()} mismatches, worst {np.abs(got - ref)[bad].max():.3g} (scale {scale:.3g})"


@pytest.mark.parametrize("case", ["rgb", "rgb_bg", "cov3d", "sh0", "sh1", "sh2", "sh3"])
def test_backward_matches_autograd(case):
    kw = dict(rgb={}, rgb_bg=dict(bg=(0.3, 0.6, 0.9)), cov3d=dict(use_cov3D=True),
              sh0=dict(sh_degree=0), sh1=dict(sh_degree=1), sh2=dict(sh_degree=2),
              sh3=dict(sh_degree=3))[case]
    g, ref, st = _autograd_case(seed=7, **kw)
    vis = st["radii"] > 0
    assert vis.sum() > 10
    _close("means2D", g["means2D"][:, :2], ref["means2D"])
    assert not g["means2D"][:, 2].any()
    _close("opacities", g["opacities"], ref["opacities"])
    _close("means3D", g["means3D"], ref["means3D"])
    _close("cov3D", g["cov3D"][vis], ref["cov3D"][vis])
    if "scales" in ref:
        _close("scales", g["scales"], ref["scales"])
        _close("rotations", g["rotations"], ref["rotations"])
    if "sh" in ref:
        _close("sh", g["sh"], ref["sh"])
    else:
        _close("colors", g["colors"], ref["colors"])
