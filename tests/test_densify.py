"""Densification with Adam state surgery.

CPU: the numpy oracle (oracle/densify_oracle.py) reproduces the reference's densify_gaussians
(external.py:211-314, run by tests/golden/gen_golden.py on seeded data with a populated torch Adam)
at i = 500 / 3000 / 5000: every parameter row, Adam moment and statistic bit-exact, except the split
copies' means (R q * sample: matrix-product rounding, <= 1e-6 absolute) and log-scales (exp / log
rounding, <= 1e-6 absolute).  GPU (-m gpu): splat_densify through the C ABI against the same golden
outputs (fed the reference's recorded torch.normal draw), against the oracle on a 200k-Gaussian
random cloud, and the statistics kernels against the reference's densify statistics sequence.
"""
import os

import numpy as np
import pytest
import torch

from oracle import densify_oracle as DO

GOLD = np.load(os.path.join(os.path.dirname(__file__), "golden", "reference_harness.npz"))
SPLIT_TOL = 1e-6
LR = {"means": 0.00016, "colors": 0.0025, "segmentation_masks": 0.0, "rotation_quaternions": 0.001,
      "opacity_logits": 0.05, "log_scales": 0.001, "camera_matrices": 1e-4, "camera_center": 1e-4}


def _case(c):
    pre = f"dens{c}_pre_"
    keys = [k[len(pre):] for k in GOLD.files if k.startswith(pre) and not k.startswith(pre + "m_")
            and not k.startswith(pre + "v_")]
    g = {k: GOLD[pre + k] for k in keys}
    m = {k: GOLD[pre + "m_" + k] for k in keys if k not in DO.GAUSSIAN_EXCLUDED}
    v = {k: GOLD[pre + "v_" + k] for k in keys if k not in DO.GAUSSIAN_EXCLUDED}
    return keys, g, m, v


def _compare(keys, got_p, got_m, got_v, c, n_base):
    """n_base = rows before the split copies (originals + clones kept): the split rows follow."""
    for k in keys:
        ref = GOLD[f"dens{c}_out_{k}"]
        got = np.asarray(got_p[k])
        assert got.shape == ref.shape, (k, got.shape, ref.shape)
        if k in ("means", "log_scales"):
            np.testing.assert_array_equal(got[:n_base], ref[:n_base], err_msg=k)
            np.testing.assert_allclose(got[n_base:], ref[n_base:], rtol=0, atol=SPLIT_TOL, err_msg=k)
        else:
            np.testing.assert_array_equal(got, ref, err_msg=k)
        if k in got_m:
            np.testing.assert_array_equal(np.asarray(got_m[k]), GOLD[f"dens{c}_out_m_{k}"], err_msg=k)
            np.testing.assert_array_equal(np.asarray(got_v[k]), GOLD[f"dens{c}_out_v_{k}"], err_msg=k)


@pytest.mark.parametrize("c", range(3))
def test_oracle_matches_reference_densify(c):
    keys, g, m, v = _case(c)
    p2, m2, v2, acc, cnt, mr, info = DO.densify(
        g, m, v, GOLD[f"dens{c}_in_acc"], GOLD[f"dens{c}_in_count"], GOLD[f"dens{c}_in_max_radii"],
        GOLD[f"dens{c}_in_vis"], GOLD[f"dens{c}_in_m2grad"], float(GOLD[f"dens{c}_scene_radius"]),
        int(GOLD[f"dens{c}_iter"]), GOLD[f"dens{c}_samples"])
    assert info["n_clone"] > 0 and info["n_split"] > 0
    _compare(keys, p2, m2, v2, c, _first_split_row(g, c))
    for nm, a in {"acc": acc, "count": cnt, "max_radii": mr}.items():
        np.testing.assert_array_equal(a, GOLD[f"dens{c}_out_{nm}"])


def _first_split_row(g, c):
    """Row index where the split copies begin in the densified arrays (after kept originals and kept
    clones): recomputed from the oracle's own decisions."""
    acc = GOLD[f"dens{c}_in_acc"].copy()
    cnt = GOLD[f"dens{c}_in_count"].copy()
    acc, cnt = DO.accumulate_grads(GOLD[f"dens{c}_in_vis"], GOLD[f"dens{c}_in_m2grad"], acc, cnt)
    with np.errstate(invalid="ignore", divide="ignore"):
        avg = acc / cnt
    avg[np.isnan(avg)] = 0
    i = int(GOLD[f"dens{c}_iter"])
    sr = float(GOLD[f"dens{c}_scene_radius"])
    ms = np.exp(g["log_scales"]).max(1)
    hot = avg >= np.float32(0.0002)
    clone = hot & (ms <= np.float32(0.01 * sr))
    split = hot & (ms > np.float32(0.01 * sr))
    pr = (1 / (1 + np.exp(-g["opacity_logits"][:, 0])) < np.float32(0.25 if i == 5000 else 0.005))
    if i >= 3000:
        pr = pr | (ms > np.float32(0.1 * sr))
    return int((~split & ~pr).sum() + (clone & ~pr).sum())


def test_oracle_statistics_match_reference():
    radii, grads = GOLD["dstat_in_radii"], GOLD["dstat_in_grad"]
    P = radii.shape[1]
    mr, acc, cnt = np.zeros(P, np.float32), np.zeros(P, np.float32), np.zeros(P, np.float32)
    for r, g in zip(radii, grads):
        mr, vis = DO.update_max_radii(r, mr)
        acc, cnt = DO.accumulate_grads(vis, g, acc, cnt)
    np.testing.assert_array_equal(mr, GOLD["dstat_out_max_radii"])
    np.testing.assert_array_equal(cnt, GOLD["dstat_out_visibility_count"])
    np.testing.assert_allclose(acc, GOLD["dstat_out_grad_accum"], rtol=1e-6)


# ------------------------------------------------------------------------------------------------
def _gpu_setup(cuda, keys, g, m, v, step=2.0):
    params = {k: torch.nn.Parameter(torch.from_numpy(g[k]).to(cuda).contiguous()) for k in keys}
    opt = torch.optim.Adam([{"params": [p], "name": k, "lr": LR.get(k, 1e-3)} for k, p in params.items()],
                           lr=0.0, eps=1e-15)
    for k in m:
        opt.state[params[k]] = {"step": torch.tensor(step), "exp_avg": torch.from_numpy(m[k]).to(cuda),
                                "exp_avg_sq": torch.from_numpy(v[k]).to(cuda)}
    return params, opt


def _dv(cuda, acc, cnt, mr, vis, m2grad):
    from splat_densify import DensificationVariables
    m2 = torch.zeros(len(acc), 3, device=cuda, requires_grad=True)
    m2.grad = torch.from_numpy(m2grad).to(cuda)
    return DensificationVariables(
        visibility_count=torch.from_numpy(cnt).to(cuda).clone(),
        mean_2d_gradients_accumulated=torch.from_numpy(acc).to(cuda).clone(),
        max_2d_radii=torch.from_numpy(mr).to(cuda).clone(),
        gaussian_is_visible_mask=torch.from_numpy(vis).to(cuda), means_2d=m2)


@pytest.mark.gpu
@pytest.mark.parametrize("c", range(3))
def test_gpu_densify_matches_reference(cuda, c):
    import splat_densify
    keys, g, m, v = _case(c)
    params, opt = _gpu_setup(cuda, keys, g, m, v)
    dv = _dv(cuda, GOLD[f"dens{c}_in_acc"], GOLD[f"dens{c}_in_count"], GOLD[f"dens{c}_in_max_radii"],
             GOLD[f"dens{c}_in_vis"], GOLD[f"dens{c}_in_m2grad"])
    samples = torch.from_numpy(GOLD[f"dens{c}_samples"]).to(cuda)
    seen = {}

    def sample_fn(mean, std):
        seen["std"] = std.cpu().numpy()
        assert mean.shape == std.shape == samples.shape
        return samples.clone()

    splat_densify.densify_gaussians(params, dv, float(GOLD[f"dens{c}_scene_radius"]), opt,
                                    int(GOLD[f"dens{c}_iter"]), sample_fn=sample_fn)
    torch.cuda.synchronize()
    got_p = {k: params[k].detach().cpu().numpy() for k in keys}
    got_m = {k: opt.state[params[k]]["exp_avg"].cpu().numpy() for k in m}
    got_v = {k: opt.state[params[k]]["exp_avg_sq"].cpu().numpy() for k in m}
    _compare(keys, got_p, got_m, got_v, c, _first_split_row(g, c))
    for k in m:
        assert float(opt.state[params[k]]["step"]) == float(GOLD[f"dens{c}_out_step_{k}"])
        assert opt.param_groups[[gr["name"] for gr in opt.param_groups].index(k)]["params"][0] is params[k]
    np.testing.assert_array_equal(dv.visibility_count.cpu().numpy(), GOLD[f"dens{c}_out_count"])
    np.testing.assert_array_equal(dv.mean_2d_gradients_accumulated.cpu().numpy(), GOLD[f"dens{c}_out_acc"])
    np.testing.assert_array_equal(dv.max_2d_radii.cpu().numpy(), GOLD[f"dens{c}_out_max_radii"])
    # the std handed to torch.normal is exp(log_scales) of the split rows, twice (external.py:257-259)
    _, _, _, _, _, _, info = DO.densify(g, m, v, GOLD[f"dens{c}_in_acc"], GOLD[f"dens{c}_in_count"],
                                        GOLD[f"dens{c}_in_max_radii"], GOLD[f"dens{c}_in_vis"],
                                        GOLD[f"dens{c}_in_m2grad"], float(GOLD[f"dens{c}_scene_radius"]),
                                        int(GOLD[f"dens{c}_iter"]), GOLD[f"dens{c}_samples"])
    np.testing.assert_allclose(seen["std"], info["stds"], rtol=1e-6, atol=0)


@pytest.mark.gpu
def test_gpu_densify_large_random_vs_oracle(cuda):
    import splat_densify
    rng = np.random.default_rng(5)
    P, sr, it = 200_000, 3.0, 3000
    g = {"means": rng.standard_normal((P, 3), np.float32), "colors": rng.random((P, 3), np.float32),
         "segmentation_masks": rng.random((P, 3), np.float32),
         "rotation_quaternions": rng.standard_normal((P, 4), np.float32),
         "opacity_logits": (3 * rng.standard_normal((P, 1))).astype(np.float32),
         "log_scales": (np.log(0.03) + 0.8 * rng.standard_normal((P, 3))).astype(np.float32),
         "camera_matrices": np.zeros((50, 3), np.float32), "camera_center": np.zeros((50, 3), np.float32)}
    keys = list(g)
    m = {k: rng.standard_normal(g[k].shape).astype(np.float32) * 1e-3 for k in keys if k not in DO.GAUSSIAN_EXCLUDED}
    v = {k: rng.random(g[k].shape, np.float32) * 1e-6 for k in m}
    cnt = rng.integers(0, 6, P).astype(np.float32)
    acc = (cnt * 4e-4 * rng.random(P)).astype(np.float32)
    vis = rng.random(P) > 0.3
    m2g = (3e-4 * rng.standard_normal((P, 3))).astype(np.float32)
    mr = rng.integers(0, 9, P).astype(np.float32)
    params, opt = _gpu_setup(cuda, keys, g, m, v)
    dv = _dv(cuda, acc, cnt, mr, vis, m2g)
    drawn = {}

    def sample_fn(mean, std):
        drawn["s"] = torch.normal(mean=mean, std=std)
        return drawn["s"]

    info = splat_densify.densify_gaussians(params, dv, sr, opt, it, sample_fn=sample_fn)
    assert info["n_split"] > 1000 and info["n_keep_clone"] > 1000
    p2, m2, v2, *_ = DO.densify(g, m, v, acc, cnt, mr, vis, m2g, sr, it, drawn["s"].cpu().numpy())
    n_base = info["n_keep_orig"] + info["n_keep_clone"]
    for k in keys:
        got, ref = params[k].detach().cpu().numpy(), p2[k]
        assert got.shape == ref.shape, k
        if k in ("means", "log_scales"):
            np.testing.assert_array_equal(got[:n_base], ref[:n_base], err_msg=k)
            np.testing.assert_allclose(got[n_base:], ref[n_base:], rtol=0, atol=4e-6, err_msg=k)
        else:
            np.testing.assert_array_equal(got, ref, err_msg=k)
        if k in m2:
            np.testing.assert_array_equal(opt.state[params[k]]["exp_avg"].cpu().numpy(), m2[k])
            np.testing.assert_array_equal(opt.state[params[k]]["exp_avg_sq"].cpu().numpy(), v2[k])


@pytest.mark.gpu
def test_gpu_densify_c3_size_vs_oracle(cuda):
    """BASELINE configs[2]'s densify.py clone / split at its size: the bench's 1M-Gaussian densify
    event (bench.py densify_call_site: densify.py's parameter dict, statistics scaled so ~20 % of the
    seen Gaussians pass the 0.0002 threshold, scene radius at 100 x the median maximum scale, i = 600)
    through the native path against the golden-pinned numpy restatement of external.py:211-314
    (oracle/densify_oracle.py) with the split samples shared: row counts bit-exact, every row and
    Adam moment bit-exact except the split copies' means / log-scales (<= 4e-6 absolute)."""
    import splat_densify
    import splat_scenes as S
    P, it = 1_000_000, 600
    base = S.synthetic_cloud(P, 0.005, seed=0, device="cpu")
    rng = np.random.default_rng(7)
    g = {"means": base["means"].numpy(), "colors": base["colors"].numpy(),
         "segmentation_masks": np.repeat((rng.random((P, 1)) > 0.5).astype(np.float32), 3, 1),
         "rotation_quaternions": base["rotation_quaternions"].numpy(),
         "opacity_logits": base["opacity_logits"].numpy(), "log_scales": base["log_scales"].numpy(),
         "camera_matrices": np.zeros((50, 3), np.float32), "camera_center": np.zeros((50, 3), np.float32)}
    keys = list(g)
    m = {k: (rng.standard_normal(g[k].shape) * 1e-3).astype(np.float32) for k in keys if k not in DO.GAUSSIAN_EXCLUDED}
    v = {k: (rng.random(g[k].shape) * 1e-6).astype(np.float32) for k in m}
    cnt = rng.integers(0, 6, P).astype(np.float32)
    avg = rng.random(P).astype(np.float32) * np.float32(2.5e-4)  # ~20 % of the seen rows >= 0.0002
    acc = (avg * cnt).astype(np.float32)
    vis = rng.random(P) > 0.4
    m2g = (3e-4 * rng.standard_normal((P, 3))).astype(np.float32)
    mr = rng.integers(0, 9, P).astype(np.float32)
    sr = float(100.0 * np.median(np.exp(g["log_scales"]).max(axis=1)))
    params, opt = _gpu_setup(cuda, keys, g, m, v)
    dv = _dv(cuda, acc, cnt, mr, vis, m2g)
    drawn = {}

    def sample_fn(mean, std):
        drawn["s"] = torch.normal(mean=mean, std=std)
        return drawn["s"]

    info = splat_densify.densify_gaussians(params, dv, sr, opt, it, sample_fn=sample_fn)
    torch.cuda.synchronize()
    p2, m2, v2, acc2, cnt2, mr2, oinfo = DO.densify(g, m, v, acc, cnt, mr, vis, m2g, sr, it, drawn["s"].cpu().numpy())
    assert info["n_split"] > 10_000 and info["n_keep_clone"] > 10_000
    assert info["n_split"] == oinfo["n_split"] and oinfo["n_clone"] >= info["n_keep_clone"]
    assert info["P_out"] == p2["means"].shape[0] > P
    n_base = info["n_keep_orig"] + info["n_keep_clone"]
    for k in keys:
        got, ref = params[k].detach().cpu().numpy(), p2[k]
        assert got.shape == ref.shape, k
        if k in ("means", "log_scales"):
            np.testing.assert_array_equal(got[:n_base], ref[:n_base], err_msg=k)
            np.testing.assert_allclose(got[n_base:], ref[n_base:], rtol=0, atol=4e-6, err_msg=k)
        else:
            np.testing.assert_array_equal(got, ref, err_msg=k)
        if k in m2:
            np.testing.assert_array_equal(opt.state[params[k]]["exp_avg"].cpu().numpy(), m2[k])
            np.testing.assert_array_equal(opt.state[params[k]]["exp_avg_sq"].cpu().numpy(), v2[k])
    np.testing.assert_array_equal(dv.visibility_count.cpu().numpy(), cnt2)
    np.testing.assert_array_equal(dv.mean_2d_gradients_accumulated.cpu().numpy(), acc2)
    np.testing.assert_array_equal(dv.max_2d_radii.cpu().numpy(), mr2)


@pytest.mark.gpu
def test_gpu_statistics_match_reference(cuda):
    import splat_densify
    radii, grads = GOLD["dstat_in_radii"], GOLD["dstat_in_grad"]
    P = radii.shape[1]
    dv = splat_densify.DensificationVariables(visibility_count=torch.zeros(P, device=cuda),
                                             mean_2d_gradients_accumulated=torch.zeros(P, device=cuda),
                                             max_2d_radii=torch.zeros(P, device=cuda))
    for r, gr in zip(radii, grads):
        splat_densify.update_max_2d_radii_and_visibility_mask(torch.from_numpy(r).to(cuda), dv)
        m2 = torch.zeros(P, 3, device=cuda, requires_grad=True)
        m2.grad = torch.from_numpy(gr).to(cuda)
        dv.means_2d = m2
        splat_densify.accumulate_mean_2d_gradients(dv)
    np.testing.assert_array_equal(dv.max_2d_radii.cpu().numpy(), GOLD["dstat_out_max_radii"])
    np.testing.assert_array_equal(dv.visibility_count.cpu().numpy(), GOLD["dstat_out_visibility_count"])
    np.testing.assert_allclose(dv.mean_2d_gradients_accumulated.cpu().numpy(), GOLD["dstat_out_grad_accum"],
                               rtol=1e-6)


@pytest.mark.gpu
def test_gpu_densify_off_schedule_and_empty(cuda):
    """i = 550: statistics only; i = 600 with no hot Gaussians: unchanged rows, statistics reset."""
    import splat_densify
    keys, g, m, v = _case(0)
    params, opt = _gpu_setup(cuda, keys, g, m, v)
    P = g["means"].shape[0]
    dv = _dv(cuda, np.zeros(P, np.float32), np.zeros(P, np.float32), np.zeros(P, np.float32),
             np.ones(P, bool), np.zeros((P, 3), np.float32))
    assert splat_densify.densify_gaussians(params, dv, 2.0, opt, 550) is None
    assert float(dv.visibility_count.sum()) == P
    info = splat_densify.densify_gaussians(params, dv, 2.0, opt, 600)
    assert info["n_split"] == 0 and info["n_keep_clone"] == 0
    pr = 1 / (1 + np.exp(-g["opacity_logits"][:, 0])) < np.float32(0.005)
    np.testing.assert_array_equal(params["colors"].detach().cpu().numpy(), g["colors"][~pr])
    assert float(dv.visibility_count.abs().sum()) == 0 and dv.visibility_count.numel() == int((~pr).sum())


def test_oracle_opacity_reset_only_at_3000():
    """external.py:306-314 sits inside `if i <= 5000:` (external.py:218): the opacity reset fires at
    i = 3000 and never again (i = 6000, 9000, ... leave opacity_logits and its moments alone)."""
    keys, g, m, v = _case(0)
    P = g["means"].shape[0]
    z = np.zeros(P, np.float32)
    for i, resets in ((3000, True), (6000, False), (9000, False), (27000, False)):
        p2, m2, v2, *_ = DO.densify(g, m, v, z, z, z, np.zeros(P, bool), np.zeros((P, 3), np.float32), 2.0, i,
                                    np.zeros((0, 3), np.float32))
        if resets:
            assert np.allclose(1 / (1 + np.exp(-p2["opacity_logits"])), 0.01, atol=1e-6)
            assert not m2["opacity_logits"].any()
        else:
            np.testing.assert_array_equal(p2["opacity_logits"], g["opacity_logits"])
            np.testing.assert_array_equal(m2["opacity_logits"], m["opacity_logits"])
            np.testing.assert_array_equal(v2["opacity_logits"], v["opacity_logits"])


@pytest.mark.gpu
def test_gpu_opacity_reset_only_at_3000(cuda):
    import splat_densify
    keys, g, m, v = _case(0)
    P = g["means"].shape[0]
    for i, resets in ((6000, False), (9000, False), (3000, True)):
        params, opt = _gpu_setup(cuda, keys, g, m, v)
        dv = _dv(cuda, np.zeros(P, np.float32), np.zeros(P, np.float32), np.zeros(P, np.float32),
                 np.zeros(P, bool), np.zeros((P, 3), np.float32))
        splat_densify.densify_gaussians(params, dv, 2.0, opt, i)
        ol = params["opacity_logits"].detach().cpu().numpy()
        st = opt.state[params["opacity_logits"]]
        if resets:
            assert np.allclose(1 / (1 + np.exp(-ol)), 0.01, atol=1e-6) and not st["exp_avg"].any()
        else:
            np.testing.assert_array_equal(ol, g["opacity_logits"])
            np.testing.assert_array_equal(st["exp_avg"].cpu().numpy(), m["opacity_logits"])
