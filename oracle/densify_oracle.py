"""CPU oracle of Gaussian densification with Adam state surgery (numpy float32).

TEST INFRASTRUCTURE ONLY: imported by ``tests/`` as the checker, never as the thing measured or
shipped.

Restates, array by array:
  * ``update_max_2d_radii_and_visibility_mask`` (densify.py:154-162) and
    ``accumulate_mean_2d_gradients`` (external.py:113-124);
  * ``densify_gaussians`` (external.py:211-314) with ``cat_params_to_optimizer`` (:144-170),
    ``remove_points`` (:173-204) and ``update_params_and_optimizer`` (:127-141): clone small
    high-gradient Gaussians, split large ones into two samples of N(0, scale) rotated by
    ``build_rotation`` (:27-46) with scales / 1.6, drop the split originals, prune by opacity (and
    big world-space scale from i = 3000), reset Adam moments of new rows to zero, reset the
    statistics, and reset opacities at i = 3000 (the reset sits inside ``if i <= 5000``).

The split samples are an input (the reference draws them with ``torch.normal``; the tests feed the
values the reference drew).  Pinned against the reference's own outputs in
tests/golden/reference_harness.npz (tests/golden/gen_golden.py imports external.py / densify.py).
"""
from __future__ import annotations

import numpy as np

GAUSSIAN_EXCLUDED = ("camera_matrices", "camera_center")
f32 = np.float32


def update_max_radii(radii, max_radii):
    """densify.py:154-162 -> (max_radii', visible)."""
    vis = radii > 0
    out = max_radii.copy()
    out[vis] = np.maximum(radii[vis].astype(f32), max_radii[vis])
    return out, vis


def accumulate_grads(vis, m2grad, acc, count):
    """external.py:113-124."""
    acc, count = acc.copy(), count.copy()
    g = m2grad[vis, :2].astype(f32)
    acc[vis] += np.sqrt(g[:, 0] * g[:, 0] + g[:, 1] * g[:, 1]).astype(f32)
    count[vis] += f32(1)
    return acc, count


def build_rotation(q):
    """external.py:27-46 (float32, normalised)."""
    q = q.astype(f32)
    norm = np.sqrt(q[:, 0] * q[:, 0] + q[:, 1] * q[:, 1] + q[:, 2] * q[:, 2] + q[:, 3] * q[:, 3])
    q = q / norm[:, None]
    r, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    R = np.zeros((q.shape[0], 3, 3), f32)
    R[:, 0, 0] = 1 - 2 * (y * y + z * z)
    R[:, 0, 1] = 2 * (x * y - r * z)
    R[:, 0, 2] = 2 * (x * z + r * y)
    R[:, 1, 0] = 2 * (x * y + r * z)
    R[:, 1, 1] = 1 - 2 * (x * x + z * z)
    R[:, 1, 2] = 2 * (y * z - r * x)
    R[:, 2, 0] = 2 * (x * z - r * y)
    R[:, 2, 1] = 2 * (y * z + r * x)
    R[:, 2, 2] = 1 - 2 * (x * x + y * y)
    return R


def _sigmoid(x):
    return (f32(1) / (f32(1) + np.exp(-x.astype(f32)))).astype(f32)


def densify(params, m, v, acc, count, max_radii, vis, m2grad, scene_radius, i, samples):
    """external.py:211-314.  ``params``/``m``/``v``: dicts name -> float32 array (m/v: Adam exp_avg /
    exp_avg_sq, absent for a parameter without optimizer state).  Returns (params, m, v, acc, count,
    max_radii, info) as the reference leaves them."""
    params = {k: a.copy() for k, a in params.items()}
    m = {k: a.copy() for k, a in m.items()}
    v = {k: a.copy() for k, a in v.items()}
    keys = [k for k in params if k not in GAUSSIAN_EXCLUDED]
    info = {}
    if i <= 5000:
        acc, count = accumulate_grads(vis, m2grad, acc, count)
        if i >= 500 and i % 100 == 0:
            thr = f32(0.0002)
            with np.errstate(invalid="ignore", divide="ignore"):
                avg = (acc / count).astype(f32)
            avg[np.isnan(avg)] = 0.0
            ls = params["log_scales"]
            max_scales = np.exp(ls).max(axis=1)
            small = f32(0.01 * scene_radius)
            to_clone = (avg >= thr) & (max_scales <= small)
            # clones appended (cat_params_to_optimizer): zero Adam moments
            nc = int(to_clone.sum())
            for k in keys:
                params[k] = np.concatenate([params[k], params[k][to_clone]])
                if k in m:
                    z = np.zeros((nc,) + m[k].shape[1:], f32)
                    m[k], v[k] = np.concatenate([m[k], z]), np.concatenate([v[k], z])
            n1 = params["means"].shape[0]
            padded = np.zeros(n1, f32)
            padded[:avg.shape[0]] = avg
            to_split = (padded >= thr) & (np.exp(params["log_scales"]).max(axis=1) > small)
            S = int(to_split.sum())
            stds = np.tile(np.exp(params["log_scales"])[to_split], (2, 1))
            if callable(samples):  # drawn now from the split rows' stds (e.g. a broadcast draw)
                samples = np.asarray(samples(stds), np.float32)
            assert samples.shape == (2 * S, 3), (samples.shape, S)
            new = {k: np.tile(params[k][to_split], (2, 1)) for k in keys}
            rots = np.tile(build_rotation(params["rotation_quaternions"][to_split]), (2, 1, 1))
            new["means"] = (new["means"] + np.einsum("nij,nj->ni", rots.astype(np.float64),
                                                     samples.astype(np.float64)).astype(f32)).astype(f32)
            new["log_scales"] = np.log((np.exp(new["log_scales"]) / f32(0.8 * 2)).astype(f32)).astype(f32)
            for k in keys:
                params[k] = np.concatenate([params[k], new[k]])
                if k in m:
                    m[k] = np.concatenate([m[k], np.zeros_like(new[k])])
                    v[k] = np.concatenate([v[k], np.zeros_like(new[k])])
            n2 = params["means"].shape[0]
            acc, count, max_radii = np.zeros(n2, f32), np.zeros(n2, f32), np.zeros(n2, f32)
            to_remove = np.concatenate([to_split, np.zeros(2 * S, bool)])
            keep = ~to_remove
            for k in keys:
                params[k] = params[k][keep]
                if k in m:
                    m[k], v[k] = m[k][keep], v[k][keep]
            acc, count, max_radii = acc[keep], count[keep], max_radii[keep]
            remove_threshold = 0.25 if i == 5000 else 0.005
            to_remove = (_sigmoid(params["opacity_logits"]) < f32(remove_threshold)).squeeze(-1)
            if i >= 3000:
                big = np.exp(params["log_scales"]).max(axis=1) > f32(0.1 * scene_radius)
                to_remove = to_remove | big
            keep = ~to_remove
            for k in keys:
                params[k] = params[k][keep]
                if k in m:
                    m[k], v[k] = m[k][keep], v[k][keep]
            acc, count, max_radii = acc[keep], count[keep], max_radii[keep]
            info = {"n_clone": int(to_clone.sum()), "n_split": S, "stds": stds}
        if i > 0 and i % 3000 == 0:  # external.py:306-314, inside `if i <= 5000` (i = 3000 only)
            x = np.full_like(params["opacity_logits"], f32(0.01))
            params["opacity_logits"] = np.log(x / (f32(1) - x)).astype(f32)
            if "opacity_logits" in m:
                m["opacity_logits"] = np.zeros_like(params["opacity_logits"])
                v["opacity_logits"] = np.zeros_like(params["opacity_logits"])
    return params, m, v, acc, count, max_radii, info
