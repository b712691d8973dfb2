"""Densification on the HIP kernels of ``libgsr.so``.

Drop-ins with the reference's names, signatures and effects:

* ``update_max_2d_radii_and_visibility_mask(radii, densification_variables)`` -- densify.py:154-162
* ``accumulate_mean_2d_gradients(densification_variables)`` -- external.py:113-124
* ``densify_gaussians(gaussian_cloud_parameters, densification_variables, scene_radius, optimizer, i)``
  -- external.py:211-314: every 100 iterations in [500, 5000] clone small high-gradient Gaussians,
  split large ones in two, drop the split originals, prune transparent (and from i = 3000 huge)
  ones, with the optimizer's Adam moments carried along (``cat_params_to_optimizer`` /
  ``remove_points``, external.py:144-204) and the statistics reset; at i = 3000 reset the
  opacities (external.py:306-314).

The reference runs ~60 torch ops per densification, reallocating every parameter and both Adam
moments three times; here one plan kernel pair decides every row's fate (one host sync for the
output size, as the reference's boolean indexing has) and one apply kernel writes each output row
and moment once.  Split samples are drawn with ``torch.normal`` exactly as the reference draws them
(same shapes, same generator), so a seeded run matches it.  ``optimizer`` is a ``torch.optim.Adam``
(or ``splat_adam.FusedAdam``) whose param groups are named after the parameters (densify.py:68-86).
There is no CPU path.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import torch

from diff_gaussian_rasterization import _C

__all__ = ["DensificationVariables", "update_max_2d_radii_and_visibility_mask", "accumulate_mean_2d_gradients",
           "densify_gaussians", "inverse_sigmoid"]


@dataclass
class DensificationVariables:
    """shared.py:21-27 (same fields and defaults)."""
    visibility_count: torch.Tensor
    mean_2d_gradients_accumulated: torch.Tensor
    max_2d_radii: torch.Tensor
    gaussian_is_visible_mask: torch.Tensor = None
    means_2d: torch.Tensor = None


GAUSSIAN_EXCLUDED = ("camera_matrices", "camera_center")  # external.py:236,250,180
ROLES = {"means": 1, "log_scales": 2}  # enum gsr_densify_role


class _Settings(ctypes.Structure):
    _fields_ = [("P", ctypes.c_int), ("grad_threshold", ctypes.c_float), ("small_scale", ctypes.c_float),
                ("big_scale", ctypes.c_float), ("remove_opacity", ctypes.c_float), ("prune_big", ctypes.c_int),
                ("split_divisor", ctypes.c_float), ("grad_accum", ctypes.c_void_p),
                ("vis_count", ctypes.c_void_p), ("log_scales", ctypes.c_void_p),
                ("opacity_logits", ctypes.c_void_p), ("rotation_quaternions", ctypes.c_void_p)]


class _Counts(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in ("n_keep_orig", "n_keep_clone", "n_split", "n_keep_split", "P_out")]


class _Column(ctypes.Structure):
    _fields_ = [("width", ctypes.c_int), ("role", ctypes.c_int)] + [
        (n, ctypes.c_void_p) for n in ("src", "exp_avg", "exp_avg_sq", "dst", "dst_exp_avg", "dst_exp_avg_sq")]


_bound = False


def _lib():
    global _bound
    L = _C.load_library()
    if not _bound:
        vp, i = ctypes.c_void_p, ctypes.c_int
        L.gsr_densify_update_radii.argtypes = [i, vp, vp, vp, vp]
        L.gsr_densify_accumulate_grads.argtypes = [i, vp, vp, vp, vp, vp]
        L.gsr_densify_workspace_bytes.restype = ctypes.c_size_t
        L.gsr_densify_workspace_bytes.argtypes = [i]
        L.gsr_densify_plan.argtypes = [ctypes.POINTER(_Settings), vp, ctypes.POINTER(_Counts), vp]
        L.gsr_densify_split_stds.argtypes = [ctypes.POINTER(_Settings), vp, vp, vp]
        L.gsr_densify_apply.argtypes = [ctypes.POINTER(_Settings), vp, ctypes.POINTER(_Counts), vp, i,
                                        ctypes.POINTER(_Column), vp]
        for n in ("gsr_densify_update_radii", "gsr_densify_accumulate_grads", "gsr_densify_plan",
                  "gsr_densify_split_stds", "gsr_densify_apply"):
            getattr(L, n).restype = i
        _bound = True
    return L


def _dev_ptr(t, dtype=torch.float32):
    if not t.is_cuda:
        raise RuntimeError("splat_densify: tensors must be on the GPU (no CPU path)")
    if t.dtype != dtype or not t.is_contiguous():
        raise RuntimeError(f"splat_densify: expected a contiguous {dtype} tensor, got {t.dtype}")
    return t.data_ptr() if t.numel() else None


def update_max_2d_radii_and_visibility_mask(radii, densification_variables):
    """densify.py:154-162."""
    dv = densification_variables
    L = _lib()
    P = radii.numel()
    r = radii.contiguous().to(torch.int32)
    visible = torch.empty(P, dtype=torch.bool, device=radii.device)
    _C._check(L.gsr_densify_update_radii(P, _dev_ptr(r, torch.int32), _dev_ptr(dv.max_2d_radii),
                                         _dev_ptr(visible, torch.bool), _C._stream_ptr(radii.device)))
    dv.gaussian_is_visible_mask = visible


def accumulate_mean_2d_gradients(densification_variables):
    """external.py:113-124: grad_accum[vis] += |means2D.grad[vis, :2]|, visibility_count[vis] += 1."""
    dv = densification_variables
    L = _lib()
    vis = dv.gaussian_is_visible_mask.contiguous()
    if vis.dtype != torch.bool:
        raise RuntimeError("gaussian_is_visible_mask must be a bool mask")
    grad = dv.means_2d.grad.contiguous().float()
    P = vis.numel()
    _C._check(L.gsr_densify_accumulate_grads(P, _dev_ptr(vis, torch.bool), _dev_ptr(grad),
                                             _dev_ptr(dv.mean_2d_gradients_accumulated), _dev_ptr(dv.visibility_count),
                                             _C._stream_ptr(vis.device)))


def inverse_sigmoid(x):
    """external.py:207-208."""
    return torch.log(x / (1 - x))


def _group_of(optimizer, name):
    return [g for g in optimizer.param_groups if g["name"] == name][0]


def _install(params, optimizer, name, new_value, new_m, new_v):
    """Swap a parameter (and its Adam moments) in the dict and the optimizer, as
    cat_params_to_optimizer / remove_points do (external.py:144-204)."""
    group = _group_of(optimizer, name)
    old = group["params"][0]
    stored = optimizer.state.get(old, None)
    new_p = torch.nn.Parameter(new_value.requires_grad_(True))
    if stored is not None:
        stored["exp_avg"], stored["exp_avg_sq"] = new_m, new_v
        del optimizer.state[old]
        optimizer.state[new_p] = stored
    group["params"][0] = new_p
    params[name] = new_p


def _densify(params, dv, scene_radius, optimizer, i, sample_fn):
    L = _lib()
    dev = params["means"].device
    keys = [k for k in params.keys() if k not in GAUSSIAN_EXCLUDED]
    if len(keys) > 8:
        raise RuntimeError("splat_densify: at most 8 per-Gaussian parameters")
    P = params["means"].shape[0]
    ls = params["log_scales"].detach().contiguous()
    ol = params["opacity_logits"].detach().contiguous()
    rq = params["rotation_quaternions"].detach().contiguous()
    acc = dv.mean_2d_gradients_accumulated.contiguous()
    cnt = dv.visibility_count.contiguous()
    st = _Settings(P, 0.0002, 0.01 * scene_radius, 0.1 * scene_radius, 0.25 if i == 5000 else 0.005,
                   int(i >= 3000), 0.8 * 2, _dev_ptr(acc), _dev_ptr(cnt), _dev_ptr(ls), _dev_ptr(ol), _dev_ptr(rq))
    stream = _C._stream_ptr(dev)
    ws = torch.empty(L.gsr_densify_workspace_bytes(P), dtype=torch.uint8, device=dev)
    counts = _Counts()
    _C._check(L.gsr_densify_plan(ctypes.byref(st), ws.data_ptr(), ctypes.byref(counts), stream))
    S = counts.n_split
    stds = torch.empty((2 * S, 3), dtype=torch.float32, device=dev)
    if S:
        _C._check(L.gsr_densify_split_stds(ctypes.byref(st), ws.data_ptr(), stds.data_ptr(), stream))
    means = torch.zeros((stds.size(0), 3), device=dev)
    samples = (sample_fn or torch.normal)(mean=means, std=stds).float().contiguous()  # external.py:260-261
    P_out = counts.P_out
    cols, outs, keep = [], {}, [ws, samples, ls, ol, rq, acc, cnt]
    for k in keys:
        src = params[k].detach().contiguous()
        width = src.numel() // max(P, 1)
        stored = optimizer.state.get(_group_of(optimizer, k)["params"][0], None)
        dst = torch.empty((P_out,) + tuple(src.shape[1:]), dtype=torch.float32, device=dev)
        m = v = dm = dv_ = None
        if stored is not None and "exp_avg" in stored:
            m, v = stored["exp_avg"].contiguous(), stored["exp_avg_sq"].contiguous()
            dm, dv_ = torch.empty_like(dst), torch.empty_like(dst)
        outs[k] = (dst, dm, dv_)
        keep += [src, m, v]
        cols.append(_Column(width, ROLES.get(k, 0), _dev_ptr(src), m.data_ptr() if m is not None else None,
                            v.data_ptr() if v is not None else None, dst.data_ptr() if P_out else None,
                            dm.data_ptr() if dm is not None and P_out else None,
                            dv_.data_ptr() if dv_ is not None and P_out else None))
    if P_out:
        arr = (_Column * len(cols))(*cols)
        _C._check(L.gsr_densify_apply(ctypes.byref(st), ws.data_ptr(), ctypes.byref(counts),
                                      samples.data_ptr() if S else None, len(cols), arr, stream))
    for k in keys:
        dst, dm, dv_ = outs[k]
        _install(params, optimizer, k, dst, dm, dv_)
    z = lambda: torch.zeros(P_out, device=dev)  # noqa: E731 - statistics restart (external.py:273-281)
    dv.mean_2d_gradients_accumulated, dv.visibility_count, dv.max_2d_radii = z(), z(), z()
    return {"n_keep_orig": counts.n_keep_orig, "n_keep_clone": counts.n_keep_clone, "n_split": S,
            "n_keep_split": counts.n_keep_split, "P_out": P_out}


def densify_gaussians(gaussian_cloud_parameters, densification_variables, scene_radius, optimizer, i,
                      sample_fn=None, accumulate=True):
    """external.py:211-314.  ``sample_fn`` (optional, default ``torch.normal``) draws the split
    samples; tests pass the reference's recorded draw, the data-parallel path a rank-0 draw broadcast
    to every rank (splat_dp.broadcast_normal).  ``accumulate=False`` skips the per-call
    accumulate_mean_2d_gradients (external.py:219) for callers that accumulated their views' statistics
    already (splat_dp.DensifyStats).  Returns the row counts when this call densified, else None."""
    info = None
    if i <= 5000:
        if accumulate:
            accumulate_mean_2d_gradients(densification_variables)
        if (i >= 500) and (i % 100 == 0):
            info = _densify(gaussian_cloud_parameters, densification_variables, scene_radius, optimizer, i,
                            sample_fn)
        if i > 0 and i % 3000 == 0:
            # opacity reset (external.py:306-314, nested in `if i <= 5000`: it fires at i = 3000 only):
            # a new tensor, zeroed moments
            p = gaussian_cloud_parameters["opacity_logits"]
            new = inverse_sigmoid(torch.ones_like(p) * 0.01)
            group = _group_of(optimizer, "opacity_logits")
            stored = optimizer.state.get(group["params"][0], None)
            if stored is not None:
                _install(gaussian_cloud_parameters, optimizer, "opacity_logits", new, torch.zeros_like(new),
                         torch.zeros_like(new))
            else:
                _install(gaussian_cloud_parameters, optimizer, "opacity_logits", new, None, None)
    return info
