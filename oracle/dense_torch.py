"""Dense float64 torch restatement of the rasterizer forward, differentiated by ``torch.autograd``.

TEST INFRASTRUCTURE ONLY (checker for the C oracle's analytic backward; never shipped).

It recomputes the forward of ``oracle/gsr_oracle.c`` with differentiable torch ops and lets
autograd produce every gradient, so the oracle's hand-derived backward (render backward +
computeCov2D + projection + SH + Sigma3D chains) is checked against an independent
derivation.  The discrete decisions (tile membership, depth order, cull) are taken from the
oracle's forward state; the reference's gradient quirks are emulated explicitly:

* the alpha gradient ignores the ``min(0.99, .)`` clamp (straight-through on the clamp),
* ``means2D`` receives dL/d(pixel xy) scaled by (W/2, H/2), i.e. NDC units,
* quaternions enter Sigma3D unnormalised (no normalisation derivative),
* the depth image carries no gradient.

``threshold_margin`` reports how far every evaluated (pixel, Gaussian) pair sits from the
alpha >= 1/255 and T >= 1e-4 thresholds, so a test can make sure float32 (oracle) and float64
(here) take the same branches.
"""
from __future__ import annotations

import numpy as np
import torch

SH_C0 = 0.28209479177387814
SH_C1 = 0.4886025119029199
SH_C2 = [1.0925484305920792, -1.0925484305920792, 0.31539156525252005, -1.0925484305920792,
         0.5462742152960396]
SH_C3 = [-0.5900435899266435, 2.890611442640554, -0.4570457994644658, 0.3731763325901154,
         -0.4570457994644658, 1.445305721320277, -0.5900435899266435]


def _rot(q):
    r, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    # the kernel's R (glm column-major) equals build_rotation(q)^T for normalised q (external.py:27-46)
    R = torch.stack([
        torch.stack([1 - 2 * (y * y + z * z), 2 * (x * y + r * z), 2 * (x * z - r * y)], -1),
        torch.stack([2 * (x * y - r * z), 1 - 2 * (x * x + z * z), 2 * (y * z + r * x)], -1),
        torch.stack([2 * (x * z + r * y), 2 * (y * z - r * x), 1 - 2 * (x * x + y * y)], -1)], -2)
    return R  # R[i] maps rows: Sigma = R^T S^2 R


def cov3d_from(scales, rots, mod):
    R = _rot(rots)
    S = torch.diag_embed(mod * scales)
    M = S @ R
    Sig = M.transpose(1, 2) @ M
    return torch.stack([Sig[:, 0, 0], Sig[:, 0, 1], Sig[:, 0, 2], Sig[:, 1, 1], Sig[:, 1, 2],
                        Sig[:, 2, 2]], -1)


def sh_eval(deg, means, campos, sh):
    d = means - campos[None]
    d = d / torch.linalg.norm(d, dim=-1, keepdim=True)
    x, y, z = d[:, 0:1], d[:, 1:2], d[:, 2:3]
    res = SH_C0 * sh[:, 0]
    if deg > 0:
        res = res - SH_C1 * y * sh[:, 1] + SH_C1 * z * sh[:, 2] - SH_C1 * x * sh[:, 3]
        if deg > 1:
            xx, yy, zz, xy, yz, xz = x * x, y * y, z * z, x * y, y * z, x * z
            res = (res + SH_C2[0] * xy * sh[:, 4] + SH_C2[1] * yz * sh[:, 5] +
                   SH_C2[2] * (2 * zz - xx - yy) * sh[:, 6] + SH_C2[3] * xz * sh[:, 7] +
                   SH_C2[4] * (xx - yy) * sh[:, 8])
            if deg > 2:
                res = (res + SH_C3[0] * y * (3 * xx - yy) * sh[:, 9] + SH_C3[1] * xy * z * sh[:, 10] +
                       SH_C3[2] * y * (4 * zz - xx - yy) * sh[:, 11] +
                       SH_C3[3] * z * (2 * zz - 3 * xx - 3 * yy) * sh[:, 12] +
                       SH_C3[4] * x * (4 * zz - xx - yy) * sh[:, 13] +
                       SH_C3[5] * z * (xx - yy) * sh[:, 14] + SH_C3[6] * x * (xx - 3 * yy) * sh[:, 15])
    return torch.clamp(res + 0.5, min=0.0)


def dense_forward(st, means3D, opacities, colors=None, shs=None, scales=None, rotations=None,
                  cov3D=None):
    """Differentiable float64 forward on the oracle state ``st`` (decisions from ``st``).

    Returns (color (3,H,W), extras) where extras holds non-leaf tensors whose ``.grad`` map onto
    the oracle outputs: ``xy`` (pixel coords, -> means2D / (W/2, H/2)), ``cov3D`` and ``colors``.
    """
    W, H = st["W"], st["H"]
    vm = torch.tensor(st["vm"], dtype=torch.float64)
    pm = torch.tensor(st["pm"], dtype=torch.float64)
    Rv = torch.stack([vm[[0, 4, 8]], vm[[1, 5, 9]], vm[[2, 6, 10]]])  # p_view = Rv p + tv
    tv = vm[[12, 13, 14]]
    p_view = means3D @ Rv.T + tv
    p_hom = torch.stack([means3D @ pm[[0, 4, 8]] + pm[12], means3D @ pm[[1, 5, 9]] + pm[13],
                         means3D @ pm[[3, 7, 11]] + pm[15]], -1)
    pw = 1.0 / (p_hom[:, 2] + 1e-7)
    ndc = torch.stack([p_hom[:, 0] * pw, p_hom[:, 1] * pw], -1)
    xy = torch.stack([((ndc[:, 0] + 1.0) * W - 1.0) * 0.5, ((ndc[:, 1] + 1.0) * H - 1.0) * 0.5], -1)
    xy.retain_grad()
    if cov3D is None:
        cov3D = cov3d_from(scales, rotations, st["scale_modifier"])
    cov3D.retain_grad()
    fx = np.float32(W) / (np.float32(2.0) * np.float32(st["tanfovx"]))
    fy = np.float32(H) / (np.float32(2.0) * np.float32(st["tanfovy"]))
    limx, limy = 1.3 * st["tanfovx"], 1.3 * st["tanfovy"]
    tz = p_view[:, 2]
    tx = torch.clamp(p_view[:, 0] / tz, -limx, limx) * tz
    ty = torch.clamp(p_view[:, 1] / tz, -limy, limy) * tz
    zero = torch.zeros_like(tz)
    J = torch.stack([torch.stack([fx / tz, zero, -fx * tx / tz ** 2], -1),
                     torch.stack([zero, fy / tz, -fy * ty / tz ** 2], -1)], -2)  # (P,2,3)
    c = cov3D
    V = torch.stack([torch.stack([c[:, 0], c[:, 1], c[:, 2]], -1),
                     torch.stack([c[:, 1], c[:, 3], c[:, 4]], -1),
                     torch.stack([c[:, 2], c[:, 4], c[:, 5]], -1)], -2)
    T = J @ Rv[None]
    cov2 = T @ V @ T.transpose(1, 2)
    a = cov2[:, 0, 0] + 0.3
    b = cov2[:, 0, 1]
    cc = cov2[:, 1, 1] + 0.3
    det = a * cc - b * b
    conic = torch.stack([cc / det, -b / det, a / det], -1)
    if shs is not None:
        colors = sh_eval(st["D"], means3D, torch.tensor(st["campos"], dtype=torch.float64), shs)
    colors.retain_grad()
    bg = torch.tensor(st["bg"], dtype=torch.float64)
    gx = (W + 15) // 16
    out = torch.zeros(3, H, W, dtype=torch.float64)
    margin = np.inf
    ranges, plist = st["ranges"], st["point_list"]
    for tile in range(ranges.shape[0]):
        r0, r1 = int(ranges[tile, 0]), int(ranges[tile, 1])
        tx0, ty0 = (tile % gx) * 16, (tile // gx) * 16
        xs = torch.arange(tx0, min(tx0 + 16, W), dtype=torch.float64)
        ys = torch.arange(ty0, min(ty0 + 16, H), dtype=torch.float64)
        py, px = torch.meshgrid(ys, xs, indexing="ij")
        px, py = px.reshape(-1), py.reshape(-1)
        n = px.numel()
        Tt = torch.ones(n, dtype=torch.float64)
        C = torch.zeros(3, n, dtype=torch.float64)
        done = torch.zeros(n, dtype=torch.bool)
        for k in range(r0, r1):
            g = int(plist[k])
            dx, dy = xy[g, 0] - px, xy[g, 1] - py
            power = -0.5 * (conic[g, 0] * dx * dx + conic[g, 2] * dy * dy) - conic[g, 1] * dx * dy
            a_raw = opacities[g, 0] * torch.exp(power)
            alpha = a_raw + (torch.clamp(a_raw, max=0.99) - a_raw).detach()  # clamp ignored in grad
            with torch.no_grad():
                live = ~done & (power <= 0)
                if live.any():
                    margin = min(margin, float((torch.abs(alpha[live] * 255.0 - 1.0)).min()))
                keep = live & (alpha >= 1.0 / 255.0)
                test_T = Tt * (1 - alpha)
                if keep.any():
                    margin = min(margin, float((torch.abs(test_T[keep] / 1e-4 - 1.0)).min()))
                stop = keep & (test_T < 1e-4)
                use = keep & ~stop
            C = C + torch.where(use[None], colors[g][:, None] * alpha[None] * Tt[None], 0.0)
            Tt = torch.where(use, Tt * (1 - alpha), Tt)
            done = done | stop
        img = C + Tt[None] * bg[:, None]
        out[:, ty0:ty0 + ys.numel(), tx0:tx0 + xs.numel()] = img.reshape(3, ys.numel(), xs.numel())
    return out, {"xy": xy, "cov3D": cov3D, "colors": colors, "margin": margin}
