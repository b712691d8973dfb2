"""CPU oracle of the fused L1 + SSIM loss (numpy float64).

TEST INFRASTRUCTURE ONLY: imported by ``tests/`` and ``bench.py``'s ``cpu_baseline`` leg as the
checker, never as the thing measured or shipped.

Restates, in float64:
  * ``gaussian`` / ``create_window`` (external.py:48-65): the float32 1-D window
    exp(-(x - 5)^2 / (2 * 1.5^2)) normalised by its float32 sum; the 2-D window is its outer product;
  * ``_ssim`` (external.py:79-110): five zero-padded ("same", padding 5) 11x11 correlations of
    img1, img2, img1^2, img2^2, img1*img2 per plane, c1 = 0.01^2, c2 = 0.03^2, mean of the map;
  * ``torch.nn.functional.l1_loss`` (train.py:362, densify.py:127,149): mean |img1 - img2|;
  * the gradient of ``g_l1 * l1 + g_ssim * ssim`` with respect to img1, derived analytically (the
    same derivation the HIP backward uses; checked against torch.autograd of a float64 restatement
    and against the reference's own autograd in tests/golden).

Pinned against the reference: tests/golden/reference_harness.npz holds calc_ssim values and
gradients produced by importing external.py itself (tests/golden/gen_golden.py).
"""
from __future__ import annotations

from math import exp

import numpy as np

C1, C2 = 0.01 ** 2, 0.03 ** 2
RADIUS = 5


def window_1d() -> np.ndarray:
    """external.py:48-55 gaussian(11, 1.5): float32 values, float32 normalisation."""
    g = np.array([exp(-((x - RADIUS) ** 2) / float(2 * 1.5 ** 2)) for x in range(2 * RADIUS + 1)],
                 dtype=np.float32)
    return g / g.sum(dtype=np.float32)


def blur(x: np.ndarray) -> np.ndarray:
    """Zero-padded 11x11 correlation of every (..., H, W) plane with the outer-product window."""
    w = window_1d().astype(np.float64)
    x = np.asarray(x, dtype=np.float64)
    H, W = x.shape[-2:]
    pad = [(0, 0)] * (x.ndim - 2) + [(RADIUS, RADIUS), (RADIUS, RADIUS)]
    xp = np.pad(x, pad)
    h = np.zeros(x.shape[:-2] + (H + 2 * RADIUS, W), dtype=np.float64)
    for t in range(2 * RADIUS + 1):
        h += w[t] * xp[..., :, t:t + W]
    out = np.zeros_like(x)
    for t in range(2 * RADIUS + 1):
        out += w[t] * h[..., t:t + H, :]
    return out


def l1_ssim(img1, img2):
    """Returns (l1, ssim, state) where state carries what the gradient needs."""
    x, y = np.asarray(img1, np.float64), np.asarray(img2, np.float64)
    mu1, mu2 = blur(x), blur(y)
    s11, s22, s12 = blur(x * x), blur(y * y), blur(x * y)
    mu1_sq, mu2_sq, mu1_mu2 = mu1 * mu1, mu2 * mu2, mu1 * mu2
    A = 2 * mu1_mu2 + C1
    B = 2 * (s12 - mu1_mu2) + C2
    C = mu1_sq + mu2_sq + C1
    D = (s11 - mu1_sq) + (s22 - mu2_sq) + C2
    S = A * B / (C * D)
    st = {"x": x, "y": y, "mu1": mu1, "mu2": mu2, "A": A, "B": B, "C": C, "D": D, "S": S}
    return float(np.abs(x - y).mean()), float(S.mean()), st


def l1_ssim_grad(st, g_l1=1.0, g_ssim=1.0) -> np.ndarray:
    """d(g_l1 * l1 + g_ssim * ssim) / d img1."""
    x, y, mu1, mu2 = st["x"], st["y"], st["mu1"], st["mu2"]
    A, B, C, D, S = st["A"], st["B"], st["C"], st["D"], st["S"]
    n = x.size
    dmu1 = (2 * mu2 * (B - A) - 2 * mu1 * S * (D - C)) / (C * D)
    ds11 = -S / D
    ds12 = 2 * A / (C * D)
    g = (g_ssim / n) * (blur(dmu1) + 2 * x * blur(ds11) + y * blur(ds12))
    return g + (g_l1 / n) * np.sign(x - y)
