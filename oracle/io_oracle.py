"""CPU oracle of the view formatting of the data path, numpy.

TEST INFRASTRUCTURE ONLY: imported by ``tests/`` as the checker, never as the thing measured or
shipped.

Restates load_timestep_views' tensor arithmetic (shared.py:127-171) on the decoded 8-bit pixels:
  * image: ``torch.tensor(u8 HWC).float().cuda().permute(2, 0, 1) / 255`` (shared.py:152-160).  The
    reference runs the divide on the GPU, where torch divides by a Python scalar as a multiply by
    its float reciprocal (``x * (1.0f / 255.0f)``, ATen's div_true CUDA kernel for a CPU-scalar
    divisor): ``view_image``.  On the CPU torch divides exactly (``x / 255.0f``): ``view_image_cpu``
    -- what the golden fixtures hold, since they were made by running the reference on the CPU.
    The two differ by one ulp on 126 of the 256 byte values.
  * segmentation mask: ``m = float32(u8 HW)``; ``torch.stack((m, zeros_like(m), 1 - m))``
    (shared.py:131-143, 161-168).  Exact in either place.

Pinned against the reference: tests/golden/reference_io.npz holds the image / mask files of two
small sequences and the views the reference's own load_timestep_views built from them
(tests/golden/gen_golden.py --io).
"""
from __future__ import annotations

import numpy as np

INV_255 = np.float32(1.0) / np.float32(255.0)


def view_image(u8_hwc: np.ndarray) -> np.ndarray:
    """(H, W, 3) uint8 -> (3, H, W) float32 as the reference computes it on the GPU."""
    return np.ascontiguousarray(u8_hwc.astype(np.float32).transpose(2, 0, 1) * INV_255)


def view_image_cpu(u8_hwc: np.ndarray) -> np.ndarray:
    """The same expression evaluated by torch on the CPU (true division)."""
    return np.ascontiguousarray(u8_hwc.astype(np.float32).transpose(2, 0, 1) / np.float32(255.0))


def view_mask(u8_hw: np.ndarray) -> np.ndarray:
    """(H, W) 8-bit mask (bool for 1-bit PNGs) -> (3, H, W) float32 (m, 0, 1 - m)."""
    m = u8_hw.astype(np.float32)
    return np.stack((m, np.zeros_like(m), np.float32(1.0) - m))
