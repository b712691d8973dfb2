"""Fused L1 + SSIM image loss on the HIP kernels of ``libgsr.so``.

Drop-ins for the loss the reference computes after every render:

* ``calc_ssim(img1, img2, window_size=11, size_average=True)`` -- external.py:68-76 (+ ``_ssim``,
  external.py:79-110): mean SSIM with an 11x11 Gaussian window (sigma 1.5), zero padding.
* ``calculate_l1_and_ssim_loss``-style pair ``l1_and_ssim_loss(rendered, target)`` ->
  ``(l1_loss, 1 - ssim)`` as train.py:354-364 returns it, and ``image_loss(rendered, target)`` =
  ``0.8 * l1 + 0.2 * (1 - ssim)`` (train.py:391-392, densify.py:127-129,149-151).

One forward kernel computes both means and keeps the per-pixel SSIM derivatives; one backward
kernel blurs them and adds the L1 sign term, taking the upstream gradients from device memory.
Gradients flow to ``img1`` (the render) only; the target ``img2`` is data in every reference call
site, so a target that requires grad is rejected rather than silently given none.  There is no CPU
path: CPU tensors or a missing ``libgsr.so`` raise.
"""
from __future__ import annotations


import torch

from diff_gaussian_rasterization import _C

__all__ = ["calc_ssim", "l1_and_ssim", "l1_and_ssim_loss", "image_loss"]


def _planes(img):
    if img.dim() < 2:
        raise RuntimeError("l1_ssim: expected an image of shape (..., H, W)")
    H, W = img.shape[-2], img.shape[-1]
    planes = img.numel() // max(H * W, 1)
    return planes, H, W


class _L1SSIM(torch.autograd.Function):
    @staticmethod
    def forward(ctx, img1, img2):
        L = _C.load_library()
        if img1.shape != img2.shape:
            raise RuntimeError(f"l1_ssim: image shapes differ: {tuple(img1.shape)} vs {tuple(img2.shape)}")
        a, b = img1.contiguous(), img2.contiguous()
        for t in (a, b):
            _C._ptr(t)  # GPU + float32 checks (no CPU path)
        planes, H, W = _planes(a)
        dev = a.device
        scratch = torch.empty(L.gsr_ssim_scratch_bytes(planes, H, W), dtype=torch.uint8, device=dev)
        l1 = torch.empty((), dtype=torch.float32, device=dev)
        ssim = torch.empty((), dtype=torch.float32, device=dev)
        _C._check(L.gsr_l1_ssim_forward(planes, H, W, a.data_ptr(), b.data_ptr(), scratch.data_ptr(),
                                        l1.data_ptr(), ssim.data_ptr(), _C._stream_ptr(dev)))
        ctx.save_for_backward(a, b, scratch)
        ctx.shape = img1.shape
        ctx.set_materialize_grads(False)
        return l1, ssim

    @staticmethod
    def backward(ctx, g_l1, g_ssim):
        if g_l1 is None and g_ssim is None:
            return None, None
        L = _C.load_library()
        a, b, scratch = ctx.saved_tensors
        planes, H, W = _planes(a)
        gl = g_l1.contiguous().float() if g_l1 is not None else None
        gs = g_ssim.contiguous().float() if g_ssim is not None else None
        grad = torch.empty_like(a)
        _C._check(L.gsr_l1_ssim_backward(planes, H, W, a.data_ptr(), b.data_ptr(), scratch.data_ptr(),
                                         gl.data_ptr() if gl is not None else None,
                                         gs.data_ptr() if gs is not None else None, grad.data_ptr(),
                                         _C._stream_ptr(a.device)))
        return grad.view(ctx.shape), None


def l1_and_ssim(img1, img2):
    """``(torch.nn.functional.l1_loss(img1, img2), calc_ssim(img1, img2))`` from one kernel pair."""
    if img2.requires_grad:
        raise NotImplementedError("l1_ssim: gradients flow to img1 (the render) only; detach the target")
    return _L1SSIM.apply(img1, img2)


def calc_ssim(img1, img2, window_size=11, size_average=True):
    """external.py:68-76.  Only the configuration the reference uses is supported: window 11 with the
    scalar mean (``size_average=False`` cannot be evaluated on the reference's (3,H,W) renders)."""
    if window_size != 11 or not size_average:
        raise NotImplementedError("calc_ssim: only window_size=11, size_average=True (the reference's use)")
    return l1_and_ssim(img1, img2)[1]


def l1_and_ssim_loss(rendered, target):
    """train.py:354-364 ``calculate_l1_and_ssim_loss`` minus the render: ``(l1_loss, 1 - ssim)``."""
    l1, ssim = l1_and_ssim(rendered, target)
    return l1, 1.0 - ssim


def image_loss(rendered, target):
    """0.8 * l1 + 0.2 * (1 - ssim): train.py:391-392 and densify.py:127-129,149-151."""
    l1, ssim = l1_and_ssim(rendered, target)
    return 0.8 * l1 + 0.2 * (1.0 - ssim)
