"""Fused Adam over the per-Gaussian parameters on the HIP kernel of ``libgsr.so``.

``FusedAdam`` is a drop-in for the ``torch.optim.Adam`` of densify.py:68-86 (one named param group
per parameter, ``lr=0.0`` default, ``eps=1e-15``): same constructor arguments, ``param_groups`` and
per-parameter ``state`` (``step`` CPU scalar tensor, ``exp_avg``, ``exp_avg_sq``), so the reference's
optimizer surgery (external.py:127-204) and ``splat_densify`` work on it unchanged.  ``step()``
updates every parameter with a gradient in ONE kernel launch, with torch's ``_multi_tensor_adam``
operation order (parity within a few ulp; tests/test_adam.py).  Supported configuration: the
reference's -- no weight decay, no AMSGrad, not maximising.  There is no CPU path.
"""
from __future__ import annotations

import ctypes

import torch

from diff_gaussian_rasterization import _C

__all__ = ["FusedAdam"]


class _AdamTensor(ctypes.Structure):
    _fields_ = [("param", ctypes.c_void_p), ("grad", ctypes.c_void_p), ("exp_avg", ctypes.c_void_p),
                ("exp_avg_sq", ctypes.c_void_p), ("numel", ctypes.c_longlong), ("lr", ctypes.c_double),
                ("step", ctypes.c_double)]


_bound = False


def _lib():
    global _bound
    L = _C.load_library()
    if not _bound:
        L.gsr_adam_step.restype = ctypes.c_int
        L.gsr_adam_step.argtypes = [ctypes.c_int, ctypes.POINTER(_AdamTensor), ctypes.c_double, ctypes.c_double,
                                    ctypes.c_double, ctypes.c_void_p]
        _bound = True
    return L


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, amsgrad=False,
                 maximize=False):
        if weight_decay != 0 or amsgrad or maximize:
            raise NotImplementedError("FusedAdam: weight_decay / amsgrad / maximize are not supported "
                                      "(the reference uses plain Adam)")
        if not 0.0 <= lr or not 0.0 <= eps or not all(0.0 <= b < 1.0 for b in betas):
            raise ValueError("FusedAdam: invalid lr / eps / betas")
        super().__init__(params, dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=0.0, amsgrad=False,
                                      maximize=False))

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        L = _lib()
        by_cfg = {}
        keep = []
        for group in self.param_groups:
            b1, b2 = group["betas"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                if not p.is_cuda or p.dtype != torch.float32:
                    raise RuntimeError("FusedAdam: float32 GPU parameters only (no CPU path)")
                if p.grad.is_sparse:
                    raise RuntimeError("FusedAdam: sparse gradients are not supported")
                st = self.state[p]
                if len(st) == 0:  # torch.optim.Adam's lazy state (step on the CPU, moments like p)
                    st["step"] = torch.tensor(0.0, dtype=torch.float32)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["step"] += 1
                if not (p.is_contiguous() and st["exp_avg"].is_contiguous() and st["exp_avg_sq"].is_contiguous()):
                    raise RuntimeError("FusedAdam: contiguous parameters and moments required")
                g = p.grad if p.grad.is_contiguous() and p.grad.dtype == torch.float32 else p.grad.contiguous().float()
                keep.append(g)
                by_cfg.setdefault((b1, b2, group["eps"], p.device), []).append(
                    _AdamTensor(p.data_ptr(), g.data_ptr(), st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr(),
                                p.numel(), float(group["lr"]), float(st["step"].item())))
        for (b1, b2, eps, dev), ts in by_cfg.items():
            arr = (_AdamTensor * len(ts))(*ts)
            _C._check(L.gsr_adam_step(len(ts), arr, float(b1), float(b2), float(eps), _C._stream_ptr(dev)))
        return loss
