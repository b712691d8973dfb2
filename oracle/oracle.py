"""ctypes driver for the CPU parity oracle (``oracle/gsr_oracle.c``).

TEST INFRASTRUCTURE ONLY: imported by ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg, always as the checker, never as the thing measured or shipped.

The oracle restates the diff-gaussian-rasterization-w-depth algorithm that the reference calls at
``train.py:359-361``, ``train.py:531-533``, ``densify.py:124-126`` and ``densify.py:146-148``.  The
rasterizer's source is absent from ``/root/reference`` (empty submodule, ``.gitmodules:1-3``), so
the restatement is *parity unpinned* against the reference CUDA code; see the C file's header for
how it is pinned instead.

``forward`` / ``backward`` mirror ``_C.rasterize_gaussians`` / ``_C.rasterize_gaussians_backward``
(argument meaning and output layout), on numpy float32 arrays.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libgsr_oracle.so")
_lib = None

BLOCK_X = BLOCK_Y = 16

_f32p = ctypes.POINTER(ctypes.c_float)
_i32p = ctypes.POINTER(ctypes.c_int)
_u32p = ctypes.POINTER(ctypes.c_uint)
_u8p = ctypes.POINTER(ctypes.c_ubyte)


def build() -> str:
    """Compile the oracle with its Makefile (gcc, -ffp-contract=off)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.ora_preprocess.restype = None
        L.ora_preprocess.argtypes = [
            ctypes.c_int, ctypes.c_int, ctypes.c_int, _f32p, _f32p, ctypes.c_float, _f32p, _f32p,
            _f32p, _f32p, _f32p, _f32p, _f32p, _f32p, ctypes.c_int, ctypes.c_int, ctypes.c_float,
            ctypes.c_float, ctypes.c_int, _f32p, _i32p, _f32p, _f32p, _f32p, _f32p, _u8p, _u32p,
            _i32p]
        L.ora_bin.restype = ctypes.c_long
        L.ora_bin.argtypes = [ctypes.c_int, _f32p, _i32p, _i32p, _u32p, ctypes.c_int,
                              ctypes.c_int, _u32p, _u32p]
        L.ora_render.restype = None
        L.ora_render.argtypes = [_u32p, _u32p, ctypes.c_int, ctypes.c_int, _f32p, _f32p, _f32p,
                                 _f32p, _f32p, _f32p, _f32p, _f32p, _u32p]
        L.ora_render_backward.restype = None
        L.ora_render_backward.argtypes = [_u32p, _u32p, ctypes.c_int, ctypes.c_int, _f32p, _f32p,
                                          _f32p, _f32p, _f32p, _u32p, _f32p, _f32p, _f32p, _f32p,
                                          _f32p]
        L.ora_preprocess_backward.restype = None
        L.ora_preprocess_backward.argtypes = [
            ctypes.c_int, ctypes.c_int, ctypes.c_int, _f32p, _i32p, _f32p, _u8p, _f32p, _f32p,
            ctypes.c_float, _f32p, _f32p, _f32p, ctypes.c_int, ctypes.c_int, ctypes.c_float,
            ctypes.c_float, _f32p, _f32p, _f32p, _f32p, _f32p, _f32p, _f32p, _f32p, _f32p]
        L.ora_mark_visible.restype = None
        L.ora_mark_visible.argtypes = [ctypes.c_int, _f32p, _f32p, _f32p, _u8p]
        L.ora_set_threads.restype = ctypes.c_int
        L.ora_set_threads.argtypes = [ctypes.c_int]
        _lib = L
    return _lib


def set_threads(n: int) -> int:
    """OpenMP threads of the oracle's loops (n <= 0 leaves them); returns the count in effect."""
    return int(lib().ora_set_threads(int(n)))


def _arr(x, dtype=np.float32):
    if x is None:
        return None
    a = np.ascontiguousarray(np.asarray(x, dtype=dtype))
    return a


def _p(a, ptype=_f32p):
    if a is None or a.size == 0:
        return ctypes.cast(None, ptype)
    return a.ctypes.data_as(ptype)


def _mat(m):
    """(1,4,4) / (4,4) tensor as the 16 floats the kernel reads (``.contiguous()`` order)."""
    return _arr(np.asarray(m, dtype=np.float32).reshape(16))


def forward(bg, means3D, colors_precomp, opacities, scales, rotations, scale_modifier,
            cov3D_precomp, viewmatrix, projmatrix, tanfovx, tanfovy, image_height, image_width,
            sh, sh_degree, campos, prefiltered=False):
    """CPU restatement of ``_C.rasterize_gaussians``; returns a dict with every intermediate."""
    L = lib()
    means3D = _arr(means3D).reshape(-1, 3)
    P = means3D.shape[0]
    H, W = int(image_height), int(image_width)
    colors_precomp = _arr(colors_precomp) if colors_precomp is not None and np.size(colors_precomp) else None
    sh = _arr(sh) if sh is not None and np.size(sh) else None
    scales = _arr(scales) if scales is not None and np.size(scales) else None
    rotations = _arr(rotations) if rotations is not None and np.size(rotations) else None
    cov3D_precomp = _arr(cov3D_precomp) if cov3D_precomp is not None and np.size(cov3D_precomp) else None
    opacities = _arr(opacities).reshape(-1)
    M = sh.shape[1] if sh is not None else 0
    vm, pm = _mat(viewmatrix), _mat(projmatrix)
    campos = _arr(campos).reshape(3)
    bg = _arr(bg).reshape(3)
    st = dict(P=P, H=H, W=W, M=M, D=int(sh_degree), vm=vm, pm=pm, campos=campos, bg=bg,
              tanfovx=float(np.float32(tanfovx)), tanfovy=float(np.float32(tanfovy)),
              scale_modifier=float(np.float32(scale_modifier)), means3D=means3D, sh=sh,
              colors_precomp=colors_precomp, opacities=opacities, scales=scales,
              rotations=rotations, cov3D_precomp=cov3D_precomp)
    gx, gy = (W + BLOCK_X - 1) // BLOCK_X, (H + BLOCK_Y - 1) // BLOCK_Y
    depths = np.zeros(P, np.float32)
    radii = np.zeros(P, np.int32)
    xy = np.zeros((P, 2), np.float32)
    conic = np.zeros((P, 4), np.float32)
    rgb = np.zeros((P, 3), np.float32)
    cov3D = np.zeros((P, 6), np.float32)
    clamped = np.zeros((P, 3), np.uint8)
    tiles = np.zeros(P, np.uint32)
    rects = np.zeros((P, 4), np.int32)
    color = np.zeros((3, H, W), np.float32)
    depth = np.zeros((1, H, W), np.float32)
    final_T = np.zeros((H, W), np.float32)
    n_contrib = np.zeros((H, W), np.uint32)
    ranges = np.zeros((gx * gy, 2), np.uint32)
    point_list = np.zeros(0, np.uint32)
    K = 0
    if P > 0:
        L.ora_preprocess(P, st["D"], M, _p(means3D), _p(scales), st["scale_modifier"], _p(rotations),
                         _p(opacities), _p(sh), _p(colors_precomp), _p(cov3D_precomp), _p(vm), _p(pm),
                         _p(campos), W, H, st["tanfovx"], st["tanfovy"], int(bool(prefiltered)),
                         _p(depths), _p(radii, _i32p), _p(xy), _p(conic), _p(rgb), _p(cov3D),
                         _p(clamped, _u8p), _p(tiles, _u32p), _p(rects, _i32p))
        K = int(tiles.astype(np.int64).sum())
        point_list = np.zeros(max(K, 1), np.uint32)
        K2 = L.ora_bin(P, _p(depths), _p(radii, _i32p), _p(rects, _i32p), _p(tiles, _u32p), W, H,
                       _p(point_list, _u32p), _p(ranges, _u32p))
        assert K2 == K
        point_list = point_list[:K]
        feats = colors_precomp if colors_precomp is not None else rgb
        L.ora_render(_p(ranges, _u32p), _p(point_list, _u32p), W, H, _p(xy), _p(feats), _p(conic),
                     _p(depths), _p(bg), _p(color), _p(depth), _p(final_T), _p(n_contrib, _u32p))
    st.update(num_rendered=K, color=color, depth=depth, radii=radii, depths=depths, xy=xy,
              conic_opacity=conic, rgb=rgb, cov3D=cov3D, clamped=clamped, tiles_touched=tiles,
              rects=rects, point_list=point_list, ranges=ranges, final_T=final_T,
              n_contrib=n_contrib)
    return st


def backward(st, dL_dcolor):
    """CPU restatement of ``_C.rasterize_gaussians_backward`` on a ``forward`` state."""
    L = lib()
    P, H, W, M = st["P"], st["H"], st["W"], st["M"]
    dL_dcolor = _arr(dL_dcolor).reshape(3, H, W)
    g = dict(means2D=np.zeros((P, 3), np.float32), colors=np.zeros((P, 3), np.float32),
             opacities=np.zeros((P, 1), np.float32), means3D=np.zeros((P, 3), np.float32),
             cov3D=np.zeros((P, 6), np.float32), sh=np.zeros((P, M, 3), np.float32),
             scales=np.zeros((P, 3), np.float32), rotations=np.zeros((P, 4), np.float32),
             conic=np.zeros((P, 4), np.float32))
    if P == 0:
        return g
    feats = st["colors_precomp"] if st["colors_precomp"] is not None else st["rgb"]
    L.ora_render_backward(_p(st["ranges"], _u32p), _p(st["point_list"], _u32p), W, H, _p(st["bg"]),
                          _p(st["xy"]), _p(st["conic_opacity"]), _p(feats), _p(st["final_T"]),
                          _p(st["n_contrib"], _u32p), _p(dL_dcolor), _p(g["means2D"]), _p(g["conic"]),
                          _p(g["opacities"]), _p(g["colors"]))
    cov = st["cov3D_precomp"] if st["cov3D_precomp"] is not None else st["cov3D"]
    L.ora_preprocess_backward(P, st["D"], M, _p(st["means3D"]), _p(st["radii"], _i32p), _p(st["sh"]),
                              _p(st["clamped"], _u8p), _p(st["scales"]), _p(st["rotations"]),
                              st["scale_modifier"], _p(cov), _p(st["vm"]), _p(st["pm"]), W, H,
                              st["tanfovx"], st["tanfovy"], _p(st["campos"]), _p(g["means2D"]),
                              _p(g["conic"]), _p(g["colors"]), _p(g["means3D"]), _p(g["cov3D"]),
                              _p(g["sh"]), _p(g["scales"]), _p(g["rotations"]))
    return g


def mark_visible(means3D, viewmatrix, projmatrix):
    L = lib()
    means3D = _arr(means3D).reshape(-1, 3)
    out = np.zeros(means3D.shape[0], np.uint8)
    if means3D.shape[0]:
        L.ora_mark_visible(means3D.shape[0], _p(means3D), _p(_mat(viewmatrix)), _p(_mat(projmatrix)),
                           _p(out, _u8p))
    return out.astype(bool)
