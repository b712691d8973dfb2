"""Native entry points of the drop-in rasterizer, bound over the C ABI of ``libgsr.so``.

Same three names, argument order and return tuples as the reference extension's pybind module
``diff_gaussian_rasterization._C`` (``ext.cpp`` / ``rasterize_points.cu`` of the
diff-gaussian-rasterization-w-depth submodule, ``/root/reference/.gitmodules:1-3``):

* ``rasterize_gaussians(...) -> (num_rendered, color, radii, geomBuffer, binningBuffer, imgBuffer, depth)``
* ``rasterize_gaussians_backward(...) -> (dL_dmeans2D, dL_dcolors, dL_dopacity, dL_dmeans3D,
  dL_dcov3D, dL_dsh, dL_dscales, dL_drotations)``
* ``mark_visible(means3D, viewmatrix, projmatrix) -> bool[P]``

Tensors cross the boundary as raw device pointers (``include/gsr.h``); the three persistent
workspaces are ``torch.uint8`` tensors whose lifetime follows the autograd graph, like the reference's
``resizeFunctional`` byte buffers.  They are sized and allocated here before the native call and handed
out by ``gsr_prealloc_alloc`` (C), so a call makes no callback into Python on its usual path; a request
the pre-sized buffers do not cover (a first or redone speculative forward) falls back to a ctypes
callback.  There is no CPU path:
a missing ``libgsr.so`` or a CPU tensor raises.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GSR_LIB", os.path.join(_HERE, "libgsr.so"))

GSR_BUF_GEOM, GSR_BUF_BINNING, GSR_BUF_IMAGE, GSR_BUF_SCRATCH, GSR_BUF_SUMS = 0, 1, 2, 3, 4
EXPORTED_SYMBOLS = (
    "gsr_forward", "gsr_backward", "gsr_mark_visible", "gsr_geom_bytes", "gsr_image_bytes",
    "gsr_binning_bytes", "gsr_scratch_bytes", "gsr_last_error", "gsr_abi_version",
    "gsr_profile_enable", "gsr_profile_select", "gsr_profile_reset", "gsr_profile_read", "gsr_buffer_offsets",
    "gsr_ssim_scratch_bytes", "gsr_l1_ssim_forward", "gsr_l1_ssim_backward",
    "gsr_densify_update_radii", "gsr_densify_accumulate_grads", "gsr_densify_workspace_bytes",
    "gsr_densify_plan", "gsr_densify_split_stds", "gsr_densify_apply", "gsr_adam_step", "gsr_views_pack",
    "gsr_grad_fence", "gsr_backward_render", "gsr_backward_gaussians", "gsr_backward_items_bytes",
    "gsr_forward_info_call", "gsr_spec_stats", "gsr_sums_bytes", "gsr_prealloc_alloc", "gsr_spec_binning_bytes",
    "gsr_forward_async", "gsr_forward_resolve", "gsr_forward_release", "gsr_forward_query", "gsr_async_stats",
    "gsr_spec_keys", "gsr_async_shutdown", "gsr_debug_async_fault", "gsr_set_exact_thresholds",
)


class _Camera(ctypes.Structure):
    _fields_ = [("image_width", ctypes.c_int), ("image_height", ctypes.c_int),
                ("tan_fovx", ctypes.c_float), ("tan_fovy", ctypes.c_float),
                ("viewmatrix", ctypes.c_void_p), ("projmatrix", ctypes.c_void_p),
                ("campos", ctypes.c_void_p), ("bg", ctypes.c_void_p),
                ("prefiltered", ctypes.c_int), ("viewmatrix_stride", ctypes.c_int * 2),
                ("projmatrix_stride", ctypes.c_int * 2), ("campos_stride", ctypes.c_int)]


class _Gaussians(ctypes.Structure):
    _fields_ = [("P", ctypes.c_int), ("sh_degree", ctypes.c_int), ("sh_coeffs", ctypes.c_int),
                ("scale_modifier", ctypes.c_float), ("means3D", ctypes.c_void_p),
                ("shs", ctypes.c_void_p), ("colors_precomp", ctypes.c_void_p),
                ("opacities", ctypes.c_void_p), ("scales", ctypes.c_void_p),
                ("rotations", ctypes.c_void_p), ("cov3D_precomp", ctypes.c_void_p),
                ("activations", ctypes.c_int), ("prepare_backward", ctypes.c_int),
                ("binning_layout", ctypes.c_int)]


class _ForwardInfo(ctypes.Structure):  # gsr_forward_info (ABI 17)
    _fields_ = [("num_rendered", ctypes.c_int), ("binning_layout", ctypes.c_int), ("speculated", ctypes.c_int),
                ("pending", ctypes.c_ulonglong), ("aux_stream", ctypes.c_void_p)]


class _Resolution(ctypes.Structure):  # gsr_forward_resolution (ABI 17)
    _fields_ = [("num_rendered", ctypes.c_int), ("binning_layout", ctypes.c_int), ("binning", ctypes.c_void_p),
                ("redone", ctypes.c_int)]


class _Grads(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in (
        "dL_dmeans2D", "dL_dcolors", "dL_dopacity", "dL_dmeans3D", "dL_dcov3D", "dL_dsh",
        "dL_dscales", "dL_drotations")] + [("accumulate", ctypes.c_int)]


class _ViewGrad(ctypes.Structure):  # gsr_view_grad (ABI 12)
    _fields_ = [("cam", ctypes.POINTER(_Camera)), ("radii", ctypes.c_void_p), ("geom", ctypes.c_void_p),
                ("scratch", ctypes.c_void_p), ("num_rendered", ctypes.c_int),
                ("dL_dmeans2D", ctypes.c_void_p), ("accumulate_means2D", ctypes.c_int)]


_ALLOC_FN = ctypes.CFUNCTYPE(ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t)


class _Prealloc(ctypes.Structure):  # gsr_prealloc (ABI 16)
    _fields_ = [("ptr", ctypes.c_void_p * 5), ("bytes", ctypes.c_size_t * 5), ("fallback", _ALLOC_FN),
                ("fallback_ctx", ctypes.c_void_p), ("used", ctypes.c_int)]


_lib = None
_PREALLOC_FN = None  # gsr_prealloc_alloc as a gsr_alloc_fn (a C function: no Python on the call path)


def load_library():
    """Load ``libgsr.so`` (raises if it has not been built: there is no fallback path)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"libgsr.so not found at {LIB_PATH}: build it with `make -C animating-gaussian-splats_amd/csrc` "
            "(or __graft_entry__.build()); the rasterizer has no CPU fallback")
    L = ctypes.CDLL(LIB_PATH)
    vp, i, f = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
    L.gsr_forward.restype = i
    L.gsr_forward.argtypes = [ctypes.POINTER(_Camera), ctypes.POINTER(_Gaussians), _ALLOC_FN, vp,
                              vp, vp, vp, ctypes.POINTER(i), vp]
    L.gsr_forward_info_call.restype = i
    L.gsr_forward_info_call.argtypes = [ctypes.POINTER(_Camera), ctypes.POINTER(_Gaussians), _ALLOC_FN, vp,
                                        vp, vp, vp, i, ctypes.POINTER(_ForwardInfo), vp]
    L.gsr_spec_stats.restype = i
    L.gsr_spec_stats.argtypes = [ctypes.POINTER(i), ctypes.POINTER(i), i]
    L.gsr_spec_keys.restype = i
    L.gsr_spec_keys.argtypes = []
    L.gsr_forward_async.restype = i
    L.gsr_forward_async.argtypes = [ctypes.POINTER(_Camera), ctypes.POINTER(_Gaussians), _ALLOC_FN, vp,
                                    vp, vp, vp, ctypes.POINTER(_ForwardInfo), vp]
    L.gsr_forward_resolve.restype = i
    L.gsr_forward_resolve.argtypes = [ctypes.c_ulonglong, ctypes.POINTER(_Resolution)]
    L.gsr_forward_release.restype = i
    L.gsr_forward_release.argtypes = [ctypes.c_ulonglong]
    L.gsr_forward_query.restype = i
    L.gsr_forward_query.argtypes = [ctypes.c_ulonglong]
    L.gsr_async_stats.restype = i
    L.gsr_async_stats.argtypes = [ctypes.POINTER(i), ctypes.POINTER(i)]
    L.gsr_async_shutdown.restype = i
    L.gsr_async_shutdown.argtypes = []
    L.gsr_debug_async_fault.restype = i
    L.gsr_debug_async_fault.argtypes = [i, i, i]
    import atexit
    atexit.register(L.gsr_async_shutdown)  # the resolver thread stops before the HIP runtime goes
    L.gsr_backward.restype = i
    L.gsr_backward.argtypes = [ctypes.POINTER(_Camera), ctypes.POINTER(_Gaussians), vp, i, vp, vp, vp,
                               vp, vp, _ALLOC_FN, vp, ctypes.POINTER(_Grads), vp]
    L.gsr_backward_render.restype = i
    L.gsr_backward_render.argtypes = [ctypes.POINTER(_Camera), ctypes.POINTER(_Gaussians), vp, i, vp, vp, vp,
                                      vp, _ALLOC_FN, vp, vp]
    L.gsr_backward_gaussians.restype = i
    L.gsr_backward_gaussians.argtypes = [i, ctypes.POINTER(_ViewGrad), ctypes.POINTER(_Gaussians),
                                         ctypes.POINTER(_Grads), vp]
    L.gsr_grad_fence.restype = i
    L.gsr_grad_fence.argtypes = [ctypes.POINTER(vp), i, vp]
    L.gsr_mark_visible.restype = i
    L.gsr_mark_visible.argtypes = [i, vp, vp, vp, vp, vp]
    L.gsr_geom_bytes.restype = ctypes.c_size_t
    L.gsr_geom_bytes.argtypes = [i]
    L.gsr_binning_bytes.restype = ctypes.c_size_t
    L.gsr_binning_bytes.argtypes = [i, i]
    L.gsr_sums_bytes.restype = ctypes.c_size_t
    L.gsr_sums_bytes.argtypes = [i]
    for n in ("gsr_scratch_bytes", "gsr_backward_items_bytes"):
        getattr(L, n).restype = ctypes.c_size_t
        getattr(L, n).argtypes = [i, i, i]
    L.gsr_image_bytes.restype = ctypes.c_size_t
    L.gsr_image_bytes.argtypes = [i, i, i]
    L.gsr_last_error.restype = ctypes.c_char_p
    L.gsr_last_error.argtypes = []
    L.gsr_abi_version.restype = i
    L.gsr_profile_enable.argtypes = [i]
    L.gsr_profile_enable.restype = i
    L.gsr_profile_reset.restype = i
    L.gsr_profile_select.argtypes = [ctypes.c_char_p]
    L.gsr_profile_select.restype = i
    L.gsr_profile_read.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(i)]
    L.gsr_profile_read.restype = i
    L.gsr_buffer_offsets.restype = i
    L.gsr_buffer_offsets.argtypes = [i, i, i, i, ctypes.POINTER(ctypes.c_size_t), i]
    L.gsr_ssim_scratch_bytes.restype = ctypes.c_size_t
    L.gsr_ssim_scratch_bytes.argtypes = [i, i, i]
    L.gsr_l1_ssim_forward.restype = i
    L.gsr_l1_ssim_forward.argtypes = [i, i, i, vp, vp, vp, vp, vp, vp]
    L.gsr_l1_ssim_backward.restype = i
    L.gsr_l1_ssim_backward.argtypes = [i, i, i, vp, vp, vp, vp, vp, vp, vp]
    L.gsr_spec_binning_bytes.restype = ctypes.c_size_t
    L.gsr_spec_binning_bytes.argtypes = [i, i, i, i]
    L.gsr_set_exact_thresholds.restype = i
    L.gsr_set_exact_thresholds.argtypes = [i]
    if L.gsr_abi_version() != ABI_VERSION:
        raise RuntimeError(f"libgsr.so ABI {L.gsr_abi_version()} != binding ABI {ABI_VERSION}: rebuild it")
    global _PREALLOC_FN
    _PREALLOC_FN = _ALLOC_FN(ctypes.cast(L.gsr_prealloc_alloc, ctypes.c_void_p).value)
    _lib = L
    return L


ABI_VERSION = 21  # GSR_ABI_VERSION of include/gsr.h this binding's structs follow
ACT_SIGMOID_OPACITY, ACT_EXP_SCALES, ACT_NORMALIZE_ROTATIONS = 1, 2, 4  # enum gsr_activation
ACT_ALL = ACT_SIGMOID_OPACITY | ACT_EXP_SCALES | ACT_NORMALIZE_ROTATIONS


def set_exact_thresholds(on: bool) -> bool:
    """Exact-threshold mode (gsr_set_exact_thresholds; on by default since ABI 21): tiles where a blend
    weight within 1e-5 of the 1/255 threshold was taken are redone with such weights re-evaluated in
    the reference's expression order, so the forward and backward take the reference's decisions
    there.  Process-wide; returns the previous setting."""
    return bool(load_library().gsr_set_exact_thresholds(int(bool(on))))


def _check(rc):
    if rc != 0:
        msg = _lib.gsr_last_error().decode(errors="replace")
        raise RuntimeError(f"libgsr error {rc}: {msg}")


def _ptr(t):
    """Device pointer of a tensor, or None for an absent (empty) argument."""
    if t is None or t.numel() == 0:
        return None
    if not t.is_cuda:
        raise RuntimeError("diff_gaussian_rasterization: tensors must be on the GPU (no CPU path)")
    if t.dtype != torch.float32:
        raise RuntimeError(f"diff_gaussian_rasterization: expected float32, got {t.dtype}")
    return t.data_ptr()


def _bp(b):
    """A workspace buffer given as a tensor (its data pointer) or as a device pointer (int)."""
    return b if isinstance(b, int) else b.data_ptr()


def _f32(t):
    return t.contiguous() if t is not None and t.numel() else t


_tls = threading.local()


def _fallback_alloc(_ctx, which, nbytes):
    """The pre-allocation's fallback (a request the pre-sized buffers do not cover: a first forward,
    a redone speculation): a byte tensor on the calling thread's current pre-allocation device."""
    try:
        t = torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=_tls.device)
    except Exception:  # noqa: BLE001 - reported through the C ABI as GSR_ERR_ALLOC
        return None
    _tls.buffers[int(which)] = t
    return t.data_ptr()


_FALLBACK_FN = _ALLOC_FN(_fallback_alloc)  # one thunk for the process
_PREALLOC_ON = os.environ.get("GSR_PREALLOC", "1") != "0"  # 0: every request through the callback (A/B)


class _PreAllocator:
    """Buffers sized on the host before the native call and handed out by gsr_prealloc_alloc (C),
    so the call makes no ctypes callback (which would re-acquire the interpreter lock while other
    threads submit their views) unless a request exceeds them.  ``groups``: lists of (gsr_buffer,
    bytes); the buffers of one list are carved from ONE allocation (they share its lifetime).  After the
    call: ``ptrs`` (gsr_buffer -> device pointer handed out), ``bases`` (the allocations backing them,
    what keeps them alive) and, built on first use, ``buffers`` (gsr_buffer -> uint8 tensor view)."""

    def __init__(self, device, groups):
        self.device = device
        self.pa = _Prealloc()
        self.given = {}  # which -> (base tensor, offset, bytes)
        for group in groups if _PREALLOC_ON else ():
            offs, total = [], 0
            for which, nbytes in group:
                offs.append((which, total, nbytes))
                total += (int(nbytes) + 255) & ~255
            if total == 0:
                continue
            buf = torch.empty(total, dtype=torch.uint8, device=device)
            base = buf.data_ptr()
            for which, o, nbytes in offs:
                if nbytes > 0:
                    self.given[which] = (buf, o, int(nbytes))
                    self.pa.ptr[which] = base + o
                    self.pa.bytes[which] = int(nbytes)
        self.pa.fallback = _FALLBACK_FN
        self.cb = _PREALLOC_FN
        self.ctx = ctypes.byref(self.pa)
        self._views = None

    def __enter__(self):
        self.prev = getattr(_tls, "buffers", None), getattr(_tls, "device", None)
        _tls.buffers, _tls.device = {}, self.device
        return self

    def __exit__(self, *exc):
        got = _tls.buffers
        _tls.buffers, _tls.device = self.prev
        # what the call took: the pre-allocated buffers it was handed, and the fallback's
        used = self.pa.used
        self._took({w: g for w, g in self.given.items() if (used >> w) & 1}, got)
        return False

    def _took(self, taken, fallback):
        """``taken``: gsr_buffer -> (base tensor, offset, bytes) of the pre-allocated buffers the call
        used; ``fallback``: gsr_buffer -> tensor of the requests made through the fallback."""
        self.taken, self.fallback = taken, fallback
        self.ptrs = {w: b.data_ptr() + o for w, (b, o, _) in taken.items()}
        self.ptrs.update({w: t.data_ptr() for w, t in fallback.items()})
        bases = {id(g[0]): g[0] for g in taken.values()}
        bases.update({id(t): t for t in fallback.values()})
        self.bases = list(bases.values())
        self._views = None

    def base_of(self, which):
        """The allocation backing buffer `which` (to record it on another stream)."""
        if which in self.fallback:
            return self.fallback[which]
        g = self.taken.get(which)
        return g[0] if g is not None else None

    @property
    def buffers(self):
        if self._views is None:
            v = {w: b.narrow(0, o, n) for w, (b, o, n) in self.taken.items()}
            v.update(self.fallback)
            self._views = v
        return self._views


class _NativeAlloc(_PreAllocator):
    """What gsr_bind's calls allocated (their ``(taken, fallback)`` lists), with _PreAllocator's
    post-call interface (``ptrs``, ``bases``, ``buffers``, ``base_of``)."""

    def __init__(self, res):  # noqa: D107 - no pre-allocation here: gsr_bind made the tensors
        taken, fallback = res
        self._took({w: (b, o, n) for w, b, o, n in taken}, dict(fallback))


_native_mod = None
# GSR_NATIVE_BIND: bit mask of the calls gsr_bind takes over (1 forward, 2 render half, 4 views,
# 8 one-call backward; 0 none)
_NATIVE_PARTS = int(os.environ.get("GSR_NATIVE_BIND", "15"))
_EMPTY = torch.empty(0)  # an absent tensor argument (gsr_bind treats empty tensors as absent)


def _native():
    """The gsr_bind torch extension (gsr_bind.so next to this file, built by __graft_entry__.build():
    the two per-view calls' argument marshalling in C++), bound to this process's libgsr; None when it
    is absent or GSR_NATIVE_BIND=0 -- the ctypes path below does the same work in Python."""
    global _native_mod
    if _native_mod is None:
        _native_mod = False
        path = os.path.join(_HERE, "gsr_bind.so")
        if _NATIVE_PARTS and os.path.exists(path):
            import importlib.machinery
            import importlib.util
            L = load_library()
            import warnings
            try:  # the dlopen + PyInit happen in module_from_spec, the module body in exec_module
                spec = importlib.util.spec_from_file_location(
                    "gsr_bind", path, loader=importlib.machinery.ExtensionFileLoader("gsr_bind", path))
                m = importlib.util.module_from_spec(spec)
                spec.loader.exec_module(m)
                abi = m.abi_version() if hasattr(m, "abi_version") else None
            except (ImportError, OSError) as err:  # a stale build (another torch): ctypes, same kernels
                warnings.warn(f"gsr_bind.so not loadable ({err}); binding libgsr through ctypes instead")
                return None
            if abi != L.gsr_abi_version():  # built against another include/gsr.h: its structs differ
                warnings.warn(f"gsr_bind.so built for ABI {abi}, libgsr.so is ABI {L.gsr_abi_version()}: "
                              "binding libgsr through ctypes instead (rebuild gsr_bind)")
                return None
            m.set_functions({n: ctypes.cast(L[n], ctypes.c_void_p).value for n in (  # (L[n]: the symbol itself)
                "gsr_forward_info_call", "gsr_forward_async", "gsr_backward_render", "gsr_backward_gaussians",
                "gsr_backward", "gsr_prealloc_alloc",
                "gsr_spec_binning_bytes", "gsr_geom_bytes", "gsr_image_bytes", "gsr_scratch_bytes",
                "gsr_sums_bytes", "gsr_last_error")})
            _native_mod = m
    return _native_mod or None


_get_device = torch._C._cuda_getDevice
_raw_stream = torch._C._cuda_getCurrentRawStream


class _device_guard:
    """Make `dev` the current HIP device for the duration of a libgsr call (the library launches on
    the current device); free when it already is, which is the common case."""

    def __init__(self, dev):
        self.idx = dev.index if dev.index is not None else _get_device()
        self.prev = None

    def __enter__(self):
        cur = _get_device()
        if cur != self.idx:
            self.prev = cur
            torch.cuda.set_device(self.idx)
        return self

    def __exit__(self, *exc):
        if self.prev is not None:
            torch.cuda.set_device(self.prev)
        return False


def _stream_ptr(device):
    """The raw current HIP stream of `device` (torch's current stream)."""
    return ctypes.c_void_p(_raw_stream(device.index if device.index is not None else _get_device()))


_CAM_CACHE = {}
_CAM_CACHE_MAX = 512


def _camera(viewmatrix, projmatrix, tan_fovx, tan_fovy, image_height, image_width, campos, bg,
            prefiltered, keep):
    # the matrices and campos go in as they are (strided views included: the reference's viewmatrix
    # is a transposed view, campos a column slice) -- no per-call device copy.  The struct of a camera
    # whose tensors need no conversion is cached by the tensors' identity and data pointers (train.py
    # renders the same View.render_settings every step).
    key = (id(viewmatrix), id(projmatrix), id(campos), id(bg), image_width, image_height, tan_fovx, tan_fovy,
           prefiltered)
    e = _CAM_CACHE.get(key)
    if e is not None:
        cam, refs, ptrs = e
        if (refs[0] is viewmatrix and refs[1] is projmatrix and refs[2] is campos and refs[3] is bg and
                ptrs == (viewmatrix.data_ptr(), projmatrix.data_ptr(),
                         campos.data_ptr() if campos is not None else 0, bg.data_ptr())):
            return cam
    vm, vs = _mat16(viewmatrix)
    pm, ps = _mat16(projmatrix)
    bg_ = bg if bg.dtype == torch.float32 and bg.is_contiguous() else bg.contiguous().float()
    cp, cs = None, 0
    if campos is not None and campos.numel():
        cp = campos if campos.dtype == torch.float32 and campos.dim() == 1 else campos.reshape(-1).float()
        cs = cp.stride(0)
    keep += [vm, pm, bg_, cp]
    cam = _Camera(int(image_width), int(image_height), float(tan_fovx), float(tan_fovy),
                  _ptr(vm), _ptr(pm), _ptr(cp) if cp is not None else None,
                  _ptr(bg_), int(bool(prefiltered)))
    cam.viewmatrix_stride[0], cam.viewmatrix_stride[1] = vs
    cam.projmatrix_stride[0], cam.projmatrix_stride[1] = ps
    cam.campos_stride = cs
    if vm is viewmatrix and pm is projmatrix and bg_ is bg and (cp is campos):  # nothing converted
        if len(_CAM_CACHE) >= _CAM_CACHE_MAX:
            _CAM_CACHE.clear()
        _CAM_CACHE[key] = (cam, (viewmatrix, projmatrix, campos, bg),
                           (viewmatrix.data_ptr(), projmatrix.data_ptr(),
                            campos.data_ptr() if campos is not None else 0, bg.data_ptr()))
    return cam


def _mat16(m):
    """A 4x4 camera matrix ((4, 4) or (1, 4, 4), any strides) as (fp32 tensor whose data pointer is
    element [0][0], (row, col) element strides) -- the tensor itself when it needs no conversion."""
    if m.numel() != 16:
        raise RuntimeError("viewmatrix/projmatrix must hold 16 floats")
    if m.dtype != torch.float32:
        m = m.float()
    if m.shape in ((4, 4), (1, 4, 4)):
        return m, (m.stride(-2), m.stride(-1))
    m2 = m.reshape(4, 4)
    return m2, (m2.stride(0), m2.stride(1))


def _gaussians(means3D, sh, degree, colors, opacity, scales, rotations, scale_modifier, cov3D, keep,
               activations=0, prepare_backward=False, binning_layout=0):
    if means3D.ndimension() != 2 or means3D.size(1) != 3:
        raise RuntimeError("means3D must have dimensions (num_points, 3)")
    P = means3D.size(0)
    ts = [_f32(x) for x in (means3D, sh, colors, opacity, scales, rotations, cov3D)]
    keep += ts
    means3D, sh, colors, opacity, scales, rotations, cov3D = ts
    M = sh.size(1) if sh is not None and sh.numel() else 0
    return _Gaussians(P, int(degree), M, float(scale_modifier), _ptr(means3D), _ptr(sh), _ptr(colors),
                      _ptr(opacity), _ptr(scales), _ptr(rotations), _ptr(cov3D),
                      int(activations), int(bool(prepare_backward)), int(binning_layout or 0)), P, M


class AsyncForward:
    """An asynchronous forward's handle (gsr_forward_async): ``resolve()`` waits until its pair count is
    known and returns ``(num_rendered, binning_layout, binning_ptr)`` -- what the backward calls take
    (the BINNING buffer is the forward's own, or the library's when the speculation was redone);
    ``ready()`` says whether that would return without waiting.  The handle is released when this
    object is collected (after the backward that holds it)."""
    __slots__ = ("handle", "_res")

    def __init__(self, handle):
        self.handle = int(handle)
        self._res = None

    def __del__(self):
        _release_async(self.handle)

    def ready(self):
        return self._res is not None or load_library().gsr_forward_query(self.handle) > 0

    def resolve(self):
        if self._res is None:
            r = _Resolution()
            _check(load_library().gsr_forward_resolve(self.handle, ctypes.byref(r)))
            self._res = (r.num_rendered, r.binning_layout, r.binning, bool(r.redone))
        return self._res[:3]

    @property
    def redone(self):
        return self._res[3] if self._res is not None else None


def _release_async(handle):
    if _lib is not None:
        _lib.gsr_forward_release(handle)


def debug_async_fault(hold_next_redo_ms=0, gate_timeout_ms=0, clear=False):
    """Test hook (include/gsr.h gsr_debug_async_fault): hold the next redone asynchronous forward's gate
    closed for `hold_next_redo_ms`, time gates out after `gate_timeout_ms` (0: the default 5 s)."""
    _check(load_library().gsr_debug_async_fault(int(hold_next_redo_ms), int(gate_timeout_ms), int(bool(clear))))


def async_stats():
    """(asynchronous forwards since the last speculation_stats(reset=True), handles still held)."""
    c, p = ctypes.c_int(0), ctypes.c_int(0)
    _check(load_library().gsr_async_stats(ctypes.byref(c), ctypes.byref(p)))
    return c.value, p.value


def rasterize_gaussians(background, means3D, colors, opacity, scales, rotations, scale_modifier,
                        cov3D_precomp, viewmatrix, projmatrix, tan_fovx, tan_fovy, image_height,
                        image_width, sh, degree, campos, prefiltered, debug=False, activations=0,
                        prepare_backward=False, speculate=False, info=None, nonblocking=False):
    """``activations`` (ACT_* bits): opacity / scales / rotations hold the raw parameters of
    shared.py:29-42 and are activated inside the kernels (0 = the reference's interface).
    ``prepare_backward``: a backward will follow; the forward also builds its work-item list (the
    backward calls must then pass the same flag).  ``speculate``: queue the post-scan kernels before
    num_rendered is read back (gsr_forward_info_call, include/gsr.h); ``info`` (a dict) receives
    ``num_rendered``, ``binning_layout`` (pass it to the backward calls and decode_buffers),
    ``speculated`` and ``pending``.  ``nonblocking``: gsr_forward_async -- with a capacity from the
    pair-count history the call returns without reading num_rendered back; ``num_rendered`` is then
    -1 and ``info["pending"]`` an ``AsyncForward`` whose ``resolve()`` gives what the backward needs."""
    fi, color, radii, depth, alloc, pending = _forward(
        background, means3D, colors, opacity, scales, rotations, scale_modifier, cov3D_precomp, viewmatrix,
        projmatrix, tan_fovx, tan_fovy, image_height, image_width, sh, degree, campos, prefiltered, activations,
        prepare_backward, speculate, nonblocking)
    if info is not None:
        info.update(num_rendered=fi.num_rendered, binning_layout=fi.binning_layout, speculated=bool(fi.speculated),
                    pending=pending)
    b = alloc.buffers
    return fi.num_rendered, color, radii, b[GSR_BUF_GEOM], b[GSR_BUF_BINNING], b[GSR_BUF_IMAGE], depth


def _forward(background, means3D, colors, opacity, scales, rotations, scale_modifier, cov3D_precomp, viewmatrix,
             projmatrix, tan_fovx, tan_fovy, image_height, image_width, sh, degree, campos, prefiltered, activations,
             prepare_backward, speculate, nonblocking):
    """rasterize_gaussians without the buffer views: returns (gsr_forward_info, color, radii, depth,
    the _PreAllocator (``ptrs`` / ``bases`` of GEOM, BINNING, IMAGE), the AsyncForward or None)."""
    L = load_library()
    nat = _native() if _NATIVE_PARTS & 1 else None
    if nat is not None:
        e = _EMPTY
        (K, layout, spec, pend, aux, color, radii, depth, res) = nat.forward(
            background, means3D, e if colors is None else colors, e if opacity is None else opacity,
            e if scales is None else scales,
            e if rotations is None else rotations, float(scale_modifier), e if cov3D_precomp is None else cov3D_precomp,
            viewmatrix, projmatrix, float(tan_fovx), float(tan_fovy), int(image_height), int(image_width),
            e if sh is None else sh, int(degree), e if campos is None else campos, bool(prefiltered),
            int(activations), bool(prepare_backward), bool(speculate), bool(nonblocking), _PREALLOC_ON)
        fi = _ForwardInfo(K, layout, spec, pend, aux or None)
        alloc = _NativeAlloc(res)
    else:
        fi, color, radii, depth, alloc = _forward_ctypes(
            L, background, means3D, colors, opacity, scales, rotations, scale_modifier, cov3D_precomp, viewmatrix,
            projmatrix, tan_fovx, tan_fovy, image_height, image_width, sh, degree, campos, prefiltered, activations,
            prepare_backward, speculate, nonblocking)
    pending = AsyncForward(fi.pending) if fi.pending else None
    return fi, color, radii, depth, alloc, pending


def _forward_ctypes(L, background, means3D, colors, opacity, scales, rotations, scale_modifier, cov3D_precomp,
                    viewmatrix, projmatrix, tan_fovx, tan_fovy, image_height, image_width, sh, degree, campos,
                    prefiltered, activations, prepare_backward, speculate, nonblocking):
    """_forward's native call over ctypes (without gsr_bind)."""
    keep = []
    g, P, _ = _gaussians(means3D, sh, degree, colors, opacity, scales, rotations, scale_modifier,
                         cov3D_precomp, keep, activations, prepare_backward)
    cam = _camera(viewmatrix, projmatrix, tan_fovx, tan_fovy, image_height, image_width, campos,
                  background, prefiltered, keep)
    dev = means3D.device
    H, W = int(image_height), int(image_width)
    color = torch.empty((3, H, W), dtype=torch.float32, device=dev)
    depth = torch.empty((1, H, W), dtype=torch.float32, device=dev)
    radii = torch.empty((P,), dtype=torch.int32, device=dev)  # preprocess writes every entry
    fi = _ForwardInfo(0, 0, 0)
    with _device_guard(dev):  # launches go to dev even when another device is current
        # GEOM + IMAGE sized here in one allocation; the speculative BINNING (when this forward will
        # speculate) in its own, so that a failed speculation's buffer is released with the call
        spec = L.gsr_spec_binning_bytes(P, W, H, int(bool(prepare_backward))) if (speculate or nonblocking) and P else 0
        alloc = _PreAllocator(dev, [[(GSR_BUF_GEOM, L.gsr_geom_bytes(P)), (GSR_BUF_IMAGE, L.gsr_image_bytes(W, H, P))],
                                    [(GSR_BUF_BINNING, spec)]])
        with alloc:
            if nonblocking:
                _check(L.gsr_forward_async(ctypes.byref(cam), ctypes.byref(g), alloc.cb, alloc.ctx, color.data_ptr(),
                                           depth.data_ptr(), radii.data_ptr() if P else None, ctypes.byref(fi),
                                           _stream_ptr(dev)))
            else:
                _check(L.gsr_forward_info_call(ctypes.byref(cam), ctypes.byref(g), alloc.cb, alloc.ctx,
                                               color.data_ptr(), depth.data_ptr(), radii.data_ptr() if P else None,
                                               int(bool(speculate)), ctypes.byref(fi), _stream_ptr(dev)))
    return fi, color, radii, depth, alloc


_EXT_STREAMS = {}


def _external_stream(ptr, dev):
    """torch's handle of a raw stream (cached per device and stream).  Handle 0 is the device's default
    stream: torch.cuda.ExternalStream(0) is NOT that queue on ROCm -- work put on it ran on a separate
    hardware queue, unordered with the default stream (round 6: the held-back render halves of deferred
    views raced the forward and the per-Gaussian pass, tools/spec_half_repro.py, profiles/r06_async_race.txt)."""
    key = (dev.index if dev.index is not None else torch.cuda.current_device(), int(ptr))
    st = _EXT_STREAMS.get(key)
    if st is None:
        d = torch.device("cuda", key[0])
        st = torch.cuda.default_stream(d) if key[1] == 0 else torch.cuda.ExternalStream(key[1], device=d)
        _EXT_STREAMS[key] = st
    return st


def speculation_stats(reset=False):
    """(stood, redone) counts of speculative forwards since the last reset; ``reset`` also clears the
    pair-count history the capacities come from."""
    h, m = ctypes.c_int(0), ctypes.c_int(0)
    _check(load_library().gsr_spec_stats(ctypes.byref(h), ctypes.byref(m), int(bool(reset))))
    return h.value, m.value


def _grad_outputs(P, M, dev, colors, cov3D_precomp, scales, rotations, skip_unused, accumulate_into,
                  skip=(), overwrite=()):
    """The 8 gradient outputs of the backward (output order) and the accumulate bits: a given
    ``accumulate_into`` tensor is used in place, every other output is allocated (``skip``: output
    slots not produced at all, returned as None; ``overwrite``: slots whose given tensor receives the
    gradient without being read, i.e. no accumulate bit)."""
    e = lambda *s: torch.empty(s, dtype=torch.float32, device=dev)  # noqa: E731 - every element is written
    has = lambda t: t is not None and t.numel() > 0  # noqa: E731
    keep_col = not skip_unused or has(colors)
    keep_cov = not skip_unused or has(cov3D_precomp)
    keep_sr = not skip_unused or (has(scales) and has(rotations))
    shapes = [(P, 3), (P, 3) if keep_col else (0,), (P, 1), (P, 3), (P, 6) if keep_cov else (0,),
              (P, M, 3), (P, 3) if keep_sr else (0,), (P, 4) if keep_sr else (0,)]
    acc = list(accumulate_into or ()) + [None] * 8
    out = []
    acc_bits = given = 0
    for k, shp in enumerate(shapes):  # outputs that accumulate into a caller tensor are not allocated
        t = acc[k]
        if k in skip:
            out.append(None)
            continue
        if t is None or shp == (0,):
            out.append(e(*shp))
            continue
        if tuple(t.shape) != shp or t.dtype != torch.float32 or not t.is_contiguous() or t.device != dev:
            raise RuntimeError(f"accumulate_into[{k}]: expected a contiguous float32 {shp} tensor on {dev}")
        out.append(t)
        given |= 1 << k
        if k not in overwrite:
            acc_bits |= 1 << k
    out = tuple(out)
    if given:  # the kernel writes caller tensors on this stream: the allocator must not recycle
        cs = torch.cuda.current_stream(dev)  # them before it is done (views on several streams)
        for k in range(8):
            if given >> k & 1:
                out[k].record_stream(cs)
    return out, acc_bits


def rasterize_gaussians_backward(background, means3D, radii, colors, scales, rotations,
                                 scale_modifier, cov3D_precomp, viewmatrix, projmatrix, tan_fovx,
                                 tan_fovy, dL_dout_color, sh, degree, campos, geomBuffer, R,
                                 binningBuffer, imageBuffer, debug=False, dL_dout_depth=None,
                                 activations=0, skip_unused=False, accumulate_into=None,
                                 prepare_backward=False, needed=None, binning_layout=0, binning_ptr=None):
    """Returns the 8 gradients of the upstream binding.  ``skip_unused``: gradients of inputs that
    were not given (colours under SH, cov3D under scales/rotations and vice versa) come back as
    empty tensors and their HBM writes are skipped.  ``accumulate_into``: optional sequence of 8
    tensors (or None) in output order; a given tensor (contiguous fp32 of the output's shape) receives
    ``tensor + gradient`` in place (the kernel's single add = autograd's accumulation) and is
    returned in that slot.  ``needed``: optional 8 booleans in output order; a False slot is not
    computed into memory at all (NULL output, ABI 13) and comes back as None -- the autograd
    Function passes ``needs_input_grad`` (train.py renders frozen Gaussians: only means3D,
    rotations and means2D need a gradient there).  ``binning_ptr``: the BINNING buffer to read instead
    of ``binningBuffer``'s (an asynchronous forward's, from ``AsyncForward.resolve()``)."""
    L = load_library()
    nat = _native() if _NATIVE_PARTS & 8 else None
    if nat is not None:
        if means3D.ndimension() != 2 or means3D.size(1) != 3:
            raise RuntimeError("means3D must have dimensions (num_points, 3)")
        P, dev = means3D.size(0), means3D.device
        M = sh.size(1) if sh is not None and sh.numel() else 0
        skip = tuple(k for k in range(8) if needed is not None and not needed[k])
        out, acc_bits = _grad_outputs(P, M, dev, colors, cov3D_precomp, scales, rotations, skip_unused,
                                      accumulate_into, skip=skip)
        e = _EMPTY
        nat.backward(background, means3D, radii, e if colors is None else colors, e if scales is None else scales,
                     e if rotations is None else rotations, float(scale_modifier),
                     e if cov3D_precomp is None else cov3D_precomp, viewmatrix, projmatrix, float(tan_fovx),
                     float(tan_fovy), dL_dout_color, e if sh is None else sh, int(degree),
                     e if campos is None else campos, _bp(geomBuffer), int(R), binning_ptr or _bp(binningBuffer),
                     _bp(imageBuffer), int(activations), bool(prepare_backward), int(binning_layout or 0),
                     list(out), int(acc_bits), _PREALLOC_ON)
        return out
    keep = []
    g, P, M = _gaussians(means3D, sh, degree, colors, torch.empty(0, device=means3D.device), scales,
                         rotations, scale_modifier, cov3D_precomp, keep, activations, prepare_backward,
                         binning_layout)
    H, W = dL_dout_color.shape[-2], dL_dout_color.shape[-1]
    cam = _camera(viewmatrix, projmatrix, tan_fovx, tan_fovy, H, W, campos, background, False, keep)
    dev = means3D.device
    skip = tuple(k for k in range(8) if needed is not None and not needed[k])
    out, acc_bits = _grad_outputs(P, M, dev, colors, cov3D_precomp, scales, rotations, skip_unused,
                                  accumulate_into, skip=skip)
    if P == 0:
        return out
    dpix = dL_dout_color.contiguous().float()
    keep.append(dpix)
    grads = _Grads(*[t.data_ptr() if t is not None and t.numel() else None for t in out], acc_bits)
    alloc = _PreAllocator(dev, [[(GSR_BUF_SCRATCH, L.gsr_scratch_bytes(int(R), W, H))]])
    with _device_guard(dev), alloc:
        _check(L.gsr_backward(ctypes.byref(cam), ctypes.byref(g), radii.data_ptr(), int(R),
                              _bp(geomBuffer), binning_ptr or _bp(binningBuffer), _bp(imageBuffer),
                              dpix.data_ptr(), None, alloc.cb, alloc.ctx, ctypes.byref(grads), _stream_ptr(dev)))
    return out


def rasterize_gaussians_backward_render(background, means3D, radii, colors, scales, rotations,
                                        scale_modifier, cov3D_precomp, viewmatrix, projmatrix, tan_fovx,
                                        tan_fovy, dL_dout_color, sh, degree, campos, geomBuffer, R,
                                        binningBuffer, imageBuffer, activations=0, prepare_backward=False,
                                        binning_layout=0, binning_ptr=None):
    """The per-pixel half of ``rasterize_gaussians_backward`` (gsr_backward_render): returns the
    view's SUMS byte buffer (each Gaussian's per-(tile, Gaussian) gradient records summed, 9 x P
    floats), for ``rasterize_gaussians_backward_views``; the records' SCRATCH buffer is released here
    (its last reader is already queued on the current stream).  ``R < 0``: the speculative half of an
    asynchronous forward whose pair count is not known yet (ABI 19): sized for its capacity
    ``binning_layout`` over its own BINNING; redo it with the resolved values when
    ``AsyncForward.redone``."""
    L = load_library()
    nat = _native() if _NATIVE_PARTS & 2 else None
    if nat is not None:
        e = _EMPTY
        sums, _ = nat.backward_render(
            background, means3D, radii, e if colors is None else colors, e if scales is None else scales,
            e if rotations is None else rotations, float(scale_modifier), e if cov3D_precomp is None else cov3D_precomp,
            viewmatrix, projmatrix, float(tan_fovx), float(tan_fovy), dL_dout_color, e if sh is None else sh,
            int(degree), e if campos is None else campos, _bp(geomBuffer), int(R),
            binning_ptr or _bp(binningBuffer), _bp(imageBuffer), int(activations), bool(prepare_backward),
            int(binning_layout or 0), _PREALLOC_ON)
        return sums
    keep = []
    g, P, _ = _gaussians(means3D, sh, degree, colors, torch.empty(0, device=means3D.device), scales,
                         rotations, scale_modifier, cov3D_precomp, keep, activations, prepare_backward,
                         binning_layout)
    H, W = dL_dout_color.shape[-2], dL_dout_color.shape[-1]
    cam = _camera(viewmatrix, projmatrix, tan_fovx, tan_fovy, H, W, campos, background, False, keep)
    dev = means3D.device
    if P == 0:
        return torch.empty(1, dtype=torch.uint8, device=dev)
    dpix = dL_dout_color.contiguous().float()
    keep.append(dpix)
    # SCRATCH and SUMS as two allocations: SCRATCH is released when this returns, SUMS stays queued
    alloc = _PreAllocator(dev, [[(GSR_BUF_SCRATCH, L.gsr_scratch_bytes(int(R) if R >= 0 else int(binning_layout), W, H))],
                                [(GSR_BUF_SUMS, L.gsr_sums_bytes(P))]])
    with _device_guard(dev), alloc:
        _check(L.gsr_backward_render(ctypes.byref(cam), ctypes.byref(g), radii.data_ptr(), int(R),
                                     _bp(geomBuffer), binning_ptr or _bp(binningBuffer), _bp(imageBuffer),
                                     dpix.data_ptr(), alloc.cb, alloc.ctx, _stream_ptr(dev)))
    return alloc.buffers[GSR_BUF_SUMS]


def rasterize_gaussians_backward_views(views, means3D, colors, scales, rotations, scale_modifier,
                                       cov3D_precomp, sh, degree, activations=0, skip_unused=True,
                                       accumulate_into=None, overwrite=(), needed=None):
    """The per-Gaussian half over several views of the same Gaussians (gsr_backward_gaussians), on the
    current stream: returns the 8 gradients of ``rasterize_gaussians_backward`` summed over the views
    (slot 0, dL/dmeans2D, is None: each view's goes to its own array; ``needed`` as in
    ``rasterize_gaussians_backward``).  ``views``: dicts with the
    view's ``viewmatrix``, ``projmatrix``, ``tanfovx``, ``tanfovy``, ``image_height``, ``image_width``,
    ``campos``, ``bg``, its ``radii``, ``geomBuffer`` (a tensor or a device pointer, then ``keep``: the
    tensors backing it), ``scratch`` (from
    ``rasterize_gaussians_backward_render``) and ``num_rendered``, and optionally ``means2D_grad``, a
    contiguous (P, 3) fp32 tensor receiving its screen-space gradient (added into when
    ``accumulate_means2D``).  ``overwrite``: output slots whose ``accumulate_into`` tensor is written
    without being read (a fresh, uninitialised gradient).  The caller orders the views' render halves
    before this call."""
    L = load_library()
    keep = []
    dev = means3D.device
    g, P, M = _gaussians(means3D, sh, degree, colors, torch.empty(0, device=dev), scales, rotations,
                         scale_modifier, cov3D_precomp, keep, activations)
    skip = (0,) + tuple(k for k in range(1, 8) if needed is not None and not needed[k])
    out, acc_bits = _grad_outputs(P, M, dev, colors, cov3D_precomp, scales, rotations, skip_unused,
                                  accumulate_into, skip=skip, overwrite=overwrite)
    if P == 0 or not views:
        return out
    nat = _native() if _NATIVE_PARTS & 4 else None
    if nat is not None:
        e = _EMPTY
        nat.backward_views(list(views), means3D, e if colors is None else colors, e if scales is None else scales,
                           e if rotations is None else rotations, float(scale_modifier),
                           e if cov3D_precomp is None else cov3D_precomp, e if sh is None else sh, int(degree),
                           int(activations), list(out), int(acc_bits))
        return out
    cams = []
    vg = (_ViewGrad * len(views))()
    cs = torch.cuda.current_stream(dev)
    for k, v in enumerate(views):
        cam = _camera(v["viewmatrix"], v["projmatrix"], v["tanfovx"], v["tanfovy"], v["image_height"],
                      v["image_width"], v["campos"], v["bg"], False, keep)
        cams.append(cam)
        m2 = v.get("means2D_grad")
        if m2 is not None:
            if tuple(m2.shape) != (P, 3) or m2.dtype != torch.float32 or not m2.is_contiguous() or m2.device != dev:
                raise RuntimeError(f"views[{k}]['means2D_grad']: expected a contiguous float32 ({P}, 3) tensor on {dev}")
            m2.record_stream(cs)
        for t in (v["radii"], v["scratch"], *v.get("keep", ()),  # read on this stream, maybe allocated
                  *((v["geomBuffer"],) if isinstance(v["geomBuffer"], torch.Tensor) else ())):  # on the view's
            t.record_stream(cs)
        vg[k] = _ViewGrad(ctypes.pointer(cam), v["radii"].data_ptr(), _bp(v["geomBuffer"]),
                          v["scratch"].data_ptr(), int(v["num_rendered"]),
                          m2.data_ptr() if m2 is not None else None, int(bool(v.get("accumulate_means2D"))))
    grads = _Grads(*[t.data_ptr() if t is not None and t.numel() else None for t in out], acc_bits)
    with _device_guard(dev):
        _check(L.gsr_backward_gaussians(len(views), vg, ctypes.byref(g), ctypes.byref(grads), _stream_ptr(dev)))
    return out


def grad_fence(*grads):
    """Declare that the work queued so far on the current stream writes the gradient tensors
    ``grads`` (an all-reduce, a reset of the bucket they live in): the next rasterizer backward
    into any of them, on any stream, is ordered after it (gsr_grad_fence)."""
    grads = [g for g in grads if g is not None and g.numel()]
    if not grads:
        return
    dev = grads[0].device
    arr = (ctypes.c_void_p * len(grads))(*[g.data_ptr() for g in grads])
    with _device_guard(dev):
        _check(load_library().gsr_grad_fence(arr, len(grads), _stream_ptr(dev)))


def mark_visible(means3D, viewmatrix, projmatrix):
    L = load_library()
    P = means3D.size(0)
    present = torch.zeros((P,), dtype=torch.bool, device=means3D.device)
    if P == 0:
        return present
    m = means3D.contiguous().float()
    vm, pm = viewmatrix.contiguous().float(), projmatrix.contiguous().float()
    with _device_guard(means3D.device):
        _check(L.gsr_mark_visible(P, _ptr(m), _ptr(vm), _ptr(pm), present.data_ptr(),
                                  _stream_ptr(means3D.device)))
    return present


# ---- instrumentation (per-phase HIP-event timing inside libgsr) ----
def profile_enable(on=True):
    _check(load_library().gsr_profile_enable(int(bool(on))))


def profile_select(phases=None):
    """Record device events only for ``phases`` (iterable of names; None = all phases)."""
    _check(load_library().gsr_profile_select(",".join(phases).encode() if phases else None))


def profile_reset():
    _check(load_library().gsr_profile_reset())


def profile_read(phase=None):
    """Return (total_ms, count) of the recorded launches of ``phase`` (all phases if None)."""
    L = load_library()
    tot, cnt = ctypes.c_double(0), ctypes.c_int(0)
    _check(L.gsr_profile_read(phase.encode() if phase else None, ctypes.byref(tot), ctypes.byref(cnt)))
    return tot.value, cnt.value


def decode_buffers(P, W, H, num_rendered, geomBuffer, binningBuffer, imgBuffer, binning_layout=0):
    """Typed views of the arrays inside the forward buffers (for parity tests / debugging);
    ``binning_layout``: the forward's info["binning_layout"] when it enqueued speculatively."""
    L = load_library()
    offs = (ctypes.c_size_t * 16)()
    L.gsr_buffer_offsets(int(P), int(W), int(H), int(binning_layout or num_rendered), offs, 16)
    o = list(offs)
    T = ((W + 15) // 16) * ((H + 15) // 16)
    K = int(num_rendered)

    def view(buf, off, n, dtype, shape):
        nbytes = n * torch.tensor([], dtype=dtype).element_size()
        return buf[off:off + nbytes].view(dtype).reshape(shape)

    f32, i32, i64 = torch.float32, torch.int32, torch.int64
    rec = view(geomBuffer, o[1], 16 * P, f32, (P, 16))  # 64-byte render records
    return {
        "depth": view(geomBuffer, o[0], P, f32, (P,)),
        "rec": rec,
        "xy": rec[:, 0:2],
        "conic_opacity": torch.stack([rec[:, 12], rec[:, 13], rec[:, 14], rec[:, 5]], 1),
        "rgbd": torch.cat([rec[:, 8:11], rec[:, 6:7]], 1),
        "tau2": rec[:, 7],
        "rect": view(geomBuffer, o[2], 2 * P, i32, (P, 2)),
        "tiles_touched": view(geomBuffer, o[3], P, i32, (P,)),
        "goff": view(geomBuffer, o[4], P + 1, i32, (P + 1,)),
        "ranges": view(imgBuffer, o[5], 2 * T, i32, (T, 2)),
        "pix_end": view(imgBuffer, o[6], 4 * W * H, f32, (H, W, 4)),
        "final_T": view(imgBuffer, o[6], 4 * W * H, f32, (H, W, 4))[..., 3],
        "seg_off": view(imgBuffer, o[12], T + 1, i32, (T + 1,)),
        "n_contrib": view(imgBuffer, o[7], W * H, i32, (H, W)),
        "tile_maxc": view(imgBuffer, o[8], 4 * T, i32, (T, 4)),
        "tile_flag": view(imgBuffer, o[14], T, i32, (T,)),  # near-threshold re-evaluations (> 16: overflow tile)
        "tsat_count": view(imgBuffer, o[15], 1, i32, (1,)),  # pixels the exact saturation re-walk redid
        # per-pair records (index, depth bits, emission, 0) in tile-bucket order; keys = .x | .y << 32
        "pairs": view(binningBuffer, o[9], 4 * K, i32, (K, 4)),
        "keys": view(binningBuffer, o[9], 2 * K, i64, (K, 2))[:, 0],
        "point_list": view(binningBuffer, o[10], K, i32, (K,)),
        "slot_emit": view(binningBuffer, o[11], K, i32, (K,)),
    }
