"""CPU tests of the drop-in boundary: the C-ABI library and the Python surface (no GPU compute).

* libgsr.so loads and exports every function include/gsr.h declares;
* host-only entry points (buffer sizing, ABI version, argument validation) behave as documented,
  with the reference binding's error messages;
* the Python package exposes GaussianRasterizationSettings (the 11 keyword fields of
  shared.py:112-124 + optional debug) and GaussianRasterizer with the reference's argument
  validation, and refuses CPU tensors (there is no CPU fallback path).
"""
import ctypes
import os
import re

import pytest
import torch

from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer, _C

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "gsr.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"\b(gsr_\w+)\s*\(", src)
    return sorted(set(n for n in names if not n.endswith("_fn")))


def test_library_exports_every_declared_symbol():
    L = _C.load_library()
    decl = declared_functions()
    assert len(decl) >= 10
    for name in decl:
        assert hasattr(L, name), f"{name} declared in include/gsr.h but not exported"
    assert set(decl) == set(_C.EXPORTED_SYMBOLS)


def test_host_only_entry_points():
    L = _C.load_library()
    assert L.gsr_abi_version() == _C.ABI_VERSION == 21
    for P in (0, 1, 1000, 1_000_000):
        assert L.gsr_geom_bytes(P) % 256 == 0 and L.gsr_geom_bytes(P) >= 64 * P
    assert L.gsr_image_bytes(1920, 1080, 10) >= 1920 * 1080 * 8
    assert L.gsr_binning_bytes(100, 1000) >= 100 * 16 and L.gsr_scratch_bytes(100, 64, 48) >= 100 * 36
    assert L.gsr_sums_bytes(1000) >= 1000 * 36 and L.gsr_sums_bytes(1000) % 256 == 0  # ABI 15
    offs = (ctypes.c_size_t * 15)()
    assert L.gsr_buffer_offsets(100, 64, 48, 500, offs, 15) == 15
    assert all(o % 256 == 0 for o in offs)


def test_async_forward_handles_host_side():
    """ABI 17: the asynchronous forward's handle calls validate without a GPU -- an unknown handle is
    refused by resolve (with a message), reported unknown by query, and ignored by release; no
    forward has run, so nothing is pending."""
    L = _C.load_library()
    r = _C._Resolution()
    assert L.gsr_forward_resolve(12345, ctypes.byref(r)) == 1
    assert b"unknown or released forward 12345" in L.gsr_last_error()
    assert L.gsr_forward_query(12345) == -1
    assert L.gsr_forward_release(12345) == 0
    assert _C.async_stats() == (0, 0)
    assert L.gsr_spec_keys() == 0


def test_binning_bytes_follow_segment_length():
    """gsr_binning_bytes(K, P) (ABI 16) sizes the backward's saved blend states for the segment length
    of a P-Gaussian cloud (seg_log2, gsr_common.h): 64 list entries below 262144 Gaussians, 128 below
    524288, 256 above, one 256-pixel float4 state per segment boundary."""
    L = _C.load_library()
    K = 4_000_000
    b = {P: L.gsr_binning_bytes(K, P) for P in (262_143, 262_144, 524_287, 524_288, 2_000_000)}
    states = lambda seg: (K // seg + 1) * 256 * 16  # noqa: E731
    assert b[262_143] - b[262_144] == states(64) - states(128)
    assert b[524_287] - b[524_288] == states(128) - states(256)
    assert b[262_144] == b[524_287] and b[524_288] == b[2_000_000]


def _cam_gauss(**kw):
    dummy = ctypes.c_void_p(0x1000)  # never dereferenced: validation fails first
    cam = _C._Camera(64, 48, 0.5, 0.5, dummy, dummy, dummy, dummy, 0)
    g = _C._Gaussians(10, 0, 0, 1.0, dummy, None, dummy, dummy, dummy, dummy, None)
    for k, v in kw.items():
        setattr(g, k, v)
    return cam, g


@pytest.mark.parametrize("bad,msg", [
    (dict(colors_precomp=None), "excatly one of either SHs or precomputed colors"),
    (dict(rotations=None), "scale/rotation pair or precomputed 3D covariance"),
    (dict(cov3D_precomp=ctypes.c_void_p(0x1000)), "scale/rotation pair or precomputed 3D covariance"),
    (dict(P=-1), "P must be >= 0"),
])
def test_forward_argument_validation(bad, msg):
    L = _C.load_library()
    cam, g = _cam_gauss(**bad)
    nr = ctypes.c_int(0)
    alloc = _C._ALLOC_FN(lambda ctx, which, n: None)
    rc = L.gsr_forward(ctypes.byref(cam), ctypes.byref(g), alloc, None, ctypes.c_void_p(0x1000),
                       ctypes.c_void_p(0x1000), ctypes.c_void_p(0x1000), ctypes.byref(nr), None)
    assert rc == 1  # GSR_ERR_ARG, before any device work
    assert msg in L.gsr_last_error().decode()


def test_settings_namedtuple_matches_reference_construction():
    fields = ("image_height", "image_width", "tanfovx", "tanfovy", "bg", "scale_modifier",
              "viewmatrix", "projmatrix", "sh_degree", "campos", "prefiltered")
    assert GaussianRasterizationSettings._fields[:11] == fields
    rs = GaussianRasterizationSettings(image_height=2, image_width=3, tanfovx=0.5, tanfovy=0.5,
                                       bg=torch.zeros(3), scale_modifier=1.0, viewmatrix=torch.eye(4)[None],
                                       projmatrix=torch.eye(4)[None], sh_degree=0, campos=torch.zeros(3),
                                       prefiltered=False)
    assert rs.debug is False


def test_rasterizer_validation_and_no_cpu_path():
    rs = GaussianRasterizationSettings(image_height=8, image_width=8, tanfovx=0.5, tanfovy=0.5,
                                       bg=torch.zeros(3), scale_modifier=1.0, viewmatrix=torch.eye(4)[None],
                                       projmatrix=torch.eye(4)[None], sh_degree=0, campos=torch.zeros(3),
                                       prefiltered=False)
    r = GaussianRasterizer(raster_settings=rs)
    m = torch.zeros(4, 3)
    with pytest.raises(Exception, match="excatly one of either SHs or precomputed colors"):
        r(means3D=m, means2D=m, opacities=torch.ones(4, 1), scales=m, rotations=torch.zeros(4, 4))
    with pytest.raises(Exception, match="scale/rotation pair"):
        r(means3D=m, means2D=m, opacities=torch.ones(4, 1), colors_precomp=m, scales=m)
    with pytest.raises(RuntimeError, match="no CPU path"):
        r(means3D=m, means2D=m, opacities=torch.ones(4, 1), colors_precomp=m, scales=m,
          rotations=torch.zeros(4, 4))
    with pytest.raises(RuntimeError, match=r"means3D must have dimensions \(num_points, 3\)"):
        r(means3D=torch.zeros(4, 2), means2D=m, opacities=torch.ones(4, 1), colors_precomp=m, scales=m,
          rotations=torch.zeros(4, 4))


@pytest.mark.skipif(not os.path.exists(os.path.join(os.path.dirname(_C.__file__), "gsr_bind.so")),
                    reason="gsr_bind.so not built")
def test_native_marshalling_module_loads():
    """gsr_bind (the C++ marshalling of the per-call bindings) loads against this torch and takes the
    library's symbol addresses -- no GPU call."""
    m = _C._native()
    assert m is not None
    for name in ("forward", "backward", "backward_render", "backward_views", "set_functions"):
        assert hasattr(m, name), name
