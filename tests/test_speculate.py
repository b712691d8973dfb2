"""Speculative enqueue of the forward (-m gpu; gsr_forward_info_call, include/gsr.h ABI 14).

A forward with pair-count history for its (device, P, W, H) queues bin_emit / tile_sort / render /
items before reading num_rendered back, against a BINNING capacity of 1.25 x the largest K seen; the
kernels check k_bin_scan's verdict on the device and the host redoes them exactly when it fails.
Every output must be bitwise the exact path's: images, radii, every decoded buffer, and the backward
(which reads the BINNING arrays through the reported layout).  Cases: the first call (no history:
exact), a repeat (speculation stands), a denser view than the history (capacity exceeded: redone), a
long tile list (> 4096 pairs needs the merge sort: redone, and the next call does not speculate).
"""
import pytest
import torch

import splat_scenes as S
from diff_gaussian_rasterization import _C

pytestmark = pytest.mark.gpu


def _render(a, rs, speculate, dl):
    e = torch.empty(0, device=a["means3D"].device)
    info = {}
    out = _C.rasterize_gaussians(rs.bg, a["means3D"], a.get("colors_precomp", e), a["opacities"], a["scales"],
                                 a["rotations"], 1.0, e, rs.viewmatrix, rs.projmatrix, rs.tanfovx, rs.tanfovy,
                                 rs.image_height, rs.image_width, a.get("shs", e), rs.sh_degree, rs.campos, False,
                                 prepare_backward=True, speculate=speculate, info=info)
    K, color, radii, geom, binning, img, depth = out
    P = a["means3D"].shape[0]
    dec = _C.decode_buffers(P, rs.image_width, rs.image_height, K, geom, binning, img,
                            binning_layout=info["binning_layout"])
    g = _C.rasterize_gaussians_backward(rs.bg, a["means3D"], radii, a.get("colors_precomp", e), a["scales"],
                                        a["rotations"], 1.0, e, rs.viewmatrix, rs.projmatrix, rs.tanfovx,
                                        rs.tanfovy, dl, a.get("shs", e), rs.sh_degree, rs.campos, geom, K, binning,
                                        img, prepare_backward=True, binning_layout=info["binning_layout"])
    torch.cuda.synchronize()
    return info, color, depth, radii, dec, g


def _same(x, y):
    (ix, *rx), (iy, *ry) = x, y
    assert ix["num_rendered"] == iy["num_rendered"]
    cx, dx_, rdx, decx, gx = rx
    cy, dy_, rdy, decy, gy = ry
    assert torch.equal(cx, cy) and torch.equal(dx_, dy_) and torch.equal(rdx, rdy)
    for k in ("ranges", "point_list", "slot_emit", "n_contrib", "pix_end", "tile_maxc", "goff", "seg_off"):
        assert torch.equal(decx[k], decy[k]), k
    for a, b in zip(gx, gy):
        assert (a is None and b is None) or torch.equal(a, b)


def test_speculative_forward_is_bitwise_the_exact_path(cuda):
    P, W, H = 60_000, 640, 480
    a = {k: v for k, v in S.activated_inputs(S.synthetic_cloud(P, 0.01, sh_degree=3, seed=21, device=cuda), 3).items()
         if k != "means2D" and v is not None}
    a.pop("colors_precomp", None)
    # the same (P, W, H) key twice: the cloud as is, and with 4x the scales (each Gaussian covers more
    # tiles: K 111873 -> 256884 by the CPU oracle, longest list 2488, no merge sort)
    cam = S.render_settings(W, H, S.intrinsics(500.0, W, H), S.look_at(30, 0.2, 9.0), device=cuda, sh_degree=3)
    dense = dict(a, scales=a["scales"] * 4.0)
    dl = S.upstream_grad(H, W, device=cuda)
    _C.speculation_stats(reset=True)
    exact_far = _render(a, cam, False, dl)
    assert exact_far[0]["speculated"] is False and exact_far[0]["binning_layout"] == exact_far[0]["num_rendered"]
    first = _render(a, cam, True, dl)       # history from the exact call above: speculates
    assert first[0]["speculated"] and first[0]["binning_layout"] > first[0]["num_rendered"]
    _same(first, exact_far)
    exact_near = _render(dense, cam, False, dl)
    _C.speculation_stats(reset=True)
    _render(a, cam, False, dl)               # history: the sparse cloud only
    grown = _render(dense, cam, True, dl)    # K well above 1.25 x the history: redone exactly
    assert exact_near[0]["num_rendered"] > 1.3 * exact_far[0]["num_rendered"] + 65536
    assert grown[0]["speculated"] is False
    _same(grown, exact_near)
    again = _render(dense, cam, True, dl)    # history now holds the dense cloud: stands
    assert again[0]["speculated"]
    _same(again, exact_near)
    hits, misses = _C.speculation_stats()
    assert (hits, misses) == (1, 1)


def test_speculation_falls_back_on_long_lists(cuda):
    """A tile list past 4096 pairs needs the host-sized merge sort: a speculative call that meets one
    is redone exactly, and the key then stops speculating until a call without long lists."""
    g = torch.Generator().manual_seed(4)
    P = 12_000
    m = torch.zeros(P, 3)
    m[:, 0] = torch.rand(P, generator=g) * 0.02 - 0.01
    m[:, 1] = torch.rand(P, generator=g) * 0.02 - 0.01
    m[:, 2] = torch.rand(P, generator=g) * 2 - 1
    a = {"means3D": m, "colors_precomp": torch.rand(P, 3, generator=g), "opacities": torch.full((P, 1), 0.05),
         "scales": torch.full((P, 3), 0.004), "rotations": torch.tensor([[1.0, 0, 0, 0]]).repeat(P, 1)}
    a = {k: v.to(cuda) for k, v in a.items()}
    rs = S.render_settings(64, 64, S.intrinsics(64.0, 64, 64), S.look_at(0, 0, 4), device=cuda)
    dl = S.upstream_grad(64, 64, device=cuda)
    exact = _render(a, rs, False, dl)
    # seed a history without long lists for this (P, W, H): the same cloud spread out (x300: K 9307,
    # longest list 641 by the CPU oracle; x100 still leaves a 4186-pair tile)
    spread = dict(a, means3D=a["means3D"] * torch.tensor([300.0, 300.0, 1.0], device=cuda))
    _C.speculation_stats(reset=True)
    _render(spread, rs, False, dl)
    got = _render(a, rs, True, dl)
    assert got[0]["speculated"] is False
    _same(got, exact)
    nxt = _render(a, rs, True, dl)           # the last call saw long lists: exact, no speculation
    assert nxt[0]["speculated"] is False
    assert _C.speculation_stats() == (0, 1)
