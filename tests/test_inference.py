"""train.py's inference call site against the CPU oracle (-m gpu).

render_and_export_frame (train.py:506-547) renders each timestep through the five fixed cameras of
create_extrinsic_matrices (train.py:459-503) at 1280 x 720, under ``torch.no_grad()`` (train.py:778),
with ``Renderer(raster_settings=...)(**create_render_arguments(params))``: a forward-only call of the
drop-in module on non-leaf activations.  Checked here on a 300k-Gaussian cloud:

* radii bit-exact and colour / depth within 1e-4 (T-saturation flips allowed at 4x the measured
  rate) against the oracle, for every camera;
* no per-call workspace outlives the call: with no autograd graph the GEOM / IMAGE / BINNING buffers
  (and any speculative BINNING) are released when the call returns, so the bytes requested from the
  caching allocator (``requested_bytes``: exact sizes, not its block rounding) grow by the outputs
  alone, and return to where they were once the outputs go.
"""
import numpy as np
import pytest
import torch

import splat_scenes as S
from diff_gaussian_rasterization import GaussianRasterizer
from oracle import oracle as O
from test_gpu_parity import _close, _np

pytestmark = pytest.mark.gpu

P = 300_000
PIX_FLIP = 0.0  # round 6: the T >= 1e-4 saturation decisions are the oracle's too (k_render_tsat)


def _requested(dev):
    return torch.cuda.memory_stats(dev)["requested_bytes.all.current"]


def _cloud(dev):
    return S.synthetic_cloud(P, 0.008, sh_degree=-1, seed=2, device=dev)


def test_inference_rig_parity_and_workspace(cuda):
    params = _cloud(cuda)
    cams = S.inference_cameras(device=cuda)
    torch.cuda.synchronize()
    for i, rs in enumerate(cams):
        with torch.no_grad():
            args = S.render_arguments(params)  # create_render_arguments, per render (train.py:544)
            torch.cuda.synchronize()
            before = _requested(cuda)
            img, radii, depth = GaussianRasterizer(raster_settings=rs)(**args)
            torch.cuda.synchronize()
            after = _requested(cuda)
        assert not img.requires_grad and img.grad_fn is None
        # the oracle gets the very activations the GPU rendered (torch's GPU exp / sigmoid / normalize can
        # differ from its CPU ones by an ulp, which can move a radius across an integer)
        a = {k: v.detach().cpu() for k, v in args.items() if k != "means2D"}
        out_bytes = sum(t.untyped_storage().nbytes() for t in (img, radii, depth))
        assert after - before == out_bytes, (
            f"camera {i}: {after - before} bytes held after the call, outputs are {out_bytes}")
        r = rs._replace(viewmatrix=rs.viewmatrix.cpu(), projmatrix=rs.projmatrix.cpu(), campos=rs.campos.cpu(),
                        bg=rs.bg.cpu())
        st = O.forward(r.bg.numpy(), a["means3D"].numpy(), a["colors_precomp"].numpy(), a["opacities"].numpy(),
                       a["scales"].numpy(), a["rotations"].numpy(), 1.0, None, r.viewmatrix, r.projmatrix,
                       r.tanfovx, r.tanfovy, r.image_height, r.image_width, None, 0, r.campos.numpy())
        assert st["num_rendered"] > 0
        np.testing.assert_array_equal(_np(radii), st["radii"])
        _close("color", _np(img), st["color"], atol_frac=1e-6, max_bad_frac=PIX_FLIP)
        _close("depth", _np(depth), st["depth"], atol_frac=1e-6, max_bad_frac=PIX_FLIP)
        del img, radii, depth, st
        torch.cuda.synchronize()
        assert _requested(cuda) == before, f"camera {i}: memory not returned after the outputs went"
