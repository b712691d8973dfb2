"""Boundary callers pinned against golden vectors produced by the reference's own Python.

tests/golden/reference_harness.npz was written by tests/golden/gen_golden.py, which imports the
reference's shared.py / external.py / densify.py / train.py (CPU shims, stub open3d/wandb/imageio)
and records their outputs.  The restatements used by tests and bench (splat_scenes) and the
data-parallel densify statistics (splat_dp) must reproduce them exactly.
"""
import os

import numpy as np
import pytest
import torch

import splat_dp
import splat_scenes as S
from oracle import dense_torch as DT

GOLD = np.load(os.path.join(os.path.dirname(__file__), "golden", "reference_harness.npz"))


@pytest.mark.parametrize("c", range(int(GOLD["n_cams"])))
def test_render_settings_match_reference(c):
    """create_render_settings (shared.py:64-124): matrices bit-exact, tanfov exact."""
    W, H = (int(x) for x in GOLD[f"cam{c}_in_wh"])
    rs = S.render_settings(W, H, GOLD[f"cam{c}_in_K"], GOLD[f"cam{c}_in_w2c"], device="cpu")
    np.testing.assert_array_equal(rs.viewmatrix.contiguous().numpy(), GOLD[f"cam{c}_viewmatrix"])
    np.testing.assert_array_equal(rs.projmatrix.contiguous().numpy(), GOLD[f"cam{c}_projmatrix"])
    np.testing.assert_array_equal(rs.campos.numpy(), GOLD[f"cam{c}_campos"])
    np.testing.assert_array_equal(rs.bg.numpy(), GOLD[f"cam{c}_bg"])
    assert (rs.tanfovx, rs.tanfovy) == tuple(GOLD[f"cam{c}_tanfov"])
    h, w, shd, mod, pre = GOLD[f"cam{c}_misc"]
    assert (rs.image_height, rs.image_width, rs.sh_degree, rs.scale_modifier, float(rs.prefiltered)) == (h, w, shd, mod, pre)
    # the matrices the kernels read: 16 floats, column-major (x' = m0 x + m4 y + m8 z + m12)
    w2c = GOLD[f"cam{c}_in_w2c"].astype(np.float32)
    m = GOLD[f"cam{c}_viewmatrix"].reshape(16)
    np.testing.assert_array_equal(m[[0, 4, 8, 12]], w2c[0])


def test_inference_rig_matches_reference():
    """splat_scenes.inference_rig / inference_intrinsics restate train.py's create_extrinsic_matrices and
    render_and_export_frame's intrinsics: golden cameras 5-9 are the reference's own five, in order."""
    rig = list(S.inference_rig().values())
    assert len(rig) == 5
    for i, (w2c, aspect) in enumerate(rig):
        c = 5 + i
        np.testing.assert_array_equal(w2c, GOLD[f"cam{c}_in_w2c"])
        np.testing.assert_array_equal(S.inference_intrinsics(aspect), GOLD[f"cam{c}_in_K"])
        assert tuple(int(x) for x in GOLD[f"cam{c}_in_wh"]) == (S.INFERENCE_W, S.INFERENCE_H)
        rs = S.inference_cameras(device="cpu")[i]
        np.testing.assert_array_equal(rs.viewmatrix.contiguous().numpy(), GOLD[f"cam{c}_viewmatrix"])
        np.testing.assert_array_equal(rs.projmatrix.contiguous().numpy(), GOLD[f"cam{c}_projmatrix"])


def test_render_arguments_match_reference():
    """create_render_arguments (shared.py:29-42)."""
    params = {k[len("args_in_"):]: torch.from_numpy(GOLD[k]) for k in GOLD.files if k.startswith("args_in_")}
    ra = S.render_arguments(params)
    for k in ("means3D", "colors_precomp", "rotations", "opacities", "scales", "means2D"):
        np.testing.assert_array_equal(ra[k].detach().numpy(), GOLD[f"args_out_{k}"])
    assert ra["means2D"].requires_grad and not ra["means2D"].is_leaf


def test_quaternion_convention_matches_build_rotation():
    """Sigma3D's rotation (kernel and oracle) is build_rotation(q)^T (external.py:27-46)."""
    q = torch.from_numpy(GOLD["args_in_rotation_quaternions"]).double()
    qn = q / q.norm(dim=-1, keepdim=True)
    R = DT._rot(qn).numpy()
    np.testing.assert_allclose(np.transpose(R, (0, 2, 1)), GOLD["rot_out"], rtol=0, atol=2e-6)


def test_densify_stats_match_reference_single_process():
    """splat_dp.DensifyStats.update == densify.py:154-162 + external.py:113-124 over 6 views."""
    radii, grads = GOLD["dstat_in_radii"], GOLD["dstat_in_grad"]
    st = splat_dp.DensifyStats(radii.shape[1], "cpu")
    for r, g in zip(radii, grads):
        st.update(torch.from_numpy(r), torch.from_numpy(g))
    np.testing.assert_array_equal(st.visibility_count.numpy(), GOLD["dstat_out_visibility_count"])
    np.testing.assert_array_equal(st.max_2d_radii.numpy(), GOLD["dstat_out_max_radii"])
    np.testing.assert_allclose(st.mean_2d_gradients_accumulated.numpy(), GOLD["dstat_out_grad_accum"], rtol=1e-6, atol=0)
