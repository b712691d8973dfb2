"""Data / format path: frames -> views (splat_io + gsr_views_pack) and the
``.pth`` parameter dict.

Pinned by tests/golden/reference_io.npz: two small sequences (image / mask files stored as bytes)
with the views the reference's own load_timestep_views built from them, and a parameter file its
export_parameters wrote with the values its load_densified_initial_parameters read back.  The golden
views were made on the CPU, where torch divides by 255 exactly; on the GPU (where the reference
runs) torch multiplies by the float reciprocal -- the GPU tests compare bitwise with torch's own
GPU evaluation of the reference expression and allow exactly that 1-ulp difference from the CPU
golden.
"""
import json
import os

import numpy as np
import pytest
import torch

import splat_io
from oracle import io_oracle

GOLD = np.load(os.path.join(os.path.dirname(__file__), "golden", "reference_io.npz"))
SEQS = {"a": (40, 24, 2, 3), "b": (37, 23, 1, 2)}  # W, H, timesteps, cameras


def _sequence(tmp_path, name):
    """Write the fixture's files back into the reference's dataset layout; returns (root, meta)."""
    md = json.loads(GOLD[f"io_{name}_meta"].tobytes())
    root = tmp_path / name
    for t, fns in enumerate(md["fn"]):
        for c, fn in enumerate(fns):
            for sub, f in (("ims", fn), ("seg", fn.replace(".jpg", ".png"))):
                path = root / sub / f
                path.parent.mkdir(parents=True, exist_ok=True)
                path.write_bytes(GOLD[f"io_{name}_file_{sub}_{t}_{c}"].tobytes())
    return root, md


def _ulp_close(a, b):
    """Equal, or one float32 ulp apart (the GPU's reciprocal multiply vs the CPU's division)."""
    ai, bi = a.view(np.int32).astype(np.int64), b.view(np.int32).astype(np.int64)
    return np.abs(ai - bi).max() <= 1


# ---------------------------------------------------------------- CPU: oracle and host logic
@pytest.mark.parametrize("name", list(SEQS))
def test_oracle_reproduces_reference_views(tmp_path, name):
    root, md = _sequence(tmp_path, name)
    for t in range(SEQS[name][2]):
        for c, fn in enumerate(md["fn"][t]):
            img = splat_io.decode_frame(root / "ims" / fn)
            msk = splat_io.decode_frame(root / "seg" / fn.replace(".jpg", ".png"))
            gi, gm = GOLD[f"io_{name}_t{t}_c{c}_image"], GOLD[f"io_{name}_t{t}_c{c}_mask"]
            assert np.array_equal(io_oracle.view_image_cpu(img), gi)
            assert np.array_equal(io_oracle.view_mask(msk), gm)
            assert _ulp_close(io_oracle.view_image(img), gi)
            # odd cameras hold 1-bit PNGs (numpy reads bool): the mask is still 0 / 1
            assert set(np.unique(gm[0])) <= {0.0, 1.0}


def test_reciprocal_and_division_differ_where_documented():
    a = np.arange(256, dtype=np.uint8).reshape(16, 16, 1).repeat(3, axis=2)
    gpu, cpu = io_oracle.view_image(a), io_oracle.view_image_cpu(a)
    assert int((gpu != cpu).sum() // 3) == 126 and _ulp_close(gpu, cpu)


@pytest.mark.parametrize("name", list(SEQS))
def test_decoder_stages_every_frame(tmp_path, name):
    root, md = _sequence(tmp_path, name)
    with splat_io.TimestepDecoder(workers=3) as dec:
        for t in range(SEQS[name][2]):
            rgb, seg = dec.submit(md, t, root).result()
            W, H, _, C = SEQS[name]
            assert rgb.shape == (C, H, W, 3) and seg.shape == (C, H, W)
            for c, fn in enumerate(md["fn"][t]):
                assert np.array_equal(rgb[c].numpy(), splat_io.decode_frame(root / "ims" / fn))
                assert np.array_equal(seg[c].numpy(), splat_io.decode_frame(root / "seg" / fn.replace(".jpg", ".png")))


def test_decoder_reports_bad_frames(tmp_path):
    root, md = _sequence(tmp_path, "a")
    bad = dict(md, w=md["w"] + 1)
    with splat_io.TimestepDecoder(workers=2) as dec:
        with pytest.raises(ValueError, match="metadata says"):
            dec.submit(bad, 0, root).result()
        missing = dict(md, fn=[["nope/000000.jpg"]])
        with pytest.raises(FileNotFoundError):
            dec.submit(missing, 0, root).result()
        rgb, seg = dec.submit(dict(md, fn=[[]]), 0, root).result()  # a timestep without cameras
        assert rgb.shape[0] == 0 and seg.shape[0] == 0


def test_render_settings_follow_reference(tmp_path):
    _, md = _sequence(tmp_path, "a")
    for t in range(2):
        for c in range(3):
            rs = splat_io.create_render_settings(image_width=md["w"], image_height=md["h"],
                                                 intrinsic_matrix=md["k"][t][c],
                                                 extrinsic_matrix=md["w2c"][t][c], device="cpu")
            key = f"io_a_t{t}_c{c}"
            assert np.array_equal(rs.viewmatrix.numpy(), GOLD[key + "_viewmatrix"])
            assert np.array_equal(rs.projmatrix.numpy(), GOLD[key + "_projmatrix"])
            assert np.array_equal(rs.campos.numpy(), GOLD[key + "_campos"])
            assert [rs.tanfovx, rs.tanfovy] == GOLD[key + "_tanfov"].tolist()


def _reference_pth(tmp_path):
    seq = tmp_path / "data" / "seq"
    seq.mkdir(parents=True)
    (seq / splat_io.PARAMETERS_FILE_NAME).write_bytes(GOLD["io_pth_bytes"].tobytes())
    return tmp_path / "data"


def test_loads_parameter_file_written_by_reference(tmp_path):
    params = splat_io.load_densified_initial_parameters(_reference_pth(tmp_path), "seq", device="cpu")
    assert list(params) == json.loads(GOLD["io_pth_keys"].tobytes())
    for k, v in params.items():
        assert isinstance(v, torch.nn.Parameter) and not v.requires_grad
        assert bool(GOLD[f"io_pth_rg_{k}"]) is False
        assert np.array_equal(v.detach().numpy(), GOLD[f"io_pth_val_{k}"])


def test_export_then_load_round_trip(tmp_path):
    params = splat_io.load_densified_initial_parameters(_reference_pth(tmp_path), "seq", device="cpu")
    out = tmp_path / "out" / "seq"
    out.mkdir(parents=True)
    path = splat_io.export_parameters(out, {k: torch.nn.Parameter(v.detach().clone()) for k, v in params.items()})
    assert path.name == "densified_initial_gaussian_cloud_parameters.pth"
    again = splat_io.load_densified_initial_parameters(tmp_path / "out", "seq", device="cpu")
    assert list(again) == list(params)
    for k in params:
        assert torch.equal(again[k], params[k])
    # and the reference's loader (plain torch.load of the same path) reads what we wrote
    plain = torch.load(path, weights_only=True)
    assert all(torch.equal(plain[k], params[k]) for k in params)


def test_pack_views_has_no_cpu_path():
    with pytest.raises(RuntimeError, match="no CPU path"):
        splat_io.pack_views(torch.zeros((1, 4, 4, 3), dtype=torch.uint8))


# ---------------------------------------------------------------- GPU: the HIP path
def _torch_reference_views(rgb, seg, device):
    """The reference's expressions (shared.py:131-168) evaluated by torch on the GPU."""
    imgs, msks = [], []
    for c in range(rgb.shape[0]):
        imgs.append(torch.tensor(rgb[c]).float().to(device).permute(2, 0, 1) / 255)
        m = torch.tensor(seg[c].astype(np.float32)).float().to(device)
        msks.append(torch.stack((m, torch.zeros_like(m), 1 - m)))
    return imgs, msks


@pytest.mark.gpu
@pytest.mark.parametrize("F,H,W", [(5, 360, 640), (3, 23, 37), (2, 1, 1), (1, 1080, 1920), (4, 7, 4)])
def test_pack_views_bitwise(cuda, F, H, W):
    rng = np.random.default_rng(F * 1000 + H)
    rgb = rng.integers(0, 256, size=(F, H, W, 3), dtype=np.uint8)
    rgb[0].reshape(-1)[:256] = np.arange(256, dtype=np.uint8)[: rgb[0].size]  # every byte value
    seg = rng.integers(0, 2, size=(F, H, W), dtype=np.uint8)
    seg[-1] = rng.integers(0, 256, size=(H, W), dtype=np.uint8)  # any 8-bit mask value
    images, masks = splat_io.pack_views(torch.from_numpy(rgb).to(cuda), torch.from_numpy(seg).to(cuda))
    ref_i, ref_m = _torch_reference_views(rgb, seg, cuda)
    for c in range(F):
        assert torch.equal(images[c], ref_i[c]), c
        assert torch.equal(masks[c], ref_m[c]), c
        assert np.array_equal(images[c].cpu().numpy(), io_oracle.view_image(rgb[c]))
    im2, none = splat_io.pack_views(torch.from_numpy(rgb).to(cuda))  # images only
    assert none is None and torch.equal(im2, images)


@pytest.mark.gpu
def test_pack_views_edge_cases(cuda):
    e, m = splat_io.pack_views(torch.zeros((0, 8, 8, 3), dtype=torch.uint8, device=cuda),
                               torch.zeros((0, 8, 8), dtype=torch.uint8, device=cuda))
    assert e.shape == (0, 3, 8, 8) and m.shape == (0, 3, 8, 8)
    with pytest.raises(ValueError):
        splat_io.pack_views(torch.zeros((1, 8, 8, 3), dtype=torch.uint8, device=cuda),
                            torch.zeros((1, 8, 9), dtype=torch.uint8, device=cuda))
    with pytest.raises(ValueError):
        splat_io.pack_views(torch.zeros((1, 8, 8, 4), dtype=torch.uint8, device=cuda))


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(SEQS))
def test_load_timestep_views_matches_reference(cuda, tmp_path, name):
    root, md = _sequence(tmp_path, name)
    for t in range(SEQS[name][2]):
        views = splat_io.load_timestep_views(md, t, root, device=cuda)
        assert [v.camera_index for v in views] == list(range(SEQS[name][3]))
        for v in views:
            key = f"io_{name}_t{t}_c{v.camera_index}"
            fn = md["fn"][t][v.camera_index]
            img = splat_io.decode_frame(root / "ims" / fn)
            got = v.image.cpu().numpy()
            assert got.shape == GOLD[key + "_image"].shape
            assert np.array_equal(got, io_oracle.view_image(img))  # the reference's GPU arithmetic
            assert _ulp_close(got, GOLD[key + "_image"])           # the reference run on the CPU
            assert np.array_equal(v.segmentation_mask.cpu().numpy(), GOLD[key + "_mask"])
            rs = v.render_settings
            assert np.array_equal(rs.viewmatrix.cpu().numpy(), GOLD[key + "_viewmatrix"])
            assert np.array_equal(rs.projmatrix.cpu().numpy(), GOLD[key + "_projmatrix"])
            assert rs.viewmatrix.device.type == "cuda"


@pytest.mark.gpu
def test_load_all_views_is_timesteps_one_to_count(cuda, tmp_path):
    root, md = _sequence(tmp_path, "a")
    allv = splat_io.load_all_views(md, 1, root, device=cuda, prefetch=1)  # train.py:207-217: 1 .. count
    one = splat_io.load_timestep_views(md, 1, root, device=cuda)
    assert len(allv) == 1 and len(allv[0]) == len(one)
    for a, b in zip(allv[0], one):
        assert torch.equal(a.image, b.image) and torch.equal(a.segmentation_mask, b.segmentation_mask)


@pytest.mark.gpu
def test_parameters_load_to_gpu(cuda, tmp_path):
    params = splat_io.load_densified_initial_parameters(_reference_pth(tmp_path), "seq", device=cuda)
    for k, v in params.items():
        assert v.is_cuda and not v.requires_grad
        assert np.array_equal(v.detach().cpu().numpy(), GOLD[f"io_pth_val_{k}"])
