"""Generate golden vectors by running the REFERENCE's own Python callers of the rasterizer.

Run in the build container only (needs /root/reference, which does not exist on the GPU box):
    python tests/golden/gen_golden.py          (both files)   |   python tests/golden/gen_golden.py --io
Writes tests/golden/reference_harness.npz and reference_io.npz (data only: inputs and the
reference's outputs; the I/O fixtures hold the small image / .pth files the reference read).

What is captured:
  * create_render_settings (shared.py:64-124) for the benchmark/test cameras and the inference rig
    of train.py:460-503 (create_extrinsic_matrices / render_and_export_frame intrinsics)
  * create_render_arguments (shared.py:29-42) activations on a seeded parameter dict
  * build_rotation (external.py:27-46) - the quaternion convention of Sigma3D
  * calc_ssim (external.py:68-110) on seeded images, with its autograd gradient, and the
    0.8 * l1 + 0.2 * (1 - ssim) loss of densify.py:149-151 on a ragged binary-target pair (for the
    fused-loss row of SURVEY 8(f))
  * update_max_2d_radii_and_visibility_mask (densify.py:154-162) + accumulate_mean_2d_gradients
    (external.py:113-124) over a sequence of seeded views, and densify_gaussians
    (external.py:211-314) - the statistics the data-parallel grad/stat reduction must reproduce;
  * densify_gaussians (external.py:211-314) at i = 500 / 3000 / 5000 on a seeded parameter dict with
    a populated torch Adam (densify.py:68-86): parameters, Adam exp_avg / exp_avg_sq / step and
    densification statistics before and after, plus the torch.normal split samples it drew.

The reference needs open3d / wandb / imageio / a rasterizer and CUDA; here open3d, wandb and imageio
are empty stub modules, ``diff_gaussian_rasterization`` is this repo's drop-in (only its settings
namedtuple is used), and ``.cuda()`` / ``device="cuda"`` are redirected to the CPU.  Nothing from
the reference is copied: its modules are imported from /root/reference and only their outputs are
saved.  No bytecode is written into /root/reference.
"""
import importlib
import os
import sys
import types

import numpy as np
import torch

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path[:0] = [os.path.join(REPO, "animating-gaussian-splats_amd"), REPO]


def _install_shims():
    for name in ("open3d", "wandb", "imageio"):
        sys.modules.setdefault(name, types.ModuleType(name))
    torch.Tensor.cuda = lambda self, *a, **k: self

    def cpu(fn):
        def wrapped(*a, **k):
            if "device" in k:
                k["device"] = "cpu"
            return fn(*a, **k)
        return wrapped

    for fname in ("tensor", "zeros", "zeros_like", "ones", "ones_like", "empty", "normal", "randn"):
        setattr(torch, fname, cpu(getattr(torch, fname)))


def main():
    _install_shims()
    sys.path.insert(0, REF)
    shared = importlib.import_module("shared")
    external = importlib.import_module("external")
    densify = importlib.import_module("densify")
    train = importlib.import_module("train")
    out = {}

    # ---- cameras -------------------------------------------------------------------------
    cams = []
    for W, H, f, yaw, hgt, dist in [(256, 256, 256.0, 0.0, 0.0, 4.0), (800, 800, 800.0, 90.0, 0.0, 4.0),
                                    (1920, 1080, 1600.0, 0.0, 0.0, 4.0), (1920, 1080, 1600.0, 280.0, 0.8, 4.0),
                                    (200, 120, 150.0, 200.0, -0.8, 4.0)]:
        K = np.array([[f, 0.0, W / 2], [0.0, f, H / 2], [0.0, 0.0, 1.0]])
        cams.append((W, H, K, train.create_transformation_matrix(yaw, hgt, dist)))
    for key, (w2c, aspect) in train.create_extrinsic_matrices().items():
        W, H = 1280, 720
        K = np.array([[aspect * W, 0, W / 2], [0, aspect * W, H / 2], [0, 0, 1]])
        cams.append((W, H, K, w2c))
    for c, (W, H, K, w2c) in enumerate(cams):
        rs = shared.create_render_settings(image_width=W, image_height=H, intrinsic_matrix=K,
                                           extrinsic_matrix=w2c)
        out[f"cam{c}_in_K"] = K
        out[f"cam{c}_in_w2c"] = w2c
        out[f"cam{c}_in_wh"] = np.array([W, H])
        out[f"cam{c}_viewmatrix"] = rs.viewmatrix.contiguous().numpy()
        out[f"cam{c}_projmatrix"] = rs.projmatrix.contiguous().numpy()
        out[f"cam{c}_campos"] = rs.campos.numpy()
        out[f"cam{c}_tanfov"] = np.array([rs.tanfovx, rs.tanfovy], dtype=np.float64)
        out[f"cam{c}_bg"] = rs.bg.numpy()
        out[f"cam{c}_misc"] = np.array([rs.image_height, rs.image_width, rs.sh_degree,
                                        float(rs.scale_modifier), float(rs.prefiltered)])
    out["n_cams"] = np.array(len(cams))

    # ---- render arguments --------------------------------------------------------------------
    g = torch.Generator().manual_seed(0)
    P = 257
    params = {"means": torch.randn(P, 3, generator=g), "colors": torch.rand(P, 3, generator=g),
              "rotation_quaternions": torch.randn(P, 4, generator=g),
              "opacity_logits": torch.randn(P, 1, generator=g),
              "log_scales": torch.randn(P, 3, generator=g) - 4.0}
    for k, v in params.items():
        out[f"args_in_{k}"] = v.numpy()
    ra = shared.create_render_arguments(params)
    for k, v in ra.items():
        out[f"args_out_{k}"] = v.detach().numpy()
    out["rot_out"] = external.build_rotation(params["rotation_quaternions"]).numpy()

    # ---- SSIM ------------------------------------------------------------------------------
    img1 = torch.rand(3, 48, 64, generator=g)
    img2 = (img1 + 0.1 * torch.randn(3, 48, 64, generator=g)).clamp(0, 1)
    out["ssim_in_img1"], out["ssim_in_img2"] = img1.numpy(), img2.numpy()
    out["ssim_out"] = np.array(float(external.calc_ssim(img1, img2)))
    x = img1.clone().requires_grad_(True)
    external.calc_ssim(x, img2).backward()
    out["ssim_out_grad"] = x.grad.numpy()
    # the loss of densify.py:149-151 on a ragged segmentation-style pair (binary target), with the
    # reference's autograd through calc_ssim and torch's l1_loss
    seg = (torch.rand(3, 37, 53, generator=g) > 0.5).float()
    rend = torch.sigmoid(3.0 * torch.randn(3, 37, 53, generator=g))
    x = rend.clone().requires_grad_(True)
    l1 = torch.nn.functional.l1_loss(x, seg)
    ss = external.calc_ssim(x, seg)
    loss = 0.8 * l1 + 0.2 * (1.0 - ss)
    loss.backward()
    out["loss_in_img1"], out["loss_in_img2"] = rend.numpy(), seg.numpy()
    out["loss_out_l1"], out["loss_out_ssim"] = np.array(l1.item()), np.array(ss.item())
    out["loss_out_grad"] = x.grad.numpy()

    # ---- densification statistics over a sequence of views ----------------------------------
    P = 2000
    gp = torch.Generator().manual_seed(5)
    n_views = 6
    radii_seq = [(torch.randint(0, 6, (P,), generator=gp) * (torch.rand(P, generator=gp) > 0.3)).int()
                 for _ in range(n_views)]
    grad_seq = [torch.randn(P, 3, generator=gp) * 4e-4 for _ in range(n_views)]
    dv = shared.DensificationVariables(visibility_count=torch.zeros(P), mean_2d_gradients_accumulated=torch.zeros(P),
                                       max_2d_radii=torch.zeros(P))
    for r, gr in zip(radii_seq, grad_seq):
        densify.update_max_2d_radii_and_visibility_mask(r, dv)
        m2 = torch.zeros(P, 3, requires_grad=True)
        m2.grad = gr
        dv.means_2d = m2
        external.accumulate_mean_2d_gradients(dv)
    out["dstat_in_radii"] = torch.stack(radii_seq).numpy()
    out["dstat_in_grad"] = torch.stack(grad_seq).numpy()
    out["dstat_out_visibility_count"] = dv.visibility_count.numpy()
    out["dstat_out_grad_accum"] = dv.mean_2d_gradients_accumulated.numpy()
    out["dstat_out_max_radii"] = dv.max_2d_radii.numpy()

    # ---- densify_gaussians (external.py:211-314) with Adam state surgery ------------------------
    # i = 500: clone / split / prune (opacity < 0.005); i = 3000: + big-point prune and the opacity
    # reset of external.py:306-314; i = 5000: prune threshold 0.25.  torch.normal is recorded so the
    # build can be fed the same split samples.
    real_normal = torch.normal
    for case, (i_it, seed) in enumerate([(500, 11), (3000, 12), (5000, 13)]):
        gd = torch.Generator().manual_seed(seed)
        P, sr = 400, 2.0  # clone/split threshold 0.01 * sr = 0.02, big points > 0.1 * sr = 0.2
        raw = {"means": torch.randn(P, 3, generator=gd), "colors": torch.rand(P, 3, generator=gd),
               "segmentation_masks": torch.rand(P, 3, generator=gd),
               "rotation_quaternions": torch.randn(P, 4, generator=gd),
               "opacity_logits": 3.0 * torch.randn(P, 1, generator=gd),
               "log_scales": float(np.log(0.02)) + 0.9 * torch.randn(P, 3, generator=gd),
               "camera_matrices": torch.zeros(50, 3), "camera_center": torch.zeros(50, 3)}
        for k, v in raw.items():
            out[f"dens{case}_in_{k}"] = v.numpy()
        params = {k: torch.nn.Parameter(v.clone().requires_grad_(True)) for k, v in raw.items()}
        opt = densify.create_optimizer(params, sr)
        for _ in range(2):  # populate exp_avg / exp_avg_sq / step
            for k, p_ in params.items():
                p_.grad = 0.01 * torch.randn(p_.shape, generator=gd)
            opt.step()
        for k, p_ in params.items():
            st = opt.state[p_]
            out[f"dens{case}_pre_{k}"] = p_.detach().numpy().copy()
            out[f"dens{case}_pre_m_{k}"] = st["exp_avg"].numpy().copy()
            out[f"dens{case}_pre_v_{k}"] = st["exp_avg_sq"].numpy().copy()
        cnt = torch.randint(0, 5, (P,), generator=gd).float()
        acc = cnt * 0.0004 * torch.rand(P, generator=gd)
        dv = shared.DensificationVariables(visibility_count=cnt.clone(), mean_2d_gradients_accumulated=acc.clone(),
                                           max_2d_radii=torch.randint(0, 9, (P,), generator=gd).float())
        vis = torch.rand(P, generator=gd) > 0.3
        m2 = torch.zeros(P, 3, requires_grad=True)
        m2.grad = 3e-4 * torch.randn(P, 3, generator=gd)
        dv.gaussian_is_visible_mask, dv.means_2d = vis, m2
        out[f"dens{case}_in_count"], out[f"dens{case}_in_acc"] = cnt.numpy(), acc.numpy()
        out[f"dens{case}_in_max_radii"] = dv.max_2d_radii.numpy().copy()
        out[f"dens{case}_in_vis"], out[f"dens{case}_in_m2grad"] = vis.numpy(), m2.grad.numpy()
        samples = []

        def recording_normal(*a, **k):
            r = real_normal(*a, **k)
            samples.append(r.detach().clone())
            return r
        torch.normal = recording_normal
        torch.manual_seed(100 + case)
        external.densify_gaussians(params, dv, sr, opt, i_it)
        torch.normal = real_normal
        out[f"dens{case}_iter"] = np.array(i_it)
        out[f"dens{case}_scene_radius"] = np.array(sr)
        out[f"dens{case}_samples"] = (samples[0].numpy() if samples else np.zeros((0, 3), np.float32))
        for k, p_ in params.items():
            st = opt.state[p_]
            out[f"dens{case}_out_{k}"] = p_.detach().numpy()
            out[f"dens{case}_out_m_{k}"] = st["exp_avg"].numpy()
            out[f"dens{case}_out_v_{k}"] = st["exp_avg_sq"].numpy()
            out[f"dens{case}_out_step_{k}"] = np.array(float(st["step"]))
        out[f"dens{case}_out_count"] = dv.visibility_count.numpy()
        out[f"dens{case}_out_acc"] = dv.mean_2d_gradients_accumulated.numpy()
        out[f"dens{case}_out_max_radii"] = dv.max_2d_radii.numpy()

    np.savez_compressed(os.path.join(HERE, "reference_harness.npz"), **out)
    print(f"wrote {len(out)} arrays to tests/golden/reference_harness.npz")


def _write_sequence(root, W, H, T, C, seed):
    """A tiny camera sequence in the reference's dataset layout (train_meta.json + ims/*.jpg +
    seg/*.png), written with PIL from seeded arrays; returns the metadata dict."""
    import json
    from PIL import Image
    rng = np.random.default_rng(seed)
    os.makedirs(os.path.join(root, "ims"), exist_ok=True)
    os.makedirs(os.path.join(root, "seg"), exist_ok=True)
    md = {"w": W, "h": H, "fn": [], "k": [], "w2c": []}
    yy, xx = np.mgrid[0:H, 0:W]
    for t in range(T):
        md["fn"].append([]); md["k"].append([]); md["w2c"].append([])
        for c in range(C):
            fn = f"{c}/{t:06d}.jpg"
            os.makedirs(os.path.join(root, "ims", str(c)), exist_ok=True)
            os.makedirs(os.path.join(root, "seg", str(c)), exist_ok=True)
            base = np.stack([xx * 255 // max(W - 1, 1), yy * 255 // max(H - 1, 1), (xx + yy + 40 * c) % 256], -1)
            img = np.clip(base + rng.integers(-30, 31, size=(H, W, 3)), 0, 255).astype(np.uint8)
            Image.fromarray(img).save(os.path.join(root, "ims", fn), quality=85)
            inside = ((xx - W / 2 - 3 * t) ** 2 + (yy - H / 2 + c) ** 2) < (min(W, H) / 3) ** 2
            seg_png = os.path.join(root, "seg", fn.replace(".jpg", ".png"))
            if c % 2 == 0:
                Image.fromarray(inside.astype(np.uint8), mode="L").save(seg_png)
            else:  # 1-bit PNG: numpy reads it as bool
                Image.fromarray(inside).convert("1").save(seg_png)
            f = 0.8 * W + 10 * c
            md["fn"][t].append(fn)
            md["k"][t].append([[f, 0.0, W / 2 + c], [0.0, f, H / 2 - t], [0.0, 0.0, 1.0]])
            md["w2c"][t].append(train.create_transformation_matrix(30.0 * c + 5 * t, 0.1 * t, 4.0).tolist())
    with open(os.path.join(root, "train_meta.json"), "w") as fh:
        json.dump(md, fh)
    return md


def main_io():
    """Fixtures of the data / format row: the reference's load_timestep_views
    (shared.py:127-171) on two tiny sequences written here (one with a pixel count that is not a
    multiple of 4), and a parameter dict written by its export_parameters (densify.py:190-198) and
    read back by load_densified_initial_parameters (train.py:155-163).  The image / mask files and
    the .pth are stored as bytes (data), with the reference's outputs.  Writes reference_io.npz."""
    global train
    import json
    import tempfile
    from pathlib import Path
    _install_shims()
    sys.modules["wandb"].save = lambda *a, **k: None
    sys.path.insert(0, REF)
    shared = importlib.import_module("shared")
    densify = importlib.import_module("densify")
    train = importlib.import_module("train")
    out = {}
    with tempfile.TemporaryDirectory() as tmp:
        for name, (W, H, T, C, seed) in {"a": (40, 24, 2, 3, 1), "b": (37, 23, 1, 2, 2)}.items():
            root = os.path.join(tmp, name)
            md = _write_sequence(root, W, H, T, C, seed)
            out[f"io_{name}_meta"] = np.frombuffer(json.dumps(md).encode(), dtype=np.uint8)
            for t in range(T):
                for c, fn in enumerate(md["fn"][t]):
                    for sub, f in (("ims", fn), ("seg", fn.replace(".jpg", ".png"))):
                        with open(os.path.join(root, sub, f), "rb") as fh:
                            out[f"io_{name}_file_{sub}_{t}_{c}"] = np.frombuffer(fh.read(), dtype=np.uint8)
                views = shared.load_timestep_views(dataset_metadata=md, timestep=t, sequence_path=Path(root))
                for v in views:
                    c = v.camera_index
                    out[f"io_{name}_t{t}_c{c}_image"] = v.image.contiguous().numpy()
                    out[f"io_{name}_t{t}_c{c}_mask"] = v.segmentation_mask.contiguous().numpy()
                    out[f"io_{name}_t{t}_c{c}_image_strides"] = np.array(v.image.stride())
                    rs = v.render_settings
                    out[f"io_{name}_t{t}_c{c}_viewmatrix"] = rs.viewmatrix.numpy()
                    out[f"io_{name}_t{t}_c{c}_projmatrix"] = rs.projmatrix.numpy()
                    out[f"io_{name}_t{t}_c{c}_campos"] = rs.campos.numpy()
                    out[f"io_{name}_t{t}_c{c}_tanfov"] = np.array([rs.tanfovx, rs.tanfovy])
        # .pth parameter dict: reference export -> bytes; reference load -> values
        gd = torch.Generator().manual_seed(7)
        params = {k: torch.nn.Parameter(torch.randn(*shp, generator=gd))
                  for k, shp in (("means", (50, 3)), ("colors", (50, 3)), ("segmentation_masks", (50, 3)),
                                 ("rotation_quaternions", (50, 4)), ("opacity_logits", (50, 1)),
                                 ("log_scales", (50, 3)), ("camera_matrices", (4, 3)), ("camera_center", (4, 3)))}
        seq = Path(tmp) / "seq"
        seq.mkdir()
        densify.export_parameters(sequence_path=seq, parameters=params)
        with open(seq / "densified_initial_gaussian_cloud_parameters.pth", "rb") as fh:
            out["io_pth_bytes"] = np.frombuffer(fh.read(), dtype=np.uint8)
        loaded = train.load_densified_initial_parameters(Path(tmp), "seq")
        out["io_pth_keys"] = np.frombuffer(json.dumps(list(loaded.keys())).encode(), dtype=np.uint8)
        for k, v in loaded.items():
            out[f"io_pth_val_{k}"] = v.detach().numpy()
            out[f"io_pth_rg_{k}"] = np.array(bool(v.requires_grad))
    np.savez_compressed(os.path.join(HERE, "reference_io.npz"), **out)
    print(f"wrote {len(out)} arrays to tests/golden/reference_io.npz")


if __name__ == "__main__":
    if "--io" in sys.argv[1:]:
        main_io()
    else:
        main()
        main_io()
