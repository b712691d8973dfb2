"""Benchmark: differentiable Gaussian-splat rasterizer forward + backward (BASELINE.json metric).

Metric: Msplats/s = P x views / wall-time(forward + backward) / 1e6, P counted pre-cull
(SURVEY.md 8(d)).  Workload (BASELINE.json configs[2], the 1-GPU config the metric is quoted on):
1M synthetic Gaussians, SH degree 3, 1920x1080, f = 1600, views from the 27-camera rig of
configs[3] (heights {-0.8, 0, 0.8} x yaws {0, 40, ..., 320}).  One step = every rank renders
``--views-per-rank`` views (default 5: train.py:757 optimises on the summed losses of 5 views per
step) through the drop-in ``GaussianRasterizer`` on the render arguments of
shared.py:29-42 (activated once, before timing, and held as leaf tensors: SURVEY.md 8(d) times the
rasterizer's forward + backward), backpropagates a fixed upstream dL/dcolor into them (gradients
accumulate over the rank's views, as train.py sums view losses), and for N > 1 all-reduces (SUM)
the gradients over RCCL.  Inputs are resident in HBM before timing.

Also reported (untimed for `value`, ``call_site``): ms per view of train.py's whole render call
site, (a) the reference's way -- torch activations + their autograd + the drop-in -- and (b) the
fused ``rasterize_parameters`` path (activations inside the kernels).

N > 1: launched by torch.distributed.run, one process per GPU; the step's N * V rig cameras
(step * N * V + k) mod 27 are sharded round-robin over ranks (splat_dp.shard_views; camera data
parallelism, weak scaling: fixed views per GPU), then splat_dp.GradAllReduce sums the gradients.

Prints ONE JSON line (rank 0) with the roofline of the dominant kernel (HIP events inside libgsr on
the stream the kernel runs on) and the CPU-oracle baseline (rank 0, N = 1 only).
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(REPO, "animating-gaussian-splats_amd"), REPO]

import numpy as np  # noqa: E402
import torch  # noqa: E402

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md chip table)
# rocprofv3 FETCH_SIZE / WRITE_SIZE summary of this same command (tools/profile_round.sh): HBM bytes per
# launch of each kernel, converted per access shape (calibrated_traffic; MI355X_MICROARCH.md's 2 x
# FETCH_SIZE + WRITE_SIZE is the streaming case and is reported beside it)
PMC_SUMMARY = os.path.join(REPO, "profiles", "r06_hbm_pmc.json")
# SQ counters of the same command (tools/profile_round.sh sq passes): VALU activity per launch
SQ_SUMMARY = os.path.join(REPO, "profiles", "r06_sq_pmc.json")
VALU_PEAK_GINST = 1024 * 2.4 / 2  # wave64 f32 VALU instructions per ns: 1024 SIMDs x 2.4 GHz / 2 cycles
PHASES = ["preprocess", "bin_count", "bin_scan", "bin_emit", "tile_sort", "render_fwd", "bwd_items",
          "render_bwd", "sum_records", "gauss_bwd"]


def streamed_read_bytes(phase, P, K, N, T):
    """Lane-contiguous (streaming) reads of one launch; the rest of a render kernel's reads are 64-B
    record gathers.  profiles/r01_fetch_calib.txt: FETCH_SIZE bills streamed reads at half their bytes
    and a record gather at one whole 64-B unit, so HBM reads = FETCH_SIZE + streamed / 2."""
    if phase == "render_bwd":      # point list + slot map per pair; T, n_contrib, dL/dpix per pixel
        return K * 8 + N * 20 + T * 28
    if phase == "render_fwd":      # 16-B binning record per pair; order + range per tile
        return K * 16 + T * 12
    return None                    # streaming kernels: the guide's x2 applies to the whole FETCH_SIZE


def calibrated_traffic(pm, phase, P, K, N, T):
    """HBM bytes of one launch from the kernel's FETCH_SIZE / WRITE_SIZE (KiB averages)."""
    f = pm["FETCH_SIZE_KiB_avg"] * 1024
    w = pm["WRITE_SIZE_KiB_avg"] * 1024
    s = streamed_read_bytes(phase, P, K, N, T)
    return int((f + s / 2 if s is not None and s / 2 <= f else 2 * f) + w)


def algorithmic_bytes(phase, P, K, N, T, F, sh):
    """Compulsory HBM bytes of one launch of each kernel: its share of SURVEY.md 8(d)'s per-view byte
    model (one sort pass, no atomics, no scratch records -- the backward's per-pair partial records
    replace the reference's atomics and are this design's own traffic, not algorithmic)."""
    if phase == "preprocess":      # read means/scales/rot/opacity/features, write the geometry records
        return P * (44 + F) + P * (36 + 12 * sh)
    if phase == "render_fwd":      # per pair: id + xy + conic/op + rgb/depth gather; per pixel outputs
        return K * 44 + N * 24 + T * 16
    if phase == "render_bwd":      # per pair: 40 B gather; per pixel: dL/dpix + final T + n_contrib
        return K * 40 + N * 20 + T * 16
    if phase == "gauss_bwd":       # per Gaussian: inputs read + every gradient written
        return P * (84 + F) + P * (56 + F)
    if phase == "tile_sort":       # one sort pass over the pairs
        return K * 24
    if phase == "bin_emit":        # duplicate with keys: 12 B per emitted pair
        return K * 12
    return 0


def pipeline_bytes(P, K, N, T, F, sh):
    """B = P (220 + 3F + 12 [SH]) + 120 K + 44 N + 16 T per fwd + bwd of one view."""
    return P * (220 + 3 * F + 12 * sh) + 120 * K + 44 * N + 16 * T


FWD_KERNELS = ("k_preprocess", "k_bin_count", "k_bin_colscan", "k_bin_scan", "k_bin_emit", "k_tile_sort",
               "k_chunk_sort", "k_merge_pass", "k_render_fwd")


def step_valu(sq, views_per_gpu, median_ms, fwd_solo_ms):
    """(valu_step, valu_render_fwd) from a tools/rocprof_summary.py `sq` summary of this command: each
    kernel's SQ_INSTS_VALU per launch times its launches per view -- dispatches profiled over k_render_fwd's
    for the forward kernels and over k_render_bwd's for the backward ones (the profiled bench also runs
    forward-only probes), so k_gauss_bwd_multi counts 1/V; without dispatch counts one per view and
    k_gauss_bwd_multi one per step -- summed over the step's views, over the median step at the VALU
    issue peak."""
    fwd, bwd = sq.get("k_render_fwd"), sq.get("k_render_bwd")
    if not fwd or not bwd or "SQ_INSTS_VALU" not in fwd:
        return None, None
    per_view, kernels = 0.0, {}
    for k, v in sq.items():
        if "SQ_INSTS_VALU" not in v:
            continue
        ref = fwd if k in FWD_KERNELS else bwd
        if v.get("launches") and ref.get("launches"):
            lpv = v["launches"] / ref["launches"]
        else:
            lpv = 1.0 / views_per_gpu if k == "k_gauss_bwd_multi" else 1.0
        per_view += v["SQ_INSTS_VALU"] * lpv
        kernels[k] = round(v["SQ_INSTS_VALU"] * lpv / 1e6, 2)
    insts = per_view * views_per_gpu
    step = {"insts_per_step": int(insts), "peak_Ginst_s": VALU_PEAK_GINST,
            "issue_frac": round(insts / (VALU_PEAK_GINST * 1e9 * median_ms * 1e-3), 4),
            "M_insts_per_view_by_kernel": kernels, "source": os.path.relpath(SQ_SUMMARY, REPO)}
    f = None
    if fwd_solo_ms:
        f = {"insts_per_launch": int(fwd["SQ_INSTS_VALU"]), "solo_ms": round(fwd_solo_ms, 5),
             "issue_frac": round(fwd["SQ_INSTS_VALU"] / (VALU_PEAK_GINST * 1e9 * fwd_solo_ms * 1e-3), 4),
             "salu_per_valu": round(fwd.get("SQ_INSTS_SALU", 0) / fwd["SQ_INSTS_VALU"], 3)}
    return step, f


def cpu_baseline_oracle(cfg, params_cpu, cam_cpu, dl_cpu, threads=0):
    """The C oracle (OpenMP over tiles / Gaussians), forward + backward of ONE view of the same
    workload on this host's cores: ``threads`` OpenMP threads, 0 = every CPU this process may run on
    (os.sched_getaffinity, what `nproc` reports)."""
    from oracle import oracle as O
    import splat_scenes as S
    avail = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    share = _cpu_quota() or avail
    threads = O.set_threads(threads if threads > 0 else min(avail, share))
    a = {k: (v.detach().numpy() if isinstance(v, torch.Tensor) else v)
         for k, v in S.activated_inputs(params_cpu, cfg.sh_degree).items()}
    t0 = time.perf_counter()
    st = O.forward(cam_cpu.bg.numpy(), a["means3D"], a.get("colors_precomp"), a["opacities"],
                   a["scales"], a["rotations"], 1.0, None, cam_cpu.viewmatrix, cam_cpu.projmatrix,
                   cam_cpu.tanfovx, cam_cpu.tanfovy, cam_cpu.image_height, cam_cpu.image_width,
                   a.get("shs"), cam_cpu.sh_degree, cam_cpu.campos.numpy())
    O.backward(st, dl_cpu.numpy())
    dt = time.perf_counter() - t0
    return {"value": round(cfg.P / dt / 1e6, 6), "unit": "Msplats/s", "cores": threads, "kind": "port",
            "host_nproc": os.cpu_count(), "available_cpus": avail, "cpu_quota": share,
            "sample": f"1 view of the same workload ({cfg.P} Gaussians, {cam_cpu.image_width}x"
                      f"{cam_cpu.image_height}, SH{cfg.sh_degree}) fwd+bwd by the C oracle "
                      f"(oracle/gsr_oracle.c, OpenMP, {threads} threads = the process's CPU share: "
                      f"{avail} CPUs in its affinity mask, a cgroup quota of {share} CPUs, "
                      f"{os.cpu_count()} on the host), {dt:.2f} s"}


def _cpu_quota():
    """CPUs this process's cgroup may use (cpu.max quota / period, rounded up), or None when
    unlimited: the GPU box shows every host CPU in the affinity mask but grants a share of them, and
    an OpenMP team of the whole host's size on that share runs slower than one of the share's size
    (measured: 256 threads 2.80 s vs 16 threads 0.80 s for the same view)."""
    import math
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            q, p = open(path).read().split()[:2]
            if q != "max":
                return max(1, math.ceil(int(q) / int(p)))
        except (OSError, ValueError):
            pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        p = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        if q > 0:
            return max(1, math.ceil(q / p))
    except (OSError, ValueError):
        pass
    return None


def _torch_calc_ssim(img1, img2):
    """external.py:48-110 composed from torch ops (the reference's way: 5 grouped conv2d + elementwise),
    for the loss leg's comparison only."""
    from math import exp
    g = torch.tensor([exp(-((x - 5) ** 2) / float(2 * 1.5 ** 2)) for x in range(11)])
    g = (g / g.sum()).unsqueeze(1)
    C = img1.size(-3)
    w = g.mm(g.t()).float()[None, None].expand(C, 1, 11, 11).contiguous().to(img1.device)
    conv = lambda t: torch.nn.functional.conv2d(t, w, padding=5, groups=C)  # noqa: E731
    mu1, mu2 = conv(img1), conv(img2)
    mu1_sq, mu2_sq, mu1_mu2 = mu1.pow(2), mu2.pow(2), mu1 * mu2
    s1, s2, s12 = conv(img1 * img1) - mu1_sq, conv(img2 * img2) - mu2_sq, conv(img1 * img2) - mu1_mu2
    c1, c2 = 0.01 ** 2, 0.03 ** 2
    return (((2 * mu1_mu2 + c1) * (2 * s12 + c2)) / ((mu1_sq + mu2_sq + c1) * (s1 + s2 + c2))).mean()


def loss_call_site(steps, cam, leaves, dev):
    """ms per render-loss fwd+bwd at the bench resolution (train.py:362-363): fused L1+SSIM kernels
    (splat_loss) vs the reference's torch composition; plus the fused kernels' device times."""
    import splat_loss
    from diff_gaussian_rasterization import GaussianRasterizer, _C
    with torch.no_grad():
        img = GaussianRasterizer(raster_settings=cam)(**leaves)[0].detach()
    gen = torch.Generator(device="cpu").manual_seed(3)
    target = torch.rand(img.shape, generator=gen).to(dev)

    def run(fn):
        for _ in range(3):
            x = img.clone().requires_grad_(True)
            fn(x).backward()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(steps):
            x = img.clone().requires_grad_(True)
            fn(x).backward()
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / steps * 1e3

    fused = run(lambda x: splat_loss.image_loss(x, target))
    ref = run(lambda x: 0.8 * torch.nn.functional.l1_loss(x, target) + 0.2 * (1.0 - _torch_calc_ssim(x, target)))
    _C.profile_reset()
    _C.profile_select(["ssim_fwd", "ssim_bwd"])
    _C.profile_enable(True)
    run(lambda x: splat_loss.image_loss(x, target))
    _C.profile_enable(False)
    k = {ph: _C.profile_read(ph) for ph in ("ssim_fwd", "ssim_bwd")}
    _C.profile_select(None)
    n = img.numel()
    kms = {ph: v[0] / max(v[1], 1) for ph, v in k.items()}
    return {"image": list(img.shape), "fused_ms": round(fused, 4), "torch_reference_ms": round(ref, 4),
            "ssim_fwd_kernel_ms": round(kms["ssim_fwd"], 4), "ssim_bwd_kernel_ms": round(kms["ssim_bwd"], 4),
            # algorithmic bytes: fwd 2 reads + 3 writes, bwd 5 reads + 1 write per pixel (fp32)
            "ssim_fwd_GBps": round(20 * n / (kms["ssim_fwd"] * 1e-3) / 1e9, 1),
            "ssim_bwd_GBps": round(24 * n / (kms["ssim_bwd"] * 1e-3) / 1e9, 1), "steps": steps}


def _torch_densify_event(params, acc, cnt, scene_radius, opt, i):
    """external.py:211-304's densification as the reference composes it from torch ops (the
    comparison leg only): clone, split with torch.normal, drop split originals, prune, Adam surgery."""
    keys = [k for k in params if k not in ("camera_matrices", "camera_center")]

    def swap(new):  # cat_params_to_optimizer / remove_points: new tensor + moments per parameter
        for k, (v, m, s2) in new.items():
            grp = [g for g in opt.param_groups if g["name"] == k][0]
            st = opt.state.pop(grp["params"][0], None)
            p = torch.nn.Parameter(v.requires_grad_(True))
            if st is not None:
                st["exp_avg"], st["exp_avg_sq"] = m, s2
                opt.state[p] = st
            grp["params"][0] = params[k] = p

    def moments(k):
        st = opt.state.get([g for g in opt.param_groups if g["name"] == k][0]["params"][0], {})
        return st.get("exp_avg"), st.get("exp_avg_sq")

    avg = acc / cnt
    avg[avg.isnan()] = 0.0
    ms = torch.exp(params["log_scales"]).max(dim=1).values
    clone = (avg >= 0.0002) & (ms <= 0.01 * scene_radius)
    swap({k: (torch.cat((params[k], params[k][clone])),
              *[torch.cat((t, torch.zeros_like(params[k][clone]))) if t is not None else None for t in moments(k)])
          for k in keys})
    n = params["means"].shape[0]
    pad = torch.zeros(n, device=avg.device)
    pad[:avg.shape[0]] = avg
    split = (pad >= 0.0002) & (torch.exp(params["log_scales"]).max(dim=1).values > 0.01 * scene_radius)
    new = {k: params[k][split].repeat(2, 1) for k in keys}
    stds = torch.exp(params["log_scales"])[split].repeat(2, 1)
    samples = torch.normal(mean=torch.zeros((stds.size(0), 3), device=stds.device), std=stds)
    q = torch.nn.functional.normalize(params["rotation_quaternions"][split])
    r, x, y, z = q.unbind(-1)
    R = torch.stack([1 - 2 * (y * y + z * z), 2 * (x * y - r * z), 2 * (x * z + r * y),
                     2 * (x * y + r * z), 1 - 2 * (x * x + z * z), 2 * (y * z - r * x),
                     2 * (x * z - r * y), 2 * (y * z + r * x), 1 - 2 * (x * x + y * y)], -1).view(-1, 3, 3)
    new["means"] = new["means"] + torch.bmm(R.repeat(2, 1, 1), samples.unsqueeze(-1)).squeeze(-1)
    new["log_scales"] = torch.log(torch.exp(new["log_scales"]) / 1.6)
    swap({k: (torch.cat((params[k], new[k])),
              *[torch.cat((t, torch.zeros_like(new[k]))) if t is not None else None for t in moments(k)])
          for k in keys})
    keep = ~torch.cat((split, torch.zeros(new["means"].shape[0], dtype=torch.bool, device=split.device)))
    swap({k: (params[k][keep], *[t[keep] if t is not None else None for t in moments(k)]) for k in keys})
    keep = ~(torch.sigmoid(params["opacity_logits"]) < 0.005).squeeze()
    swap({k: (params[k][keep], *[t[keep] if t is not None else None for t in moments(k)]) for k in keys})


def densify_call_site(steps, cfg, cam, dev):
    """densify.py's loop body (densify.py:218-247) at the bench resolution on a 1M-Gaussian
    densify.py-style parameter dict: (a) the native path (splat_train.densify_iteration: fused
    activations, fused L1+SSIM, statistics kernels, FusedAdam) vs (b) the reference's composition
    (torch activations + this rasterizer + torch calc_ssim / l1 + torch statistics + torch.optim.Adam),
    ms per iteration; and one densification event (clone / split / prune + Adam surgery) each way."""
    import splat_adam
    import splat_densify
    import splat_scenes as S
    import splat_train
    from diff_gaussian_rasterization import GaussianRasterizer, _C
    P = cfg.P
    g = torch.Generator().manual_seed(7)
    base = S.synthetic_cloud(P, cfg.s0, seed=0, device="cpu")
    base["segmentation_masks"] = (torch.rand(P, 1, generator=g) > 0.5).float().repeat(1, 3)
    base["camera_matrices"] = torch.zeros(50, 3)
    base["camera_center"] = torch.zeros(50, 3)
    order = ["means", "colors", "segmentation_masks", "rotation_quaternions", "opacity_logits", "log_scales",
             "camera_matrices", "camera_center"]
    lrs = {"means": 0.00016 * 4.0, "colors": 0.0025, "segmentation_masks": 0.0, "rotation_quaternions": 0.001,
           "opacity_logits": 0.05, "log_scales": 0.001, "camera_matrices": 1e-4, "camera_center": 1e-4}
    H, W = cfg.height, cfg.width
    view = splat_train.View(0, cam, torch.rand(3, H, W, generator=g).to(dev),
                            (torch.rand(1, H, W, generator=g) > 0.5).float().repeat(3, 1, 1).to(dev))

    def fresh(opt_cls):
        params = {k: torch.nn.Parameter(base[k].to(dev).contiguous()) for k in order}
        opt = opt_cls([{"params": [params[k]], "name": k, "lr": lrs[k]} for k in order], lr=0.0, eps=1e-15)
        return params, opt, splat_train.create_densification_variables(params)

    def native(state, i):
        params, opt, dv = state
        splat_train.densify_iteration(params, view, dv, opt, 4.0, i)

    def reference(state, i):
        params, opt, dv = state
        ra = S.render_arguments(params)
        ra["means2D"].retain_grad()
        img, radii, _ = GaussianRasterizer(raster_settings=cam)(**ra)
        li = 0.8 * torch.nn.functional.l1_loss(img, view.image) + 0.2 * (1.0 - _torch_calc_ssim(img, view.image))
        rs = S.render_arguments(params)
        rs["colors_precomp"] = params["segmentation_masks"]
        seg, _, _ = GaussianRasterizer(raster_settings=cam)(**rs)
        ls = 0.8 * torch.nn.functional.l1_loss(seg, view.segmentation_mask) + \
            0.2 * (1.0 - _torch_calc_ssim(seg, view.segmentation_mask))
        pos = radii > 0
        dv.max_2d_radii[pos] = torch.max(radii[pos], dv.max_2d_radii[pos])
        (li + 3 * ls).backward()
        with torch.no_grad():
            dv.mean_2d_gradients_accumulated[pos] += torch.norm(ra["means2D"].grad[pos, :2], dim=-1)
            dv.visibility_count[pos] += 1
            opt.step()
            opt.zero_grad(set_to_none=True)

    def timed(fn, state, first):
        for i in range(2):
            fn(state, first + i)  # warm-up (off the densify schedule: i % 100 != 0)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for i in range(steps):
            fn(state, first + 2 + i)
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / steps * 1e3

    nat_state = fresh(splat_adam.FusedAdam)
    nat = timed(native, nat_state, 501)
    ref_state = fresh(torch.optim.Adam)
    ref = timed(reference, ref_state, 501)
    # One densification event each way on the statistics the timed iterations accumulated, scaled so
    # that 20 % of the seen Gaussians pass the 0.0002 gradient threshold, with a scene radius that puts
    # the 0.01 r clone / split boundary at the cloud's median maximum scale: clones AND splits happen
    # (with the bench's tiny synthetic gradients and r = 4 nothing would split).
    out = {"gaussians": P, "image": f"{W}x{H}", "native_iteration_ms": round(nat, 3),
           "reference_composition_iteration_ms": round(ref, 3), "steps": steps}
    dv0 = nat_state[2]
    seen = dv0.visibility_count > 0
    avg = dv0.mean_2d_gradients_accumulated[seen] / dv0.visibility_count[seen]
    gscale = float(2e-4 / torch.quantile(avg[:1 << 24].float(), 0.8).clamp_min(1e-30))
    radius = float(100.0 * torch.exp(nat_state[0]["log_scales"].detach()).max(dim=1).values.median())
    out["densify_event"] = {"gradient_scale": gscale, "scene_radius": radius}
    for name, state in (("native", nat_state), ("reference", ref_state)):
        params, opt, dv = state
        acc, cnt = dv.mean_2d_gradients_accumulated * gscale, dv.visibility_count.clone()
        torch.cuda.synchronize()
        t = time.perf_counter()
        if name == "native":
            _C.profile_reset()
            _C.profile_select(["densify_plan", "densify_apply"])
            _C.profile_enable(True)
            dv.mean_2d_gradients_accumulated, dv.visibility_count = acc, cnt
            info = splat_densify._densify(params, dv, radius, opt, 600, None)
        else:
            _torch_densify_event(params, acc, cnt, radius, opt, 600)
        torch.cuda.synchronize()
        out[f"{name}_densify_event_ms"] = round((time.perf_counter() - t) * 1e3, 3)
        if name == "native":
            _C.profile_enable(False)
            apply_ms = _C.profile_read("densify_apply")[0]
            _C.profile_select(None)
            out["densify_rows"] = info
            # apply: every input row read (17 floats x param + 2 moments) + every output row written
            out["densify_apply_GBps"] = round(4 * 17 * 3 * (P + info["P_out"]) / (apply_ms * 1e-3) / 1e9, 1)
    return out


def _reference_timestep_views(md, t, root, dev):
    """shared.py:127-171's per-view formatting composed from the reference's own ops (PIL on one
    thread, float on the host, one upload per tensor, permute / divide / stack on the GPU), for the
    I/O leg's comparison only."""
    import copy
    from PIL import Image
    out = []
    for c, fn in enumerate(md["fn"][t]):
        m = torch.tensor(np.array(copy.deepcopy(Image.open(os.path.join(root, "seg", fn.replace(".jpg", ".png"))))
                                  ).astype(np.float32)).float().to(dev)
        img = torch.tensor(np.array(copy.deepcopy(Image.open(os.path.join(root, "ims", fn))))).float().to(dev)
        out.append((img.permute(2, 0, 1) / 255, torch.stack((m, torch.zeros_like(m), 1 - m))))
    return out


def io_call_site(timesteps, dev, W=640, H=360, C=27):
    """Frames per second of the data path on a synthetic sequence in the
    reference's layout (27 cameras of 640 x 360 -- the dataset's frame size -- JPEG + PNG):
    splat_io.load_all_views (thread-pool decode into one pinned 8-bit batch, one upload, one
    gsr_views_pack launch per timestep) vs the reference's per-view composition; plus the pack
    kernel's device time and its GB/s over 4 B read + 24 B written per pixel."""
    import shutil
    import tempfile
    import splat_io
    import splat_scenes as S
    from PIL import Image
    from diff_gaussian_rasterization import _C
    root = tempfile.mkdtemp(prefix="gsr_io_")
    try:
        rng = np.random.default_rng(0)
        yy, xx = np.mgrid[0:H, 0:W]
        md = {"w": W, "h": H, "fn": [], "k": [], "w2c": []}
        K = S.intrinsics(0.8 * W, W, H).tolist()
        for t in range(timesteps + 1):
            md["fn"].append([]); md["k"].append([]); md["w2c"].append([])
            for c in range(C):
                fn = f"{c}/{t:06d}.jpg"
                for sub in ("ims", "seg"):
                    os.makedirs(os.path.join(root, sub, str(c)), exist_ok=True)
                base = np.stack([xx * 255 // (W - 1), yy * 255 // (H - 1), (xx + yy + 9 * c + t) % 256], -1)
                img = np.clip(base + rng.integers(-20, 21, size=(H, W, 3)), 0, 255).astype(np.uint8)
                Image.fromarray(img).save(os.path.join(root, "ims", fn), quality=90)
                inside = ((xx - W / 2) ** 2 + (yy - H / 2) ** 2) < (H / 3 + c) ** 2
                Image.fromarray(inside.astype(np.uint8), mode="L").save(os.path.join(root, "seg", fn.replace(".jpg", ".png")))
                md["fn"][t].append(fn); md["k"][t].append(K)
                md["w2c"][t].append(S.look_at(360.0 * c / C, 0.2, 4.0).tolist())
        frames = timesteps * C
        splat_io.load_all_views(md, 1, root, device=dev)  # warm: pool start, pinned allocator, kernel
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        views = splat_io.load_all_views(md, timesteps, root, device=dev)
        torch.cuda.synchronize()
        ours = time.perf_counter() - t0
        _reference_timestep_views(md, 1, root, dev)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ref = [_reference_timestep_views(md, t, root, dev) for t in range(1, timesteps + 1)]
        torch.cuda.synchronize()
        refs = time.perf_counter() - t0
        same = all(torch.equal(v.image, r[0]) and torch.equal(v.segmentation_mask, r[1])
                   for vs, rs in zip(views, ref) for v, r in zip(vs, rs))
        # device time of the pack kernel over one timestep already resident in HBM
        rgb = torch.randint(0, 256, (C, H, W, 3), dtype=torch.uint8, device=dev)
        seg = torch.randint(0, 2, (C, H, W), dtype=torch.uint8, device=dev)
        splat_io.pack_views(rgb, seg)
        _C.profile_reset(); _C.profile_select(["views_pack"]); _C.profile_enable(True)
        for _ in range(20):
            splat_io.pack_views(rgb, seg)
        _C.profile_enable(False)
        tot, n = _C.profile_read("views_pack")
        _C.profile_select(None)
        kms = tot / max(n, 1)
        return {"frames": frames, "frame": f"{W}x{H}", "cameras": C, "timesteps": timesteps,
                "workers": splat_io.TimestepDecoder().workers,
                "native_frames_per_s": round(frames / ours, 1), "reference_frames_per_s": round(frames / refs, 1),
                "bitwise_equal_to_reference_ops": bool(same),
                "pack_kernel_ms_per_timestep": round(kms, 5),
                "pack_GBps": round(28 * C * H * W / (kms * 1e-3) / 1e9, 1)}
    finally:
        shutil.rmtree(root, ignore_errors=True)


def _self_launch(n):
    """``--gpus N`` without a launcher: start N ranks with torch.distributed.run (127.0.0.1 rendezvous)
    as CHILD processes and relay their output (rank 0 prints the JSON line).  The parent never touches
    the GPU and never re-execs; it exits with the launcher's status."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd).returncode


def _dry_run(args, rank, world):
    """CPU rehearsal of the launcher and the step's control flow (no GPU, gloo): shard the config's
    views, fill a gradient bucket per view, all-reduce it once per step, report what every rank did."""
    import torch.distributed as dist
    import splat_dp
    import splat_scenes as S
    views = list(range(len(S.RIG27)))
    mine = splat_dp.shard_views(views, rank, world) if args.config == "C4" else \
        splat_dp.shard_views([(k) % len(views) for k in range(world * args.views_per_rank)], rank, world)
    bucket = torch.zeros(16)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        bucket.zero_()
        for v in mine:
            bucket += float(v + 1)
        if world > 1:
            dist.all_reduce(bucket)
    elapsed = time.perf_counter() - t0
    shards = [None] * world
    if world > 1:
        dist.all_gather_object(shards, mine)
    else:
        shards = [mine]
    expect = float(sum(v + 1 for sh in shards for v in sh))
    if rank == 0:
        print(json.dumps({"metric": "dry run (launcher + sharding + collective rehearsal, no GPU)", "value": None,
                          "unit": None, "n_gpus": world, "steps": args.steps, "dry_run": True,
                          "config": {"workload": args.config, "views_per_rank": [len(x) for x in shards]},
                          "bucket_sum_ok": bool(torch.all(bucket == expect)),
                          "ms_per_step": round(elapsed / max(args.steps, 1) * 1e3, 4)}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def step_stats(views_per_step, P, ms):
    """value / median / quartiles of per-step device intervals (ms list)."""
    ms = sorted(ms)
    med = float(np.median(ms))
    return {"Msplats_per_s": round(views_per_step * P / (med * 1e-3) / 1e6, 2), "median_ms_per_step": round(med, 4),
            "step_ms_quartiles": [round(float(np.percentile(ms, q)), 4) for q in (25, 50, 75)],
            "Msplats_per_s_quartiles": [round(views_per_step * P / (float(np.percentile(ms, q)) * 1e-3) / 1e6, 2)
                                        for q in (75, 50, 25)]}


def timed_steps(fn, steps, warmup, dev, host=None):
    """Run fn(it) warmup times, then `steps` times with an event on the current stream after each
    step: per-step device intervals (ms).  ``host``: a list that receives each step's host time (ms,
    the submitting thread's wall clock of the call): a step whose host time reaches its device time is
    host-bound."""
    for it in range(warmup):
        fn(it)
    torch.cuda.synchronize()
    s = torch.cuda.current_stream(dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
    ev[0].record(s)
    for it in range(steps):
        t = time.perf_counter()
        fn(warmup + it)
        if host is not None:
            host.append((time.perf_counter() - t) * 1e3)
        ev[it + 1].record(s)
    torch.cuda.synchronize()
    return [ev[i].elapsed_time(ev[i + 1]) for i in range(steps)]


def unchanged_call_site(steps, warmup, cfg, cams, views, dl, dev):
    """train.py's render step exactly as an unchanged train.py drives it, reported beside ``value``
    (VERDICT r03 item 1): ONE host thread, torch's current stream, no caller streams; the Gaussian
    parameters frozen (train.py:155-163 sets requires_grad = False) with the colours train.py renders
    (colors_precomp, RGB); the step's means and rotations are deep copies, ``.detach()``ed, plus 0.01 x a
    deformation output (train.py:297-308 -- a (P, 7) leaf stands in for the network, which is out of
    scope); every view builds its arguments with create_render_arguments (shared.py:29-42: normalize,
    sigmoid, exp and a fresh ``zeros_like(requires_grad=True) + 0`` means2D) and renders through
    ``GaussianRasterizer(raster_settings=...)(**args)`` (train.py:359-361); the 5 views' losses are
    stacked, summed and backpropagated once (train.py:402-418, 767).  The loss of a view is
    ``(image * dL/dimage).sum()`` with the headline's fixed upstream gradient (the L1 + SSIM and the
    rigidity loss are out of the metric's scope).  Rasterizer inputs are not leaves, so every view
    takes the immediate per-view backward.  Library defaults throughout: each forward reads its pair
    count back as the reference's does (the asynchronous forward and the library view streams are off,
    DESIGN.md 2.4d, as they measured slower on this shape)."""
    import splat_scenes as S
    from diff_gaussian_rasterization import GaussianRasterizer
    P = cfg.P
    base = S.synthetic_cloud(P, cfg.s0, sh_degree=-1, seed=0, device=dev)  # requires_grad False
    delta = torch.zeros(P, 7, device=dev, requires_grad=True)

    def one(it):
        p = {k: v.clone() for k, v in base.items()}  # copy.deepcopy (train.py:297-299)
        p["means"] = p["means"].detach()
        p["means"] += delta[:, :3] * 0.01
        p["rotation_quaternions"] = p["rotation_quaternions"].detach()
        p["rotation_quaternions"] += delta[:, 3:] * 0.01
        losses = torch.stack([(GaussianRasterizer(raster_settings=cams[ci])(**S.render_arguments(p))[0] * dl).sum()
                              for ci in views(it)])
        losses.sum(dim=0).backward()
        delta.grad = None  # optimizer.zero_grad()

    host = []
    ms = timed_steps(one, steps, warmup, dev, host)
    out = {"features": "RGB (colors_precomp, as train.py renders)", "views_per_step": len(views(0)),
           "host_ms_per_step_median": round(float(np.median(host)), 4),
           "threads": 1, "streams": "torch's current stream only", "steps": steps,
           "inputs": "non-leaf (frozen Gaussians, means/rotations = deepcopy.detach() + 0.01 delta, "
                     "per-view create_render_arguments)",
           "backward": "one backward of the stacked, summed view losses (immediate per-view rasterizer backward)"}
    out.update(step_stats(len(views(0)), P, ms))
    return out


def inference_call_site(steps, warmup, P, s0, dev):
    """train.py's inference renders (outside ``value``): render_and_export_frame
    (train.py:506-547) under torch.no_grad() (train.py:778) -- every timestep the five fixed cameras of
    create_extrinsic_matrices (train.py:459-503) at 1280 x 720, each call
    ``GaussianRasterizer(raster_settings=...)(**create_render_arguments(params))``: forward only, one host
    thread, torch's current stream, RGB colours.  One step = the five cameras; the PNG export and the
    deformation network are outside the metric.  Msplats/s = 5 P / step time."""
    import splat_scenes as S
    from diff_gaussian_rasterization import GaussianRasterizer
    params = S.synthetic_cloud(P, s0, sh_degree=-1, seed=0, device=dev)
    cams = S.inference_cameras(device=dev)

    def one(it):
        with torch.no_grad():
            for rs in cams:
                GaussianRasterizer(raster_settings=rs)(**S.render_arguments(params))

    host = []
    ms = timed_steps(one, steps, warmup, dev, host)
    out = {"workload": f"{P} Gaussians, RGB, 5 inference cameras at {S.INFERENCE_W}x{S.INFERENCE_H}, forward only "
                       "(no_grad), create_render_arguments per render", "views_per_step": len(cams),
           "threads": 1, "streams": "torch's current stream only", "steps": steps,
           "host_ms_per_step_median": round(float(np.median(host)), 4)}
    out.update(step_stats(len(cams), P, ms))
    return out


def c2_leg(steps, warmup, dev, nstreams=3):
    """BASELINE configs[1] (C2: 100k Gaussians, RGB, the 4 cameras of 800x800 at yaw 0/90/180/270),
    measured in the default run so the driver records it: one step = the 4 views rendered from ONE
    host thread over `nstreams` streams (the forwards do not wait for their pair counts, so one thread
    keeps every stream fed), their losses summed, one backward into leaf render arguments (deferred
    multi-view per-Gaussian pass), a fresh zero means2D leaf per render."""
    import splat_scenes as S
    import splat_step
    cfg = S.CONFIGS["C2"]
    params = S.synthetic_cloud(cfg.P, cfg.s0, sh_degree=-1, seed=0, device=dev)
    with torch.no_grad():
        act = S.activated_inputs(params, -1)
    leaves = {k: v.detach().clone().requires_grad_(True) for k, v in act.items()}
    cams = S.scene_cameras(cfg, device=dev)
    dl = S.upstream_grad(cfg.height, cfg.width, device=dev)
    cur = torch.cuda.current_stream(dev)
    streams = [torch.cuda.Stream(dev) for _ in range(nstreams)]
    for st in streams:
        st.wait_stream(cur)
    rstep = splat_step.RenderStep(dev, cams, lambda ci: dict(leaves, means2D=torch.zeros_like(leaves["means3D"],
                                                                                              requires_grad=True)),
                                  dl, streams, threads=False)

    def one(it):
        rstep(list(range(len(cams))))
        for st in streams:
            cur.wait_stream(st)  # the step ends on the current stream (its timing event)
        for v in leaves.values():
            v.grad = None

    host = []
    ms = timed_steps(one, steps, warmup, dev, host)
    rstep.close()
    out = {"workload": f"C2: {cfg.P} Gaussians, RGB, {cfg.width}x{cfg.height}, 4 cameras per step, fwd+bwd, "
                       "view losses summed, one backward", "views_per_step": len(cams), "steps": steps,
           "submission": f"one host thread, {nstreams} streams",
           "host_ms_per_step_median": round(float(np.median(host)), 4)}
    out.update(step_stats(len(cams), cfg.P, ms))
    return out


def train_call_site(steps, cfg, cams, views, dl, dev, streams, sh):
    """train.py's render call site with the benchmark's streams (outside ``value``): the Gaussian
    parameters are frozen (train.py:155-163 loads them with requires_grad =
    False); the means and rotations of the step are ``p.detach()`` copies plus 0.01 x a deformation
    output (train.py:297-308; here a (P, 7) leaf stands in for the network, which is out of scope);
    every view builds its arguments with create_render_arguments (shared.py:29-42: normalize / sigmoid
    / exp and a fresh ``zeros_like(requires_grad=True) + 0`` means2D); the view losses are summed and
    backpropagated once (train.py:402-418, 767).  The rasterizer's inputs are therefore NOT leaves and
    every view takes the immediate per-view backward (no deferred multi-view pass).  Unlike an
    unchanged train.py (``unchanged_call_site``), the views run on the headline's caller-owned streams
    with one submitting thread per stream.  ``sh``: False = the reference's colors_precomp (RGB,
    what train.py renders), True = SH3 coefficients passed as ``shs`` (the headline's features)."""
    import splat_scenes as S
    import splat_step
    from diff_gaussian_rasterization import _C
    P = cfg.P
    base = S.synthetic_cloud(P, cfg.s0, sh_degree=3 if sh else -1, seed=0, device=dev)  # requires_grad False
    delta = torch.zeros(P, 7, device=dev, requires_grad=True)
    cur = {}
    main = torch.cuda.current_stream(dev)

    def args_of(_ci):  # shared.py:29-42 on the step's updated parameters, per view
        a = S.render_arguments(cur["p"])
        if sh:
            a.pop("colors_precomp")
            a["shs"] = cur["p"]["shs"]
        return a

    rstep = splat_step.RenderStep(dev, cams, args_of, dl, streams, threads=True)

    def one(it):
        p = dict(base)  # update_gaussian_cloud_parameters (train.py:297-308)
        p["means"] = base["means"].clone()
        p["means"] += delta[:, :3] * 0.01
        p["rotation_quaternions"] = base["rotation_quaternions"].clone()
        p["rotation_quaternions"] += delta[:, 3:] * 0.01
        cur["p"] = p
        for s in streams:
            s.wait_stream(main)  # the step's updated parameters
        rstep(views(it))
        for s in streams:
            main.wait_stream(s)
        delta.grad = None  # optimizer.zero_grad()

    for it in range(3):
        one(it)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for it in range(steps):
        one(3 + it)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) / steps * 1e3
    # device time per launch of the path's kernels inside the same pipelined steps (HIP events on
    # each kernel's launch stream, untimed steps)
    _C.profile_reset()
    _C.profile_select(["render_fwd", "render_bwd", "gauss_bwd"])
    _C.profile_enable(True)
    for it in range(3):
        one(3 + steps + it)
    torch.cuda.synchronize()
    _C.profile_enable(False)
    _C.profile_select(None)
    phases = {ph: _C.profile_read(ph) for ph in ("render_fwd", "render_bwd", "gauss_bwd")}
    rstep.close()
    nv = len(views(0))
    return {"features": "SH3 (shs)" if sh else "RGB (colors_precomp, as train.py renders)",
            "ms_per_step": round(ms, 4), "views_per_step": nv, "Msplats_per_s": round(nv * P / ms / 1e3, 2),
            "inputs": "non-leaf (frozen Gaussians, means/rotations = detach + 0.01 delta, per-view activations)",
            "backward": "immediate per-view (rasterizer inputs are not leaves)",
            "in_step_kernel_ms_per_launch": {ph: round(v[0] / max(v[1], 1), 5) for ph, v in phases.items() if v[1]},
            "steps": steps}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None, help="timed steps (default 100; C5: 5)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed warm-up steps (default 10; C5: 1)")
    ap.add_argument("--config", default="C3", choices=["C2", "C3", "C3M", "C4", "C5"],
                    help="C3 (default): 1M Gaussians SH3 at 1080p, --views-per-rank rig views per GPU per "
                         "step (weak scaling); C2: 100k Gaussians, RGB, the 4 cameras of 800x800 per GPU per "
                         "step (weak scaling); C4: 1M Gaussians, the 27-camera rig sharded round-robin over "
                         "the ranks per step + one RCCL SUM all-reduce (strong scaling); C5: 2M Gaussians x "
                         "150-frame sequence, independent per-frame fits sharded in frame blocks, one "
                         "optimisation iteration (5 views, fused L1+SSIM, fused Adam) of every frame per step, "
                         "no collective (strong scaling); C3M: C3 with half of the means in 16 tight clusters "
                         "(a densified scene: tiles of tens of thousands of pairs)")
    ap.add_argument("--views-per-rank", type=int, default=None,
                    help="C3 / C5: views rendered per GPU per step / per frame (default 5: train.py:753 "
                         "optimises on the summed losses of 5 views per step); C2: default 4")
    ap.add_argument("--stream-priority", type=int, default=0,
                    help="HIP priority of the view streams (negative = higher than the main stream, "
                         "which runs the multi-view per-Gaussian pass and the collectives)")
    ap.add_argument("--streams", type=int, default=3,
                    help="HIP streams the step's views alternate over: one view's memory-bound "
                         "per-Gaussian backward overlaps the next view's VALU-bound render kernels; "
                         "libgsr orders the gradient writes across streams (bitwise the 1-stream result)")
    ap.add_argument("--step-shape", default="summed", choices=["summed", "per-view"],
                    help="summed (train.py:753-767): the step's view losses summed, ONE backward -- each "
                         "view's per-pixel backward runs in its node and one per-Gaussian pass covers all "
                         "views at the end of the pass (deferred multi-view backward); per-view: a "
                         "backward per view")
    ap.add_argument("--submit", default="auto", choices=["auto", "threads", "serial"],
                    help="auto: threads for the summed step (C3: +3-5 %% measured, tools/ab_args.sh), serial "
                         "for per-view and C2 (small views: one thread is faster and steadier); threads: one host thread per stream submits that stream's views, so a forward "
                         "waiting for its num_rendered read-back blocks only its own thread and the other "
                         "streams' views keep the GPU fed; serial: one thread submits every view in turn")
    ap.add_argument("--means2d", default="per-view", choices=["per-view", "shared"],
                    help="per-view (default): every render gets a fresh zero means2D leaf, as "
                         "create_render_arguments makes one per render (shared.py:38-41); shared: one "
                         "means2D leaf for all views of a step")
    ap.add_argument("--gil-switch-us", type=float, default=0.0,
                    help="sys.setswitchinterval in microseconds for the submitting threads (0: Python's "
                         "default, 5000)")
    ap.add_argument("--backend", default="nccl",
                    help="torch.distributed backend for N > 1 (nccl = RCCL over xGMI; gloo only to "
                         "rehearse the multi-rank path on one GPU)")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU rehearsal of the launcher / sharding / collective (gloo, no GPU work)")
    ap.add_argument("--pin-cpus", type=int, default=int(os.environ.get("GSR_PIN_CPUS", "8")),
                    help="pin the process's threads to this many of the least busy CPUs of the GPU's NUMA "
                         "node (this rank's share of it) before the GPU runtime starts -- a launcher's numactl; the "
                         "submitting threads otherwise wander over the shared host's 256 CPUs (0 = off; "
                         "splat_affinity.py)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="OpenMP threads of the CPU baseline (0 = every CPU this process may run on, "
                         "os.sched_getaffinity)")
    ap.add_argument("--call-site-steps", type=int, default=10,
                    help="steps timed for each call-site variant (0 = skip; N = 1, C3 only)")
    ap.add_argument("--train-steps", type=int, default=10,
                    help="steps timed for the train.py call-site legs (0 = skip; N = 1, C3 only)")
    ap.add_argument("--inference-steps", type=int, default=20,
                    help="steps of the inference_call_site leg (train.py's no_grad 5-camera renders; 0 = skip)")
    ap.add_argument("--unchanged-steps", type=int, default=30,
                    help="steps timed for the unchanged train.py call site (one thread, current stream, "
                         "non-leaf inputs, RGB; 0 = skip; N = 1, C3 only)")
    ap.add_argument("--c2-steps", type=int, default=60,
                    help="steps timed for the C2 leg (BASELINE configs[1], 4 x 800x800, 100k; 0 = skip; "
                         "N = 1, C3 only)")
    ap.add_argument("--loss-steps", type=int, default=10,
                    help="steps timed for the L1+SSIM loss legs at the bench resolution (0 = skip; N = 1, C3)")
    ap.add_argument("--densify-steps", type=int, default=5,
                    help="densify.py iterations timed per variant at the bench resolution (0 = skip; N = 1, C3)")
    ap.add_argument("--io-timesteps", type=int, default=2,
                    help="timesteps of 27 synthetic 640x360 frames loaded per variant by the data-path "
                         "leg (0 = skip; N = 1, C3)")
    ap.add_argument("--probe-steps", type=int, default=3,
                    help="untimed steps with events on every phase (per-kernel breakdown)")
    ap.add_argument("--grad-checksum", default=None,
                    help="C2 / C3 / C4: after the timed steps, one more step whose (all-reduced) gradient "
                         "bucket is saved to PATH.rank<r>.pt with the step's camera indices (a parity hook "
                         "for the multi-rank path: tests/test_dp_gpu.py)")
    args = ap.parse_args()
    c5_cfg = args.config == "C5"
    if args.steps is None:
        args.steps = 5 if c5_cfg else 100
    if args.warmup is None:
        args.warmup = 1 if c5_cfg else 10
    if args.views_per_rank is None:
        args.views_per_rank = 4 if args.config == "C2" else 5

    if args.gil_switch_us > 0:
        sys.setswitchinterval(args.gil_switch_us * 1e-6)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(_self_launch(args.gpus))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        if world > 1:
            import torch.distributed as dist
            dist.init_process_group("gloo")
        _dry_run(args, rank, world)
        return

    import splat_dp
    import splat_scenes as S
    import splat_step
    from diff_gaussian_rasterization import GaussianRasterizer, _C, rasterize_parameters

    dist = None
    local = local % max(torch.cuda.device_count(), 1)  # rehearsal: several gloo ranks on one GPU
    # host-thread placement before the GPU runtime starts, so its threads and host allocations start on
    # the chosen CPUs' node (pinning after it started: C2 399-473 vs 509-520 Msplats/s, tools/c2_pin.py)
    affinity0 = sorted(os.sched_getaffinity(0))
    pinned = []
    if args.pin_cpus > 0:
        import splat_affinity
        pinned = splat_affinity.pin_host_threads(local, local, int(os.environ.get("LOCAL_WORLD_SIZE", "1")),
                                                 args.pin_cpus)
    # under a launcher (torch.distributed.run sets WORLD_SIZE) the process group is formed even for one
    # rank, so `torchrun --nproc-per-node 1 bench.py --backend nccl` runs the RCCL path on one GPU
    if world > 1 or "TORCHELASTIC_RUN_ID" in os.environ:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(args.backend)
        world = dist.get_world_size()
        rank = dist.get_rank()
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    _C.load_library()

    if c5_cfg:
        cfg = S.SceneConfig("C5", 2_000_000, 1920, 1080, 1600.0, 0.005, views=S.RIG27)
    elif args.config == "C2":
        cfg = S.CONFIGS["C2"]
    else:
        base = S.CONFIGS["C3" if args.config == "C3M" else args.config]
        cfg = S.SceneConfig(args.config, base.P, base.width, base.height, base.focal, base.s0,
                            sh_degree=base.sh_degree, views=S.RIG27)
    if args.config == "C3M":
        params_cpu = S.clustered_cloud(cfg.P, cfg.s0, sh_degree=cfg.sh_degree, seed=0, device="cpu")
    else:
        params_cpu = S.synthetic_cloud(cfg.P, cfg.s0, sh_degree=cfg.sh_degree, seed=0, device="cpu")
    params = {k: torch.nn.Parameter(v.to(dev)) for k, v in params_cpu.items()}
    cams = S.scene_cameras(cfg, device=dev)
    dl = S.upstream_grad(cfg.height, cfg.width, device=dev)
    V = args.views_per_rank

    # the rasterizer's inputs: render arguments of shared.py:29-42, activated once, as leaves
    with torch.no_grad():
        act = S.activated_inputs(params, cfg.sh_degree)
    if cfg.sh_degree >= 0:
        act.pop("colors_precomp")
    leaves = {k: v.detach().clone().requires_grad_(True) for k, v in act.items()}
    grad_leaves = [v for k, v in leaves.items() if k != "means2D"]
    grads_of = lambda: [v.grad for v in grad_leaves]  # noqa: E731
    # N > 1 (C2 / C3 / C4): the gradients live in one flat bucket that backward accumulates into and
    # RCCL reduces in place (no pack / unpack copies)
    reducer = splat_dp.GradAllReduce(grad_leaves).attach() if dist is not None and not c5_cfg else None

    if args.config == "C4":  # the whole rig every step, sharded round-robin (4,4,4,3,3,3,3,3 at 8)
        views_per_step = len(cams)
        my_views = splat_dp.shard_views(list(range(len(cams))), rank, world)

        def views_of(it):
            return my_views
    else:
        views_per_step = world * V

        def views_of(it):  # rank r renders its round-robin share of this step's world * V cameras
            return splat_dp.shard_views([(it * world * V + k) % len(cams) for k in range(world * V)], rank, world)

    main_stream = torch.cuda.current_stream(dev)
    # side streams for the views: the main stream keeps the collectives (N > 1) out of their way
    streams = [torch.cuda.Stream(dev, priority=args.stream_priority) for _ in range(max(args.streams, 1))]
    for s in streams:
        s.wait_stream(main_stream)  # the setup's parameters, leaves and upstream gradient

    if reducer is not None:  # the bucket's zeroing (main stream) precedes the first backward
        _C.grad_fence(*grads_of())

    if args.submit == "auto":
        # threads: one submitting thread per stream pays off when a view's GPU work (~0.7 ms at C3)
        # covers the thread hand-offs; C2's views (~0.3 ms) run faster and steadier from one thread
        # (C2 threads 200-418 vs serial 265-277 Msplats/s; C3 threads +3-5 %, tools/ab_args.sh)
        args.submit = "threads" if args.step_shape == "summed" and args.config != "C2" else "serial"

    def inputs_of(ci):  # called on the view's stream (RenderStep), like the reference's per-render zeros
        if args.means2d == "shared":
            return leaves
        return dict(leaves, means2D=torch.zeros_like(leaves["means3D"], requires_grad=True))

    rstep = splat_step.RenderStep(dev, cams, inputs_of, dl, streams, threads=args.submit == "threads",
                                  shape="summed" if args.step_shape == "summed" else "per_view")

    def step(it, solo=False, keep=False):
        # No stream waits for another at the step start: libgsr orders the gradient writes across
        # streams, record_stream keeps freed gradients from early reuse, and for N > 1 the bucket's
        # all-reduce + reset on the main stream is declared with grad_fence, so the next step's
        # forwards run during the all-reduce and only its first gradient write waits for it.
        # solo: one stream, one submitting thread (per-kernel times without concurrency); keep: leave
        # the step's (reduced) gradients in place
        rstep(views_of(it), solo=solo)
        for s in streams:
            main_stream.wait_stream(s)  # the step ends on the main stream (its end event, the reduce)
        if reducer is not None:
            reducer.reduce()  # one flat-bucket all-reduce (SUM) of every gradient over RCCL
            if keep:
                return
            reducer.zero_()
            _C.grad_fence(*grads_of())
            leaves["means2D"].grad = None
        elif not keep:
            for p in leaves.values():
                p.grad = None

    fits = None
    if c5_cfg:
        import splat_adam
        import splat_frames
        import splat_loss

        def render(p, cam):
            return rasterize_parameters(p, cam)[0]
        fits = splat_frames.FrameFits(
            {k: v.to(dev) for k, v in params_cpu.items()}, cams, rank, world, V, render, splat_loss.image_loss,
            lambda p: splat_adam.FusedAdam([{"params": [v], "name": k, "lr": splat_frames.FRAME_LRS.get(k, 1e-3)}
                                            for k, v in p.items()], lr=0.0, eps=1e-15),
            streams=streams, main_stream=main_stream)
        torch.cuda.synchronize()
        views_per_step = sum(len(splat_dp.shard_frames(150, r, world)) for r in range(world)) * V

        def step(it, solo=False, keep=False):  # noqa: F811 -- every frame of this rank's block
            fits.step(it)

    def step_reference_call_site(it):  # train.py: create_render_arguments + Renderer + backward
        for ci in views_of(it):
            a = S.activated_inputs(params, cfg.sh_degree)
            if cfg.sh_degree >= 0:
                a.pop("colors_precomp")
            img, _radii, _depth = GaussianRasterizer(raster_settings=cams[ci])(**a)
            img.backward(dl)
        for p in params.values():
            p.grad = None

    def step_fused_call_site(it):  # the same through rasterize_parameters (fused activations)
        for ci in views_of(it):
            img, _radii, _depth = rasterize_parameters(params, cams[ci], shs=params.get("shs"))
            img.backward(dl)
        for p in params.values():
            p.grad = None

    def time_steps(fn, n, first):
        torch.cuda.synchronize()
        t = time.perf_counter()
        for it in range(n):
            fn(first + it)
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / n * 1e3

    for it in range(args.warmup):
        step(it)
    probe_steps = min(args.probe_steps, 1) if c5_cfg else args.probe_steps
    # untimed probe: events around every kernel (they add launch gaps, so not in the timed region)
    torch.cuda.synchronize()
    _C.profile_reset()
    _C.profile_select(None)
    _C.profile_enable(True)
    for it in range(probe_steps):
        step(args.warmup + it)
    torch.cuda.synchronize()
    _C.profile_enable(False)
    probe = {ph: _C.profile_read(ph) for ph in PHASES}
    dom = max(PHASES, key=lambda ph: probe[ph][0])
    # untimed solo probe (not C5): the same steps on one stream, one thread -- each kernel's time
    # without the other streams' kernels sharing the CUs (the roofline's kernel alone)
    solo = None
    if fits is None and probe_steps > 0:
        torch.cuda.synchronize()
        _C.profile_reset()
        _C.profile_enable(True)
        for it in range(probe_steps):
            step(args.warmup + it, solo=True)
        torch.cuda.synchronize()
        _C.profile_enable(False)
        solo = {ph: _C.profile_read(ph) for ph in PHASES}
    # timed region: HIP events only around the dominant kernel (its roofline), host timers on, and an
    # event on the main stream at every step end (the step ends there): per-step device intervals
    first = args.warmup + probe_steps
    ends = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    _C.profile_reset()
    _C.profile_select([dom])
    _C.profile_enable(True)
    t0 = time.perf_counter()
    ends[0].record(main_stream)
    for it in range(args.steps):
        step(first + it)
        ends[it + 1].record(main_stream)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    _C.profile_enable(False)
    step_ms = sorted(ends[i].elapsed_time(ends[i + 1]) for i in range(args.steps))
    median_ms = float(np.median(step_ms))
    if dist is not None:
        t = torch.tensor([elapsed, median_ms], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, median_ms = float(t[0].item()), float(t[1].item())

    # dominant kernel's device time inside the timed region (HIP events on its launch stream)
    tot_ms, cnt = _C.profile_read(dom)
    _C.profile_select(None)
    checksum = None
    if args.grad_checksum and fits is None:  # one more step, its (reduced) gradients kept and saved
        it = first + args.steps
        step(it, keep=True)
        torch.cuda.synchronize()
        flat = reducer.flat if reducer is not None else torch.cat([g.reshape(-1) for g in grads_of()])
        checksum = f"{args.grad_checksum}.rank{rank}.pt"
        torch.save({"bucket": flat.detach().cpu(), "views": views_of(it), "world": world, "rank": rank,
                    "names": [k for k in leaves if k != "means2D"]}, checksum)
        if reducer is not None:
            reducer.zero_()
        for p in leaves.values():
            if reducer is None or p is leaves["means2D"]:
                p.grad = None
    legs = world == 1 and args.config == "C3"
    call_site = None
    if legs and args.call_site_steps > 0:
        per_view = len(views_of(first))
        time_steps(step_reference_call_site, 3, first)  # warm each path's kernels and allocations
        ref_ms = time_steps(step_reference_call_site, args.call_site_steps, first)
        time_steps(step_fused_call_site, 3, first)
        fused_ms = time_steps(step_fused_call_site, args.call_site_steps, first)
        call_site = {"reference_activations_ms_per_view": round(ref_ms / per_view, 4),
                     "fused_activations_ms_per_view": round(fused_ms / per_view, 4),
                     "steps": args.call_site_steps}
    host = {ph: _C.profile_read(ph) for ph in ("host_forward", "host_wait_K", "host_backward")}
    unchanged = c2 = None
    if legs and args.unchanged_steps > 0:
        unchanged = unchanged_call_site(args.unchanged_steps, 5, cfg, cams, views_of, dl, dev)
    inference = None
    if legs and args.inference_steps > 0:
        inference = inference_call_site(args.inference_steps, 3, cfg.P, cfg.s0, dev)
    if legs and args.c2_steps > 0:
        c2 = c2_leg(args.c2_steps, 10, dev)
    train_site = None
    if legs and args.train_steps > 0:
        train_site = {k: train_call_site(args.train_steps, cfg, cams, views_of, dl, dev, streams, sh)
                      for k, sh in (("rgb", False), ("sh3", True))}
    loss_site = loss_call_site(args.loss_steps, cams[0], leaves, dev) if legs and args.loss_steps > 0 else None
    dens_site = densify_call_site(args.densify_steps, cfg, cams[0], dev) if legs and args.densify_steps > 0 else None
    io_site = io_call_site(args.io_timesteps, dev) if legs and args.io_timesteps > 0 else None
    # untimed forwards over the cameras the timed steps used: mean pair count K for the byte model
    used = fits.used_views() if fits else \
        sorted({ci for it in range(first, first + args.steps) for ci in views_of(it)})
    Ks, max_tile = [], 0
    with torch.no_grad():
        if fits:
            import splat_frames
            a = S.activated_inputs(splat_frames.frame_truth(fits.params[fits.frames[0]], fits.phi, fits.frames[0],
                                                            fits.n_frames), -1)
        else:
            a = S.activated_inputs(params, cfg.sh_degree)
        if cfg.sh_degree >= 0:
            a.pop("colors_precomp")
        e = torch.empty(0, device=dev)
        colors = a.get("colors_precomp")
        for ci in used:
            c = cams[ci]
            r = _C.rasterize_gaussians(c.bg, a["means3D"].detach(), colors.detach() if colors is not None else e,
                                       a["opacities"].detach(), a["scales"].detach(), a["rotations"].detach(), 1.0, e,
                                       c.viewmatrix, c.projmatrix, c.tanfovx, c.tanfovy,
                                       cfg.height, cfg.width, a.get("shs", e), c.sh_degree,
                                       c.campos, False)
            Ks.append(r[0])
            rg = _C.decode_buffers(a["means3D"].shape[0], cfg.width, cfg.height, r[0], r[3], r[4], r[5])["ranges"]
            max_tile = max(max_tile, int((rg[:, 1] - rg[:, 0]).max()))
    K = float(np.mean(Ks))
    N = cfg.width * cfg.height
    T = ((cfg.width + 15) // 16) * ((cfg.height + 15) // 16)
    F = 12 * (cfg.sh_degree + 1) ** 2 if cfg.sh_degree >= 0 else 12
    SH = int(cfg.sh_degree >= 0)
    avg_ms = tot_ms / max(cnt, 1)
    traffic = traffic_2x = None
    if os.path.exists(PMC_SUMMARY):
        pm = json.load(open(PMC_SUMMARY)).get("k_" + dom)
        if pm and args.config == "C3":
            traffic_2x = int(pm["hbm_bytes_per_launch_corrected"])
            traffic = calibrated_traffic(pm, dom, cfg.P, K, N, T)
    valu = None
    solo_ms = solo[dom][0] / solo[dom][1] if solo and solo[dom][1] else None
    if os.path.exists(SQ_SUMMARY) and args.config == "C3":
        q = json.load(open(SQ_SUMMARY)).get("k_" + dom)
        if q and "SQ_INSTS_VALU" in q:
            # the kernel's wave64 VALU instructions (profile of this command) over its live duration,
            # vs one per 2 cycles on every SIMD (the v_fma_f32 rate; transcendentals, DPP and permlane
            # ops occupy the pipe 2-4x longer: tools/valu_rate_probe.hip), so issue_frac is a floor
            # on the VALU pipe's busy share
            rate = q["SQ_INSTS_VALU"] / ((solo_ms or avg_ms) * 1e-3) / 1e9
            valu = {"insts_per_launch": int(q["SQ_INSTS_VALU"]),
                    "trans_insts_per_launch": int(q.get("SQ_INSTS_VALU_TRANS_F32", 0)),
                    "achieved_Ginst_s": round(rate, 1), "peak_Ginst_s": VALU_PEAK_GINST,
                    "issue_frac": round(rate / VALU_PEAK_GINST, 4),
                    "source": os.path.relpath(SQ_SUMMARY, REPO)}
            if q.get("clock_ghz"):  # GRBM_GUI_ACTIVE / 8 / duration in the profile pass: the clock held
                pk = 1024 * q["clock_ghz"] / 2  # Ginst/s at that clock
                valu["profile_clock_ghz"] = round(q["clock_ghz"], 3)
                valu["issue_frac_at_profile_clock"] = round(rate / pk, 4)
    valu_step = valu_fwd = None
    if os.path.exists(SQ_SUMMARY) and args.config == "C3" and args.step_shape == "summed":
        valu_step, valu_fwd = step_valu(json.load(open(SQ_SUMMARY)), views_per_step / world, median_ms,
                                        solo["render_fwd"][0] / solo["render_fwd"][1]
                                        if solo and solo["render_fwd"][1] else None)
    bytes_launch = algorithmic_bytes(dom, cfg.P, K, N, T, F, SH)
    # the roofline uses the kernel's own duration: the solo probe (one stream, nothing else on the chip)
    # when there is one; the in-step event interval (which overlaps the other streams' kernels) is
    # reported beside it, labelled as such
    kernel_ms = solo_ms if solo_ms else avg_ms
    achieved = bytes_launch / (kernel_ms * 1e-3) / 1e9
    ms_per_step = elapsed / args.steps * 1e3
    # value: the median step (median of >= 20 reps) -- per-step device intervals
    # between the step-end events on the main stream; the mean over the timed region beside it
    value = views_per_step * cfg.P / (median_ms * 1e-3) / 1e6
    value_mean = views_per_step * cfg.P / (elapsed / args.steps) / 1e6
    pipe_b = pipeline_bytes(cfg.P, K, N, T, F, SH)
    pipe_gbps = pipe_b * views_per_step / world / (median_ms * 1e-3) / 1e9
    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            yaw, hgt = cfg.views[0]
            cam_cpu = S.render_settings(cfg.width, cfg.height, S.intrinsics(cfg.focal, cfg.width, cfg.height),
                                        S.look_at(yaw, hgt, cfg.distance), device="cpu",
                                        sh_degree=max(cfg.sh_degree, 0))
            if pinned:  # the CPU baseline gets the process's whole CPU share back
                splat_affinity.unpin_host_threads(affinity0)
            cpu = cpu_baseline_oracle(cfg, params_cpu, cam_cpu, dl.cpu(), args.cpu_threads)
            if pinned:
                splat_affinity.unpin_host_threads(pinned)
        workload = {
            "C2": f"C2: {cfg.P} Gaussians, RGB, {cfg.width}x{cfg.height}, the 4 cameras (yaw 0/90/180/270) "
                  f"per GPU per step, fwd+bwd" + (", RCCL SUM all-reduce of the gradients" if world > 1 else ""),
            "C3": f"C3: {cfg.P} Gaussians, SH{cfg.sh_degree}, {cfg.width}x{cfg.height}, 27-camera rig, "
                  f"{V} view(s)/GPU/step, fwd+bwd" + (", RCCL SUM all-reduce of the gradients" if world > 1 else ""),
            "C3M": f"C3M: C3 with half of the {cfg.P} means in 16 tight clusters (densified-scene stand-in), "
                   f"SH{cfg.sh_degree}, {cfg.width}x{cfg.height}, {V} view(s)/GPU/step, fwd+bwd",
            "C4": f"C4: {cfg.P} Gaussians, RGB, {cfg.width}x{cfg.height}, the 27-camera rig per step sharded "
                  f"round-robin over {world} GPU(s), fwd+bwd" + (", one RCCL SUM all-reduce" if world > 1 else ""),
            "C5": f"C5: {cfg.P} Gaussians x 150 frames, RGB, {cfg.width}x{cfg.height}, independent per-frame "
                  f"fits (own parameters + Adam state per frame), frames sharded in blocks over {world} GPU(s); "
                  f"one step = one optimisation iteration of every frame ({V} rig views fwd + fused L1/SSIM "
                  f"+ bwd + fused Adam); no collective",
        }[args.config]
        shape = ("view losses summed, one backward (deferred multi-view per-Gaussian pass)"
                 if args.step_shape == "summed" else "one backward per view")
        out = {
            "metric": "Msplats/sec fwd+bwd @1080p (1M gauss)" if args.config in ("C3", "C3M", "C4") else
                      "Msplats/sec fwd+bwd @800x800 (100k gauss, 4 cameras)" if args.config == "C2" else
                      "Msplats/sec fwd+bwd @1080p (2M gauss per-frame fits)",
            "value": round(value, 3), "unit": "Msplats/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
            "scaling": "strong" if args.config in ("C4", "C5") else "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic",
            "value_definition": "views x Gaussians / median step (device intervals between the step-end "
                                "events on the main stream; max over ranks)",
            "median_ms_per_step": round(median_ms, 4), "value_mean": round(value_mean, 3),
            "step_ms_quartiles": [round(float(np.percentile(step_ms, q)), 4) for q in (25, 50, 75)],
            "config": {"workload": workload, "gaussians": cfg.P, "views_per_step": views_per_step,
                       "views_per_gpu": [len(splat_dp.shard_views(list(range(views_per_step)), r, world))
                                         for r in range(world)],
                       "image": f"{cfg.width}x{cfg.height}", "sh_degree": cfg.sh_degree,
                       "mean_num_rendered": int(K), "max_tile_pairs": max_tile,
                       "parallelism": f"frame-dp{world}" if c5_cfg else f"camera-dp{world}",
                       "streams_per_gpu": len(streams),
                       "step_shape": "per frame: view losses summed, one backward, one Adam step" if c5_cfg else shape,
                       "submission": "one host thread per stream" if rstep.pool is not None else "one host thread",
                       "means2D": None if c5_cfg else ("one fresh zero leaf per render (shared.py:38-41)"
                                                       if args.means2d == "per-view" else "one leaf shared by the step's views"),
                       "backend": args.backend if dist is not None else None,
                       "host_cpus": pinned or "unpinned"},
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 2),
                         "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBPS, 5), "traffic": traffic,
                         "traffic_source": os.path.relpath(PMC_SUMMARY, REPO) if traffic else None,
                         "traffic_2x_fetch": traffic_2x,
                         "traffic_calibration": "profiles/r01_fetch_calib.txt" if traffic else None,
                         "avg_kernel_ms": round(kernel_ms, 5), "algorithmic_bytes": int(bytes_launch),
                         "duration_basis": ("solo probe: the kernel alone on one stream, HIP events on its launch "
                                            "stream inside libgsr" if solo_ms else "in-step event interval"),
                         # the interval between HIP events around the kernel inside the pipelined step: it
                         # overlaps the other streams' kernels, so it is not the kernel's own time
                         "in_step_interval_ms": round(avg_ms, 5),
                         "in_step_frac": round(bytes_launch / (avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 5),
                         "algorithmic_bytes_formula": {"render_bwd": "K*40 + N*20 + T*16",
                                                       "render_fwd": "K*44 + N*24 + T*16",
                                                       "gauss_bwd": "P*(84+F) + P*(56+F)"}.get(dom),
                         "binding_resource": "VALU issue (blend evaluations: ~256 pixel-Gaussian pairs per "
                                             "pair record); HBM traffic is a small share of the kernel time",
                         "valu": valu,
                         # the step's binding resource: every library kernel's wave64
                         # VALU instructions per step (profiled per launch) over the median step time, against
                         # one instruction per 2 cycles on every SIMD at 2.4 GHz
                         "valu_step": valu_step,
                         "valu_render_fwd": valu_fwd,
                         "pipeline": {"bytes_per_view": int(pipe_b),
                                      "formula": "P*(220 + 3F + 12*SH) + 120*K + 44*N + 16*T (SURVEY.md 8(d))",
                                      "achieved_GBps_per_gpu": round(pipe_gbps, 1),
                                      "frac": round(pipe_gbps / HBM_PEAK_GBPS, 4)}},
            "phase_ms_per_launch": {ph: round(probe[ph][0] / max(probe[ph][1], 1), 5) for ph in PHASES},
            "phase_ms_per_launch_solo": {ph: round(solo[ph][0] / max(solo[ph][1], 1), 5) for ph in PHASES}
            if solo else None,
            "host_ms_per_call": {ph: round(host[ph][0] / max(host[ph][1], 1), 5) for ph in host},
            "cpu_baseline": cpu,
            "unchanged_call_site": unchanged,
            "inference_call_site": inference,
            "c2": c2,
            "train_call_site": train_site,
            "call_site": call_site,
            "loss_call_site": loss_site,
            "densify_call_site": dens_site,
            "io_call_site": io_site,
            "grad_checksum": checksum,
        }
        print(json.dumps(out), flush=True)
    rstep.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
