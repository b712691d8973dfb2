"""Per-wave timing of the render kernels (diagnostic; needs `make -C animating-gaussian-splats_amd/csrc trace`).

Loads tools/libgsr_trace.so (render kernels stamp (start, end, HW_ID) per wave with s_memrealtime,
100 MHz) instead of libgsr.so, renders the bench workload's views once each (forward + backward)
and prints, per kernel: span, wave-duration percentiles, the active-wave profile over time and the
tail (time from 90 % of waves finished to the last one).  Output: stdout + gpurun_out/render_trace.json.

usage (GPU box): python tools/render_trace.py [--config C3] [--cams 5,6,7,8]
"""
import argparse
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["GSR_LIB"] = os.environ.get("GSR_TRACE_LIB", os.path.join(REPO, "tools", "libgsr_trace.so"))
sys.path[:0] = [os.path.join(REPO, "animating-gaussian-splats_amd"), REPO]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def analyse(buf, n_waves, label):
    a = buf[: 4 * n_waves].reshape(n_waves, 4).astype(np.int64)
    a = a[a[:, 0] > 0]
    if not len(a):
        return {}
    t0 = a[:, 0].min()
    st, en = (a[:, 0] - t0) / 100.0, (a[:, 1] - t0) / 100.0  # microseconds
    dur = en - st
    span = en.max()
    order = np.sort(en)
    t90 = order[int(0.9 * (len(order) - 1))]
    bins = np.linspace(0, span, 21)
    active = [int(((st < b1) & (en > b0)).sum()) for b0, b1 in zip(bins[:-1], bins[1:])]
    out = {"waves": int(len(a)), "span_us": round(float(span), 1),
           "dur_us_p50_p90_max": [round(float(np.percentile(dur, q)), 1) for q in (50, 90, 100)],
           "mean_dur_us": round(float(dur.mean()), 1),
           "sum_dur_over_span": round(float(dur.sum() / span), 1),
           "t90_us": round(float(t90), 1), "tail_us": round(float(span - t90), 1),
           "last_start_us": round(float(st.max()), 1), "active_waves_per_20th": active}
    print(f"[{label}] " + json.dumps(out))
    return out


def analyse_emit(buf, label):
    """k_bin_emit per-block stamps (start, LDS count done, slabs reserved, end), microseconds."""
    a = buf.reshape(-1, 4).astype(np.int64)
    a = a[a[:, 0] > 0]
    if not len(a):
        return {}
    t0 = a[:, 0].min()
    rel = (a - t0) / 100.0
    ph = np.diff(rel, axis=1)  # count, reserve, scatter
    pct = lambda x: [round(float(np.percentile(x, q)), 1) for q in (50, 90, 100)]  # noqa: E731
    out = {"blocks": int(len(a)), "span_us": round(float(rel[:, 3].max()), 1),
           "start_us_p50_p90_max": pct(rel[:, 0]), "count_us": pct(ph[:, 0]), "reserve_us": pct(ph[:, 1]),
           "scatter_us": pct(ph[:, 2])}
    print(f"[{label}] " + json.dumps(out))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--cams", default="5,6,7,8")
    args = ap.parse_args()
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    import splat_scenes as S
    from diff_gaussian_rasterization import GaussianRasterizer, _C
    L = _C.load_library()
    dev = torch.device("cuda", 0)
    base = S.CONFIGS["C3" if args.config == "C3M" else args.config]
    cfg = S.SceneConfig(base.name, base.P, base.width, base.height, base.focal, base.s0,
                        sh_degree=base.sh_degree, views=S.RIG27)
    gen = S.clustered_cloud if args.config == "C3M" else S.synthetic_cloud
    params = {k: v.to(dev) for k, v in gen(cfg.P, cfg.s0, sh_degree=cfg.sh_degree, seed=0, device="cpu").items()}
    with torch.no_grad():
        act = S.activated_inputs(params, cfg.sh_degree)
    if cfg.sh_degree >= 0:
        act.pop("colors_precomp")
    leaves = {k: v.detach().clone().requires_grad_(True) for k, v in act.items()}
    cams = S.scene_cameras(cfg, device=dev)
    dl = S.upstream_grad(cfg.height, cfg.width, device=dev)
    T = ((cfg.width + 15) // 16) * ((cfg.height + 15) // 16)
    fbuf = torch.zeros(2 * 4 * 4 * T, dtype=torch.int64, device=dev)  # the view's launch, then k_render_fwd_long
    bbuf = torch.zeros(4 * 16 * T, dtype=torch.int64, device=dev)  # (tile, segment) items
    L.gsr_debug_trace_fwd.argtypes = [ctypes.c_void_p]
    L.gsr_debug_trace_bwd.argtypes = [ctypes.c_void_p]
    L.gsr_debug_trace_emit.argtypes = [ctypes.c_void_p]
    ebuf = torch.zeros(4 * 4096, dtype=torch.int64, device=dev)
    for ci in [int(c) for c in args.cams.split(",")]:  # warm-up
        GaussianRasterizer(raster_settings=cams[ci])(**leaves)[0].backward(dl)
    torch.cuda.synchronize()
    report = {}
    for ci in [int(c) for c in args.cams.split(",")]:
        fbuf.zero_(); bbuf.zero_(); ebuf.zero_()
        assert L.gsr_debug_trace_fwd(fbuf.data_ptr()) == 0 and L.gsr_debug_trace_bwd(bbuf.data_ptr()) == 0
        assert L.gsr_debug_trace_emit(ebuf.data_ptr()) == 0
        img, radii, _ = GaussianRasterizer(raster_settings=cams[ci])(**leaves)
        img.backward(dl)
        torch.cuda.synchronize()
        L.gsr_debug_trace_fwd(None); L.gsr_debug_trace_bwd(None); L.gsr_debug_trace_emit(None)
        np.save(os.path.join(REPO, "gpurun_out", f"trace_bwd_cam{ci}.npy"), bbuf.cpu().numpy())
        np.save(os.path.join(REPO, "gpurun_out", f"trace_fwd_cam{ci}.npy"), fbuf.cpu().numpy())
        report[ci] = {"emit": analyse_emit(ebuf.cpu().numpy(), f"cam{ci} emit"),
                      "fwd": analyse(fbuf.cpu().numpy(), 8 * T, f"cam{ci} fwd"),
                      "fwd_view": analyse(fbuf.cpu().numpy(), 4 * T, f"cam{ci} fwd view launch"),
                      "fwd_long": analyse(fbuf.cpu().numpy()[16 * T:], 4 * T, f"cam{ci} fwd long lists"),
                      "bwd": analyse(bbuf.cpu().numpy(), 16 * T, f"cam{ci} bwd")}
    out = os.path.join(REPO, "gpurun_out")
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, "render_trace.json"), "w") as f:
        json.dump(report, f, indent=1)


if __name__ == "__main__":
    main()
