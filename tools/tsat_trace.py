"""Per-pixel timing of the exact T-saturation re-walk (k_render_tsat; diagnostic, needs
`make -C animating-gaussian-splats_amd/csrc trace`).  Renders the inference rig's 5 views (no_grad, 1280x720)
and one C3 view with tools/libgsr_trace.so and prints, per view: flagged pixels, the spread of their
start times, their durations and the slowest pixels' list lengths.  usage (GPU box): python tools/tsat_trace.py"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["GSR_LIB"] = os.environ.get("GSR_TRACE_LIB", os.path.join(REPO, "tools", "libgsr_trace.so"))
sys.path[:0] = [os.path.join(REPO, "animating-gaussian-splats_amd"), REPO]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def report(buf, T, label):
    a = buf[16 * T:].reshape(-1, 4).astype(np.int64)
    a = a[a[:, 0] > 0]
    if not len(a):
        print(f"[{label}] no flagged pixel")
        return
    t0 = a[:, 0].min()
    st, en = (a[:, 0] - t0) / 100.0, (a[:, 1] - t0) / 100.0
    dur = en - st
    nf, n = a[:, 2] & 0xFFFFFFFF, a[:, 2] >> 32
    chain = (a[:, 3] & 0xFFFFFFFF) / 100.0
    pct = lambda x: [round(float(np.percentile(x, q)), 1) for q in (50, 90, 99, 100)]  # noqa: E731
    print(f"[{label}] pixels {len(a)} span_us {en.max():.1f} start_us p50/90/99/max {pct(st)} "
          f"dur_us {pct(dur)} chain_us {pct(chain)} nf {pct(nf)} list {pct(n)}")
    k = np.argsort(-dur)[:6]
    print(f"[{label}] slowest: " + ", ".join(f"{dur[i]:.1f}us nf={nf[i]} n={n[i]} start={st[i]:.1f}" for i in k))
    c = np.corrcoef(nf, dur)[0, 1] if len(a) > 2 else float("nan")
    print(f"[{label}] corr(nf, dur) {c:.2f}; us per 64 entries (median) {np.median(dur / np.maximum(nf / 64, 1)):.2f}")


def main():
    import splat_scenes as S
    from diff_gaussian_rasterization import GaussianRasterizer, _C
    L = _C.load_library()
    L.gsr_debug_trace_fwd.argtypes = [ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    cfg = S.CONFIGS["C3"]
    params = S.synthetic_cloud(cfg.P, cfg.s0, sh_degree=-1, seed=0, device=dev)
    runs = [("inference", rs, S.INFERENCE_W, S.INFERENCE_H) for rs in S.inference_cameras(device=dev)]
    runs += [("C3", S.scene_cameras(cfg, device=dev)[0], cfg.width, cfg.height)]
    for k, (name, rs, W, H) in enumerate(runs):
        T = ((W + 15) // 16) * ((H + 15) // 16)
        buf = torch.zeros(32 * T, dtype=torch.int64, device=dev)
        with torch.no_grad():
            GaussianRasterizer(raster_settings=rs)(**S.render_arguments(params))  # warm-up
            torch.cuda.synchronize()
            assert L.gsr_debug_trace_fwd(buf.data_ptr()) == 0
            GaussianRasterizer(raster_settings=rs)(**S.render_arguments(params))
            torch.cuda.synchronize()
            L.gsr_debug_trace_fwd(None)
        report(buf.cpu().numpy(), T, f"{name} view {k}")


if __name__ == "__main__":
    main()
