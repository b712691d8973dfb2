"""Step-time jitter probe (GPU box): the bench's default C3 step (RenderStep, 5 rig views, 3 streams,
threaded forwards, summed backward) for N steps, recording per step the host submission time and the
device interval between step-end events on the main stream; prints both distributions and how often
a slow device step follows a slow host step.  --gc: off | on | freeze (Python's cyclic collector)."""
import argparse
import gc
import os
import sys
import time

import numpy as np
import torch

sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "animating-gaussian-splats_amd"),
                os.path.join(os.path.dirname(__file__), "..")]
import splat_scenes as S  # noqa: E402
import splat_step  # noqa: E402
from diff_gaussian_rasterization import _C  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--gc", default="on", choices=["on", "off", "freeze"])
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    _C.load_library()
    cfg = S.CONFIGS["C3"]
    cfg = S.SceneConfig("C3", cfg.P, cfg.width, cfg.height, cfg.focal, cfg.s0, sh_degree=cfg.sh_degree, views=S.RIG27)
    p = S.synthetic_cloud(cfg.P, cfg.s0, sh_degree=3, seed=0, device=dev)
    with torch.no_grad():
        act = S.activated_inputs(p, 3)
    act.pop("colors_precomp")
    leaves = {k: v.detach().clone().requires_grad_(True) for k, v in act.items()}
    cams = S.scene_cameras(cfg, device=dev)
    dl = S.upstream_grad(cfg.height, cfg.width, device=dev)
    main_s = torch.cuda.current_stream(dev)
    streams = [torch.cuda.Stream(dev) for _ in range(3)]
    for s in streams:
        s.wait_stream(main_s)
    rstep = splat_step.RenderStep(dev, cams, lambda ci: leaves, dl, streams, threads=True)

    def step(it):
        rstep([(it * 5 + k) % len(cams) for k in range(5)])
        for s in streams:
            main_s.wait_stream(s)
        for v in leaves.values():
            v.grad = None

    for it in range(10):
        step(it)
    torch.cuda.synchronize()
    if a.gc == "off":
        gc.disable()
    elif a.gc == "freeze":
        gc.collect()
        gc.freeze()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps + 1)]
    host = []
    ev[0].record(main_s)
    for it in range(a.steps):
        t = time.perf_counter()
        step(10 + it)
        ev[it + 1].record(main_s)
        host.append((time.perf_counter() - t) * 1e3)
    torch.cuda.synchronize()
    dev_ms = np.array([ev[i].elapsed_time(ev[i + 1]) for i in range(a.steps)])
    host = np.array(host)
    rstep.close()
    q = lambda x: np.percentile(x, [10, 25, 50, 75, 90]).round(3).tolist()  # noqa: E731
    print(f"gc={a.gc} device ms: mean {dev_ms.mean():.3f} quantiles {q(dev_ms)}")
    print(f"gc={a.gc} host ms:   mean {host.mean():.3f} quantiles {q(host)}")
    slow = dev_ms > np.median(dev_ms) * 1.08
    print(f"slow device steps {slow.mean():.2f}; corr(host, device) {np.corrcoef(host, dev_ms)[0, 1]:.2f}; "
          f"Msplats/s mean {5e3 / dev_ms.mean():.1f} median {5e3 / np.median(dev_ms):.1f}")
    print("first 40 device ms:", dev_ms[:40].round(2).tolist())
    print("first 40 host ms:  ", host[:40].round(2).tolist())


if __name__ == "__main__":
    main()
