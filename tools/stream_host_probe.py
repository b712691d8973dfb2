"""Probe: host time of each rasterizer call in the bench step with views over S streams."""
import os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "animating-gaussian-splats_amd"), REPO]
import numpy as np
import torch
import splat_scenes as S
from diff_gaussian_rasterization import GaussianRasterizer, _C

dev = torch.device("cuda", 0)
_C.load_library()
base = S.CONFIGS["C3"]
cfg = S.SceneConfig(base.name, base.P, base.width, base.height, base.focal, base.s0, sh_degree=base.sh_degree, views=S.RIG27)
params = S.synthetic_cloud(cfg.P, cfg.s0, sh_degree=cfg.sh_degree, seed=0, device="cpu")
with torch.no_grad():
    act = S.activated_inputs({k: v.to(dev) for k, v in params.items()}, cfg.sh_degree)
act.pop("colors_precomp")
leaves = {k: v.detach().clone().requires_grad_(True) for k, v in act.items()}
cams = S.scene_cameras(cfg, device=dev)
dl = S.upstream_grad(cfg.height, cfg.width, device=dev)
nstreams = int(sys.argv[1]) if len(sys.argv) > 1 else 2
main = torch.cuda.current_stream()
streams = [main] + [torch.cuda.Stream() for _ in range(nstreams - 1)]
rec = []
def step(it, log):
    t_s = time.perf_counter()
    for s in streams[1:]:
        s.wait_stream(main)
    for k in range(5):
        ci = (it * 5 + k) % len(cams)
        with torch.cuda.stream(streams[k % nstreams]):
            t0 = time.perf_counter()
            img, _, _ = GaussianRasterizer(raster_settings=cams[ci])(**leaves)
            t1 = time.perf_counter()
            img.backward(dl)
            t2 = time.perf_counter()
        if log:
            rec.append((k, t1 - t0, t2 - t1))
    for s in streams[1:]:
        main.wait_stream(s)
    t3 = time.perf_counter()
    for p in leaves.values():
        p.grad = None
    t4 = time.perf_counter()
    if log:
        rec.append((9, t3 - t_s, t4 - t3))
for it in range(5):
    step(it, False)
torch.cuda.synchronize()
t = time.perf_counter()
for it in range(20):
    step(it, True)
torch.cuda.synchronize()
print("ms/step", (time.perf_counter() - t) / 20 * 1e3)
r = np.array(rec)
for k in list(range(5)) + [9]:
    m = r[r[:, 0] == k]
    print(k, "fwd ms mean %.3f max %.3f | bwd ms mean %.3f max %.3f" % (m[:, 1].mean() * 1e3, m[:, 1].max() * 1e3, m[:, 2].mean() * 1e3, m[:, 2].max() * 1e3))
