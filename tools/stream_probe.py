"""Probe: step time of the bench workload with views alternating over S HIP streams (timing only --
without libgsr's cross-stream accumulation ordering, gradients of concurrent views may race)."""
import os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "animating-gaussian-splats_amd"), REPO]
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
for nstreams, summed in ((1, False), (2, False), (1, True), (2, True), (3, True)):
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(nstreams - 1)]
    main = torch.cuda.current_stream()
    def step(it):
        for s in streams[1:]:
            s.wait_stream(main)
        imgs = []
        for k in range(5):
            ci = (it * 5 + k) % len(cams)
            with torch.cuda.stream(streams[k % nstreams]):
                img, _, _ = GaussianRasterizer(raster_settings=cams[ci])(**leaves)
                if summed:
                    imgs.append(img)
                else:
                    img.backward(dl)
        if summed:  # train.py: the summed loss of the step's views, one backward
            torch.autograd.backward(imgs, [dl] * len(imgs))
        for s in streams[1:]:
            main.wait_stream(s)
        for p in leaves.values():
            p.grad = None
    for it in range(5):
        step(it)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for it in range(20):
        step(it)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / 20
    print(f"streams={nstreams} summed={summed} ms/step {dt*1e3:.3f}  Msplats/s {5*cfg.P/dt/1e6:.1f}", flush=True)
