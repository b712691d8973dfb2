"""The C2 summed step's gradients with gsr_bind's forward against the ctypes forward (diagnostic):
one stream / three streams with threads, speculation history fresh each time.  usage (GPU box)"""
import os
import sys

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(REPO, "animating-gaussian-splats_amd"), REPO]
import torch  # noqa: E402

import splat_scenes as S  # noqa: E402
import splat_step  # noqa: E402
from diff_gaussian_rasterization import _C  # noqa: E402

cuda = torch.device("cuda", 0)
cfg = S.CONFIGS["C2"]
p = S.synthetic_cloud(cfg.P, cfg.s0, sh_degree=-1, seed=0, device=cuda)
with torch.no_grad():
    act = S.activated_inputs(p, -1)
cams = S.scene_cameras(cfg, device=cuda)
dl = S.upstream_grad(cfg.height, cfg.width, device=cuda)


def step(ns, threads, parts, reps):
    _C._NATIVE_PARTS = parts
    _C.speculation_stats(reset=True)
    out = []
    for _ in range(reps):
        leaves = {k: v.detach().clone().requires_grad_(True) for k, v in act.items()}
        streams = [torch.cuda.Stream() for _ in range(ns)]
        for s in streams:
            s.wait_stream(torch.cuda.current_stream())
        st = splat_step.RenderStep(cuda, cams, lambda ci: leaves, dl, streams, threads=threads)
        try:
            st(list(range(len(cams))))
        finally:
            st.close()
        torch.cuda.synchronize()
        out.append({k: v.grad.clone() for k, v in leaves.items()})
    return out


for ns, threads in ((1, False), (3, False), (3, True)):
    ref = step(ns, threads, 0, 3)
    for parts in (1, 2, 4):
        got = step(ns, threads, parts, 3)
        d = [{k: int((r[k] != g[k]).sum()) for k in r if int((r[k] != g[k]).sum())} for r, g in zip(ref, got)]
        print(f"streams {ns} threads {threads} parts {parts}: per rep differing {d}", flush=True)
