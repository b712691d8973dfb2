"""A/B of the unchanged train.py call shape (bench.py unchanged_call_site) and the headline step under
the round-4 switches, one configuration per process (GSR_ITEMS_AUX is read when libgsr loads).

usage (GPU box): python tools/callshape_probe.py NAME [--no-async] [--no-view-streams] [--steps N]
prints one JSON line: ms per step (median, quartiles) of the unchanged shape, and of the C2 leg."""
import argparse
import json
import os
import sys
import time

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(REPO, "animating-gaussian-splats_amd"), REPO]
import splat_affinity  # noqa: E402
splat_affinity.pin_host_threads(0, 0, 1, int(os.environ.get("GSR_PIN_CPUS", "8")))  # as bench.py does
import torch  # noqa: E402

import bench  # noqa: E402
import splat_dp  # noqa: E402
import splat_scenes as S  # noqa: E402
import diff_gaussian_rasterization as dgr  # noqa: E402
from diff_gaussian_rasterization import _C  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("name")
ap.add_argument("--no-async", action="store_true")
ap.add_argument("--no-view-streams", action="store_true")
ap.add_argument("--steps", type=int, default=30)
ap.add_argument("--c2", action="store_true")
ap.add_argument("--profile", action="store_true", help="per-phase device times + host wait inside the leg")
args = ap.parse_args()
dgr.set_async_forward(not args.no_async)
dgr.set_view_streams(not args.no_view_streams)
dev = torch.device("cuda", 0)
_C.load_library()
base = S.CONFIGS["C3"]
cfg = S.SceneConfig("C3", base.P, base.width, base.height, base.focal, base.s0, sh_degree=base.sh_degree,
                    views=S.RIG27)
cams = S.scene_cameras(cfg, device=dev)
dl = S.upstream_grad(cfg.height, cfg.width, device=dev)


def views_of(it):
    return splat_dp.shard_views([(it * 5 + k) % len(cams) for k in range(5)], 0, 1)


out = {"name": args.name, "async": not args.no_async, "view_streams": not args.no_view_streams,
       "items_aux": os.environ.get("GSR_ITEMS_AUX", "1")}
t0 = time.perf_counter()
if args.profile:
    _C.profile_reset()
    _C.profile_enable(True)
u = bench.unchanged_call_site(args.steps, 5, cfg, cams, views_of, dl, dev)
if args.profile:
    _C.profile_enable(False)
    out["phase_ms"] = {ph: round(v[0] / max(v[1], 1), 4) for ph in bench.PHASES + ["host_forward", "host_wait_K", "host_backward"]
                       for v in [_C.profile_read(ph)]}
out["wall_s"] = round(time.perf_counter() - t0, 2)
out["unchanged"] = {k: u[k] for k in ("Msplats_per_s", "median_ms_per_step", "step_ms_quartiles", "host_ms_per_step_median")}
if args.c2:
    c = bench.c2_leg(60, 10, dev)
    out["c2"] = {k: c[k] for k in ("Msplats_per_s", "median_ms_per_step", "step_ms_quartiles", "host_ms_per_step_median")}
print(json.dumps(out), flush=True)
