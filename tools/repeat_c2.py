"""Run the C2 summed step (tests/test_repeatability.py's shape) N times in one process and count the
gradient values that differ from the first run (diagnostic).  usage (GPU box): python tools/repeat_c2.py [N]"""
import os
import sys

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(REPO, "animating-gaussian-splats_amd"), REPO, os.path.join(REPO, "tests")]
import torch  # noqa: E402

import splat_scenes as S  # noqa: E402
from test_repeatability import _step  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
cuda = torch.device("cuda", 0)
cfg = S.CONFIGS["C2"]
views = list(range(len(cfg.views)))
ref = _step(cfg, views, cuda, cfg.sh_degree)
for r in range(1, n):
    got = _step(cfg, views, cuda, cfg.sh_degree)
    dimg = sum(int((x != y).sum()) for x, y in zip(ref[0], got[0]))
    dg = {k: int((ref[1][k] != got[1][k]).sum()) for k in ref[1]}
    print(f"run {r}: image values differing {dimg}, gradients {dg}", flush=True)
