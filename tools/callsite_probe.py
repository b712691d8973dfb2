"""The train.py call-site leg of bench.py alone (GPU box), for rocprofv3: RGB or SH3 features,
N steps of 5 views each (bench.train_call_site).  usage: python tools/callsite_probe.py [--sh] [--steps N]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402  (puts the package on sys.path)
import torch  # noqa: E402

import splat_dp  # noqa: E402
import splat_scenes as S  # noqa: E402
from diff_gaussian_rasterization import _C  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sh", action="store_true")
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    _C.load_library()
    base = S.CONFIGS["C3"]
    cfg = S.SceneConfig("C3", base.P, base.width, base.height, base.focal, base.s0, sh_degree=base.sh_degree,
                        views=S.RIG27)
    cams = S.scene_cameras(cfg, device=dev)
    dl = S.upstream_grad(cfg.height, cfg.width, device=dev)
    streams = [torch.cuda.Stream(dev) for _ in range(3)]

    def views_of(it):
        return splat_dp.shard_views([(it * 5 + k) % len(cams) for k in range(5)], 0, 1)
    r = bench.train_call_site(a.steps, cfg, cams, views_of, dl, dev, streams, a.sh)
    print(r)


if __name__ == "__main__":
    main()
