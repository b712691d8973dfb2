"""Which tiles make the render_fwd tail (diagnostic, CPU).

Runs the CPU oracle's forward on one view of a config and prints, per tile, the list length n, its rank in
the render's longest-first order, and the walk length -- the list position where the tile's last pixel is
done (its n_contrib when it saturates, the whole list when it never does): the forward's per-tile time is
about proportional to it (~0.1 us per entry for a quarter wave that still blends).  CPU; a minute or two.

usage: python tools/long_tiles.py [--config C3M] [--cam 0] [--top 25]
"""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "animating-gaussian-splats_amd"), REPO]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3M")
    ap.add_argument("--cam", type=int, default=0)
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--ranks", default="", help="also describe the tiles at these longest-first ranks")
    args = ap.parse_args()
    import splat_scenes as S
    from oracle import oracle as O
    base = S.CONFIGS["C3" if args.config == "C3M" else args.config]
    cfg = S.SceneConfig(base.name, base.P, base.width, base.height, base.focal, base.s0,
                        sh_degree=base.sh_degree, views=S.RIG27)
    gen = S.clustered_cloud if args.config == "C3M" else S.synthetic_cloud
    p = gen(cfg.P, cfg.s0, sh_degree=cfg.sh_degree, seed=0, device="cpu")
    a = {k: (v.detach() if hasattr(v, "detach") else v) for k, v in S.activated_inputs(p, cfg.sh_degree).items()}
    rs = S.scene_cameras(cfg, device="cpu")[args.cam]
    W, H = cfg.width, cfg.height
    shs = a["shs"].numpy() if cfg.sh_degree >= 0 else None
    col = None if cfg.sh_degree >= 0 else a["colors_precomp"].numpy()
    st = O.forward(rs.bg.numpy(), a["means3D"].numpy(), col, a["opacities"].numpy(), a["scales"].numpy(),
                   a["rotations"].numpy(), 1.0, None, rs.viewmatrix, rs.projmatrix, rs.tanfovx, rs.tanfovy, H, W,
                   shs, max(cfg.sh_degree, 0), rs.campos.numpy())
    rg = st["ranges"].astype(np.int64)
    n = rg[:, 1] - rg[:, 0]
    gx = (W + 15) // 16
    nc = st["n_contrib"].reshape(H, W).astype(np.int64)
    Tf = st["final_T"].reshape(H, W)
    walk = np.zeros(len(n), np.int64)
    for t in np.nonzero(n)[0]:
        ty, tx = divmod(int(t), gx)
        sl = (slice(16 * ty, min(16 * ty + 16, H)), slice(16 * tx, min(16 * tx + 16, W)))
        # saturated (stopped: its final T is the one before the stopping entry, in [1e-4, 1e-2) as alpha <= 0.99),
        # else it walks the whole list
        done = Tf[sl] < 1e-2
        walk[t] = int(np.where(done, nc[sl], n[t]).max())
    order = np.argsort(-n, kind="stable")
    rank = np.empty_like(order)
    rank[order] = np.arange(len(order))
    print(f"{args.config} cam {args.cam}: tiles {len(n)}, lists > 4096: {(n > 4096).sum()}, > 16384: {(n > 16384).sum()}, "
          f"longest {n.max()}, K {n.sum()}")
    for t in np.argsort(-walk)[: args.top]:
        print(f"tile {t:6d} rank {rank[t]:5d} n {n[t]:7d} walk {walk[t]:7d}")
    for r in [int(x) for x in args.ranks.split(",") if x]:
        t = int(order[r])
        ty, tx = divmod(t, gx)
        sl = (slice(16 * ty, min(16 * ty + 16, H)), slice(16 * tx, min(16 * tx + 16, W)))
        und = Tf[sl] >= 1e-2
        print(f"rank {r}: tile {t} n {n[t]} unsaturated pixels {und.sum()} (quarters "
              f"{[int(und[8 * (q >> 1):8 * (q >> 1) + 8, 8 * (q & 1):8 * (q & 1) + 8].sum()) for q in range(4)]}), "
              f"n_contrib max {nc[sl].max()} median {int(np.median(nc[sl]))}, final T min {Tf[sl].min():.3g} max {Tf[sl].max():.3g}")
    for thr in (1024, 2048, 4096, 8192):
        sel = walk > thr
        print(f"walk > {thr}: {sel.sum()} tiles, their n: min {n[sel].min() if sel.any() else 0}")


if __name__ == "__main__":
    main()
