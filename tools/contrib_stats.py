"""How many (pair, quarter) evaluations of the backward blend have no contributing pixel (diagnostic).

Runs the CPU oracle's forward on one C3 view and, for a sample of tiles, counts per (list entry,
16x4 quarter) whether any pixel passes the blend test geometrically (power <= 0, alpha >= 1/255:
what the tile cull + quarter maxima admit, up to the cull's margin) and whether any pixel actually
contributed in the forward (the same test AND entry < the pixel's n_contrib).  The ratio is what a
forward-recorded contributor mask would save the backward.  CPU only; minutes.

usage: python tools/contrib_stats.py [--config C3] [--tiles 300]
"""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "animating-gaussian-splats_amd"), REPO]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--tiles", type=int, default=300)
    args = ap.parse_args()
    import splat_scenes as S
    from oracle import oracle as O
    cfg = S.CONFIGS[args.config]
    p = S.synthetic_cloud(cfg.P, cfg.s0, sh_degree=cfg.sh_degree, seed=0, device="cpu")
    a = {k: (v.detach() if hasattr(v, "detach") else v) for k, v in S.activated_inputs(p, cfg.sh_degree).items()}
    rs = S.render_settings(cfg.width, cfg.height, S.intrinsics(cfg.focal, cfg.width, cfg.height),
                           S.look_at(0.0, 0.0, cfg.distance), device="cpu", sh_degree=max(cfg.sh_degree, 0))
    n = lambda k: a[k].numpy() if a.get(k) is not None else None  # noqa: E731
    st = O.forward(rs.bg.numpy(), a["means3D"].numpy(), n("colors_precomp"), a["opacities"].numpy(),
                   n("scales"), n("rotations"), rs.scale_modifier, None, rs.viewmatrix, rs.projmatrix,
                   rs.tanfovx, rs.tanfovy, rs.image_height, rs.image_width, n("shs"), rs.sh_degree,
                   rs.campos.numpy())
    W, H = st["W"], st["H"]
    gx = (W + 15) // 16
    ranges, pl, xy, co, nc = st["ranges"], st["point_list"], st["xy"], st["conic_opacity"], st["n_contrib"]
    T = ranges.shape[0]
    rng = np.random.default_rng(0)
    nonempty = np.nonzero(ranges[:, 1] > ranges[:, 0])[0]
    tiles = rng.choice(nonempty, size=min(args.tiles, len(nonempty)), replace=False)
    tot = dict(entries=0, pq_geom=0, pq_live=0, pairs_geom=0, pairs_live=0, pix_geom=0, pix_live=0)
    for t in tiles:
        r0, r1 = int(ranges[t, 0]), int(ranges[t, 1])
        tx, ty = t % gx, t // gx
        ys, xs = np.mgrid[ty * 16:ty * 16 + 16, tx * 16:tx * 16 + 16]
        inside = (xs < W) & (ys < H)
        lc = np.where(inside, nc[np.minimum(ys, H - 1), np.minimum(xs, W - 1)], 0).astype(np.int64)
        maxc = int(lc.max())
        if maxc == 0:
            continue
        g = pl[r0:r0 + maxc]
        dx = (xy[g, 0][:, None, None] - xs[None].astype(np.float32)).astype(np.float32)
        dy = (xy[g, 1][:, None, None] - ys[None].astype(np.float32)).astype(np.float32)
        A, B, C, o = (co[g, k][:, None, None] for k in range(4))
        power = (np.float32(-0.5) * (A * dx * dx + C * dy * dy) - B * dx * dy).astype(np.float32)
        alpha = np.minimum(np.float32(0.99), o * np.exp(power)).astype(np.float32)
        geom = (power <= 0) & (alpha >= np.float32(1 / 255)) & inside[None]
        pidx = np.arange(maxc)[:, None, None]
        live = geom & (pidx < lc[None])
        qmax = np.array([lc[4 * k:4 * k + 4].max() for k in range(4)])
        gq = geom.reshape(maxc, 4, 64).any(-1) & (pidx[:, :, 0] < qmax[None])
        lq = live.reshape(maxc, 4, 64).any(-1)
        tot["entries"] += maxc
        tot["pq_geom"] += int(gq.sum()); tot["pq_live"] += int(lq.sum())
        tot["pairs_geom"] += int(gq.any(1).sum()); tot["pairs_live"] += int(lq.any(1).sum())
        tot["pix_geom"] += int(geom.sum()); tot["pix_live"] += int(live.sum())
        # 8x8 blocks instead of 16x4 strips
        b8 = geom.reshape(maxc, 2, 8, 2, 8).transpose(0, 1, 3, 2, 4).reshape(maxc, 4, 64)
        lc8 = lc.reshape(2, 8, 2, 8).transpose(0, 2, 1, 3).reshape(4, 64).max(-1)
        tot["pq8_geom"] = tot.get("pq8_geom", 0) + int((b8.any(-1) & (pidx[:, :, 0] < lc8[None])).sum())
    print(tot)
    print("quarters per entry: geom %.3f live %.3f; pairs walked geom %.3f live %.3f; live/geom (pair,quarter) %.3f; 8x8 blocks per entry %.3f"
          % (tot["pq_geom"] / tot["entries"], tot["pq_live"] / tot["entries"], tot["pairs_geom"] / tot["entries"],
             tot["pairs_live"] / tot["entries"], tot["pq_live"] / max(tot["pq_geom"], 1), tot["pq8_geom"] / tot["entries"]))


if __name__ == "__main__":
    main()
