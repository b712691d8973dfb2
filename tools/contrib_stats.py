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
        # 8x4 half-quarters (two per 8x8 quarter)
        b84 = geom.reshape(maxc, 4, 4, 2, 8).transpose(0, 1, 3, 2, 4).reshape(maxc, 8, 32)
        lc84 = lc.reshape(4, 4, 2, 8).transpose(0, 2, 1, 3).reshape(8, 32).max(-1)
        tot["pq84_geom"] = tot.get("pq84_geom", 0) + int((b84.any(-1) & (pidx[:, :, 0] < lc84[None])).sum())
        # backward split into two 16x8 halves walking their own lists in one wave: steps per 64-entry batch
        # = max over the halves of the entries each half walks (vs entries the whole tile walks)
        top = geom[:, :8, :].reshape(maxc, -1).any(-1) & (np.arange(maxc) < lc[:8].max())
        bot = geom[:, 8:, :].reshape(maxc, -1).any(-1) & (np.arange(maxc) < lc[8:].max())
        anyq = gq.any(1)
        steps = 0
        # 16x2 strips of each half (rows 2k, 2k+1): a lane's 4 pixels share a column
        st = geom.reshape(maxc, 2, 4, 2, 16).any(-1).any(-1)  # (entry, half, strip)
        lch = lc.reshape(2, 4, 2, 16).max(-1).max(-1)          # (half, strip) max n_contrib
        st = st & (np.arange(maxc)[:, None, None] < lch[None])
        ev = 0
        for b0 in range(0, maxc, 64):
            ia = [e for e in range(b0, min(b0 + 64, maxc)) if top[e]]
            ib = [e for e in range(b0, min(b0 + 64, maxc)) if bot[e]]
            steps += max(len(ia), len(ib))
            for t in range(max(len(ia), len(ib))):
                ma = st[ia[t], 0] if t < len(ia) else np.zeros(4, bool)
                mb = st[ib[t], 1] if t < len(ib) else np.zeros(4, bool)
                ev += int((ma | mb).sum())
        tot["half_evals"] = tot.get("half_evals", 0) + ev
        # forward: each 8x8 quarter's wave split into two 8x4 halves walking their own lists
        fs = 0
        h84 = b84.any(-1)  # (entry, 8 halves): index = 4-row block * 2 + 8-column block
        for q in range(4):
            qy, qx = q >> 1, q & 1
            i0, i1 = (2 * qy) * 2 + qx, (2 * qy + 1) * 2 + qx
            ha = h84[:, i0] & (np.arange(maxc) < lc84[i0])
            hb = h84[:, i1] & (np.arange(maxc) < lc84[i1])
            for b0 in range(0, maxc, 64):
                fs += max(int(ha[b0:b0 + 64].sum()), int(hb[b0:b0 + 64].sum()))
        tot["fwd_half_steps"] = tot.get("fwd_half_steps", 0) + fs
        tot["half_steps"] = tot.get("half_steps", 0) + steps
        tot["half_pairs"] = tot.get("half_pairs", 0) + int(top.sum() + bot.sum())
    print(tot)
    print("split-wave backward: half-pair walks per entry %.3f, wave steps per entry %.3f (now %.3f), "
          "strip evaluations per entry %.3f (now %.3f quarter evaluations)"
          % (tot["half_pairs"] / tot["entries"], tot["half_steps"] / tot["entries"], tot["pairs_geom"] / tot["entries"],
             tot["half_evals"] / tot["entries"], tot["pq_geom"] / tot["entries"]))
    print("forward with 8x4 half-waves: wave steps per entry %.3f (8x8 quarters now %.3f)"
          % (tot["fwd_half_steps"] / tot["entries"], tot["pq8_geom"] / tot["entries"]))
    print("quarters per entry: geom %.3f live %.3f; pairs walked geom %.3f live %.3f; live/geom (pair,quarter) %.3f; 8x8 blocks per entry %.3f, 8x4 halves per entry %.3f"
          % (tot["pq_geom"] / tot["entries"], tot["pq_live"] / tot["entries"], tot["pairs_geom"] / tot["entries"],
             tot["pairs_live"] / tot["entries"], tot["pq_live"] / max(tot["pq_geom"], 1), tot["pq8_geom"] / tot["entries"], tot["pq84_geom"] / tot["entries"]))


if __name__ == "__main__":
    main()
