"""Repro of tests/test_async_forward.py::test_speculative_render_half_bitwise[True] (diagnostic, GPU).

Renders the test's 5 views of a denser cloud (scales x3) with blocking forwards (twice) and with
asynchronous forwards whose speculation fails (several times, spec render halves on and off), and reports
per gradient the max difference to the first blocking run and the number of differing Gaussians.

usage (GPU box): python tools/spec_half_repro.py [--reps 4]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "animating-gaussian-splats_amd"), REPO]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--halves", default="1,0", help="spec_half settings to run (1 = on, 0 = held back)")
    ap.add_argument("--history-scale", type=float, default=1.0,
                    help="scale of the blocking step that sets the pair-count history (3.0: every speculation stands)")
    ap.add_argument("--views", type=int, default=5)
    ap.add_argument("--no-busy", action="store_true")
    ap.add_argument("--blocking", action="store_true", help="the measured step with blocking forwards too")
    ap.add_argument("--stash", action="store_true",
                    help="keep every render half's SUMS (no synchronisation) and compare them after the step")
    ap.add_argument("--nofresh", action="store_true", help="zero-filled gradient targets (_defer['fresh'] off)")
    ap.add_argument("--views-twice", action="store_true",
                    help="after the per-Gaussian pass, synchronise and run it again into zeroed targets, compare")
    ap.add_argument("--hold", default="", help="keep extra references: 'fwd' (every _C._forward result), "
                    "'half' (every render half's return), 'both'")
    ap.add_argument("--probe", action="store_true",
                    help="in the end-of-pass callback, redo every held-back render half after a device "
                         "synchronisation and compare the two SUMS buffers")
    args = ap.parse_args()
    import splat_scenes as S
    import diff_gaussian_rasterization as dgr
    from diff_gaussian_rasterization import GaussianRasterizer, _C
    cuda = torch.device("cuda", 0)
    P, W, H = 80_000, 480, 320
    base = S.synthetic_cloud(P, 0.01, seed=7, device=cuda)
    cams = [S.render_settings(W, H, S.intrinsics(400.0, W, H), S.look_at(yaw, 0.2, 8.0), device=cuda)
            for yaw in (0, 72, 144, 216, 288)][: args.views]
    dl = S.upstream_grad(H, W, device=cuda)
    with torch.no_grad():
        act = S.activated_inputs(base, -1)

    def step(scale, busy):
        leaves = {k: v.detach().clone().requires_grad_(True) for k, v in act.items()}
        with torch.no_grad():
            leaves["scales"].mul_(scale)
        if busy:
            torch.cuda._sleep(50_000_000)
        if args.probe:
            print(f"  forward stream {torch.cuda.current_stream().cuda_stream:#x}", flush=True)
        imgs = [GaussianRasterizer(raster_settings=rs)(**dict(leaves, means2D=torch.zeros_like(
            leaves["means3D"], requires_grad=True)))[0] for rs in cams]
        torch.stack([(i * dl).sum() for i in imgs]).sum().backward()
        torch.cuda.synchronize()
        return [i.detach() for i in imgs], {k: v.grad for k, v in leaves.items() if v.grad is not None}

    with torch.no_grad():  # visibility in any view (radii > 0 of a blocking forward at scale 3)
        lv = {k: v.detach().clone() for k, v in act.items()}
        lv["scales"].mul_(3.0)
        vis = torch.zeros(P, dtype=torch.bool, device=cuda)
        for rs in cams:
            vis |= GaussianRasterizer(raster_settings=rs)(**dict(lv, means2D=torch.zeros_like(lv["means3D"])))[1] > 0
    print(f"visible in some view: {int(vis.sum())} of {P}", flush=True)
    if args.nofresh:
        dgr._defer["fresh"] = False
    if args.views_twice:
        orig_views = _C.rasterize_gaussians_backward_views

        def views_twice(views, *a, accumulate_into=None, overwrite=(), needed=None, **k):
            r = orig_views(views, *a, accumulate_into=accumulate_into, overwrite=overwrite, needed=needed, **k)
            torch.cuda.synchronize()
            first = [None if t is None else t.clone() for t in accumulate_into]
            fresh = [None if t is None else torch.zeros_like(t) for t in accumulate_into]
            vs = [dict(v, means2D_grad=None) for v in views]
            orig_views(vs, *a, accumulate_into=fresh, overwrite=(), needed=needed, **k)
            torch.cuda.synchronize()
            d = [None if f is None else float((f - g).abs().nan_to_num(1e30).max()) for f, g in zip(first, fresh)]
            print(f"  views pass: {len(views)} views, K {[v['num_rendered'] for v in views]}; again after a sync "
                  f"into zeroed targets, max diff per slot {d}", flush=True)
            return r
        _C.rasterize_gaussians_backward_views = views_twice

    def cmp(label, ref, got):
        im = all(torch.equal(x, y) for x, y in zip(ref[0], got[0]))
        parts = []
        for k in ref[1]:
            d = (ref[1][k] - got[1][k]).abs().nan_to_num(1e30)
            bad = d.reshape(d.shape[0], -1).amax(1) > 0
            nd = int(bad.sum())
            parts.append(f"{k}: max {float(d.max()):.3g} n {nd} (visible {int((bad & vis).sum())})")
        print(f"{label}: images equal {im}; " + "; ".join(parts), flush=True)

    if args.probe:
        orig = dgr._run_group
        orig_defer = dgr._try_defer
        snaps = []

        def cells(fn, depth=0):  # the tensors a closure holds (two levels: render_half -> args_kw)
            out = []
            for c in (fn.__closure__ or ()):
                try:
                    x = c.cell_contents
                except ValueError:
                    continue
                if isinstance(x, torch.Tensor):
                    out.append(x)
                elif callable(x) and depth < 1 and getattr(x, "__closure__", None):
                    out += cells(x, depth + 1)
            return out

        def spy(ctx, gauss, radii, geomBuffer, leaf_inputs, nodes, need, render_fn, keep=()):
            ts = cells(render_fn)
            snaps.append([(t, t.detach().clone()) for t in ts if t.is_cuda])
            return orig_defer(ctx, gauss, radii, geomBuffer, leaf_inputs, nodes, need, render_fn, keep)
        dgr._try_defer = spy

        def probed(grp, created, post):
            print(f"  callback: current stream {torch.cuda.current_stream().cuda_stream:#x}", flush=True)
            torch.cuda.synchronize()
            for k, sn in enumerate(snaps):
                bad = [(tuple(t.shape), float((t.float() - c.float()).abs().max())) for t, c in sn
                       if t.shape == c.shape and not torch.equal(t, c)]
                print(f"  view {k}: {len(sn)} closure tensors, changed since the backward: {bad}", flush=True)
            snaps.clear()
            for v in grp["views"]:
                fn = v.get("render_fn")
                if v.get("scratch") is None and fn is not None:
                    def wrapped(fn=fn, v=v):
                        print(f"  view stream {v['stream']:#x}; pending ready before: "
                              f"{v.get('spec') is None}", flush=True)
                        sc, K = fn()
                        first = sc.clone()
                        torch.cuda.synchronize()
                        again = sc.clone()
                        sc2, K2 = fn()
                        torch.cuda.synchronize()
                        print(f"  render half K {K}/{K2}: first vs after sync equal {torch.equal(first, again)}; "
                              f"vs a second half {torch.equal(again, sc2)}", flush=True)
                        return sc, K
                    v["render_fn"] = wrapped
            return orig(grp, created, post)
        dgr._run_group = probed
    held = []
    if args.hold in ("fwd", "both"):
        orig_fwd = _C._forward

        def fwd_hold(*a, **k):
            r = orig_fwd(*a, **k)
            held.append(r)
            return r
        _C._forward = fwd_hold
    if args.hold in ("half", "both"):
        for name in ("rasterize_gaussians_backward_render",):
            orig_h = getattr(_C, name)

            def half_hold(*a, _o=orig_h, **k):
                r = _o(*a, **k)
                held.append((a, k, r))
                return r
            setattr(_C, name, half_hold)
    stash = []
    if args.stash:
        orig_defer2 = dgr._try_defer

        def spy2(ctx, gauss, radii, geomBuffer, leaf_inputs, nodes, need, render_fn, keep=()):
            def wrapped(spec=False, fn=render_fn, radii=radii):
                sc, K = fn(spec)
                stash.append((spec, K, sc, radii))
                return sc, K
            return orig_defer2(ctx, gauss, radii, geomBuffer, leaf_inputs, nodes, need, wrapped, keep)
        dgr._try_defer = spy2
    ref_sums = {}

    def check_sums(label):
        for spec, K, sc, radii in stash:
            f = sc.view(torch.float32)[: 9 * P]
            key = (int(radii.sum()),)
            if key not in ref_sums:
                ref_sums[key] = f.clone()
                print(f"  {label}: SUMS reference for radii sum {key[0]} (K {K})", flush=True)
            else:
                r = ref_sums[key]
                print(f"  {label}: SUMS (spec {spec}, K {K}) vs reference: equal {torch.equal(r, f)}, "
                      f"NaNs {int(f.isnan().sum())}, differing {int((r != f).sum())}", flush=True)
        stash.clear()
    prev_async, prev_half = dgr.set_async_forward(False), dgr._defer["spec_half"]
    try:
        ref = step(3.0, False)
        check_sums("ref")
        cmp("blocking again", ref, step(3.0, False))
        cmp("blocking, busy", ref, step(3.0, True))
        for half in [h == "1" for h in args.halves.split(",")]:
            dgr._defer["spec_half"] = half
            for r in range(args.reps):
                dgr.set_async_forward(False)
                _C.speculation_stats(reset=True)
                step(args.history_scale, False)
                dgr.set_async_forward(not args.blocking)
                q0, r0 = dgr._spec_half_stats["queued"], dgr._spec_half_stats["redone"]
                stash.clear()
                got = step(3.0, not args.no_busy)
                check_sums(f"rep {r}")
                q, rd = dgr._spec_half_stats["queued"] - q0, dgr._spec_half_stats["redone"] - r0
                cmp(f"{'blocking' if args.blocking else 'async'} spec_half={half} rep {r} (halves queued {q}, redone {rd}, "
                    f"spec stats {_C.speculation_stats()})", ref, got)
    finally:
        dgr.set_async_forward(prev_async)
        dgr._defer["spec_half"] = prev_half


if __name__ == "__main__":
    main()
