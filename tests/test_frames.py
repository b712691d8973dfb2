"""Frame-sharded independent per-frame fits (splat_frames.FrameFits, bench.py --config C5) on the CPU
with a stand-in render / loss engine, world_size 2 over gloo: the 150 frames split into contiguous
blocks (75 + 75), every frame owns its parameter set and optimiser state, one step runs one
train.py:738-776 iteration of every frame of the rank's block, and no collective is issued
(per-frame fits are replicas with no exchange)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import splat_frames


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class _Cam:
    def __init__(self, w):
        self.w = w


def _render(p, cam):  # differentiable stand-in for the rasterizer: a 2x2 "image" of the parameters
    m = p["means"]
    return torch.stack([(m * cam.w).sum(), (p["log_scales"] * cam.w).sum(),
                        p["opacity_logits"].sum(), p["colors"].sum() * cam.w]).view(2, 2)


def _loss(img, tgt):
    return ((img - tgt) ** 2).mean()


def _base(P=6):
    g = torch.Generator().manual_seed(0)
    return {"means": torch.randn(P, 3, generator=g), "log_scales": torch.randn(P, 3, generator=g),
            "rotation_quaternions": torch.randn(P, 4, generator=g), "opacity_logits": torch.randn(P, 1, generator=g),
            "colors": torch.rand(P, 3, generator=g)}


def _fits(rank, world):
    cams = [_Cam(1.0 + 0.1 * k) for k in range(27)]
    return splat_frames.FrameFits(_base(), cams, rank, world, 5, _render, _loss,
                                  lambda p: torch.optim.Adam(list(p.values()), lr=1e-2), n_frames=150)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        fits = _fits(rank, world)

        def refuse(*a, **k):
            raise AssertionError("a per-frame fit step issued a collective")
        real = (dist.all_reduce, dist.broadcast, dist.all_gather)
        dist.all_reduce = dist.broadcast = dist.all_gather = refuse
        try:
            before = {t: {k: v.detach().clone() for k, v in fits.params[t].items()} for t in fits.frames}
            fits.step(0)
            fits.step(1)
        finally:
            dist.all_reduce, dist.broadcast, dist.all_gather = real
        moved = {t: float(sum((fits.params[t][k] - before[t][k]).abs().sum() for k in before[t])) for t in fits.frames}
        q.put((rank, list(fits.frames), moved,
               {t: {k: v.detach().numpy().copy() for k, v in fits.params[t].items()} for t in fits.frames[:2]}))
    finally:
        dist.destroy_process_group()


def test_frame_blocks_are_independent_fits_without_exchange():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        r, frames, moved, sample = q.get(timeout=120)
        res[r] = (frames, moved, sample)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0][0] == list(range(0, 75)) and res[1][0] == list(range(75, 150))
    for r in range(world):
        assert all(v > 0 for v in res[r][1].values()), "every frame of the block is optimised each step"
    # each frame's fit equals the same frame fitted alone in one process: independent of the split
    solo = _fits(0, 1)
    for r in range(world):
        for t, params in res[r][2].items():
            one = splat_frames.FrameFits(_base(), solo.cams, 0, 1, 5, _render, _loss,
                                         lambda p: torch.optim.Adam(list(p.values()), lr=1e-2), n_frames=150)
            one.frames = [t]
            one.step(0)
            one.step(1)
            for k in params:
                assert torch.equal(torch.from_numpy(params[k]), one.params[t][k].detach()), (t, k)


def test_frame_targets_and_views():
    fits = _fits(1, 8)
    assert fits.frames == list(range(19, 38))  # 150 = 19 x 6 + 18 x 2: rank 1's block
    assert len(fits.params) == 19 and len({id(p["means"]) for p in fits.params.values()}) == 19
    assert fits.frame_views(19) == [(19 * 5 + j) % 27 for j in range(5)]
    # targets: renders of each frame's displaced ground truth, made before the fit
    assert set(fits.targets) == {(t, ci) for t in fits.frames for ci in fits.frame_views(t)}
    t0 = splat_frames.frame_truth(_base(), fits.phi, 0, 150)["means"]
    assert torch.allclose(t0, _base()["means"] + 0.05 * torch.sin(fits.phi))
    t1 = splat_frames.frame_truth(_base(), fits.phi, 1, 150)["means"]
    assert not torch.equal(t0, t1)
