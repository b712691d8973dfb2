"""Camera / frame data parallelism around the rasterizer (BASELINE.json north_star).

The reference is single-process.  Its training steps SUM the losses of several
views before one backward (train.py:413-418: ``losses.sum(dim=0)``), and densify.py accumulates
per-view screen-space gradient norms and visibility counts (external.py:113-124) and the maximum
radii (densify.py:154-162).  Sharding the views of a step over ranks and all-reducing therefore
reproduces the single-process result exactly (up to summation order):

* ``shard_views``      round-robin camera sharding (27-camera rig over 8 ranks -> 4,4,4,3,3,3,3,3)
* ``shard_frames``     contiguous frame blocks for independent per-frame fits (replicas, no exchange)
* ``GradAllReduce``    ONE flat-bucket all-reduce (SUM) of the Gaussian-parameter gradients per step
                       over RCCL (``backend="nccl"``) / gloo; either packs ``.grad`` into a reused
                       bucket, or (``attach``) keeps the gradients IN the bucket so backward
                       accumulates into it and the collective runs in place
* ``DensifyStats``     per-rank view-level accumulation of the densify statistics with the
                       reference's own formulas, then SUM (norm accumulator, visibility count) / MAX
                       (radii) reductions before the clone/split/prune decision, so every rank takes
                       identical densification decisions
* ``broadcast_normal`` the split samples (external.py:260-261 ``torch.normal``) drawn on one rank and
                       broadcast, so the split copies -- and from then on every parameter -- stay
                       identical on all ranks
* ``densify_gaussians`` the DP densification step: all-reduced statistics + broadcast samples around
                       ``splat_densify.densify_gaussians``

The data path has exactly one collective per step (the gradient all-reduce); the densify-stat
reduction runs only when densification happens (every 100 iterations in densify.py).
"""
from __future__ import annotations

from typing import Iterable, Sequence

import torch
import torch.distributed as dist


def shard_views(views: Sequence, rank: int, world: int) -> list:
    """Round-robin shard of a camera list (rank r gets views r, r + world, ...)."""
    return list(views[rank::world])


def shard_frames(n_frames: int, rank: int, world: int) -> range:
    """Contiguous block of frames for this rank (sizes differ by at most one)."""
    q, r = divmod(n_frames, world)
    start = rank * q + min(rank, r)
    return range(start, start + q + (1 if rank < r else 0))


class GradAllReduce:
    """Sum the gradients of ``params`` over ranks with one flat-bucket all-reduce per step.

    The flat bucket (one contiguous fp32 buffer, allocated on first use and reused) makes the step's
    exchange a single large collective, which is what RCCL's ring/direct algorithms over xGMI run
    at link rate; small per-tensor collectives would be latency bound.
    """

    def __init__(self, params: Iterable[torch.Tensor], group=None):
        self.params = list(params)
        self.group = group
        self.flat = None
        self.work = None

    def _pack(self):
        n = sum(p.numel() for p in self.params)
        dev = self.params[0].device
        if self.flat is None or self.flat.numel() != n or self.flat.device != dev:
            self.flat = torch.empty(n, dtype=torch.float32, device=dev)
        o = 0
        for p in self.params:
            k = p.numel()
            if p.grad is None:
                self.flat[o:o + k].zero_()
            else:
                self.flat[o:o + k].copy_(p.grad.reshape(-1))
            o += k

    def _unpack(self):
        o = 0
        for p in self.params:
            k = p.numel()
            if p.grad is None:
                p.grad = torch.empty_like(p)
            p.grad.copy_(self.flat[o:o + k].view_as(p))
            o += k

    def start(self):
        """Pack the local gradients and launch the all-reduce (asynchronously)."""
        self._pack()
        if dist.is_initialized() and dist.get_world_size(self.group) > 1:
            self.work = dist.all_reduce(self.flat, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        return self

    def finish(self):
        """Wait for the collective and write the summed gradients back into ``p.grad``."""
        if self.work is not None:
            self.work.wait()
            self.work = None
        self._unpack()

    def __call__(self):
        self.start().finish()

    # ---- in-place mode: the gradients live in the bucket (no pack / unpack copies) ----
    def attach(self):
        """Make every ``p.grad`` a view of the flat bucket (zeroed).  Autograd then accumulates each
        backward straight into the bucket, ``reduce()`` all-reduces it in place and ``zero_()``
        clears it for the next step -- 2 x bucket bytes less HBM traffic per step than pack/unpack."""
        n = sum(p.numel() for p in self.params)
        dev = self.params[0].device
        self.flat = torch.zeros(n, dtype=torch.float32, device=dev)
        o = 0
        for p in self.params:
            k = p.numel()
            p.grad = self.flat[o:o + k].view_as(p)
            o += k
        return self

    def reduce(self):
        """In-place SUM all-reduce of the attached bucket (synchronous on the current stream)."""
        if dist.is_initialized() and dist.get_world_size(self.group) > 1:
            dist.all_reduce(self.flat, op=dist.ReduceOp.SUM, group=self.group)

    def zero_(self):
        self.flat.zero_()


class DensifyStats:
    """Densification statistics of densify.py / external.py, accumulated per view on each rank.

    ``update(radii, means2D_grad)`` applies, for one rendered view, the reference's
    update_max_2d_radii_and_visibility_mask (densify.py:154-162) and accumulate_mean_2d_gradients
    (external.py:113-124): for Gaussians with radii > 0, max_2d_radii = max(radii, max_2d_radii),
    grad_accum += ||means2D.grad[:, :2]||, visibility_count += 1.  ``allreduce()`` combines the
    ranks (SUM, SUM, MAX) so that every rank holds the statistics of all views.
    """

    def __init__(self, P: int, device):
        self.visibility_count = torch.zeros(P, device=device)
        self.mean_2d_gradients_accumulated = torch.zeros(P, device=device)
        self.max_2d_radii = torch.zeros(P, device=device)

    def update(self, radii: torch.Tensor, means2D_grad: torch.Tensor):
        vis = radii > 0
        self.max_2d_radii[vis] = torch.max(radii[vis].to(self.max_2d_radii.dtype), self.max_2d_radii[vis])
        self.mean_2d_gradients_accumulated[vis] += torch.norm(means2D_grad[vis, :2], dim=-1)
        self.visibility_count[vis] += 1

    def allreduce(self, group=None):
        if not (dist.is_initialized() and dist.get_world_size(group) > 1):
            return self
        packed = torch.stack([self.mean_2d_gradients_accumulated, self.visibility_count])
        dist.all_reduce(packed, op=dist.ReduceOp.SUM, group=group)
        self.mean_2d_gradients_accumulated.copy_(packed[0])
        self.visibility_count.copy_(packed[1])
        dist.all_reduce(self.max_2d_radii, op=dist.ReduceOp.MAX, group=group)
        return self


def broadcast_normal(group=None, src: int = 0):
    """A ``sample_fn`` for ``splat_densify.densify_gaussians``: ``torch.normal(mean, std)`` drawn on
    rank ``src`` only and broadcast to every rank.  The reference draws the split offsets with an
    unseeded ``torch.normal`` (external.py:260-261); drawn independently per rank they would make the
    replicas' split copies -- and every later gradient -- diverge."""
    def draw(mean, std):
        if not (dist.is_initialized() and dist.get_world_size(group) > 1):
            return torch.normal(mean=mean, std=std)
        out = torch.normal(mean=mean, std=std) if dist.get_rank(group) == src else torch.empty_like(std)
        dist.broadcast(out, src=src, group=group)
        return out
    return draw


def densify_gaussians(params, stats: "DensifyStats", scene_radius, optimizer, i, group=None, densify_fn=None):
    """Camera-DP densification (densify.py:218-247 + external.py:211-314 on sharded views): the
    ranks' view statistics are reduced (``DensifyStats.allreduce``: SUM, SUM, MAX) and handed to
    ``densify_fn`` (default ``splat_densify.densify_gaussians`` with ``accumulate=False`` -- the views
    were accumulated by ``stats.update``) together with a ``broadcast_normal`` sampler, so every rank
    makes the same clone / split / prune decisions and draws the same split offsets."""
    stats.allreduce(group)
    if densify_fn is None:
        import splat_densify
        dv = splat_densify.DensificationVariables(visibility_count=stats.visibility_count,
                                                  mean_2d_gradients_accumulated=stats.mean_2d_gradients_accumulated,
                                                  max_2d_radii=stats.max_2d_radii)
        info = splat_densify.densify_gaussians(params, dv, scene_radius, optimizer, i,
                                               sample_fn=broadcast_normal(group), accumulate=False)
        stats.visibility_count, stats.mean_2d_gradients_accumulated, stats.max_2d_radii = \
            dv.visibility_count, dv.mean_2d_gradients_accumulated, dv.max_2d_radii
        return info
    return densify_fn(params, stats, scene_radius, optimizer, i, broadcast_normal(group))
