"""Bookkeeping of the deferred multi-view backward's queue (diff_gaussian_rasterization/__init__.py),
on CPU with stand-in autograd nodes: each backward pass (graph task) flushes only its own queued
views -- a reentrant inner pass (torch.utils.checkpoint, use_reentrant=True) must not drop the outer
pass's views -- and a pass that raises drops its views through the callback's finalizer instead of
keeping their SCRATCH buffers alive."""
import pytest
import torch

import diff_gaussian_rasterization as D


class _Queue(torch.autograd.Function):
    """Backward queues one stand-in view under the running graph task, as _try_defer does."""

    @staticmethod
    def forward(ctx, x, tag):
        ctx.tag = tag
        return x.clone()

    @staticmethod
    def backward(ctx, g):
        task = torch._C._current_graph_task_id()
        with D._pending_lock:
            grp = D._pending.setdefault((task, "stand-in"), {"views": []})
            grp["views"].append(ctx.tag)
            queue = task not in D._queued
            D._queued.add(task)
        if queue:
            D._queue_flush(task)
        return g, None


class _Boom(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return x.clone()

    @staticmethod
    def backward(ctx, g):
        raise RuntimeError("boom")


@pytest.fixture
def flushed(monkeypatch):
    runs = []
    monkeypatch.setattr(D, "_run_group", lambda grp, created, post: runs.append(list(grp["views"])))
    D.clear_pending()
    yield runs
    D.clear_pending()


def test_each_pass_flushes_only_its_views(flushed):
    x = torch.ones(4, requires_grad=True)
    # another (still running / concurrent) task's queued view must survive this pass's flush
    with D._pending_lock:
        D._pending[(10 ** 15, "other")] = {"views": ["other"]}
    _Queue.apply(x, "a").sum().backward()
    assert flushed == [["a"]]
    assert D.pending_views() == 1


def test_reentrant_inner_pass_keeps_outer_views(flushed):
    from torch.utils.checkpoint import checkpoint
    x = torch.ones(4, requires_grad=True)
    y = torch.ones(4, requires_grad=True)
    inner = checkpoint(lambda t: _Queue.apply(t * 2, "inner"), y, use_reentrant=True)
    outer = _Queue.apply(x, "outer")  # created last: its node runs (and queues) before the checkpoint's
    (inner.sum() + outer.sum()).backward()
    assert sorted(map(tuple, flushed)) == [("inner",), ("outer",)]
    assert D.pending_views() == 0
    assert torch.equal(y.grad, torch.full((4,), 2.0)) and torch.equal(x.grad, torch.ones(4))


def test_raising_pass_drops_its_views(flushed):
    x = torch.ones(4, requires_grad=True)
    boom = _Boom.apply(x)          # created first: runs after the queueing node
    q = _Queue.apply(x, "lost")
    with pytest.raises(RuntimeError, match="boom"):
        (boom.sum() + q.sum()).backward()
    assert flushed == []
    assert D.pending_views() == 0  # finalizer of the never-run callback
    _Queue.apply(x, "next").sum().backward()
    assert flushed == [["next"]]
