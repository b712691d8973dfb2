"""MI355X-native drop-in for ``diff_gaussian_rasterization`` (diff-gaussian-rasterization-w-depth).

The reference imports exactly these names: ``GaussianRasterizer`` (``train.py:16``,
``densify.py:9``) and ``GaussianRasterizationSettings`` (``shared.py:9``, constructed by keyword with
11 fields at ``shared.py:112-124``).  ``GaussianRasterizer(raster_settings=...)(**render_args)``
returns ``(color (3,H,W), radii (P,) int32, depth (1,H,W))`` (``train.py:354-361``,
``densify.py:120-126``); ``means2D.grad`` receives the screen-space gradient in NDC units that
``external.py:113-124`` accumulates for densification.

Python surface and error behaviour follow the upstream binding; the native
work runs in hand-written HIP kernels for gfx950 behind the C ABI of ``include/gsr.h``.
"""
from __future__ import annotations

import os
import threading
import weakref
from typing import NamedTuple

import torch
import torch.nn as nn
from torch.autograd.graph import get_gradient_edge

from . import _C

__all__ = ["GaussianRasterizationSettings", "GaussianRasterizer", "rasterize_gaussians",
           "rasterize_parameters", "set_deferred_backward", "set_speculative_forward", "set_async_forward", "async_forward", "set_exact_thresholds",
           "pending_views", "clear_pending"]


class GaussianRasterizationSettings(NamedTuple):
    image_height: int
    image_width: int
    tanfovx: float
    tanfovy: float
    bg: torch.Tensor
    scale_modifier: float
    viewmatrix: torch.Tensor
    projmatrix: torch.Tensor
    sh_degree: int
    campos: torch.Tensor
    prefiltered: bool
    debug: bool = False


def _engine_accumulates(t, node=None):
    """True when the running backward pass will execute ``t``'s AccumulateGrad node, i.e. write
    ``t.grad``: ``loss.backward()`` does; ``torch.autograd.grad(...)`` never does (the engine refuses
    the query for its inputs) and ``loss.backward(inputs=[...])`` only for the listed leaves.
    ``node``: that AccumulateGrad node when the caller already has it (``_input_nodes``)."""
    try:
        return bool(torch._C._will_engine_execute_node(node if node is not None else get_gradient_edge(t).node))
    except RuntimeError:  # autograd.grad(): the gradient is returned, .grad is left alone
        return False


def _tensor_positions(args):
    """Input index -> position in the Function node's ``next_functions`` (tensor inputs only)."""
    pos, k = {}, 0
    for i, a in enumerate(args):
        if isinstance(a, torch.Tensor):
            pos[i] = k
            k += 1
    return pos


def _input_nodes(ctx, inputs):
    """The graph edges of the given input indices, read off the backward node itself: for a leaf
    that requires grad, its AccumulateGrad node (``get_gradient_edge(t).node``, ~8 us per call,
    would cost ~50 us per backward on the host thread that feeds the GPU)."""
    nf = ctx.next_functions
    pos = ctx.tensor_pos
    return [nf[pos[i]][0] if i in pos and pos[i] < len(nf) else None for i in inputs]


def _accumulation_target(t, node=None, create=False):
    """The leaf's existing ``.grad`` when the backward kernel may add into it in place (and the
    Function then returns None for it): a leaf requiring grad whose gradient is a contiguous fp32
    tensor of its shape, with no hooks that autograd's accumulation would have run, in a backward
    pass that will accumulate into that leaf (``_engine_accumulates``) without building a graph of
    the gradient (``create_graph``).  Gives the same value as autograd's AccumulateGrad (one fp32
    add, ``grad += new``) without its separate read-read-write pass; every other case returns the
    gradient to autograd as stock Functions do.  ``create``: a leaf that qualifies but has no
    ``.grad`` yet comes back as ``_Fresh(leaf)``: its gradient is allocated (uninitialised) when the
    deferred pass runs and written there without a read (what AccumulateGrad would have stored)."""
    if t is None or not isinstance(t, torch.Tensor) or t.numel() == 0 or not t.is_leaf or not t.requires_grad:
        return None
    g = t.grad
    if g is None and not (create and t.dtype == torch.float32 and t.is_contiguous()):
        return None
    if g is not None and (g.dtype != torch.float32 or not g.is_contiguous() or g.shape != t.shape or g.requires_grad):
        return None
    if t._backward_hooks or getattr(t, "_post_accumulate_grad_hooks", None):
        return None
    if torch.is_grad_enabled() or not _engine_accumulates(t, node):
        return None
    if g is None:
        if not _defer["fresh"]:  # (A/B switch: zero-filled gradient, read back by the pass)
            t.grad = g = torch.zeros_like(t)
            return g
        return _Fresh(t)
    return g


class _Fresh:
    """A deferred gradient target whose leaf had no ``.grad``: instead of a zero fill that the
    per-Gaussian pass would read back, the flush allocates it and the first launch writing it
    overwrites it."""
    __slots__ = ("leaf",)

    def __init__(self, leaf):
        self.leaf = leaf


def _fresh_target(t, created, post):
    """Resolve a deferred target at the flush -> (tensor, overwrite).  ``created``: ids of leaves
    whose .grad this flush allocated and no launch has written yet; ``post``: (leaf, tensor) pairs
    to add into a .grad that appeared meanwhile in an unusable form."""
    if not isinstance(t, _Fresh):
        return t, False
    leaf = t.leaf
    g = leaf.grad
    if g is None:  # still absent: allocate, the first writer overwrites
        leaf.grad = g = torch.empty_like(leaf, memory_format=torch.contiguous_format)
        created.add(id(leaf))
    elif id(leaf) not in created and (g.dtype != torch.float32 or not g.is_contiguous() or
                                      g.shape != leaf.shape or g.requires_grad):
        tmp = torch.zeros_like(leaf, memory_format=torch.contiguous_format)  # set by autograd meanwhile
        post.append((leaf, tmp))
        return tmp, False
    return g, id(leaf) in created


# ---- deferred multi-view per-Gaussian backward ------------------------------------------------
# train.py:753-767 sums the losses of 5 views and runs ONE backward.  When every gradient a view's
# backward produces lands in a leaf's .grad (the in-place accumulation above), the per-Gaussian half
# of the backward can wait until the pass has run every view: each view's backward node runs only
# the per-pixel half (gsr_backward_render) and queues its records; a callback at the end of the
# backward pass (the engine's final callbacks, which run on the caller's current streams after the
# leaf streams are synchronised) runs ONE per-Gaussian pass over all the queued views of the same
# Gaussians (gsr_backward_gaussians), reading the parameters and read-modify-writing every gradient
# array once instead of once per view.  .grad holds the summed result when backward() returns, as
# with stock autograd; the fp32 additions are grouped differently (views summed first).  Queued views
# are keyed by the engine's graph-task id and each pass flushes only its own: a reentrant backward
# inside the pass (torch.utils.checkpoint(use_reentrant=True)) or a pass run concurrently from another
# thread is a different graph task with its own views and callback.  A pass that raises never runs
# its callback; the engine then destroys the callback object, whose finalizer drops that pass's
# queued views (and the SCRATCH buffers they hold) at once.  AccumulateGrad *node* hooks
# (node.register_hook / register_prehook, e.g. DDP's reducer) cannot be seen from Python: such
# callers read .grad during the pass and must run with set_deferred_backward(False).
_defer = {"on": os.environ.get("GSR_DEFER_BACKWARD", "1") != "0",
          "fresh": os.environ.get("GSR_FRESH_GRADS", "1") != "0",
          # forwards queue their post-scan kernels before num_rendered is read back (include/gsr.h,
          # gsr_forward_info_call): the stream does not idle while the host reads K and launches
          "speculate": os.environ.get("GSR_SPECULATE", "1") != "0",
          # forwards with a pair-count history return without reading num_rendered back
          # (gsr_forward_async): one host thread keeps queueing views on several streams while the
          # GPU renders.  Off by default: on one stream (train.py's shape) and with one submitting
          # thread per stream (the headline) the host wait for K is already hidden, and the asynchronous
          # bookkeeping cost 1-3 % there; ``async_forward(True)`` / the env switch turn
          # it on for one-thread multi-stream submission (splat_step.RenderStep does)
          "async": os.environ.get("GSR_ASYNC_FORWARD", "0") == "1",
          # a deferred view whose asynchronous forward has no pair count yet queues its render half at
          # once against the forward's capacity (ABI 19) instead of holding it back to the end of the
          # pass; the end-of-pass callback only checks the device's verdict and redoes the rare miss
          "spec_half": os.environ.get("GSR_SPEC_RENDER_HALF", "1") != "0"}
_async_tls = threading.local()  # async_forward(): a per-thread override of _defer["async"]
_pending_lock = threading.Lock()
_pending = {}  # (graph task id, group key) -> {"views": [...], "gauss": (...), "targets": [...], ...}
_queued = set()  # graph tasks whose flush callback is queued
_spec_half_stats = {"queued": 0, "redone": 0}  # speculative render halves (diagnostics / tests)


def set_deferred_backward(on: bool) -> bool:
    """Enable / disable the deferred multi-view per-Gaussian backward; returns the previous setting."""
    prev = _defer["on"]
    _defer["on"] = bool(on)
    return prev


def set_speculative_forward(on: bool) -> bool:
    """Enable / disable the forward's speculative enqueue (gsr_forward_info_call); returns the
    previous setting.  The outputs are bitwise the same either way."""
    prev = _defer["speculate"]
    _defer["speculate"] = bool(on)
    return prev


def set_exact_thresholds(on: bool) -> bool:
    """Exact-threshold mode (include/gsr.h gsr_set_exact_thresholds, on by default): near-threshold
    blend weights re-evaluated as the reference computes them, in the few tiles that have one;
    returns the previous setting.  It applies to forwards queued after the call (a backward follows
    the choice its forward made)."""
    return _C.set_exact_thresholds(on)


def set_async_forward(on: bool) -> bool:
    """Enable / disable the asynchronous forward (gsr_forward_async: no host wait for num_rendered when
    the pair-count history gives a capacity); returns the previous setting.  Outputs are bitwise the
    same either way."""
    prev = _defer["async"]
    _defer["async"] = bool(on)
    return prev


class async_forward:
    """Context manager: the asynchronous forward on (or off) for the calls this thread makes inside it,
    whatever the process-wide setting (set_async_forward)."""

    def __init__(self, on: bool = True):
        self.on = bool(on)

    def __enter__(self):
        self.prev = getattr(_async_tls, "on", None)
        _async_tls.on = self.on
        return self

    def __exit__(self, *exc):
        _async_tls.on = self.prev
        return False


def _async_on():
    o = getattr(_async_tls, "on", None)
    return _defer["async"] if o is None else o


def _buffer_ptrs(alloc):
    """(GEOM, BINNING, IMAGE) device pointers of a forward's workspaces (_C._forward)."""
    p = alloc.ptrs
    return p[_C.GSR_BUF_GEOM], p[_C.GSR_BUF_BINNING], p[_C.GSR_BUF_IMAGE]


def _resolved(ctx):
    """(num_rendered, binning_layout, binning pointer or None) of the forward behind ``ctx``: an
    asynchronous forward is resolved here (waits for its pair count if the GPU has not produced it)."""
    if ctx.pending is not None:
        return ctx.pending.resolve()
    return ctx.num_rendered, ctx.binning_layout, None


def pending_views() -> int:
    """Views queued for a deferred per-Gaussian pass that has not run yet (0 between backward passes)."""
    with _pending_lock:
        return sum(len(g["views"]) for g in _pending.values())


def clear_pending() -> None:
    """Drop every queued view (their SCRATCH buffers are freed); a pass still running loses them."""
    with _pending_lock:
        _pending.clear()
        _queued.clear()


def _drop_task(task):
    with _pending_lock:
        for k in [k for k in _pending if k[0] == task]:
            del _pending[k]
        _queued.discard(task)


class _TaskFlush:
    """The end-of-pass callback of one graph task.  The engine holds the only reference: after a
    successful pass it has run (and flushed the task's views); after a pass that raised it is
    released without running, and the finalizer registered beside it drops the task's views."""
    __slots__ = ("task", "__weakref__")

    def __init__(self, task):
        self.task = task

    def __call__(self):
        _flush_pending(self.task)


def _queue_flush(task):
    """Queue ``task``'s end-of-pass flush on the running backward pass (once per pass)."""
    cb = _TaskFlush(task)
    weakref.finalize(cb, _drop_task, task)
    torch.autograd.Variable._execution_engine.queue_callback(cb)


def _flush_pending(task):
    """Final callback of a backward pass: one per-Gaussian pass per group of this pass's views."""
    with _pending_lock:
        groups = [g for (t, _), g in _pending.items() if t == task]
        for k in [k for k in _pending if k[0] == task]:
            del _pending[k]
        _queued.discard(task)
    created, post = set(), []
    for grp in groups:
        _run_group(grp, created, post)
    for leaf, tmp in post:
        leaf.grad = leaf.grad + tmp


def _run_group(grp, created, post):
    """One multi-view per-Gaussian pass over a group of queued views of the same Gaussians."""
    dev = grp["device"]
    with torch.cuda.device(dev):
        cur = torch.cuda.current_stream(dev)
        for v in grp["views"]:
            pend = v.pop("spec", None)
            if pend is not None:  # a speculative render half: it stands unless its forward was redone
                K, _, _ = pend.resolve()
                if pend.redone:
                    v["scratch"] = None
                    _spec_half_stats["redone"] += 1
                else:
                    v["num_rendered"] = K
                    v.pop("render_fn")
            # render halves held back while their forward's pair count was unknown, or redone
            if v["scratch"] is None:
                with torch.cuda.stream(_C._external_stream(v["stream"], dev)):
                    v["scratch"], v["num_rendered"] = v.pop("render_fn")()
        cur_ptr = cur.cuda_stream
        for s in grp["streams"]:  # every view's render half precedes the per-Gaussian pass
            if s != cur_ptr:
                cur.wait_stream(_C._external_stream(s, dev))
        (means3D, colors, scales, rotations, scale_modifier, cov3D, sh, degree, act) = grp["gauss"]
        targets, over = [None] * 8, []
        for k in range(1, 8):
            targets[k], ow = _fresh_target(grp["targets"][k], created, post)
            if ow:
                over.append(k)
        views = []
        for v in grp["views"]:  # each view's screen-space gradient: overwrite a fresh one first
            m2, ow = _fresh_target(v["means2D_grad"], created, post)
            views.append(dict(v, means2D_grad=m2, accumulate_means2D=not ow))
            if ow:
                created.discard(id(v["means2D_grad"].leaf))
        # slots without a target are gradients no input asked for (_try_defer queues a view only
        # when every needed gradient has one): not computed into memory
        needed = [k == 0 or grp["targets"][k] is not None for k in range(8)]
        _C.rasterize_gaussians_backward_views(views, means3D, colors, scales, rotations,
                                              scale_modifier, cov3D, sh, degree, activations=act,
                                              skip_unused=True, accumulate_into=targets, overwrite=over,
                                              needed=needed)
        for k in over:  # written: later launches add into it
            created.discard(id(grp["targets"][k].leaf))


def _try_defer(ctx, gauss, radii, geomBuffer, leaf_inputs, nodes, need, render_fn, keep=()):
    """Queue this view for the end-of-pass per-Gaussian backward when every gradient it must produce
    can go into a leaf's .grad; returns True when queued (the Function then returns None for all).
    ``render_fn(spec=False)`` runs the view's per-pixel half and returns ``(SUMS buffer, num_rendered)``.
    When the view's forward was asynchronous and its pair count is not known yet (the GPU has not
    reached its tile scan -- the pass's first nodes belong to the step's last views), the half is
    queued speculatively (``render_fn(True)``: against the forward's capacity, its kernels return at
    once if the device's speculation failed) and the end-of-pass callback resolves the forward,
    redoing the half only when the forward was redone; with ``_defer["spec_half"]`` off it is held back
    until that callback instead, so the earlier views' render halves are queued first."""
    if not _defer["on"]:
        return False
    means3D, colors, scales, rotations, scale_modifier, cov3D, sh, degree, act = gauss
    P = means3D.shape[0]
    if P == 0 or not means3D.is_cuda or (sh.numel() and sh.shape[1] not in (1, 4, 9, 16)):
        return False
    task = torch._C._current_graph_task_id()
    if task < 0:
        return False
    op = ctx.leaves[2]
    if need[leaf_inputs[2]] and (op is None or tuple(op.shape) != (P, 1)):
        return False
    targets = [None] * 8
    for k, (t, i, node) in enumerate(zip(ctx.leaves, leaf_inputs, nodes)):
        if i is None or not need[i]:
            continue
        tgt = _accumulation_target(t, node, create=True)
        if tgt is None:
            return False  # autograd must receive this gradient: immediate path
        targets[k] = tgt
    rs = ctx.raster_settings
    # the view's stream as its raw handle (torch.cuda.current_stream builds a Stream object per call)
    dix = means3D.device.index
    stream = _C._raw_stream(dix if dix is not None else _C._get_device())
    spec = None
    if ctx.pending is None or ctx.pending.ready():
        scratch, K = render_fn()
    elif _defer["spec_half"]:
        scratch, K = render_fn(True)
        spec = ctx.pending
        _spec_half_stats["queued"] += 1
    else:
        scratch, K = None, -1
    ptr = lambda t: t.data_ptr() if t is not None and t.numel() else 0  # noqa: E731
    tkey = lambda t: ("fresh", id(t.leaf)) if isinstance(t, _Fresh) else ptr(t)  # noqa: E731
    key = (means3D.device, P, ptr(means3D), ptr(scales), ptr(rotations), ptr(cov3D), ptr(sh), ptr(colors),
           int(degree), float(scale_modifier), int(act)) + tuple(tkey(t) for t in targets[1:])
    view = {"viewmatrix": rs.viewmatrix, "projmatrix": rs.projmatrix, "tanfovx": rs.tanfovx,
            "tanfovy": rs.tanfovy, "image_height": rs.image_height, "image_width": rs.image_width,
            "campos": rs.campos, "bg": rs.bg, "radii": radii, "geomBuffer": geomBuffer, "scratch": scratch,
            "num_rendered": K, "means2D_grad": targets[0], "accumulate_means2D": True, "stream": stream,
            "keep": keep}
    if scratch is None or spec is not None:
        view["render_fn"] = render_fn
    if spec is not None:
        view["spec"] = spec
    with _pending_lock:
        grp = _pending.get((task, key))
        if grp is None:
            grp = _pending[(task, key)] = {"device": means3D.device, "views": [], "gauss": gauss,
                                           "targets": targets, "streams": []}
        grp["views"].append(view)
        if stream not in grp["streams"]:
            grp["streams"].append(stream)
        queue = task not in _queued
        _queued.add(task)
    if queue:
        _queue_flush(task)
    return True


def rasterize_gaussians(means3D, means2D, sh, colors_precomp, opacities, scales, rotations,
                        cov3Ds_precomp, raster_settings):
    args = (means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp)
    return _RasterizeGaussians.apply(*args, raster_settings, torch.is_grad_enabled())


class _RasterizeGaussians(torch.autograd.Function):
    @staticmethod
    def forward(ctx, means3D, means2D, sh, colors_precomp, opacities, scales, rotations,
                cov3Ds_precomp, raster_settings, grad_mode=False):
        rs = raster_settings
        args = (rs.bg, means3D, colors_precomp, opacities, scales, rotations, rs.scale_modifier,
                cov3Ds_precomp, rs.viewmatrix, rs.projmatrix, rs.tanfovx, rs.tanfovy,
                rs.image_height, rs.image_width, sh, rs.sh_degree, rs.campos, rs.prefiltered)
        # a backward can follow (grad mode at the call, an input requiring grad): the forward
        # prepares it
        ctx.prep = bool(grad_mode) and any(ctx.needs_input_grad)
        fi, color, radii, depth, alloc, pending = _C._forward(
            *args, 0, ctx.prep, _defer["speculate"], _async_on())
        ctx.raster_settings = rs
        ctx.num_rendered = fi.num_rendered
        ctx.binning_layout = fi.binning_layout
        ctx.pending = pending  # an asynchronous forward: resolved by the backward
        ctx.bufs = _buffer_ptrs(alloc)  # GEOM, BINNING, IMAGE device pointers (the bases are saved)
        # leaves whose existing gradient the backward kernel may accumulate into (grad output order)
        ctx.leaves = (means2D, colors_precomp, opacities, means3D, cov3Ds_precomp, sh, scales, rotations)
        ctx.tensor_pos = _tensor_positions((means3D, means2D, sh, colors_precomp, opacities, scales,
                                            rotations, cov3Ds_precomp))
        ctx.save_for_backward(colors_precomp, means3D, scales, rotations, cov3Ds_precomp, radii, sh,
                              *alloc.bases)
        ctx.mark_non_differentiable(radii)
        ctx.set_materialize_grads(False)  # no zero-filled gradients for the unused depth output
        return color, radii, depth

    @staticmethod
    def backward(ctx, grad_out_color, _grad_radii, grad_depth):
        if grad_out_color is None:  # only depth was used: it carries no gradient (-w-depth)
            return (None,) * 10
        rs = ctx.raster_settings
        saved = ctx.saved_tensors
        colors_precomp, means3D, scales, rotations, cov3Ds_precomp, radii, sh = saved[:7]
        bases = saved[7:]
        geomBuffer, binningBuffer, imgBuffer = ctx.bufs

        def args_kw(spec=False):  # the forward's pair count and BINNING (an asynchronous forward resolves
            # here; ``spec``: not yet -- its capacity and own BINNING, the speculative render half)
            K, layout, bptr = (-1, ctx.binning_layout, None) if spec else _resolved(ctx)
            return ((rs.bg, means3D, radii, colors_precomp, scales, rotations, rs.scale_modifier,
                     cov3Ds_precomp, rs.viewmatrix, rs.projmatrix, rs.tanfovx, rs.tanfovy, grad_out_color,
                     sh, rs.sh_degree, rs.campos, geomBuffer, K, binningBuffer, imgBuffer),
                    {"prepare_backward": ctx.prep, "binning_layout": layout, "binning_ptr": bptr})

        def render_half(spec=False):
            a, k = args_kw(spec)
            return _C.rasterize_gaussians_backward_render(*a, **k), a[17]
        inputs = (1, 3, 4, 0, 7, 2, 5, 6)  # input index of each leaf (grad output order)
        nodes = _input_nodes(ctx, inputs)
        gauss = (means3D, colors_precomp, scales, rotations, rs.scale_modifier, cov3Ds_precomp, sh,
                 rs.sh_degree, 0)
        if _try_defer(ctx, gauss, radii, geomBuffer, inputs, nodes, ctx.needs_input_grad, render_half, bases):
            return (None,) * 10  # every gradient is added into its leaf's .grad at the end of the pass
        args, kw = args_kw()
        need = [ctx.needs_input_grad[i] for i in inputs]
        acc = [_accumulation_target(t, node) if n else None for t, n, node in zip(ctx.leaves, need, nodes)]
        g = list(_C.rasterize_gaussians_backward(*args, skip_unused=True, accumulate_into=acc, needed=need, **kw))
        for k, t in enumerate(acc):
            if t is not None:
                g[k] = None  # already accumulated into the leaf's .grad
        (grad_means2D, grad_colors_precomp, grad_opacities, grad_means3D, grad_cov3Ds_precomp,
         grad_sh, grad_scales, grad_rotations) = g
        return (grad_means3D, grad_means2D, grad_sh, grad_colors_precomp, grad_opacities,
                grad_scales, grad_rotations, grad_cov3Ds_precomp, None, None)


class GaussianRasterizer(nn.Module):
    def __init__(self, raster_settings):
        super().__init__()
        self.raster_settings = raster_settings

    def markVisible(self, positions):
        # near-plane frustum test of every point (a bool mask)
        with torch.no_grad():
            rs = self.raster_settings
            visible = _C.mark_visible(positions, rs.viewmatrix, rs.projmatrix)
        return visible

    def forward(self, means3D, means2D, opacities, shs=None, colors_precomp=None, scales=None,
                rotations=None, cov3D_precomp=None):
        rs = self.raster_settings
        if (shs is None and colors_precomp is None) or (shs is not None and colors_precomp is not None):
            raise Exception('Please provide excatly one of either SHs or precomputed colors!')
        if ((scales is None or rotations is None) and cov3D_precomp is None) or \
                ((scales is not None or rotations is not None) and cov3D_precomp is not None):
            raise Exception('Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!')
        empty = torch.Tensor([])
        if shs is None:
            shs = empty
        if colors_precomp is None:
            colors_precomp = empty
        if scales is None:
            scales = empty
        if rotations is None:
            rotations = empty
        if cov3D_precomp is None:
            cov3D_precomp = empty
        return rasterize_gaussians(means3D, means2D, shs, colors_precomp, opacities, scales,
                                   rotations, cov3D_precomp, rs)


def rasterize_parameters(params, raster_settings, means2D=None, shs=None):
    """Fused ``create_render_arguments`` (shared.py:29-42) + ``GaussianRasterizer`` call
    (train.py:359-361, densify.py:124-126): the caller's normalize / sigmoid / exp activations run
    inside the preprocess kernel and their derivatives inside the per-Gaussian backward kernel, so
    no activated copies or autograd nodes are created and gradients land directly on
    ``params["means"]``, ``params["rotation_quaternions"]``, ``params["opacity_logits"]``,
    ``params["log_scales"]`` and ``params["colors"]`` (or ``shs`` when given).

    ``means2D``: optional (P, 3) tensor requiring grad; it receives the screen-space (NDC) gradient
    that the reference reads through ``means2D.retain_grad()`` (densify.py:119, external.py:117).
    Returns ``(color (3,H,W), radii (P,), depth (1,H,W))`` like ``GaussianRasterizer``.
    """
    means = params["means"]
    if means2D is None:
        means2D = torch.empty(0, device=means.device)
    colors = params["colors"] if shs is None else torch.empty(0, device=means.device)
    if shs is None:
        shs = torch.empty(0, device=means.device)
    return _RasterizeGaussianParameters.apply(means, means2D, shs, colors, params["opacity_logits"],
                                              params["log_scales"], params["rotation_quaternions"],
                                              raster_settings, torch.is_grad_enabled())


class _RasterizeGaussianParameters(torch.autograd.Function):
    @staticmethod
    def forward(ctx, means, means2D, sh, colors, opacity_logits, log_scales, quaternions, raster_settings,
                grad_mode=False):
        rs = raster_settings
        empty = torch.empty(0, device=means.device)
        ctx.prep = bool(grad_mode) and any(ctx.needs_input_grad)  # a backward can follow
        fi, color, radii, depth, alloc, pending = _C._forward(
            rs.bg, means, colors, opacity_logits, log_scales, quaternions, rs.scale_modifier, empty,
            rs.viewmatrix, rs.projmatrix, rs.tanfovx, rs.tanfovy, rs.image_height, rs.image_width, sh,
            rs.sh_degree, rs.campos, rs.prefiltered, _C.ACT_ALL, ctx.prep, _defer["speculate"], _async_on())
        ctx.raster_settings = rs
        ctx.num_rendered = fi.num_rendered
        ctx.binning_layout = fi.binning_layout
        ctx.pending = pending
        ctx.bufs = _buffer_ptrs(alloc)
        ctx.opacity_shape = opacity_logits.shape
        ctx.leaves = (means2D, colors, opacity_logits, means, None, sh, log_scales, quaternions)
        ctx.tensor_pos = _tensor_positions((means, means2D, sh, colors, opacity_logits, log_scales, quaternions))
        ctx.save_for_backward(colors, means, log_scales, quaternions, radii, sh, *alloc.bases)
        ctx.mark_non_differentiable(radii)
        ctx.set_materialize_grads(False)
        return color, radii, depth

    @staticmethod
    def backward(ctx, grad_out_color, _grad_radii, _grad_depth):
        if grad_out_color is None:
            return (None,) * 9
        rs = ctx.raster_settings
        saved = ctx.saved_tensors
        colors, means, log_scales, quaternions, radii, sh = saved[:6]
        bases = saved[6:]
        geomBuffer, binningBuffer, imgBuffer = ctx.bufs
        empty = torch.empty(0, device=means.device)
        need = ctx.needs_input_grad
        inputs = (1, 3, 4, 0, None, 2, 5, 6)  # input index of each leaf (grad output order; no cov3D)
        nodes = _input_nodes(ctx, [i for i in inputs if i is not None])
        nodes.insert(4, None)
        gauss = (means, colors, log_scales, quaternions, rs.scale_modifier, empty, sh, rs.sh_degree, _C.ACT_ALL)
        def render_half(spec=False):
            K, layout, bptr = (-1, ctx.binning_layout, None) if spec else _resolved(ctx)
            return _C.rasterize_gaussians_backward_render(
                rs.bg, means, radii, colors, log_scales, quaternions, rs.scale_modifier, empty,
                rs.viewmatrix, rs.projmatrix, rs.tanfovx, rs.tanfovy, grad_out_color, sh,
                rs.sh_degree, rs.campos, geomBuffer, K, binningBuffer, imgBuffer,
                activations=_C.ACT_ALL, prepare_backward=ctx.prep, binning_layout=layout, binning_ptr=bptr), K
        if _try_defer(ctx, gauss, radii, geomBuffer, inputs, nodes, need, render_half, bases):
            return (None,) * 9
        K, layout, bptr = _resolved(ctx)
        acc = [_accumulation_target(t, node) if i is not None and need[i] else None
               for t, i, node in zip(ctx.leaves, inputs, nodes)]
        if acc[2] is not None and acc[2].shape != (means.shape[0], 1):
            acc[2] = None
        needed = [i is not None and need[i] for i in inputs]
        (g_means2D, g_colors, g_opacity, g_means, _g_cov3D, g_sh, g_scales, g_rot) = \
            _C.rasterize_gaussians_backward(
                rs.bg, means, radii, colors, log_scales, quaternions, rs.scale_modifier, empty,
                rs.viewmatrix, rs.projmatrix, rs.tanfovx, rs.tanfovy, grad_out_color, sh, rs.sh_degree,
                rs.campos, geomBuffer, K, binningBuffer, imgBuffer,
                activations=_C.ACT_ALL, skip_unused=True, accumulate_into=acc, prepare_backward=ctx.prep,
                needed=needed, binning_layout=layout, binning_ptr=bptr)
        done = [t is not None or not n for t, n in zip(acc, needed)]  # in the leaf's .grad / not needed: None
        return (None if done[3] else g_means, None if (done[0] or not need[1]) else g_means2D,
                None if (done[5] or not sh.numel()) else g_sh,
                None if (done[1] or not colors.numel()) else g_colors,
                None if done[2] else g_opacity.view(ctx.opacity_shape),
                None if done[6] else g_scales, None if done[7] else g_rot, None, None)
