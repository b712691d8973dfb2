"""One training step's render work over several views, pipelined across HIP streams.

train.py computes the losses of 5 views, sums them and runs ONE backward per step
(train.py:753-767, ``losses.sum(dim=0)`` at train.py:413-418); densify.py sums its colour and
segmentation losses the same way (densify.py:237).  ``RenderStep`` runs that shape through the
drop-in ``GaussianRasterizer`` for the benchmark and the parity tests alike:

* the views alternate over ``streams`` (one view's memory-bound kernels overlap the next view's
  VALU-bound blend kernels; libgsr orders the gradient writes across streams, so the result is
  bitwise that of one stream -- ``tests/test_streams.py``); ``rotate``: the assignment starts one
  stream further every call, so with 5 views on 3 streams the streams carry 2, 2, 1 views in turn
  instead of the first two always carrying two (their serial kernel chains bound the step);
* ``threads``: one host thread per stream submits that stream's forwards, so a forward waiting for
  its ``num_rendered`` read-back (the reference's host sync) blocks only its own stream; without
  threads (one host thread for several streams) the forwards are asynchronous
  (``diff_gaussian_rasterization.async_forward``: no host wait for the pair count), so that one thread
  keeps every stream fed;
* ``summed``: the views' images are backpropagated together (``torch.autograd.backward`` of all
  images with the fixed upstream gradient = the summed loss), so the deferred multi-view
  per-Gaussian pass covers every view when the inputs are leaves; ``per_view``: one backward per
  view (the reference's densify.py shape for a single render).

``inputs_of(view)`` returns the rasterizer's keyword arguments for a view: the same leaf dict for
every view (the benchmark), a dict with that view's own ``means2D`` leaf (create_render_arguments
makes a fresh one per render, shared.py:38-41), or freshly activated non-leaf arguments (the
reference's call site, train.py:354-364).
"""
from __future__ import annotations

import os
from concurrent.futures import ThreadPoolExecutor
from contextlib import nullcontext as _nullcontext
from typing import Callable, Sequence

import torch

from diff_gaussian_rasterization import GaussianRasterizer, async_forward


class RenderStep:
    def __init__(self, device, cams: Sequence, inputs_of: Callable, dl: torch.Tensor, streams: Sequence,
                 threads: bool = True, shape: str = "summed", rotate: bool | None = None):
        if shape not in ("summed", "per_view"):
            raise ValueError(f"shape: 'summed' or 'per_view', got {shape!r}")
        self.device, self.cams, self.inputs_of, self.dl = device, cams, inputs_of, dl
        self.streams = list(streams)
        self.shape = shape
        self.rotate = os.environ.get("GSR_STREAM_ROTATE", "1") != "0" if rotate is None else rotate
        self.calls = 0
        # one single-thread executor per stream: a stream's views are always submitted by the same
        # thread, so the autograd nodes' sequence numbers (per-thread counters) and with them the order
        # in which the backward visits the views do not depend on which idle pool thread took which
        # task (the deferred multi-view pass also sums a launch's views in a camera-fixed order,
        # k_gauss_bwd_multi's view_order, so the gradients do not depend on it either)
        self.pool = ([ThreadPoolExecutor(max_workers=1) for _ in self.streams]
                     if threads and len(self.streams) > 1 else None)

    def close(self):
        if self.pool is not None:
            for ex in self.pool:
                ex.shutdown()
            self.pool = None

    def _forwards(self, vs, s):  # one stream's share of a summed step's forwards
        torch.cuda.set_device(self.device)
        with torch.cuda.stream(s):
            return [GaussianRasterizer(raster_settings=self.cams[ci])(**self.inputs_of(ci))[0] for ci in vs]

    def _fwd_bwd(self, vs, s):  # one stream's share of a per-view step, fwd + bwd per view
        torch.cuda.set_device(self.device)
        with torch.cuda.stream(s):
            for ci in vs:
                img = GaussianRasterizer(raster_settings=self.cams[ci])(**self.inputs_of(ci))[0]
                img.backward(self.dl)

    def __call__(self, views: Sequence[int], solo: bool = False):
        """Render ``views`` (camera indices) forward + backward.  ``solo``: one stream, one submitting
        thread (per-kernel times without concurrency).  Returns the rendered images (summed shape) in
        the order of ``views``."""
        ns = 1 if solo else len(self.streams)
        pool = None if solo else self.pool
        off = self.calls % ns if self.rotate else 0  # stream of this call's first view
        self.calls += 1
        streams = self.streams[off:ns] + self.streams[:off] if ns > 1 else self.streams[:1]
        with async_forward(True) if pool is None and ns > 1 else _nullcontext():
            return self._run(views, ns, pool, streams)

    def _run(self, views, ns, pool, streams):
        if self.shape == "summed":
            if pool is not None:
                futs = [pool[self.streams.index(streams[k])].submit(self._forwards, views[k::ns], streams[k])
                        for k in range(min(ns, len(views)))]
                imgs = [None] * len(views)
                for k, f in enumerate(futs):
                    imgs[k::ns] = f.result()
            else:  # one submitting thread: the device once, the stream switched per view; both restored
                imgs = []
                prev_dev = torch.cuda.current_device()
                torch.cuda.set_device(self.device)
                cur = torch.cuda.current_stream(self.device)
                try:
                    for k, ci in enumerate(views):
                        torch.cuda.set_stream(streams[k % ns])
                        imgs.append(GaussianRasterizer(raster_settings=self.cams[ci])(**self.inputs_of(ci))[0])
                finally:
                    torch.cuda.set_stream(cur)
                    torch.cuda.set_device(prev_dev)
            torch.autograd.backward(imgs, [self.dl] * len(imgs))
            return [img.detach() for img in imgs]
        elif pool is not None:
            futs = [pool[self.streams.index(streams[k])].submit(self._fwd_bwd, views[k::ns], streams[k])
                    for k in range(min(ns, len(views)))]
            for f in futs:
                f.result()
        else:
            for k, ci in enumerate(views):
                self._fwd_bwd([ci], streams[k % ns])
        return None
