"""Frame-sharded per-frame fits (BASELINE.json configs[4]).

A dynamic sequence of ``n_frames`` frames, each fitted by its OWN Gaussian parameter set and Adam
state: the per-timestep optimisation of train.py:738-776 (render ``V`` views, L1 + SSIM losses
summed over the views, one backward, one Adam step) run for every frame independently.  Frames are
split over the ranks in contiguous blocks (``splat_dp.shard_frames``: 150 frames over 8 ranks ->
19 x 6 + 18 x 2); there is no exchange between ranks -- each rank's frames are independent fits.

One ``step()`` = one optimisation iteration of EVERY frame of this rank's block, so the work of a
step is the whole sequence's and ``--gpus N`` divides it (strong scaling).  Frame ``t``'s parameter
set starts from the initial cloud (train.py's timestep t starts from the densified cloud too) and its
targets are renders of the frame's ground-truth cloud, made before timing (a real sequence's
captured images are resident in HBM as well: train.py:723-727 preloads every timestep).

The render / loss / optimiser engine is injected, so the control flow (frame split, independent
parameter sets, no collective) is testable on the CPU with stand-ins (tests/test_frames.py); the
benchmark passes the HIP path: ``rasterize_parameters`` (fused activations), ``splat_loss.image_loss``
(fused L1 + SSIM) and ``splat_adam.FusedAdam``.
"""
from __future__ import annotations

import math
from typing import Callable, Dict, Sequence

import torch

import splat_dp

# densify.py:68-86 learning rates (camera parameters are not rendered)
FRAME_LRS = {"means": 0.00016, "colors": 0.0025, "rotation_quaternions": 0.001, "opacity_logits": 0.05,
             "log_scales": 0.001, "shs": 0.0025}


def frame_displacement(P: int, device, seed: int = 2) -> torch.Tensor:
    """Per-Gaussian phase phi ~ U(0, 2 pi) (seed 2)."""
    g = torch.Generator().manual_seed(seed)
    return (torch.rand(P, 1, generator=g) * 2 * math.pi).to(device)


def frame_truth(base: Dict[str, torch.Tensor], phi: torch.Tensor, t: int, n_frames: int) -> Dict[str, torch.Tensor]:
    """Frame t's ground-truth cloud: means + 0.05 sin(2 pi t / n_frames + phi)."""
    p = dict(base)
    p["means"] = base["means"] + 0.05 * torch.sin(2 * math.pi * t / n_frames + phi)
    return p


class FrameFits:
    """Independent per-frame fits of this rank's frame block.

    render(params, cam) -> image; loss(image, target) -> scalar; make_optimizer(param dict) -> optimiser;
    ``streams``: the views of one frame alternate over them (None: the current stream).
    """

    def __init__(self, base: Dict[str, torch.Tensor], cams: Sequence, rank: int, world: int, views: int,
                 render: Callable, loss: Callable, make_optimizer: Callable, n_frames: int = 150,
                 streams: Sequence = None, main_stream=None):
        self.cams, self.V = cams, views
        self.render, self.loss = render, loss
        self.n_frames = n_frames
        self.frames = list(splat_dp.shard_frames(n_frames, rank, world))
        self.streams = list(streams) if streams else None
        dev = base["means"].device
        # the stream the per-frame backward + Adam run on: the caller's, or the current one
        self.main = main_stream if main_stream is not None or not self.streams else torch.cuda.current_stream(dev)
        self.phi = frame_displacement(base["means"].shape[0], dev)
        self.params, self.opts, self.targets = {}, {}, {}
        with torch.no_grad():
            for t in self.frames:
                self.params[t] = {k: torch.nn.Parameter(v.detach().clone()) for k, v in base.items()}
                self.opts[t] = make_optimizer(self.params[t])
                gt = frame_truth(base, self.phi, t, n_frames)
                for ci in self.frame_views(t):
                    self.targets[(t, ci)] = render(gt, cams[ci]).detach()

    def frame_views(self, t: int) -> list:
        """The V rig cameras frame t is fitted on (a fixed, frame-dependent subset of the rig)."""
        return [(t * self.V + j) % len(self.cams) for j in range(self.V)]

    def used_views(self) -> list:
        return sorted({ci for t in self.frames for ci in self.frame_views(t)})

    def frame_step(self, t: int):
        """One train.py:738-776 iteration of frame t: V renders, summed losses, backward, Adam."""
        params = self.params[t]
        losses = []
        if self.streams:
            for s in self.streams:
                s.wait_stream(self.main)  # the previous frame's Adam update
        for k, ci in enumerate(self.frame_views(t)):
            if self.streams:
                with torch.cuda.stream(self.streams[k % len(self.streams)]):
                    losses.append(self.loss(self.render(params, self.cams[ci]), self.targets[(t, ci)]))
            else:
                losses.append(self.loss(self.render(params, self.cams[ci]), self.targets[(t, ci)]))
        if self.streams:
            for s in self.streams:
                self.main.wait_stream(s)
        sum(losses).backward()  # train.py:757-767: the views' losses summed, one backward
        self.opts[t].step()
        self.opts[t].zero_grad(set_to_none=True)

    def step(self, it: int = 0):
        """One optimisation iteration of every frame of this rank's block (no collective)."""
        for t in self.frames:
            self.frame_step(t)
