"""Data / format path: camera frames -> view tensors, and the ``.pth``
parameter dict.

Reference behaviour restated here (same names, arguments and results):

* ``load_timestep_views(dataset_metadata, timestep, sequence_path)`` (shared.py:127-171): one
  ``View`` per camera of the timestep; ``image`` = the JPEG ``ims/<fn>`` as (3, H, W) float / 255,
  ``segmentation_mask`` = (m, 0, 1 - m) of the PNG ``seg/<fn with .png>`` as float (not scaled),
  ``render_settings`` = ``create_render_settings(w, h, k[t][c], w2c[t][c])``.
* ``load_all_views(dataset_metadata, timestep_count, sequence_path)`` (train.py:207-217): the lists
  of timesteps 1 .. timestep_count.
* ``export_parameters(sequence_path, parameters)`` (densify.py:190-198) and
  ``load_densified_initial_parameters(data_directory_path, sequence_name)`` (train.py:155-163):
  ``torch.save`` / ``torch.load`` of the parameter dict as
  ``densified_initial_gaussian_cloud_parameters.pth`` -- the same file format both ways (the
  loader uses ``weights_only=True``; ``wandb.save`` is out of scope).

How it is done on MI355X: the reference decodes each frame with PIL on one thread, then per view
builds float tensors on the host (4 B per channel byte), copies them to the GPU one by one and runs
the permute / divide / stack as separate torch kernels.  Here the frames of a timestep are decoded
by a thread pool (PIL -- the reference's own decoder, so the 8-bit pixels are identical -- releases
the GIL while decoding) straight into ONE pinned 8-bit staging buffer, uploaded with one
asynchronous copy (a quarter of the reference's bytes), and ``gsr_views_pack`` (csrc/gsr_io.hip)
writes every view's planar float image and 3-channel mask in one launch.  ``load_all_views``
decodes the next timesteps while the current one uploads.  Entropy decoding is serial per JPEG
scan and stays on the host cores.

Values are bitwise the reference's on the GPU (torch divides by the Python scalar 255 as a multiply
by ``1.0f / 255``); the reference's ``image`` comes out of ``permute(...) / 255`` with HWC strides,
ours is contiguous (3, H, W) -- same values and shape, the layout the loss kernels read.
"""
from __future__ import annotations

import concurrent.futures as cf
import ctypes
import os
import threading
from pathlib import Path

import numpy as np
import torch

from diff_gaussian_rasterization import _C
from splat_scenes import render_settings as create_render_settings
from splat_train import View

__all__ = ["View", "decode_frame", "pack_views", "TimestepDecoder", "load_timestep_views",
           "load_all_views", "export_parameters", "load_densified_initial_parameters",
           "PARAMETERS_FILE_NAME"]

PARAMETERS_FILE_NAME = "densified_initial_gaussian_cloud_parameters.pth"  # densify.py:194-196
_bound = False


def _lib():
    global _bound
    L = _C.load_library()
    if not _bound:
        vp = ctypes.c_void_p
        L.gsr_views_pack.restype = ctypes.c_int
        L.gsr_views_pack.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, vp, vp, vp, vp, vp]
        _bound = True
    return L


def decode_frame(path) -> np.ndarray:
    """8-bit pixels of one image file, as the reference reads them (``np.array(Image.open(...))``,
    shared.py:131-141, 152-157).  Mode "1" PNGs become 0/1 bytes (numpy gives bool there)."""
    from PIL import Image  # imported lazily: only the loader needs it
    with Image.open(path) as im:
        a = np.asarray(im)
    if a.dtype == np.bool_:
        a = a.astype(np.uint8)
    if a.dtype != np.uint8:
        raise ValueError(f"{path}: {a.dtype} pixels; the view loader handles 8-bit frames")
    return a


def pack_views(rgb: torch.Tensor, seg: torch.Tensor | None = None):
    """(F, H, W, 3) uint8 frames (+ (F, H, W) uint8 masks) on the GPU -> ``images`` (F, 3, H, W)
    float32 = rgb / 255 and ``masks`` (F, 3, H, W) float32 = (m, 0, 1 - m), or None without seg.
    One ``gsr_views_pack`` launch on the current stream."""
    if not rgb.is_cuda:
        raise RuntimeError("pack_views: frames must be on the GPU (no CPU path)")
    if rgb.dtype != torch.uint8 or rgb.dim() != 4 or rgb.size(3) != 3:
        raise ValueError(f"pack_views: expected (F, H, W, 3) uint8 frames, got {tuple(rgb.shape)} {rgb.dtype}")
    F, H, W, _ = rgb.shape
    rgb = rgb.contiguous()
    images = torch.empty((F, 3, H, W), dtype=torch.float32, device=rgb.device)
    masks = None
    if seg is not None:
        if seg.dtype != torch.uint8 or tuple(seg.shape) != (F, H, W) or seg.device != rgb.device:
            raise ValueError(f"pack_views: expected ({F}, {H}, {W}) uint8 masks on {rgb.device}, "
                             f"got {tuple(seg.shape)} {seg.dtype} on {seg.device}")
        seg = seg.contiguous()
        masks = torch.empty((F, 3, H, W), dtype=torch.float32, device=rgb.device)
    if F * H * W:
        _C._check(_lib().gsr_views_pack(F, H, W, rgb.data_ptr(), seg.data_ptr() if seg is not None else None,
                                        images.data_ptr(), masks.data_ptr() if masks is not None else None,
                                        _C._stream_ptr(rgb.device)))
    return images, masks


def _frame_paths(dataset_metadata, timestep: int, sequence_path: Path):
    """(image path, mask path) of every camera of a timestep (shared.py:129-137, 154-156)."""
    sequence_path = Path(sequence_path)
    return [(sequence_path / "ims" / fn, sequence_path / "seg" / fn.replace(".jpg", ".png"))
            for fn in dataset_metadata["fn"][timestep]]


class TimestepDecoder:
    """Thread pool decoding the frames of a timestep into one pinned 8-bit staging pair.

    ``submit(dataset_metadata, timestep, sequence_path)`` returns a future of
    ``(rgb (F, H, W, 3) uint8, seg (F, H, W) uint8)`` host tensors in pinned memory (when a GPU is
    present), ready for one asynchronous upload."""

    def __init__(self, workers: int | None = None):
        self.workers = workers or min(16, os.cpu_count() or 1)
        self.pool = cf.ThreadPoolExecutor(self.workers)

    def close(self):
        self.pool.shutdown(wait=True)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def submit(self, dataset_metadata, timestep: int, sequence_path) -> cf.Future:
        W, H = int(dataset_metadata["w"]), int(dataset_metadata["h"])
        paths = _frame_paths(dataset_metadata, timestep, sequence_path)
        F = len(paths)
        pin = torch.cuda.is_available()
        rgb = torch.empty((F, H, W, 3), dtype=torch.uint8, pin_memory=pin)
        seg = torch.empty((F, H, W), dtype=torch.uint8, pin_memory=pin)
        rgb_np, seg_np = rgb.numpy(), seg.numpy()

        def one(c):
            img, msk = decode_frame(paths[c][0]), decode_frame(paths[c][1])
            if img.shape != (H, W, 3):
                raise ValueError(f"{paths[c][0]}: {img.shape} pixels, metadata says ({H}, {W}, 3)")
            if msk.shape != (H, W):
                raise ValueError(f"{paths[c][1]}: {msk.shape} mask, expected ({H}, {W})")
            rgb_np[c] = img
            seg_np[c] = msk

        done = cf.Future()
        if F == 0:
            done.set_result((rgb, seg))
            return done
        lock, left, errs = threading.Lock(), [F], []

        def finish(j):
            with lock:
                if j.exception() is not None:
                    errs.append(j.exception())
                left[0] -= 1
                last = left[0] == 0
            if last:  # exactly one callback gets here
                if errs:
                    done.set_exception(errs[0])
                else:
                    done.set_result((rgb, seg))

        for c in range(F):
            self.pool.submit(one, c).add_done_callback(finish)
        return done


def _views_from_staging(dataset_metadata, timestep: int, rgb, seg, device):
    """Upload one timestep's staging pair and build its views (shared.py:144-170)."""
    d_rgb = rgb.to(device, non_blocking=True)
    d_seg = seg.to(device, non_blocking=True)
    images, masks = pack_views(d_rgb, d_seg)
    views = []
    for c in range(images.size(0)):
        views.append(View(
            camera_index=c,
            render_settings=create_render_settings(
                image_width=dataset_metadata["w"], image_height=dataset_metadata["h"],
                intrinsic_matrix=dataset_metadata["k"][timestep][c],
                extrinsic_matrix=dataset_metadata["w2c"][timestep][c], device=device),
            image=images[c], segmentation_mask=masks[c]))
    # the staging buffers must outlive the asynchronous copies
    torch.cuda.current_stream(torch.device(device)).synchronize()
    return views


def load_timestep_views(dataset_metadata, timestep: int, sequence_path, device="cuda",
                        decoder: TimestepDecoder | None = None):
    """shared.py:127-171 on the native path (see the module docstring)."""
    own = decoder is None
    dec = decoder or TimestepDecoder()
    try:
        rgb, seg = dec.submit(dataset_metadata, timestep, sequence_path).result()
    finally:
        if own:
            dec.close()
    return _views_from_staging(dataset_metadata, timestep, rgb, seg, device)


def load_all_views(dataset_metadata, timestep_count: int, sequence_path, device="cuda",
                   decoder: TimestepDecoder | None = None, prefetch: int = 2):
    """train.py:207-217: ``[load_timestep_views(t) for t in 1 .. timestep_count]``, with the next
    ``prefetch`` timesteps decoding while the current one uploads and packs."""
    own = decoder is None
    dec = decoder or TimestepDecoder()
    try:
        steps = list(range(1, timestep_count + 1))
        pending = {t: dec.submit(dataset_metadata, t, sequence_path) for t in steps[:prefetch + 1]}
        out = []
        for k, t in enumerate(steps):
            nxt = k + prefetch + 1
            if nxt < len(steps):
                pending[steps[nxt]] = dec.submit(dataset_metadata, steps[nxt], sequence_path)
            rgb, seg = pending.pop(t).result()
            out.append(_views_from_staging(dataset_metadata, t, rgb, seg, device))
        return out
    finally:
        if own:
            dec.close()


def export_parameters(sequence_path, parameters: dict) -> Path:
    """densify.py:190-198 without the wandb upload: ``torch.save`` of the parameter dict."""
    path = Path(sequence_path) / PARAMETERS_FILE_NAME
    torch.save(parameters, path)
    return path


def load_densified_initial_parameters(data_directory_path, sequence_name: str, device="cuda"):
    """train.py:155-163: the saved dict with ``requires_grad`` cleared.  Loaded with
    ``weights_only=True`` (no code from the file runs) and memory-mapped, each storage copied once
    to ``device``."""
    path = Path(data_directory_path) / sequence_name / PARAMETERS_FILE_NAME
    parameters = torch.load(path, weights_only=True, mmap=True, map_location=device)
    for parameter in parameters.values():
        parameter.requires_grad = False
    return parameters
