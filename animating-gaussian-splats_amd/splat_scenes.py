"""Synthetic Gaussian clouds and cameras for parity tests and the benchmark.

Cameras are built exactly as the reference builds them, restated here because ``/root/reference``
is absent on the GPU box:

* ``look_at``         restates ``create_transformation_matrix`` (``train.py:446-457``)
* ``render_settings`` restates ``create_render_settings`` (``shared.py:64-124``): the 11-field
  ``GaussianRasterizationSettings`` with the transposed (1,4,4) view matrix, the OpenGL-style
  projection with near 1 / far 100, ``projmatrix = viewmatrix.bmm(proj)``, ``campos =
  inverse(w2c)[:3, 3]``, ``tanfov = W / (2 fx)``, zero background, ``sh_degree`` 0 unless given.
* ``render_arguments`` restates ``create_render_arguments`` (``shared.py:29-42``): normalised
  quaternions, sigmoid opacities, exp scales and a non-leaf zero ``means2D``.

The restatement is pinned against vectors produced by the reference's own functions
(``tests/golden/``).  Inputs follow SURVEY.md 8(d): CPU ``torch.Generator`` seeded 0, fp32.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
import torch

from diff_gaussian_rasterization import GaussianRasterizationSettings


def look_at(yaw_degrees: float, height: float, distance_to_center: float) -> np.ndarray:
    y = np.radians(yaw_degrees)
    return np.array([[np.cos(y), 0.0, -np.sin(y), 0.0],
                     [0.0, 1.0, 0.0, height],
                     [np.sin(y), 0.0, np.cos(y), distance_to_center],
                     [0.0, 0.0, 0.0, 1.0]])


def intrinsics(focal: float, width: int, height: int) -> np.ndarray:
    return np.array([[focal, 0.0, width / 2], [0.0, focal, height / 2], [0.0, 0.0, 1.0]])


def render_settings(image_width, image_height, intrinsic_matrix, extrinsic_matrix, device="cuda",
                    near=1.0, far=100.0, sh_degree=0):
    fx, fy = intrinsic_matrix[0][0], intrinsic_matrix[1][1]
    cx, cy = intrinsic_matrix[0][2], intrinsic_matrix[1][2]
    w2c = torch.tensor(extrinsic_matrix).float()
    campos = torch.inverse(w2c)[:3, 3]
    view = w2c.unsqueeze(0).transpose(1, 2)
    proj = torch.tensor([[2 * fx / image_width, 0.0, -(image_width - 2 * cx) / image_width, 0.0],
                         [0.0, 2 * fy / image_height, -(image_height - 2 * cy) / image_height, 0.0],
                         [0.0, 0.0, far / (far - near), -(far * near) / (far - near)],
                         [0.0, 0.0, 1.0, 0.0]]).float().unsqueeze(0).transpose(1, 2)
    full = view.bmm(proj)
    return GaussianRasterizationSettings(
        image_height=image_height, image_width=image_width,
        tanfovx=image_width / (2 * fx), tanfovy=image_height / (2 * fy),
        bg=torch.zeros(3, dtype=torch.float32).to(device), scale_modifier=1.0,
        viewmatrix=view.to(device), projmatrix=full.to(device), sh_degree=sh_degree,
        campos=campos.to(device), prefiltered=False)


def render_arguments(params: dict) -> dict:
    return {
        "means3D": params["means"],
        "colors_precomp": params["colors"],
        "rotations": torch.nn.functional.normalize(params["rotation_quaternions"]),
        "opacities": torch.sigmoid(params["opacity_logits"]),
        "scales": torch.exp(params["log_scales"]),
        "means2D": torch.zeros_like(params["means"], requires_grad=True) + 0,
    }


@dataclass(frozen=True)
class SceneConfig:
    name: str
    P: int
    width: int
    height: int
    focal: float
    s0: float
    sh_degree: int = -1          # -1: precomputed RGB colours
    views: tuple = ((0.0, 0.0),)  # (yaw degrees, height)
    distance: float = 4.0


# SURVEY.md 8(d) / BASELINE.json configs
RIG27 = tuple((float(yaw), h) for h in (-0.8, 0.0, 0.8) for yaw in range(0, 360, 40))
CONFIGS = {
    "C1": SceneConfig("C1", 10_000, 256, 256, 256.0, 0.02),
    "C2": SceneConfig("C2", 100_000, 800, 800, 800.0, 0.01,
                      views=((0.0, 0.0), (90.0, 0.0), (180.0, 0.0), (270.0, 0.0))),
    "C3": SceneConfig("C3", 1_000_000, 1920, 1080, 1600.0, 0.005, sh_degree=3),
    "C4": SceneConfig("C4", 1_000_000, 1920, 1080, 1600.0, 0.005, views=RIG27),
}


def synthetic_cloud(P: int, s0: float, sh_degree: int = -1, seed: int = 0, device="cuda") -> dict:
    """Leaf parameters of a random cloud, generated on CPU in the SURVEY 8(d) order, then moved."""
    g = torch.Generator().manual_seed(seed)
    means = torch.empty(P, 3)
    means[:, 0] = torch.rand(P, generator=g) * 4.4 - 2.2
    means[:, 1] = torch.rand(P, generator=g) * 2.5 - 1.25
    means[:, 2] = torch.rand(P, generator=g) * 2.0 - 1.0
    log_scales = math.log(s0) + 0.3 * torch.randn(P, 3, generator=g)
    quats = torch.nn.functional.normalize(torch.randn(P, 4, generator=g), dim=-1)
    opacity_logits = torch.randn(P, 1, generator=g)
    colors = torch.rand(P, 3, generator=g)
    out = {"means": means, "log_scales": log_scales, "rotation_quaternions": quats,
           "opacity_logits": opacity_logits, "colors": colors}
    if sh_degree >= 0:
        M = (sh_degree + 1) ** 2
        sh = 0.05 * torch.randn(P, M, 3, generator=g)
        sh[:, 0, :] = (torch.rand(P, 3, generator=g) - 0.5) / 0.28209479
        out["shs"] = sh
    return {k: v.float().contiguous().to(device) for k, v in out.items()}


def clustered_cloud(P: int, s0: float, sh_degree: int = -1, seed: int = 0, clusters: int = 16,
                    spread: float = 0.03, device="cuda") -> dict:
    """A densified-scene stand-in: the synthetic_cloud parameters with half of the means moved into
    `clusters` tight Gaussian blobs (std `spread`, centres uniform in the same box), so the tiles over
    a blob hold tens of thousands of Gaussian-tile pairs (the long-list sort and the backward's
    segment items at work) while the rest of the image stays like the uniform cloud."""
    out = synthetic_cloud(P, s0, sh_degree=sh_degree, seed=seed, device="cpu")
    g = torch.Generator().manual_seed(seed + 1000)
    lo = torch.tensor([-2.2, -1.25, -1.0])
    hi = torch.tensor([2.2, 1.25, 1.0])
    centres = lo + (hi - lo) * torch.rand(clusters, 3, generator=g)
    m = P // 2
    which = torch.randint(0, clusters, (m,), generator=g)
    means = out["means"].clone()
    means[:m] = centres[which] + spread * torch.randn(m, 3, generator=g)
    out["means"] = means.contiguous()
    return {k: v.to(device) for k, v in out.items()}


def upstream_grad(H: int, W: int, seed: int = 1, device="cuda") -> torch.Tensor:
    g = torch.Generator().manual_seed(seed)
    return torch.randn(3, H, W, generator=g).to(device)


def scene_cameras(cfg: SceneConfig, device="cuda"):
    K = intrinsics(cfg.focal, cfg.width, cfg.height)
    sh = max(cfg.sh_degree, 0)
    return [render_settings(cfg.width, cfg.height, K, look_at(yaw, h, cfg.distance), device=device,
                            sh_degree=sh) for yaw, h in cfg.views]


# The inference renders of train.py (render_and_export_frame, train.py:506-547, under torch.no_grad() at
# train.py:778): five fixed cameras (create_extrinsic_matrices, train.py:459-503) at 1280 x 720 with the
# intrinsic [[a W, 0, W / 2], [0, a W, H / 2], [0, 0, 1]] of each camera's aspect ratio a (train.py:512-525).
INFERENCE_W, INFERENCE_H = 1280, 720


def inference_rig() -> dict:
    """name -> (w2c, aspect ratio), restating create_extrinsic_matrices (train.py:459-503)."""
    d, h = 2.4, 1.3
    top = np.array([[1.0, 0.0, 0.0, 0.0], [0.0, 0.0, -1.0, 0.0], [0.0, 1.0, 0.0, 4.5], [0.0, 0.0, 0.0, 1.0]])
    return {"000": (look_at(0, h, d), 0.82), "090": (look_at(90, h, d), 0.52), "180": (look_at(180, h, d), 0.52),
            "270": (look_at(270, h, d), 0.52), "top": (top, 0.35)}


def inference_intrinsics(aspect: float, width: int = INFERENCE_W, height: int = INFERENCE_H) -> np.ndarray:
    return np.array([[aspect * width, 0, width / 2], [0, aspect * width, height / 2], [0, 0, 1]])


def inference_cameras(device="cuda"):
    """The five GaussianRasterizationSettings render_and_export_frame builds (sh_degree 0, zero bg)."""
    return [render_settings(INFERENCE_W, INFERENCE_H, inference_intrinsics(a), w2c, device=device)
            for w2c, a in inference_rig().values()]


def activated_inputs(params: dict, sh_degree: int = -1) -> dict:
    """Rasterizer inputs (``create_render_arguments`` plus SH when configured) as plain tensors."""
    a = render_arguments(params)
    if sh_degree >= 0:
        a["shs"] = params["shs"]
        a["colors_precomp"] = None
    return a
