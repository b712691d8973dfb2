"""One densify.py iteration on the native path (the caller side of SURVEY.md 8(a) + rows 8(f) 1-3).

``densify_iteration`` is the body of densify.py's loop (densify.py:218-247) with every piece on the
HIP kernels of ``libgsr.so``:

=====================================================  ============================================
reference (densify.py / external.py / shared.py)       here
=====================================================  ============================================
create_render_arguments + Renderer (image)  :110-126    rasterize_parameters (activations fused)
0.8 l1 + 0.2 (1 - calc_ssim)                :127-129    splat_loss.image_loss (fused L1 + SSIM)
segmentation render + loss                  :132-151    rasterize_parameters(colors = masks) + loss
update_max_2d_radii_and_visibility_mask     :154-162    splat_densify (statistics kernel)
total_loss.backward()                       :237        same (native backward kernels)
densify_gaussians                           :239-245    splat_densify.densify_gaussians
optimizer.step(); zero_grad(set_to_none)    :246-247    splat_adam.FusedAdam (one launch)
=====================================================  ============================================

``View`` restates shared.py:13-18.  The image-render ``means2D`` is a leaf that receives the same
screen-space (NDC) gradient the reference reads through ``retain_grad`` (densify.py:119).
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

import splat_densify
import splat_loss
from diff_gaussian_rasterization import GaussianRasterizationSettings, rasterize_parameters

__all__ = ["View", "densify_iteration", "create_densification_variables"]


@dataclass
class View:
    """shared.py:13-18."""
    camera_index: int
    render_settings: GaussianRasterizationSettings
    image: torch.Tensor
    segmentation_mask: torch.Tensor


def create_densification_variables(params):
    """densify.py:89-106."""
    P = params["means"].shape[0]
    dev = params["means"].device
    return splat_densify.DensificationVariables(visibility_count=torch.zeros(P, device=dev),
                                                mean_2d_gradients_accumulated=torch.zeros(P, device=dev),
                                                max_2d_radii=torch.zeros(P, device=dev))


def densify_iteration(params, view, densification_variables, optimizer, scene_radius, i, sample_fn=None):
    """densify.py:218-247 for one view.  Returns (total_loss, image_loss, segmentation_loss) as
    detached scalars (no host sync) and the densify row counts when this iteration densified."""
    rs = view.render_settings
    dv = densification_variables
    means2D = torch.zeros_like(params["means"], requires_grad=True)
    image, radii, _ = rasterize_parameters(params, rs, means2D=means2D)
    image_loss = splat_loss.image_loss(image, view.image)
    seg_params = dict(params)
    seg_params["colors"] = params["segmentation_masks"]
    seg, _, _ = rasterize_parameters(seg_params, rs)
    segmentation_loss = splat_loss.image_loss(seg, view.segmentation_mask)
    dv.means_2d = means2D  # gradient only from the colour render (densify.py:130-133)
    splat_densify.update_max_2d_radii_and_visibility_mask(radii, dv)
    total = image_loss + 3 * segmentation_loss
    total.backward()
    with torch.no_grad():
        info = splat_densify.densify_gaussians(params, dv, scene_radius, optimizer, i, sample_fn=sample_fn)
        optimizer.step()
        optimizer.zero_grad(set_to_none=True)
    return (total.detach(), image_loss.detach(), segmentation_loss.detach()), info
