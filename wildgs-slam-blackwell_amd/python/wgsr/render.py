"""The reference ``render()`` contract, for callers without the reference.

``thirdparty/gaussian_splatting/gaussian_renderer/__init__.py:24-153`` is the
only caller of the rasteriser in WildGS-SLAM.  The reference module cannot
travel to the GPU box (it imports the GaussianModel, open3d, plyfile ...), so
this is the equivalent caller used by the GPU tests and the bench: the same
tensor preparation (activated parameters, ``means2D = zeros + 0`` with
``retain_grad``, tangents from the camera FoV, the 13 settings fields, pose
deltas ``theta``/``rho``) and the same result dict.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import torch

from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer

from .camera import PinholeCamera


@dataclass
class DeviceCamera:
    """``src/utils/camera_utils.py:Camera`` fields the renderer reads."""

    FoVx: float
    FoVy: float
    image_height: int
    image_width: int
    world_view_transform: torch.Tensor
    full_proj_transform: torch.Tensor
    projection_matrix: torch.Tensor
    camera_center: torch.Tensor
    cam_rot_delta: torch.Tensor = field(default=None)
    cam_trans_delta: torch.Tensor = field(default=None)

    @staticmethod
    def from_pinhole(cam: PinholeCamera, device) -> "DeviceCamera":
        return DeviceCamera(
            FoVx=cam.FoVx, FoVy=cam.FoVy, image_height=cam.H, image_width=cam.W,
            world_view_transform=cam.world_view_transform.to(device),
            full_proj_transform=cam.full_proj_transform.to(device),
            projection_matrix=cam.projection_matrix.to(device),
            camera_center=cam.camera_center.to(device),
            cam_rot_delta=torch.zeros(3, device=device, requires_grad=True),
            cam_trans_delta=torch.zeros(3, device=device, requires_grad=True))


def render(viewpoint_camera: DeviceCamera, means3D, opacity, scales, rotations, shs, sh_degree,
           bg_color: torch.Tensor, scaling_modifier: float = 1.0, colors_precomp=None):
    """Same steps and outputs as the reference ``render`` (no mask branch)."""
    if means3D.shape[0] == 0:
        return None
    screenspace_points = torch.zeros_like(means3D, dtype=means3D.dtype, requires_grad=True,
                                          device=means3D.device) + 0
    try:
        screenspace_points.retain_grad()
    except Exception:
        pass
    tanfovx = math.tan(viewpoint_camera.FoVx * 0.5)
    tanfovy = math.tan(viewpoint_camera.FoVy * 0.5)
    raster_settings = GaussianRasterizationSettings(
        image_height=int(viewpoint_camera.image_height),
        image_width=int(viewpoint_camera.image_width),
        tanfovx=tanfovx, tanfovy=tanfovy, bg=bg_color, scale_modifier=scaling_modifier,
        viewmatrix=viewpoint_camera.world_view_transform,
        projmatrix=viewpoint_camera.full_proj_transform,
        projmatrix_raw=viewpoint_camera.projection_matrix,
        sh_degree=sh_degree, campos=viewpoint_camera.camera_center,
        prefiltered=False, debug=False)
    rasterizer = GaussianRasterizer(raster_settings=raster_settings)
    rendered_image, radii, depth, opacity_img, n_touched = rasterizer(
        means3D=means3D, means2D=screenspace_points,
        shs=shs if colors_precomp is None else None, colors_precomp=colors_precomp,
        opacities=opacity, scales=scales, rotations=rotations, cov3D_precomp=None,
        theta=viewpoint_camera.cam_rot_delta, rho=viewpoint_camera.cam_trans_delta)
    return {
        "render": rendered_image,
        "viewspace_points": screenspace_points,
        "visibility_filter": radii > 0,
        "radii": radii,
        "depth": depth,
        "opacity": opacity_img,
        "n_touched": n_touched,
    }
