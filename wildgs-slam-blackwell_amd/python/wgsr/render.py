"""The reference ``render()`` contract, for callers without the reference.

``thirdparty/gaussian_splatting/gaussian_renderer/__init__.py:24-153`` is the
only caller of the rasteriser in WildGS-SLAM.  The reference module cannot
travel to the GPU box (it imports the GaussianModel, open3d, plyfile ...), so
this is the equivalent caller used by the GPU tests and the bench: the same
tensor preparation (activated parameters, ``means2D = zeros + 0`` with
``retain_grad``, tangents from the camera FoV, the 13 settings fields, pose
deltas ``theta``/``rho``) and the same result dict.

``render_model`` is the whole reference ``render()`` on a GaussianModel-like
object (raw parameters + the activations of gaussian_model.py:54-106,
including the ``pipe.compute_cov3D_python`` / ``convert_SHs_python``
branches); ``tests/golden/make_render_fixtures.py`` pins it against the
reference's own render() + GaussianModel executed in the build container.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import torch

import torch.nn.functional as F

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


# --- gaussian_splatting utils restated (general_utils.py:97-186, sh_utils.py:24-119)

SH_C0 = 0.28209479177387814
SH_C1 = 0.4886025119029199
SH_C2 = (1.0925484305920792, -1.0925484305920792, 0.31539156525252005, -1.0925484305920792, 0.5462742152960396)
SH_C3 = (-0.5900435899266435, 2.890611442640554, -0.4570457994644658, 0.3731763325901154, -0.4570457994644658,
         1.445305721320277, -0.5900435899266435)


def build_rotation(r: torch.Tensor) -> torch.Tensor:
    """general_utils.py:113-136: quaternion (w, x, y, z), normalised inside."""
    norm = torch.sqrt(r[:, 0] * r[:, 0] + r[:, 1] * r[:, 1] + r[:, 2] * r[:, 2] + r[:, 3] * r[:, 3])
    q = r / norm[:, None]
    w, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    rows = (1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y),
            2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x),
            2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y))
    return torch.stack(rows, dim=1).reshape(-1, 3, 3)


def build_scaling_rotation(s: torch.Tensor, r: torch.Tensor) -> torch.Tensor:
    """general_utils.py:177-186: R @ diag(s)."""
    return build_rotation(r) @ torch.diag_embed(s)


def strip_symmetric(L: torch.Tensor) -> torch.Tensor:
    """general_utils.py:97-110: the 6 upper-triangle entries."""
    return torch.stack([L[:, 0, 0], L[:, 0, 1], L[:, 0, 2], L[:, 1, 1], L[:, 1, 2], L[:, 2, 2]], dim=1)


def eval_sh(deg: int, sh: torch.Tensor, dirs: torch.Tensor) -> torch.Tensor:
    """sh_utils.py:54-119 for degrees 0-3; ``sh`` is [..., C, K]."""
    assert 0 <= deg <= 3 and sh.shape[-1] >= (deg + 1) ** 2
    result = SH_C0 * sh[..., 0]
    if deg > 0:
        x, y, z = dirs[..., 0:1], dirs[..., 1:2], dirs[..., 2:3]
        result = result - SH_C1 * y * sh[..., 1] + SH_C1 * z * sh[..., 2] - SH_C1 * x * sh[..., 3]
        if deg > 1:
            xx, yy, zz, xy, yz, xz = x * x, y * y, z * z, x * y, y * z, x * z
            c = SH_C2
            result = (result + c[0] * xy * sh[..., 4] + c[1] * yz * sh[..., 5]
                      + c[2] * (2.0 * zz - xx - yy) * sh[..., 6] + c[3] * xz * sh[..., 7]
                      + c[4] * (xx - yy) * sh[..., 8])
            if deg > 2:
                c = SH_C3
                result = (result + c[0] * y * (3 * xx - yy) * sh[..., 9] + c[1] * xy * z * sh[..., 10]
                          + c[2] * y * (4 * zz - xx - yy) * sh[..., 11]
                          + c[3] * z * (2 * zz - 3 * xx - 3 * yy) * sh[..., 12]
                          + c[4] * x * (4 * zz - xx - yy) * sh[..., 13] + c[5] * z * (xx - yy) * sh[..., 14]
                          + c[6] * x * (xx - 3 * yy) * sh[..., 15])
    return result


class GaussianParams:
    """The raw parameter store of ``GaussianModel`` (gaussian_model.py:35-106)
    with its activation properties -- what ``render()`` reads."""

    def __init__(self, xyz, features_dc, features_rest, opacity, scaling, rotation, max_sh_degree: int,
                 active_sh_degree: int = 0):
        self._xyz, self._features_dc, self._features_rest = xyz, features_dc, features_rest
        self._opacity, self._scaling, self._rotation = opacity, scaling, rotation
        self.max_sh_degree, self.active_sh_degree = int(max_sh_degree), int(active_sh_degree)

    @property
    def get_xyz(self):
        return self._xyz

    @property
    def get_scaling(self):
        return torch.exp(self._scaling)

    @property
    def get_rotation(self):
        return F.normalize(self._rotation)

    @property
    def get_opacity(self):
        return torch.sigmoid(self._opacity)

    @property
    def get_features(self):
        return torch.cat((self._features_dc, self._features_rest), dim=1)

    def get_covariance(self, scaling_modifier=1.0):
        """gaussian_model.py:69-75,99-102 (the RAW rotation goes in; build_rotation normalises)."""
        L = build_scaling_rotation(scaling_modifier * self.get_scaling, self._rotation)
        return strip_symmetric(L @ L.transpose(1, 2))


def render_model(viewpoint_camera: DeviceCamera, pc: GaussianParams, pipe, bg_color: torch.Tensor,
                 scaling_modifier: float = 1.0, override_color=None):
    """gaussian_renderer/__init__.py:24-153 on a ``GaussianParams``: the same
    branches (python covariance / SH colours, override colour), the same
    rasteriser call and result dict (no mask branch: unreachable upstream)."""
    if pc.get_xyz.shape[0] == 0:
        return None
    means3D = pc.get_xyz
    scales = rotations = cov3D_precomp = None
    if getattr(pipe, "compute_cov3D_python", False):
        cov3D_precomp = pc.get_covariance(scaling_modifier)
    else:
        scales = pc.get_scaling
        if scales.shape[-1] == 1:
            scales = scales.repeat(1, 3)
        rotations = pc.get_rotation
    shs = colors_precomp = None
    if override_color is not None:
        colors_precomp = override_color
    elif getattr(pipe, "convert_SHs_python", False):
        feats = pc.get_features
        shs_view = feats.transpose(1, 2).view(-1, 3, (pc.max_sh_degree + 1) ** 2)
        dir_pp = means3D - viewpoint_camera.camera_center.repeat(feats.shape[0], 1)
        dir_pp_normalized = dir_pp / dir_pp.norm(dim=1, keepdim=True)
        colors_precomp = torch.clamp_min(eval_sh(pc.active_sh_degree, shs_view, dir_pp_normalized) + 0.5, 0.0)
    else:
        shs = pc.get_features
    screenspace_points = torch.zeros_like(means3D, dtype=means3D.dtype, requires_grad=True,
                                          device=means3D.device) + 0
    try:
        screenspace_points.retain_grad()
    except Exception:
        pass
    raster_settings = GaussianRasterizationSettings(
        image_height=int(viewpoint_camera.image_height), image_width=int(viewpoint_camera.image_width),
        tanfovx=math.tan(viewpoint_camera.FoVx * 0.5), tanfovy=math.tan(viewpoint_camera.FoVy * 0.5),
        bg=bg_color, scale_modifier=scaling_modifier, viewmatrix=viewpoint_camera.world_view_transform,
        projmatrix=viewpoint_camera.full_proj_transform, projmatrix_raw=viewpoint_camera.projection_matrix,
        sh_degree=pc.active_sh_degree, campos=viewpoint_camera.camera_center, prefiltered=False, debug=False)
    rendered_image, radii, depth, opacity_img, n_touched = GaussianRasterizer(raster_settings=raster_settings)(
        means3D=means3D, means2D=screenspace_points, shs=shs, colors_precomp=colors_precomp,
        opacities=pc.get_opacity, scales=scales, rotations=rotations, cov3D_precomp=cov3D_precomp,
        theta=viewpoint_camera.cam_rot_delta, rho=viewpoint_camera.cam_trans_delta)
    return {"render": rendered_image, "viewspace_points": screenspace_points, "visibility_filter": radii > 0,
            "radii": radii, "depth": depth, "opacity": opacity_img, "n_touched": n_touched}
