"""Camera matrices exactly as WildGS-SLAM's ``Camera`` builds them.

The rasteriser consumes five camera tensors (``GaussianRasterizationSettings``
fields ``viewmatrix``, ``projmatrix``, ``projmatrix_raw``, ``campos`` and the
two tangents).  This module reproduces how the reference derives them so that
tests and the bench feed the HIP path the same bytes the mapper would:

* ``getWorld2View2``      - thirdparty/gaussian_splatting/utils/graphics_utils.py:33-46
* ``getProjectionMatrix2``- thirdparty/gaussian_splatting/utils/graphics_utils.py:72-93
* ``focal2fov``           - thirdparty/gaussian_splatting/utils/graphics_utils.py:100-101
* ``world_view_transform``/``full_proj_transform``/``camera_center``
                           - src/utils/camera_utils.py:137-151
* ``SE3_exp``/``update_pose`` - src/utils/pose_utils.py:17-98

Everything here is float32 torch on the CPU (the reference builds them on the
device, but the values are identical); callers move them with ``.to(device)``.
The fixture script ``tests/golden/make_fixtures.py`` checks these restatements
against the reference helpers themselves.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch


def focal2fov(focal: float, pixels: float) -> float:
    """graphics_utils.py:100-101."""
    return 2 * math.atan(pixels / (2 * focal))


def get_world2view2(R: torch.Tensor, t: torch.Tensor) -> torch.Tensor:
    """graphics_utils.py:33-46 (translate=0, scale=1): Rt, inverted twice."""
    Rt = torch.zeros((4, 4), dtype=torch.float32)
    Rt[:3, :3] = R
    Rt[:3, 3] = t
    Rt[3, 3] = 1.0
    C2W = torch.linalg.inv(Rt)
    return torch.linalg.inv(C2W)


def get_projection_matrix2(znear, zfar, cx, cy, fx, fy, W, H) -> torch.Tensor:
    """graphics_utils.py:72-93 (column-vector convention, not transposed)."""
    left = ((2 * cx - W) / W - 1.0) * W / 2.0
    right = ((2 * cx - W) / W + 1.0) * W / 2.0
    top = ((2 * cy - H) / H + 1.0) * H / 2.0
    bottom = ((2 * cy - H) / H - 1.0) * H / 2.0
    left = znear / fx * left
    right = znear / fx * right
    top = znear / fy * top
    bottom = znear / fy * bottom
    z_sign = 1.0
    # (the entries in double, each rounded to fp32 once: as the reference's
    # element assignments into a zero fp32 tensor; one tensor construction)
    return torch.tensor([[2.0 * znear / (right - left), 0.0, (right + left) / (right - left), 0.0],
                         [0.0, 2.0 * znear / (top - bottom), (top + bottom) / (top - bottom), 0.0],
                         [0.0, 0.0, z_sign * zfar / (zfar - znear), -(zfar * znear) / (zfar - znear)],
                         [0.0, 0.0, z_sign, 0.0]], dtype=torch.float32)


def raster_fields_batched(R: torch.Tensor, T: torch.Tensor, fx, fy, cx, cy, W: int, H: int, znear: float = 0.01,
                          zfar: float = 100.0) -> dict:
    """PinholeCamera.raster_fields of n cameras sharing intrinsics in one
    pass: R [n, 3, 3], T [n, 3] -> viewmatrix / projmatrix [n, 4, 4],
    projmatrix_raw [4, 4], campos [n, 3].  The same operations batched
    (torch's batched 4x4 inverses and products on the CPU give the
    per-camera results bit for bit; tests/test_camera_host.py)."""
    n = R.shape[0]
    Rt = torch.zeros((n, 4, 4), dtype=torch.float32)
    Rt[:, :3, :3] = R
    Rt[:, :3, 3] = T
    Rt[:, 3, 3] = 1.0
    wv = torch.linalg.inv(torch.linalg.inv(Rt)).transpose(1, 2)
    proj = get_projection_matrix2(znear, zfar, cx, cy, fx, fy, W, H).transpose(0, 1)
    return dict(viewmatrix=wv, projmatrix=wv.bmm(proj.unsqueeze(0).expand(n, 4, 4)), projmatrix_raw=proj,
                campos=wv.inverse()[:, 3, :3])


def skew(x: torch.Tensor) -> torch.Tensor:
    """pose_utils.py:17-27."""
    m = torch.zeros(3, 3, dtype=x.dtype)
    m[0, 1] = -x[2]
    m[0, 2] = x[1]
    m[1, 0] = x[2]
    m[1, 2] = -x[0]
    m[2, 0] = -x[1]
    m[2, 1] = x[0]
    return m


def se3_exp(tau: torch.Tensor) -> torch.Tensor:
    """pose_utils.py:30-78: tau = [rho(3), theta(3)] -> 4x4 SE(3)."""
    rho, theta = tau[:3], tau[3:]
    W = skew(theta)
    W2 = W @ W
    angle = torch.norm(theta)
    I = torch.eye(3, dtype=tau.dtype)
    if angle < 1e-5:
        R = I + W + 0.5 * W2
        V = I + 0.5 * W + (1.0 / 6.0) * W2
    else:
        R = I + (torch.sin(angle) / angle) * W + ((1 - torch.cos(angle)) / angle**2) * W2
        V = I + W * ((1.0 - torch.cos(angle)) / angle**2) + W2 * ((angle - torch.sin(angle)) / angle**3)
    T = torch.eye(4, dtype=tau.dtype)
    T[:3, :3] = R
    T[:3, 3] = V @ rho
    return T


@dataclass
class PinholeCamera:
    """The subset of ``src/utils/camera_utils.py:Camera`` the rasteriser reads."""

    R: torch.Tensor  # [3,3] world->camera rotation
    T: torch.Tensor  # [3]   world->camera translation
    fx: float
    fy: float
    cx: float
    cy: float
    W: int
    H: int
    znear: float = 0.01
    zfar: float = 100.0

    @property
    def FoVx(self) -> float:
        return focal2fov(self.fx, self.W)

    @property
    def FoVy(self) -> float:
        return focal2fov(self.fy, self.H)

    @property
    def projection_matrix(self) -> torch.Tensor:
        # camera_utils.py:123-125 / mapper.py:111-121: stored transposed.
        return get_projection_matrix2(
            self.znear, self.zfar, self.cx, self.cy, self.fx, self.fy, self.W, self.H
        ).transpose(0, 1)

    @property
    def world_view_transform(self) -> torch.Tensor:
        return get_world2view2(self.R, self.T).transpose(0, 1)

    @property
    def full_proj_transform(self) -> torch.Tensor:
        return (
            self.world_view_transform.unsqueeze(0).bmm(self.projection_matrix.unsqueeze(0))
        ).squeeze(0)

    @property
    def camera_center(self) -> torch.Tensor:
        return self.world_view_transform.inverse()[3, :3]

    def raster_fields(self) -> dict:
        """The camera-derived ``GaussianRasterizationSettings`` fields
        (gaussian_renderer/__init__.py:55-72); the properties' operations,
        each matrix formed once."""
        wv = self.world_view_transform
        proj = self.projection_matrix
        return dict(
            image_height=int(self.H),
            image_width=int(self.W),
            tanfovx=math.tan(self.FoVx * 0.5),
            tanfovy=math.tan(self.FoVy * 0.5),
            viewmatrix=wv,
            projmatrix=wv.unsqueeze(0).bmm(proj.unsqueeze(0)).squeeze(0),
            projmatrix_raw=proj,
            campos=wv.inverse()[3, :3],
        )


def synthetic_camera(W: int, H: int, view: int = 0) -> PinholeCamera:
    """BASELINE.md synthetic camera: fx = fy = 0.9 W, centred principal point.

    View k (multi-view config) is rotated k * 2 degrees about y and translated
    0.05 k along x ("Synthetic inputs").
    """
    ang = math.radians(2.0 * view)
    c, s = math.cos(ang), math.sin(ang)
    R = torch.tensor([[c, 0.0, s], [0.0, 1.0, 0.0], [-s, 0.0, c]], dtype=torch.float32)
    T = torch.tensor([0.05 * view, 0.0, 0.0], dtype=torch.float32)
    f = 0.9 * W
    return PinholeCamera(R=R, T=T, fx=f, fy=f, cx=W / 2.0, cy=H / 2.0, W=W, H=H)
