"""Synthetic Gaussian scenes (BASELINE.md "Synthetic inputs").

The reference ships no dataset-free workload, so every config of
BASELINE.json is a seeded synthetic scene generated here.  Arrays are
produced on the CPU with ``torch.Generator().manual_seed(seed)`` in float32
and are the *activated* tensors that ``render()`` hands the rasteriser
(gaussian_renderer/__init__.py:76-111): scales after ``exp``, rotations after
``normalize``, opacity after ``sigmoid``, features after ``cat``.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch


@dataclass
class GaussianScene:
    means3D: torch.Tensor    # [P,3]
    scales: torch.Tensor     # [P,3]
    rotations: torch.Tensor  # [P,4] unit quaternion (w, x, y, z)
    opacities: torch.Tensor  # [P,1]
    shs: torch.Tensor        # [P,M,3]
    sh_degree: int

    @property
    def P(self) -> int:
        return self.means3D.shape[0]

    def to(self, device) -> "GaussianScene":
        return GaussianScene(
            self.means3D.to(device), self.scales.to(device), self.rotations.to(device),
            self.opacities.to(device), self.shs.to(device), self.sh_degree,
        )


def make_scene(P: int, W: int, H: int, sh_degree: int, seed: int = 0,
               fov_margin: float = 1.1, fx_factor: float = 0.9,
               opacity_range=(0.05, 0.95),
               log_scale_range=(math.log(0.004), math.log(0.03))) -> GaussianScene:
    """BASELINE.md synthetic scene in the identity camera's frame.

    z ~ U[2, 8]; x = u z tanfovx * margin, y = v z tanfovy * margin with
    u, v ~ U[-1, 1]; log-scale ~ U[ln .004, ln .03]; quaternion ~ N(0, 1)^4
    normalised; opacity ~ U[.05, .95]; SH DC ~ N(0, .5), rest ~ N(0, .1).
    """
    g = torch.Generator().manual_seed(seed)
    tanx = W / (2.0 * fx_factor * W)
    tany = H / (2.0 * fx_factor * W)
    z = 2.0 + 6.0 * torch.rand(P, generator=g)
    u = torch.rand(P, generator=g) * 2 - 1
    v = torch.rand(P, generator=g) * 2 - 1
    means = torch.stack([u * z * tanx * fov_margin, v * z * tany * fov_margin, z], dim=1)
    lo, hi = log_scale_range
    scales = torch.exp(lo + (hi - lo) * torch.rand(P, 3, generator=g))
    q = torch.randn(P, 4, generator=g)
    q = q / q.norm(dim=1, keepdim=True)
    olo, ohi = opacity_range
    opac = olo + (ohi - olo) * torch.rand(P, 1, generator=g)
    M = (sh_degree + 1) ** 2
    shs = torch.randn(P, M, 3, generator=g) * 0.1
    shs[:, 0, :] = torch.randn(P, 3, generator=g) * 0.5
    return GaussianScene(means.float().contiguous(), scales.float().contiguous(),
                         q.float().contiguous(), opac.float().contiguous(),
                         shs.float().contiguous(), sh_degree)


def make_upstream_grads(W: int, H: int, seed: int = 1):
    """dL/dcolour [3,H,W] and dL/ddepth [1,H,W] ~ N(0, 1)."""
    g = torch.Generator().manual_seed(seed)
    gc = torch.randn(3, H, W, generator=g)
    gd = torch.randn(1, H, W, generator=g)
    return gc.float().contiguous(), gd.float().contiguous()


def make_points(P: int, seed: int = 0, extent: float = 4.0) -> torch.Tensor:
    """Point cloud for distCUDA2: uniform in a box plus some exact duplicates."""
    g = torch.Generator().manual_seed(seed)
    pts = (torch.rand(P, 3, generator=g) * 2 - 1) * extent
    if P >= 8:
        n_dup = max(1, P // 64)
        src = torch.randint(0, P, (n_dup,), generator=g)
        dst = torch.randint(0, P, (n_dup,), generator=g)
        pts[dst] = pts[src]
    return pts.float().contiguous()
