#!/usr/bin/env python
"""One WildGS mapping iteration end to end on the MI355X path.

The reference's inner mapping loop (src/mapper.py:1083-1219, non-uncertainty
branch) per iteration: render() -> get_loss_mapping_rgbd (exposure-corrected
image; 0.8 L1 + 0.2 (1 - SSIM) on rgb, masked depth L1; slam_utils.py:107-143)
+ 10 x isotropic scale loss -> backward -> max_radii2D / densification
statistics (gaussian_model.py:745-749) -> Adam step + zero_grad.

Three compositions around the SAME rasteriser (diff_gaussian_rasterization on
libwgsr): "fused" is wgsr.mapping.MappingStep (~15 launches per iteration);
"mi355x" is the reference's autograd composition with the fused HIP SSIM
(wgsr.loss.ssim) and the one-launch Adam (wgsr.optim.FusedAdam); "torch" uses
the reference's conv2d SSIM (loss_utils.py:72-99) and torch.optim.Adam, as
the reference runs them.
Synthetic scene/targets (BASELINE.md distribution); device time per iteration.
"""
import argparse
import json
import math
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
for p in (os.path.join(ROOT, "wildgs-slam-blackwell_amd", "python"), ROOT, os.path.dirname(__file__)):
    sys.path.insert(0, p)

import torch  # noqa: E402
from torch import nn  # noqa: E402

from bench_f2 import torch_ssim, window  # noqa: E402


def inverse_sigmoid(x):
    return torch.log(x / (1 - x))


class Model:
    """GaussianModel's parameter groups and densification state."""

    def __init__(self, sc, dev, opt_cls):
        M = sc.shs.shape[1]
        self.xyz = nn.Parameter(sc.means3D.to(dev).clone())
        self.f_dc = nn.Parameter(sc.shs[:, :1].to(dev).clone().contiguous())
        self.f_rest = nn.Parameter(sc.shs[:, 1:M].to(dev).clone().contiguous())
        self.opacity = nn.Parameter(inverse_sigmoid(sc.opacities.to(dev).clamp(1e-4, 1 - 1e-4)))
        self.scaling = nn.Parameter(torch.log(sc.scales.to(dev)))
        self.rotation = nn.Parameter(sc.rotations.to(dev).clone())
        P = self.xyz.shape[0]
        self.max_radii2D = torch.zeros(P, device=dev)
        self.xyz_gradient_accum = torch.zeros(P, 1, device=dev)
        self.denom = torch.zeros(P, 1, device=dev)
        groups = [{"params": [self.xyz], "lr": 1.6e-4, "name": "xyz"},
                  {"params": [self.f_dc], "lr": 2.5e-3, "name": "f_dc"},
                  {"params": [self.f_rest], "lr": 2.5e-3 / 20.0, "name": "f_rest"},
                  {"params": [self.opacity], "lr": 5e-2, "name": "opacity"},
                  {"params": [self.scaling], "lr": 5e-3, "name": "scaling"},
                  {"params": [self.rotation], "lr": 1e-3, "name": "rotation"}]
        self.optimizer = opt_cls(groups, lr=0.0, eps=1e-15)  # gaussian_model.py:309


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, default=1_000_000)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--only", choices=("fused", "mi355x", "torch"), default=None)
    a = ap.parse_args()
    from wgsr.camera import synthetic_camera
    from wgsr.loss import ssim as fused_ssim
    from wgsr.optim import FusedAdam
    from wgsr.render import DeviceCamera, render
    from wgsr.scene import make_scene
    dev = torch.device("cuda:0")
    P, W, H, deg = a.P, a.width, a.height, 3
    sc = make_scene(P, W, H, deg, seed=0)
    cam = DeviceCamera.from_pinhole(synthetic_camera(W, H, 0), dev)
    g = torch.Generator().manual_seed(7)
    gt_image = torch.rand(3, H, W, generator=g).to(dev)
    gt_depth = (2 + 6 * torch.rand(1, H, W, generator=g)).to(dev)
    exposure_a = torch.zeros(1, device=dev, requires_grad=True)
    exposure_b = torch.zeros(1, device=dev, requires_grad=True)
    bg = torch.zeros(3, device=dev)
    w11 = window(11, 3, dev)
    alpha, lam, rgb_th = 0.95, 0.2, 0.01

    def run(opt_cls, ssim_fn):
        m = Model(sc, dev, opt_cls)

        def it():
            pkg = render(cam, m.xyz, torch.sigmoid(m.opacity), torch.exp(m.scaling),
                         torch.nn.functional.normalize(m.rotation), torch.cat((m.f_dc, m.f_rest), dim=1), deg, bg)
            image, vpt, vis, radii, depth = (pkg["render"], pkg["viewspace_points"], pkg["visibility_filter"],
                                             pkg["radii"], pkg["depth"])
            image_ab = torch.exp(exposure_a) * image + exposure_b
            ssim_loss = 1.0 - ssim_fn(image_ab, gt_image)
            mask = (gt_image.sum(dim=0) > rgb_th).view(1, H, W)
            l1_rgb = torch.abs(image_ab * mask - gt_image * mask)
            loss = (1.0 - lam) * l1_rgb + lam * ssim_loss
            dmask = (gt_depth > 0.01).view(*depth.shape)
            l1_depth = torch.abs(depth * dmask - gt_depth * dmask)
            loss_mapping = alpha * loss.mean() + (1 - alpha) * l1_depth.mean()
            scaling = torch.exp(m.scaling)
            loss_mapping = loss_mapping + 10 * torch.abs(scaling - scaling.mean(dim=1).view(-1, 1)).mean()
            loss_mapping.backward()
            with torch.no_grad():
                m.max_radii2D[vis] = torch.max(m.max_radii2D[vis], radii[vis].float())
                m.xyz_gradient_accum[vis] += torch.norm(vpt.grad[vis, :2], dim=-1, keepdim=True)
                m.denom[vis] += 1
                m.optimizer.step()
                m.optimizer.zero_grad(set_to_none=True)

        for _ in range(a.warmup):
            it()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.iters):
            it()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / a.iters

    def run_fused():
        from wgsr.mapping import MappingStep
        ms = MappingStep(sc.means3D.to(dev), sc.shs[:, :1].to(dev), sc.shs[:, 1:].to(dev),
                         inverse_sigmoid(sc.opacities.to(dev).clamp(1e-4, 1 - 1e-4)), torch.log(sc.scales.to(dev)),
                         sc.rotations.to(dev), deg)
        f = synthetic_camera(W, H, 0).raster_fields()
        camd = {k: (v.to(dev) if torch.is_tensor(v) else v) for k, v in f.items()}
        ea, eb = exposure_a.detach(), exposure_b.detach()

        def it():
            ms.step(camd, gt_image, gt_depth, ea, eb, bg, alpha=alpha, lambda_dssim=lam, rgb_threshold=rgb_th)

        for _ in range(a.warmup):
            it()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.iters):
            it()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / a.iters

    ms_fused = run_fused() if a.only in (None, "fused") else float("nan")
    ms_ours = run(FusedAdam, lambda x, y: fused_ssim(x, y)) if a.only in (None, "mi355x") else float("nan")
    ms_torch = run(torch.optim.Adam, lambda x, y: torch_ssim(x, y, w11)) if a.only in (None, "torch") else float("nan")
    print(json.dumps({"workload": f"mapping iteration, {P} Gaussians, {W}x{H}, SH{deg}",
                      "ms_per_iter_fused_mapping_step": ms_fused,
                      "ms_per_iter_autograd_fused_ssim_adam": ms_ours,
                      "ms_per_iter_autograd_torch_ssim_adam": ms_torch,
                      "speedup_fused_vs_torch": ms_torch / ms_fused,
                      "note": "same rasteriser in all three; fused = wgsr.mapping.MappingStep (activations, loss, "
                              "statistics and Adam as fused launches); autograd = the reference's torch composition "
                              "with our SSIM + FusedAdam, or with conv2d SSIM + torch.optim.Adam"}))


if __name__ == "__main__":
    main()
