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

``--loss uncertainty`` times the reference's DEFAULT branch instead
(uncertainty_params.activate, mapper.py:1120-1138): the uncertainty MLP
(uncertainty_model.py: 384 -> 64 -> 64 -> 1, ReLU, dropout 0.2, softplus) on
[H/14, W/14, 384] features, get_loss_mapping_uncertainty (slam_utils.py:
146-258 with mapping_utils.compute_mapping_loss_components, restated below in
the reference's torch ops) and the MLP's Adam step.  "fused" then runs the MLP
in torch and MappingStep.forward_backward_uncertainty; "torch" runs the
restated reference composition with conv2d SSIM and torch.optim.Adam.
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
    ap.add_argument("--loss", choices=("rgbd", "uncertainty"), default="rgbd")
    ap.add_argument("--torch-mlp", action="store_true",
                    help="uncertainty mode, fused path: keep the MLP in torch (default: wgsr.mlp + FusedAdam)")
    a = ap.parse_args()
    if a.loss == "uncertainty":
        return main_uncertainty(a)
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


# --------------------------------------------------------------------------
# the reference's uncertainty-aware mapping loss, in its own torch ops
# (slam_utils.py:146-258, mapping_utils.py:99-323, median_filter.py:9-52)
def _win(ws, C, dev):
    g = torch.tensor([math.exp(-((x - ws // 2) ** 2) / float(2 * 1.5 ** 2)) for x in range(ws)])
    g = g / g.sum()
    return (g[:, None] @ g[None, :]).expand(C, 1, ws, ws).contiguous().to(dev)


def ref_components(img1, img2, w7):
    F = torch.nn.functional
    a, b = img1[None], img2[None]
    mu1, mu2 = F.conv2d(a, w7, padding=3, groups=3), F.conv2d(b, w7, padding=3, groups=3)
    mu1_sq, mu2_sq, mu1_mu2 = mu1.pow(2), mu2.pow(2), mu1 * mu2
    s1 = F.conv2d(a * a, w7, padding=3, groups=3) - mu1_sq
    s2 = F.conv2d(b * b, w7, padding=3, groups=3) - mu2_sq
    s12 = F.conv2d(a * b, w7, padding=3, groups=3) - mu1_mu2
    eps = torch.tensor([torch.finfo(torch.float32).eps]).to(a.device)
    s1, s2 = torch.maximum(eps, s1), torch.maximum(eps, s2)
    s12 = torch.sign(s12) * torch.minimum(torch.sqrt(s1 * s2), torch.abs(s12))
    lum = (2 * mu1_mu2 + 1e-4) / (mu1_sq + mu2_sq + 1e-4)
    con = torch.clamp((2 * torch.sqrt(s1) * torch.sqrt(s2) + 9e-4) / (s1 + s2 + 9e-4), max=0.98)
    st = torch.clamp((s12 + 4.5e-4) / (torch.sqrt(s1) * torch.sqrt(s2) + 4.5e-4), max=0.98)
    return lum.mean(1).squeeze(), con.mean(1).squeeze(), st.mean(1).squeeze()


def ref_uncer_loss(image, depth, opacity, gt, ref_depth, ea, eb, uncertainty, w11, w7, tf=0.3, sf=0.3):
    F = torch.nn.functional
    bias = lambda x, s: x / (1 + (1 - x) * (1 / s - 2))  # noqa: E731

    def rs(t, shape, mode="bilinear"):
        return F.interpolate(t.view((1, 1) + t.shape[:2]), size=shape, mode=mode).squeeze(0).squeeze(0)

    img = torch.exp(ea) * image + eb
    _, h, w = gt.shape
    mask = (gt.sum(dim=0) > 0.01).view(1, h, w)
    ssim_loss = 1.0 - torch_ssim(img, gt, w11)
    rgb_l1 = torch.abs(img * mask - gt * mask)
    med = ref_depth.median()
    thr = min(10 * med, 50)
    dmask = ((ref_depth > 0.01) & (ref_depth < thr)).view(*depth.shape)
    depth_l1 = torch.abs(depth * dmask - ref_depth * dmask)
    pu = torch.clip(uncertainty, min=0.1) + 1e-3
    ru = (rs(pu.detach(), (h, w)) - 0.1) * (1 + bias(tf, 0.8)) + 0.1
    rop = opacity.detach().view((h, w))
    sop = rs(rop, uncertainty.shape)
    lum, con, st = ref_components(gt, img, w7)
    sl = torch.clip(rop * (100 + 900 * bias(sf, 0.8)) * (1 - lum) * (1 - st) * (1 - con), max=5.0)
    ss = rs(sl.detach(), uncertainty.shape)
    x = F.pad(ss[None, None], (2, 2, 2, 2), mode="reflect").unfold(2, 5, 1).unfold(3, 5, 1)
    filt = x.contiguous().view(x.size()[:4] + (-1,)).median(dim=-1)[0].squeeze(0).squeeze(0)
    sdl = rs(torch.clip(depth_l1.squeeze(), max=5.0).detach(), uncertainty.shape, "bicubic")
    sd = rs(ref_depth.squeeze().detach(), uncertainty.shape, "bicubic")
    sdl[sd > thr] = 0.0
    ul = filt / pu ** 2 + 0.5 * torch.log(pu) + 0.2 * sdl / pu ** 2
    ul[sop < 0.9] = 0
    rgb_loss = 0.8 * rgb_l1 + 0.2 * ssim_loss
    weights = 0.5 / (ru.unsqueeze(0)) ** 2
    weights = torch.where(weights < 0.1, 0.0, weights)
    rgb_loss = weights * rgb_loss
    um = ref_depth < depth.detach() + 1.0
    depth_l1[um] = weights[um] * depth_l1[um]
    return 0.5 * rgb_loss.mean() + 0.5 * depth_l1.mean() + 0.5 * ul.mean()


class UncerMLP(nn.Module):
    """uncertainty_model.MLPNetwork (384 -> 64 -> 64 -> 1, dropout 0.2, softplus)."""

    def __init__(self, c=384):
        super().__init__()
        self.l1, self.l2, self.out = nn.Linear(c, 64), nn.Linear(64, 64), nn.Linear(64, 1)

    def forward(self, x):
        F = torch.nn.functional
        H, W, C = x.shape
        y = x.view(-1, C)
        for layer in (self.l1, self.l2):
            y = F.dropout(F.relu(layer(y)), p=0.2)
        return F.softplus(self.out(y)).view(H, W)


def main_uncertainty(a):
    from wgsr.camera import synthetic_camera
    from wgsr.mapping import MappingStep
    from wgsr.render import DeviceCamera, render
    from wgsr.scene import make_scene
    dev = torch.device("cuda:0")
    P, W, H, deg = a.P, a.width, a.height, 3
    h, w = H // 14, W // 14
    sc = make_scene(P, W, H, deg, seed=0)
    cam = DeviceCamera.from_pinhole(synthetic_camera(W, H, 0), dev)
    g = torch.Generator().manual_seed(7)
    gt_image = torch.rand(3, H, W, generator=g).to(dev)
    gt_depth = (2 + 6 * torch.rand(1, H, W, generator=g)).to(dev)
    feats = torch.randn(h, w, 384, generator=g).to(dev)
    bg = torch.zeros(3, device=dev)
    w11, w7 = _win(11, 3, dev), _win(7, 3, dev)

    def timed(it):
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

    def run_torch():
        m = Model(sc, dev, torch.optim.Adam)
        torch.manual_seed(0)
        net = UncerMLP().to(dev)
        uopt = torch.optim.Adam(net.parameters(), lr=4e-4, weight_decay=1e-5)
        ea = torch.zeros(1, device=dev, requires_grad=True)
        eb = torch.zeros(1, device=dev, requires_grad=True)
        kopt = torch.optim.Adam([ea, eb], lr=0.01)

        def it():
            pkg = render(cam, m.xyz, torch.sigmoid(m.opacity), torch.exp(m.scaling),
                         torch.nn.functional.normalize(m.rotation), torch.cat((m.f_dc, m.f_rest), dim=1), deg, bg)
            vpt, vis, radii = pkg["viewspace_points"], pkg["visibility_filter"], pkg["radii"]
            img = torch.exp(ea) * pkg["render"] + eb  # map_opt_online's pre-exposed input (mapper.py:1129)
            lm = ref_uncer_loss(img, pkg["depth"], pkg["opacity"], gt_image, gt_depth, ea, eb, net(feats),
                                w11, w7)
            scaling = torch.exp(m.scaling)
            lm = lm + 10 * torch.abs(scaling - scaling.mean(dim=1).view(-1, 1)).mean()
            lm.backward()
            with torch.no_grad():
                m.max_radii2D[vis] = torch.max(m.max_radii2D[vis], radii[vis].float())
                m.xyz_gradient_accum[vis] += torch.norm(vpt.grad[vis, :2], dim=-1, keepdim=True)
                m.denom[vis] += 1
                m.optimizer.step()
                m.optimizer.zero_grad(set_to_none=True)
                kopt.step()
                kopt.zero_grad(set_to_none=True)
                uopt.step()
                uopt.zero_grad()
        return timed(it)

    def run_fused():
        ms = MappingStep(sc.means3D.to(dev), sc.shs[:, :1].to(dev), sc.shs[:, 1:].to(dev),
                         inverse_sigmoid(sc.opacities.to(dev).clamp(1e-4, 1 - 1e-4)), torch.log(sc.scales.to(dev)),
                         sc.rotations.to(dev), deg)
        f = synthetic_camera(W, H, 0).raster_fields()
        camd = {k: (v.to(dev) if torch.is_tensor(v) else v) for k, v in f.items()}
        torch.manual_seed(0)
        from wgsr.optim import FusedAdam
        if a.torch_mlp:
            net = UncerMLP().to(dev)
            uopt = torch.optim.Adam(net.parameters(), lr=4e-4, weight_decay=1e-5)
        else:
            from wgsr.mlp import UncertaintyMLP
            net = UncertaintyMLP(384).to(dev)
            uopt = FusedAdam(net.parameters(), lr=4e-4, weight_decay=1e-5)
        ea = torch.zeros(1, device=dev, requires_grad=True)
        eb = torch.zeros(1, device=dev, requires_grad=True)
        kopt = (torch.optim.Adam if a.torch_mlp else FusedAdam)([ea, eb], lr=0.01)  # keyframe exposure optimiser
        med = gt_depth.median()  # constant per keyframe

        def it():
            out = ms.forward_backward_uncertainty(camd, gt_image, gt_depth, ea, eb, bg, net(feats), 0.3, 0.3,
                                                  median_depth=med)
            ms.optimizer_step()
            ea.grad, eb.grad = out["dexposure_a"], out["dexposure_b"]
            kopt.step()
            uopt.step()
            uopt.zero_grad()
        return timed(it)

    ms_fused = run_fused() if a.only in (None, "fused") else float("nan")
    ms_torch = run_torch() if a.only in (None, "torch") else float("nan")
    print(json.dumps({"workload": f"uncertainty-aware mapping iteration, {P} Gaussians, {W}x{H}, SH{deg}, "
                                  f"features {h}x{w}x384",
                      "ms_per_iter_fused_mapping_step": ms_fused,
                      "ms_per_iter_reference_torch_composition": ms_torch,
                      "speedup_fused_vs_torch": ms_torch / ms_fused,
                      "mlp": "torch" if a.torch_mlp else "wgsr.mlp (HIP) + FusedAdam",
                      "note": "same rasteriser in both; fused = MLP + MappingStep.forward_backward_uncertainty"
                              " + fused Adam; torch = the reference's ops (conv2d SSIM and components, interpolate, "
                              "unfold median, torch.optim.Adam)"}))


if __name__ == "__main__":
    main()
