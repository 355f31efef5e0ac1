"""ORACLE (test infrastructure only) - the uncertainty-aware mapping loss of
SURVEY.md 8(f) row f2.  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import this module, and only as the
checker; the product path (``wgsr.mapping`` over libwgsr.so) never imports it.

A torch restatement (CPU or GPU, fp32, autograd) of

* ``compute_mapping_loss_components`` -- src/utils/dyn_uncertainty/
  mapping_utils.py:206-323 (with ``MedianPool2d``, median_filter.py:9-52, and
  ``resample_tensor_to_shape``, mapping_utils.py:10-31), and
* ``get_loss_mapping_uncertainty`` -- src/utils/slam_utils.py:146-258 (the
  ``full_resolution: False`` branch, configs/wildgs_slam.yaml:11),

taking the uncertainty map (the MLP output) as a tensor instead of running the
network, so that the loss, and by autograd its gradients with respect to the
rendered image, depth, exposure and the uncertainty map, are deterministic.

Pinning: tests/golden/make_uncer_fixtures.py runs the reference's OWN
functions on CPU in the build container (loss_utils' cv2 import stubbed, a
stand-in viewpoint and a network that returns a fixed map) and commits
inputs, loss and gradients in tests/golden/uncer_cases.npz;
tests/test_oracle_uncer.py checks this restatement against them.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

EPS32 = float(torch.finfo(torch.float32).eps)
SSIM_C1, SSIM_C2 = 0.01 ** 2, 0.03 ** 2
SSIM_C3 = SSIM_C2 / 2
CLIP = 0.98

# configs/wildgs_slam.yaml:11-77 (mapping section)
DEFAULT_CONFIG = {
    "Training": {"alpha": 0.5, "rgb_boundary_threshold": 0.01, "ssim_loss": True},
    "opt_params": {"lambda_dssim": 0.2},
    "uncertainty_params": {"ssim_window_size": 7, "ssim_median_filter_size": 5, "opacity_th_for_uncer_loss": 0.9,
                           "ssim_mult": 0.5, "uncer_depth_mult": 0.2},
    "full_resolution": False,
}


def bias_factor(x: float, s: float) -> float:
    """compute_bias_factor (mapping_utils.py:44-57)."""
    return x / (1 + (1 - x) * (1 / s - 2))


def _window(ws: int, sigma: float = 1.5) -> torch.Tensor:
    g = torch.tensor([math.exp(-((x - ws // 2) ** 2) / float(2 * sigma ** 2)) for x in range(ws)])
    g = g / g.sum()
    return g[:, None].mm(g[None, :]).float()


def _conv(x, w2, C):
    ws = w2.shape[-1]
    return F.conv2d(x, w2.expand(C, 1, ws, ws).contiguous(), padding=ws // 2, groups=C)


def ssim_components(img1, img2, ws):
    """compute_ssim_components / _ssim (mapping_utils.py:99-204) for [C,H,W]."""
    C = img1.shape[-3]
    w2 = _window(ws).to(img1)[None, None]
    a, b = img1[None], img2[None]
    mu1, mu2 = _conv(a, w2, C), _conv(b, w2, C)
    mu1_sq, mu2_sq, mu1_mu2 = mu1.pow(2), mu2.pow(2), mu1 * mu2
    s1 = _conv(a * a, w2, C) - mu1_sq
    s2 = _conv(b * b, w2, C) - mu2_sq
    s12 = _conv(a * b, w2, C) - mu1_mu2
    eps = torch.tensor([EPS32], device=a.device)
    s1, s2 = torch.maximum(eps, s1), torch.maximum(eps, s2)
    s12 = torch.sign(s12) * torch.minimum(torch.sqrt(s1 * s2), torch.abs(s12))
    lum = (2 * mu1_mu2 + SSIM_C1) / (mu1_sq + mu2_sq + SSIM_C1)
    con = (2 * torch.sqrt(s1) * torch.sqrt(s2) + SSIM_C2) / (s1 + s2 + SSIM_C2)
    st = (s12 + SSIM_C3) / (torch.sqrt(s1) * torch.sqrt(s2) + SSIM_C3)
    con, st = torch.clamp(con, max=CLIP), torch.clamp(st, max=CLIP)
    return lum.mean(1).squeeze(), con.mean(1).squeeze(), st.mean(1).squeeze()


def ssim_standard(img1, img2, ws=11):
    """loss_utils.ssim (thirdparty/gaussian_splatting/utils/loss_utils.py:61-101), size_average."""
    C = img1.shape[-3]
    w2 = _window(ws).to(img1)[None, None]
    a, b = img1[None], img2[None]
    mu1, mu2 = _conv(a, w2, C), _conv(b, w2, C)
    mu1_sq, mu2_sq, mu1_mu2 = mu1.pow(2), mu2.pow(2), mu1 * mu2
    s1 = _conv(a * a, w2, C) - mu1_sq
    s2 = _conv(b * b, w2, C) - mu2_sq
    s12 = _conv(a * b, w2, C) - mu1_mu2
    m = ((2 * mu1_mu2 + SSIM_C1) * (2 * s12 + SSIM_C2)) / ((mu1_sq + mu2_sq + SSIM_C1) * (s1 + s2 + SSIM_C2))
    return m.mean()


def _resample(t, shape, mode="bilinear"):
    """resample_tensor_to_shape (mapping_utils.py:10-31)."""
    t = t.view((1, 1) + t.shape[:2])
    return F.interpolate(t, size=shape, mode=mode).squeeze(0).squeeze(0)


def _median_pool(x, k):
    """MedianPool2d(k, stride 1, padding 0, same=True) (median_filter.py:9-52)."""
    ph = pw = max(k - 1, 0)
    pad = (pw // 2, pw - pw // 2, ph // 2, ph - ph // 2)
    x = F.pad(x, pad, mode="reflect")
    x = x.unfold(2, k, 1).unfold(3, k, 1)
    return x.contiguous().view(x.size()[:4] + (-1,)).median(dim=-1)[0]


def mapping_loss_components(gt_img, rendered_img, ref_depth, rendered_depth, uncertainty, opacity, train_fraction,
                            ssim_fraction, ucfg, mask):
    """compute_mapping_loss_components (mapping_utils.py:206-323)."""
    _, h, w = gt_img.shape
    rgb_l1 = torch.abs(rendered_img * mask - gt_img * mask)
    median_depth = ref_depth.median()
    depth_threshold = min(10 * median_depth, 50)
    depth_mask = ((ref_depth > 0.01) & (ref_depth < depth_threshold)).view(*rendered_depth.shape)
    depth_l1 = torch.abs(rendered_depth * depth_mask - ref_depth * depth_mask)
    pu = torch.clip(uncertainty, min=0.1) + 1e-3
    ru = _resample(pu.detach(), (h, w))
    data_rate = 1 + 1 * bias_factor(train_fraction, 0.8)
    ru = (ru - 0.1) * data_rate + 0.1
    r_op = opacity.detach().view((h, w))
    small_op = _resample(r_op, uncertainty.shape)
    ssim_weight = 100 + 900 * bias_factor(ssim_fraction, 0.8)
    lum, con, st = ssim_components(gt_img, rendered_img, ucfg["ssim_window_size"])
    ssim_loss = torch.clip(r_op * ssim_weight * (1 - lum) * (1 - st) * (1 - con), max=5.0)
    small_ssim = _resample(ssim_loss.detach(), uncertainty.shape)
    filtered = _median_pool(small_ssim[None, None], ucfg["ssim_median_filter_size"]).squeeze(0).squeeze(0)
    small_dl = _resample(torch.clip(depth_l1.squeeze(), max=5.0).detach(), uncertainty.shape, "bicubic")
    small_depth = _resample(ref_depth.squeeze().detach(), uncertainty.shape, "bicubic")
    small_dl[small_depth > depth_threshold] = 0.0
    ul = filtered / pu ** 2 + 0.5 * torch.log(pu) + ucfg["uncer_depth_mult"] * small_dl / pu ** 2
    ul[small_op < ucfg["opacity_th_for_uncer_loss"]] = 0
    return ul, ru, rgb_l1, depth_l1


def loss_mapping_uncertainty(config, rendered_img, rendered_depth, gt_img, ref_depth, exposure_a, exposure_b,
                             opacity, uncertainty, train_frac, ssim_frac, initialization=False,
                             freeze_uncertainty_loss=False):
    """get_loss_mapping_uncertainty (slam_utils.py:146-258), full_resolution
    False; ``uncertainty`` is the network's output map."""
    if not initialization:
        rendered_img = torch.exp(exposure_a) * rendered_img + exposure_b
    alpha = config["Training"].get("alpha", 0.95)
    thr = config["Training"]["rgb_boundary_threshold"]
    _, h, w = gt_img.shape
    mask = (gt_img.sum(dim=0) > thr).view(1, h, w)
    ssim_loss = 1.0 - ssim_standard(rendered_img, gt_img) if config["Training"]["ssim_loss"] else 0.0
    ul, ru, l1_rgb, l1_depth = mapping_loss_components(gt_img, rendered_img, ref_depth, rendered_depth, uncertainty,
                                                       opacity.view(1, h, w), train_frac, ssim_frac,
                                                       config["uncertainty_params"], mask)
    if config["Training"]["ssim_loss"]:
        lam = config["opt_params"]["lambda_dssim"]
        rgb_loss = (1.0 - lam) * l1_rgb + lam * ssim_loss
    else:
        rgb_loss = l1_rgb
    weights = 0.5 / (ru.unsqueeze(0)) ** 2
    weights = torch.where(weights < 0.1, 0.0, weights)
    rgb_loss = weights * rgb_loss
    um = ref_depth < rendered_depth.detach() + 1.0
    l1_depth[um] = weights[um] * l1_depth[um]
    if freeze_uncertainty_loss:
        ul = ul.detach()
    return (alpha * rgb_loss.mean() + (1 - alpha) * l1_depth.mean()
            + config["uncertainty_params"]["ssim_mult"] * ul.mean())
