"""Measure SURVEY.md 8(f) row f2 on the GPU: the fused SSIM (wgsr.loss)
against the reference's torch formulation on configs[2]'s frame size
(3 x 1080 x 1920 fp32).

* ssim fwd+bwd: loss_utils.ssim(rendered, gt) forward and the backward of
  1 - ssim (slam_utils.py:130, 200), window 11.
  Algorithmic bytes per plane pixel: forward 8 read + 12 written (the three
  derivative maps), backward 20 read + 4 written = 44 B.
* components: mapping_utils.compute_ssim_components(gt, rendered, 7), forward
  only: 8 B read per plane pixel + 12 B written per pixel.
Prints one JSON line; HBM peak 8 TB/s (MI355X_MICROARCH.md).
"""
import json
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "wildgs-slam-blackwell_amd", "python"))

from wgsr.loss import ssim, ssim_components  # noqa: E402

HBM_PEAK = 8.0e12


def window(ws, C, dev):
    import math
    g = torch.tensor([math.exp(-((x - ws // 2) ** 2) / float(2 * 1.5 ** 2)) for x in range(ws)])
    g = g / g.sum()
    return (g[:, None] @ g[None, :]).expand(C, 1, ws, ws).contiguous().to(dev)


def torch_ssim(img1, img2, w, ws=11):
    """loss_utils._ssim (loss_utils.py:72-99) as the reference runs it."""
    C = img1.size(-3)
    mu1 = F.conv2d(img1, w, padding=ws // 2, groups=C)
    mu2 = F.conv2d(img2, w, padding=ws // 2, groups=C)
    mu1_sq, mu2_sq, mu1_mu2 = mu1.pow(2), mu2.pow(2), mu1 * mu2
    s11 = F.conv2d(img1 * img1, w, padding=ws // 2, groups=C) - mu1_sq
    s22 = F.conv2d(img2 * img2, w, padding=ws // 2, groups=C) - mu2_sq
    s12 = F.conv2d(img1 * img2, w, padding=ws // 2, groups=C) - mu1_mu2
    return (((2 * mu1_mu2 + 1e-4) * (2 * s12 + 9e-4)) / ((mu1_sq + mu2_sq + 1e-4) * (s11 + s22 + 9e-4))).mean()


def torch_components(img1, img2, w, ws=7):
    """mapping_utils._ssim (mapping_utils.py:125-204) as the reference runs it."""
    img1, img2 = img1.unsqueeze(0), img2.unsqueeze(0)
    C = img1.size(1)
    mu1 = F.conv2d(img1, w, padding=ws // 2, groups=C)
    mu2 = F.conv2d(img2, w, padding=ws // 2, groups=C)
    mu1_sq, mu2_sq, mu1_mu2 = mu1.pow(2), mu2.pow(2), mu1 * mu2
    s11 = F.conv2d(img1 * img1, w, padding=ws // 2, groups=C) - mu1_sq
    s22 = F.conv2d(img2 * img2, w, padding=ws // 2, groups=C) - mu2_sq
    s12 = F.conv2d(img1 * img2, w, padding=ws // 2, groups=C) - mu1_mu2
    eps = torch.tensor([torch.finfo(torch.float32).eps], device=img1.device)
    s11, s22 = torch.maximum(eps, s11), torch.maximum(eps, s22)
    s12 = torch.sign(s12) * torch.minimum(torch.sqrt(s11 * s22), torch.abs(s12))
    lum = (2 * mu1_mu2 + 1e-4) / (mu1_sq + mu2_sq + 1e-4)
    con = torch.clamp((2 * torch.sqrt(s11) * torch.sqrt(s22) + 9e-4) / (s11 + s22 + 9e-4), max=0.98)
    st = torch.clamp((s12 + 4.5e-4) / (torch.sqrt(s11) * torch.sqrt(s22) + 4.5e-4), max=0.98)
    return lum.mean(1).squeeze(), con.mean(1).squeeze(), st.mean(1).squeeze()


def time_it(fn, iters=50, warmup=5):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    dev = torch.device("cuda")
    C, H, W = 3, 1080, 1920
    g = torch.Generator(device="cpu").manual_seed(0)
    gt = torch.rand(C, H, W, generator=g).to(dev)
    ren = (gt + 0.05 * torch.randn(C, H, W, generator=g).to(dev)).clamp(0, 1)
    w11, w7 = window(11, C, dev), window(7, C, dev)

    def fused():
        x = ren.detach().requires_grad_(True)
        (1.0 - ssim(x, gt)).backward()

    def ref():
        x = ren.detach().requires_grad_(True)
        (1.0 - torch_ssim(x, gt, w11)).backward()

    px = C * H * W
    res = {"workload": f"{C}x{H}x{W} fp32 (configs[2] frame)"}
    t_f, t_r = time_it(fused), time_it(ref)
    res.update(ssim_fwd_bwd_fused_ms=t_f, ssim_fwd_bwd_torch_ms=t_r, ssim_speedup=t_r / t_f,
               ssim_fused_GBps=44 * px / (t_f * 1e-3) / 1e9, ssim_fused_frac=44 * px / (t_f * 1e-3) / HBM_PEAK)
    t_cf = time_it(lambda: ssim_components(gt, ren, 7))
    with torch.no_grad():
        t_cr = time_it(lambda: torch_components(gt, ren, w7))
    cb = 8 * px + 12 * H * W
    res.update(components_fused_ms=t_cf, components_torch_ms=t_cr, components_speedup=t_cr / t_cf,
               components_fused_GBps=cb / (t_cf * 1e-3) / 1e9)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
