"""Generate tests/golden/ssim_cases.npz (run in the build container, where
/root/reference exists): inputs and outputs of the reference's OWN SSIM code
for SURVEY.md 8(f) row f2.

* ``win{ws}``: mapping_utils.create_2d_gaussian_window(ws, 1)
  (src/utils/dyn_uncertainty/mapping_utils.py:80-96; the same construction as
  loss_utils.create_window, loss_utils.py:40-58).
* ``comp_*``: mapping_utils.compute_ssim_components (:99-204) on [3, H, W]
  and [2, 3, H, W] images, window 7 (configs/wildgs_slam.yaml:71) and 11.
* ``ident_*``: single-channel pairs on which no clip / epsilon is active, with
  the reference's luminance * contrast * structure -- equal to loss_utils'
  standard SSIM map there (C3 = C2 / 2), which pins the standard SSIM
  restatement (loss_utils.py imports cv2, absent from this image).

Usage:  python tests/golden/make_ssim_fixtures.py
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"


def main():
    sys.path.insert(0, REF)
    from src.utils.dyn_uncertainty import mapping_utils as mu

    out = {}
    for ws in (3, 5, 7, 9, 11):
        out[f"win{ws}"] = mu.create_2d_gaussian_window(ws, 1)[0, 0].numpy()
    g = torch.Generator().manual_seed(21)
    H, W = 37, 53
    gt = torch.rand(3, H, W, generator=g)
    gt[:, 5:20, 10:30] = 0.25           # flat patch: epsilon and clips active
    ren = (gt + 0.08 * torch.randn(3, H, W, generator=g)).clamp(0, 1)
    ren[:, 25:, :12] = 0.7              # flat rendered region
    out["comp_gt"], out["comp_ren"] = gt.numpy(), ren.numpy()
    for ws in (7, 11):
        l, c, s = mu.compute_ssim_components(gt, ren, window_size=ws)
        out[f"comp{ws}_l"], out[f"comp{ws}_c"], out[f"comp{ws}_s"] = l.numpy(), c.numpy(), s.numpy()
    gtb = torch.rand(2, 3, 24, 31, generator=g)
    renb = (gtb + 0.1 * torch.randn(2, 3, 24, 31, generator=g)).clamp(0, 1)
    out["compb_gt"], out["compb_ren"] = gtb.numpy(), renb.numpy()
    l, c, s = mu.compute_ssim_components(gtb, renb, window_size=7)
    out["compb7_l"], out["compb7_c"], out["compb7_s"] = l.numpy(), c.numpy(), s.numpy()

    for ws in (7, 11):
        # zero-mean planes, so the zero padding adds no correlated edge
        x = torch.rand(1, 40, 48, generator=g) - 0.5
        y = 0.3 * x + 0.4 * (torch.rand(1, 40, 48, generator=g) - 0.5)
        l, c, s = mu.compute_ssim_components(x, y, window_size=ws)
        assert float(c.max()) < 0.98 and float(s.max()) < 0.98, "a clip is active: pick other inputs"
        out[f"ident{ws}_x"], out[f"ident{ws}_y"] = x.numpy(), y.numpy()
        out[f"ident{ws}_map"] = (l * c * s).numpy()
    np.savez_compressed(os.path.join(HERE, "ssim_cases.npz"), **out)
    print("wrote", os.path.join(HERE, "ssim_cases.npz"), sorted(out))


if __name__ == "__main__":
    main()
