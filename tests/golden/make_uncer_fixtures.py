"""Generate tests/golden/uncer_cases.npz (run in the build container, where
/root/reference exists): inputs, loss and gradients of the reference's OWN
uncertainty-aware mapping loss for SURVEY.md 8(f) row f2.

* ``get_loss_mapping_uncertainty`` (src/utils/slam_utils.py:146-258) with the
  mapping config of configs/wildgs_slam.yaml (alpha 0.5, lambda_dssim 0.2,
  rgb_boundary_threshold 0.01, ssim window 7, median filter 5, opacity
  threshold 0.9, ssim_mult 0.5, uncer_depth_mult 0.2), on CPU.  Stand-ins:
  a viewpoint object (original_image whose ``.cuda()`` returns the CPU
  tensor, depth as numpy, exposure_a/b leaves, features) and a network that
  returns a fixed uncertainty leaf (the reference MLP applies dropout
  unconditionally, uncertainty_model.py:55, so its output is not
  reproducible).  ``loss.backward()`` gives the gradients with respect to the
  rendered image, depth, exposures and uncertainty map.
* ``compute_mapping_loss_components`` (mapping_utils.py:206-323) outputs of
  the same case (uncertainty loss map, resized uncertainty, L1 maps).

loss_utils.py imports cv2 (absent here; unused by ssim) -- a stub module is
put in sys.modules for the import only.

Usage:  python tests/golden/make_uncer_fixtures.py
"""
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"

CONFIG = {
    "Training": {"alpha": 0.5, "rgb_boundary_threshold": 0.01, "ssim_loss": True},
    "opt_params": {"lambda_dssim": 0.2},
    "uncertainty_params": {"ssim_window_size": 7, "ssim_median_filter_size": 5, "opacity_th_for_uncer_loss": 0.9,
                           "ssim_mult": 0.5, "uncer_depth_mult": 0.2},
    "full_resolution": False,
}


class _Img:
    def __init__(self, t):
        self.t = t

    def cuda(self):
        return self.t


def make_case(g, H, W, h, w):
    gt = torch.rand(3, H, W, generator=g)
    gt[:, :4, :9] = 0.0                                    # below the rgb boundary threshold
    ren = (gt + 0.1 * torch.randn(3, H, W, generator=g)).clamp(0, 1)
    ref = 1.0 + 3.0 * torch.rand(1, H, W, generator=g)
    ref[:, 5:9, 20:30] = 0.0                               # invalid depth
    ref[:, -6:, -10:] = 80.0                               # beyond min(10 median, 50)
    dep = ref + 1.5 * torch.randn(1, H, W, generator=g)    # both sides of ref < depth + 1
    opa = torch.rand(1, H, W, generator=g) * 0.3 + 0.7     # around the 0.9 threshold
    unc = torch.rand(h, w, generator=g) * 2.5              # some < 0.1 (clip), some -> weight < 0.1
    unc[0, 0] = 0.05
    ea = torch.tensor([0.05]) * torch.randn(1, generator=g)
    eb = torch.tensor([0.02]) * torch.randn(1, generator=g)
    return gt, ren, ref, dep, opa, unc, ea, eb


def main():
    sys.path.insert(0, REF)
    sys.modules.setdefault("cv2", types.ModuleType("cv2"))
    from src.utils import slam_utils
    from src.utils.dyn_uncertainty import mapping_utils as mu

    out = {}
    g = torch.Generator().manual_seed(33)
    for ci, (H, W, h, w, tf, sf, init, freeze) in enumerate(
            [(56, 70, 4, 5, 0.3, 0.3, False, False), (60, 66, 5, 6, 0.7, 0.2, False, False),
             (42, 56, 3, 4, 0.3, 0.3, True, True)]):
        gt, ren, ref, dep, opa, unc, ea, eb = make_case(g, H, W, h, w)
        r = ren.clone().requires_grad_(True)
        d = dep.clone().requires_grad_(True)
        u = unc.clone().requires_grad_(True)
        a = ea.clone().requires_grad_(True)
        b = eb.clone().requires_grad_(True)
        vp = types.SimpleNamespace(original_image=_Img(gt), depth=ref[0].numpy().copy(), exposure_a=a,
                                   exposure_b=b, features=torch.zeros(h, w, 4))
        uncertainty, loss = slam_utils.get_loss_mapping_uncertainty(
            CONFIG, r, d, vp, opa, lambda feats: u, tf, sf, initialization=init, freeze_uncertainty_loss=freeze)
        loss.backward()
        k = f"c{ci}_"
        for name, t in (("gt", gt), ("ren", ren), ("ref", ref), ("dep", dep), ("opa", opa), ("unc", unc),
                        ("ea", ea), ("eb", eb)):
            out[k + name] = t.numpy()
        out[k + "meta"] = np.array([tf, sf, float(init), float(freeze)])
        out[k + "loss"] = np.array(float(loss))
        out[k + "g_ren"] = r.grad.numpy()
        out[k + "g_dep"] = d.grad.numpy()
        out[k + "g_unc"] = u.grad.numpy() if u.grad is not None else np.zeros_like(unc.numpy())
        out[k + "g_ea"] = a.grad.numpy() if a.grad is not None else np.zeros(1, np.float32)
        out[k + "g_eb"] = b.grad.numpy() if b.grad is not None else np.zeros(1, np.float32)
        with torch.no_grad():
            ren_ab = ren if init else torch.exp(ea) * ren + eb
            mask = (gt.sum(dim=0) > 0.01).view(1, H, W)
            ul, ru, l1r, l1d = mu.compute_mapping_loss_components(gt, ren_ab, ref, dep, unc, opa, tf, sf,
                                                                  CONFIG["uncertainty_params"], mask)
        out[k + "comp_ul"], out[k + "comp_ru"] = ul.numpy(), ru.numpy()
        out[k + "comp_l1r"], out[k + "comp_l1d"] = l1r.numpy(), l1d.numpy()
    np.savez_compressed(os.path.join(HERE, "uncer_cases.npz"), **out)
    print("wrote", os.path.join(HERE, "uncer_cases.npz"), len(out), "arrays")


if __name__ == "__main__":
    main()
