"""Generate tests/golden/track_cases.npz (run in the build container, where
/root/reference exists): inputs, loss and gradients of the reference's OWN
get_loss_tracking (src/utils/slam_utils.py:47-82; mapper.py:896-903 calls it
with config["mapping"] and the keyframe's resized uncertainty) on CPU, for
SURVEY.md 8(f) row f2 (tracking half).

Stand-ins: a viewpoint object (original_image whose ``.cuda()`` returns the
CPU tensor, grad_mask, exposure_a/b leaves).  loss_utils.py imports cv2
(absent here, unused by this function) -- a stub module is put in
sys.modules for the import only.

Usage:  python tests/golden/make_track_fixtures.py
"""
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
CONFIG = {"Training": {"rgb_boundary_threshold": 0.01}}


class _Img:
    def __init__(self, t):
        self.t = t

    def cuda(self):
        return self.t


def main():
    sys.path.insert(0, REF)
    sys.modules.setdefault("cv2", types.ModuleType("cv2"))
    from src.utils import slam_utils

    out = {}
    g = torch.Generator().manual_seed(44)
    for ci, (H, W, with_unc) in enumerate([(40, 52, True), (33, 47, False)]):
        gt = torch.rand(3, H, W, generator=g)
        gt[:, :3, :7] = 0.0                                   # below the boundary threshold
        ren = (gt + 0.1 * torch.randn(3, H, W, generator=g)).clamp(0, 1)
        opa = torch.rand(1, H, W, generator=g)
        gm = (torch.rand(1, H, W, generator=g) > 0.5).float()
        gm[:, -2:, :] = torch.rand(1, 2, W, generator=g)     # non-binary rows (outside the 32 x 32 block grid)
        unc = torch.rand(H, W, generator=g) * 2.5 + 0.05 if with_unc else None
        ea = 0.05 * torch.randn(1, generator=g)
        eb = 0.02 * torch.randn(1, generator=g)
        r = ren.clone().requires_grad_(True)
        o = opa.clone().requires_grad_(True)
        a = ea.clone().requires_grad_(True)
        b = eb.clone().requires_grad_(True)
        vp = types.SimpleNamespace(original_image=_Img(gt), grad_mask=gm, exposure_a=a, exposure_b=b)
        loss = slam_utils.get_loss_tracking(CONFIG, r, None, o, vp, uncertainty=unc)
        loss.backward()
        k = f"t{ci}_"
        for name, t in (("gt", gt), ("ren", ren), ("opa", opa), ("gm", gm), ("ea", ea), ("eb", eb)):
            out[k + name] = t.numpy()
        if unc is not None:
            out[k + "unc"] = unc.numpy()
        out[k + "loss"] = np.array(float(loss.detach()))
        out[k + "g_ren"], out[k + "g_opa"] = r.grad.numpy(), o.grad.numpy()
        out[k + "g_ea"], out[k + "g_eb"] = a.grad.numpy(), b.grad.numpy()
    np.savez_compressed(os.path.join(HERE, "track_cases.npz"), **out)
    print("wrote", os.path.join(HERE, "track_cases.npz"), len(out), "arrays")


if __name__ == "__main__":
    main()
