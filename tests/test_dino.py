"""CPU parity of the DINO regulariser restatement (wgsr.uncertainty.
dino_regularization_loss) against the reference's own
compute_dino_regularization_loss outputs (tests/golden/dino_cases.npz, made
by tests/golden/make_dino_fixtures.py).  Pure torch (no kernel of ours):
value rel 1e-6, gradient w.r.t. the uncertainty rel-L1 1e-6."""
import os

import numpy as np
import torch

from _util import GOLDEN, rel_l1


def test_dino_regularizer_matches_reference():
    from wgsr.uncertainty import dino_regularization_loss
    z = np.load(os.path.join(GOLDEN, "dino_cases.npz"))
    for ci in range(3):
        k = f"c{ci}_"
        unc = torch.from_numpy(z[k + "unc"]).requires_grad_(True)
        feat = torch.from_numpy(z[k + "feat"])
        if bool(z[k + "as_list"]):
            loss = dino_regularization_loss([unc.unsqueeze(-1)], [feat])
        else:
            loss = dino_regularization_loss(unc, feat)
        loss.backward()
        ref = float(z[k + "loss"])
        assert abs(float(loss) - ref) <= 1e-6 * abs(ref), (ci, float(loss), ref)
        assert rel_l1(unc.grad.numpy(), z[k + "grad"]) <= 1e-6, ci
