"""The tracking-loss oracle (oracle/tracking.py) against the reference's own
get_loss_tracking outputs (tests/golden/track_cases.npz, made by
tests/golden/make_track_fixtures.py), and the grad-mask restatement's block
semantics on hand-built images.  CPU only."""
import os
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import tracking as ot  # noqa: E402

FIX = np.load(os.path.join(ROOT, "tests", "golden", "track_cases.npz"))
CASES = sorted({k.split("_")[0] for k in FIX.files})


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.abs(a - b).sum() / max(np.abs(b).sum(), 1e-30)


@pytest.mark.parametrize("k", CASES)
def test_loss_and_gradients_match_reference(k):
    c = {n[len(k) + 1:]: FIX[n] for n in FIX.files if n.startswith(k + "_")}
    t = {n: torch.from_numpy(c[n].copy()) for n in ("gt", "ren", "opa", "gm", "ea", "eb")}
    r, o, a, b = (t[n].clone().requires_grad_(True) for n in ("ren", "opa", "ea", "eb"))
    unc = torch.from_numpy(c["unc"].copy()) if "unc" in c else None
    loss = ot.loss_tracking(r, o, t["gt"], a, b, t["gm"], unc)
    loss.backward()
    assert abs(float(loss) - float(c["loss"])) <= 1e-6 * abs(float(c["loss"]))
    for got, want in ((r.grad, c["g_ren"]), (o.grad, c["g_opa"]), (a.grad, c["g_ea"]), (b.grad, c["g_eb"])):
        assert _rel(got, want) <= 1e-6


def test_grad_mask_block_semantics():
    """A vertical step edge: inside each grid block the pixels above 4 x the
    block median become 1, the rest 0; a block whose threshold is >= 1 becomes
    all 0 (the reference's second assignment also clears the new 1s); rows /
    columns outside the 32 x 32 grid keep the raw intensity."""
    H, W = 330, 330                     # 10 x 10 pixel blocks; rows / cols 320..329 outside the grid
    img = torch.full((3, H, W), 0.5)
    img[:, :, 150:] = 0.9               # edge between columns 149 and 150
    m = ot.compute_grad_mask(img, 4)
    inten_edge = 0.4 * 16 / 32          # Scharr response of a 0.4 step, / 32
    inner = m[0, :320, :320]
    assert set(torch.unique(inner).tolist()) <= {0.0, 1.0}
    # the blocks holding the edge columns have median 0 -> threshold 0 -> edge pixels 1
    assert float(inner[:, 149].min()) == 1.0 and float(inner[:, 150].min()) == 1.0
    assert float(inner[:, :148].max()) == 0.0 and float(inner[:, 152:].max()) == 0.0
    # outside the grid: raw intensity
    torch.testing.assert_close(m[0, 320:, 149], torch.full((10,), inten_edge))
    assert abs(float(m[0, 10, 325])) <= 1e-6  # flat region (rounding of the grey mean only)
    # every pixel of a block above threshold 1: all zero
    img2 = torch.rand(3, 64, 64, generator=torch.Generator().manual_seed(0)) * 400 + 1
    m2 = ot.compute_grad_mask(img2, 4)
    assert float(m2.abs().sum()) == 0.0
