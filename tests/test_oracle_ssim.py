"""CPU: the SSIM oracle (oracle/ssim.py) against the reference's own outputs
(tests/golden/ssim_cases.npz, made by tests/golden/make_ssim_fixtures.py from
src/utils/dyn_uncertainty/mapping_utils.py) and the host-side checks of
wgsr.loss (no GPU)."""
import os

import numpy as np
import pytest
import torch

from oracle import ssim as osim

GOLD = np.load(os.path.join(os.path.dirname(__file__), "golden", "ssim_cases.npz"))


@pytest.mark.parametrize("ws", [3, 5, 7, 9, 11])
def test_window_matches_reference_bit_exact(ws):
    assert np.array_equal(osim.window_2d(ws), GOLD[f"win{ws}"])


# The reference ran in fp32.  Where both window variances exceed 1e-3 it is
# accurate to fp32 rounding of O(1) values (STRICT, 121-term fp32 window sums); in flat regions
# E[x^2] - E[x]^2 cancels and the reference itself is only good to ~1e-3
# (LOOSE; those pixels are in the fixture on purpose: flat patches).
STRICT, LOOSE = 5e-5, 2e-3


def check_components(mine, ref, ok):
    d = np.abs(np.asarray(mine, np.float64) - ref)
    assert d[..., ok].max() <= STRICT, d[..., ok].max()
    assert d.max() <= LOOSE, d.max()


@pytest.mark.parametrize("ws", [7, 11])
def test_components_match_reference(ws):
    gt, ren = GOLD["comp_gt"], GOLD["comp_ren"]
    l, c, s = osim.ssim_components_f64(gt, ren, ws)
    ok = osim.well_conditioned(gt, ren, ws)
    assert 0.3 < ok.mean() < 0.99
    for mine, key in ((l, "l"), (c, "c"), (s, "s")):
        check_components(mine, GOLD[f"comp{ws}_{key}"], ok)
    assert (GOLD[f"comp{ws}_c"] == np.float32(0.98)).any()  # the clips are exercised


def test_components_batch_matches_reference():
    gt, ren = GOLD["compb_gt"], GOLD["compb_ren"]
    for n in range(gt.shape[0]):
        l, c, s = osim.ssim_components_f64(gt[n], ren[n], 7)
        ok = osim.well_conditioned(gt[n], ren[n], 7)
        for mine, key in ((l, "l"), (c, "c"), (s, "s")):
            check_components(mine, GOLD[f"compb7_{key}"][n], ok)


@pytest.mark.parametrize("ws", [7, 11])
def test_standard_ssim_pinned_by_component_identity(ws):
    x, y = GOLD[f"ident{ws}_x"], GOLD[f"ident{ws}_y"]
    np.testing.assert_allclose(osim.ssim_map_f64(x, y, ws)[0], GOLD[f"ident{ws}_map"], rtol=0, atol=2e-5)


def test_torch_restatement_matches_f64():
    g = torch.Generator().manual_seed(0)
    a = torch.rand(2, 3, 29, 41, generator=g)
    b = (a + 0.1 * torch.randn(2, 3, 29, 41, generator=g)).clamp(0, 1)
    ref = osim.ssim_f64(a.numpy(), b.numpy(), 11)
    assert abs(float(osim.ssim_torch(a, b, 11)) - ref) < 1e-6
    per = osim.ssim_torch(a, b, 11, size_average=False)
    exp = osim.ssim_map_f64(a.numpy(), b.numpy(), 11).reshape(2, -1).mean(1)
    np.testing.assert_allclose(per.numpy(), exp, atol=1e-6)


def test_wgsr_loss_refuses_cpu_and_bad_windows():
    from wgsr import loss
    a = torch.rand(3, 8, 8)
    with pytest.raises(RuntimeError):
        loss.ssim(a, a)
    with pytest.raises(ValueError):
        loss.ssim(a, a, window_size=4)
    with pytest.raises(ValueError):
        loss.ssim(a, torch.rand(3, 8, 9))
    with pytest.raises(RuntimeError):
        loss.ssim_components(a, a)
