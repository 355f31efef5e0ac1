"""The uncertainty-aware mapping-loss oracle (oracle/uncertainty.py) against
the reference's own get_loss_mapping_uncertainty / compute_mapping_loss_components
outputs (tests/golden/uncer_cases.npz, made by tests/golden/make_uncer_fixtures.py).
CPU only."""
import os
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import uncertainty as ou  # noqa: E402

FIX = np.load(os.path.join(ROOT, "tests", "golden", "uncer_cases.npz"))
CASES = sorted({k.split("_")[0] for k in FIX.files})


def _case(k):
    return {n[len(k) + 1:]: FIX[n] for n in FIX.files if n.startswith(k + "_")}


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.abs(a - b).sum() / max(np.abs(b).sum(), 1e-30)


@pytest.mark.parametrize("k", CASES)
def test_loss_and_gradients_match_reference(k):
    c = _case(k)
    tf, sf, init, freeze = c["meta"]
    t = {n: torch.from_numpy(c[n].copy()) for n in ("gt", "ren", "ref", "dep", "opa", "unc", "ea", "eb")}
    r = t["ren"].clone().requires_grad_(True)
    d = t["dep"].clone().requires_grad_(True)
    u = t["unc"].clone().requires_grad_(True)
    a = t["ea"].clone().requires_grad_(True)
    b = t["eb"].clone().requires_grad_(True)
    loss = ou.loss_mapping_uncertainty(ou.DEFAULT_CONFIG, r, d, t["gt"], t["ref"], a, b, t["opa"], u, float(tf),
                                       float(sf), initialization=bool(init), freeze_uncertainty_loss=bool(freeze))
    loss.backward()
    assert abs(float(loss) - float(c["loss"])) <= 1e-6 * abs(float(c["loss"]))
    assert _rel(r.grad, c["g_ren"]) <= 1e-6
    assert _rel(d.grad, c["g_dep"]) <= 1e-6
    if freeze:
        assert u.grad is None or float(u.grad.abs().sum()) == 0.0
        assert np.abs(c["g_unc"]).sum() == 0.0
    else:
        assert _rel(u.grad, c["g_unc"]) <= 1e-6
    if not init:
        assert abs(float(a.grad) - float(c["g_ea"][0])) <= 1e-5 * max(abs(float(c["g_ea"][0])), 1e-6)
        assert abs(float(b.grad) - float(c["g_eb"][0])) <= 1e-5 * max(abs(float(c["g_eb"][0])), 1e-6)


@pytest.mark.parametrize("k", CASES)
def test_components_match_reference(k):
    c = _case(k)
    tf, sf, init, _ = c["meta"]
    t = {n: torch.from_numpy(c[n].copy()) for n in ("gt", "ren", "ref", "dep", "opa", "unc", "ea", "eb")}
    ren_ab = t["ren"] if init else torch.exp(t["ea"]) * t["ren"] + t["eb"]
    H, W = t["gt"].shape[-2:]
    mask = (t["gt"].sum(dim=0) > 0.01).view(1, H, W)
    ul, ru, l1r, l1d = ou.mapping_loss_components(t["gt"], ren_ab, t["ref"], t["dep"], t["unc"], t["opa"], float(tf),
                                                  float(sf), ou.DEFAULT_CONFIG["uncertainty_params"], mask)
    np.testing.assert_allclose(ul.numpy(), c["comp_ul"], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(ru.numpy(), c["comp_ru"], rtol=1e-6, atol=1e-7)
    np.testing.assert_array_equal(l1r.numpy(), c["comp_l1r"])
    np.testing.assert_array_equal(l1d.numpy(), c["comp_l1d"])


def test_fixture_exercises_every_branch():
    """The committed cases reach the clip, threshold and mask branches."""
    seen = dict(weight_zero=False, weight_live=False, opacity_masked=False, clip_low=False, beyond_thr=False)
    for k in CASES:
        c = _case(k)
        tf = float(c["meta"][0])
        pu = np.maximum(c["unc"], 0.1) + 1e-3
        seen["clip_low"] |= bool((c["unc"] < 0.1).any())
        ru = c["comp_ru"]
        w = 0.5 / ru ** 2
        seen["weight_zero"] |= bool((w < 0.1).any())
        seen["weight_live"] |= bool((w >= 0.1).any())
        seen["opacity_masked"] |= bool((c["comp_ul"] == 0).any())
        seen["beyond_thr"] |= bool((c["ref"] > min(10 * np.median(c["ref"]), 50)).any())
        assert pu.shape == c["unc"].shape and tf >= 0
    assert all(seen.values()), seen
