"""Host-side logic of the configs[4]-shaped loop, on CPU (no GPU): the
numpy-median point size, the deformation's 4x4 / quaternion formation and
the per-row rigid update restated in torch, each against the fixtures made
by executing the reference's own code (tests/golden/make_online_fixtures.py).
"""
import os

import numpy as np
import pytest
import torch

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.mark.parametrize("shape", [(4, 6), (5, 7), (1, 1), (2, 1), (61, 77), (96, 128)])
def test_np_median_semantics(shape):
    """gaussian_model.py:150 uses np.median: the mean of the two middle
    values for an even count (torch.median returns the lower one)."""
    from wgsr.online import OnlineMapper
    g = torch.Generator().manual_seed(shape[0] * 100 + shape[1])
    x = torch.rand(shape, generator=g) * 5
    x[0, 0] = 0.0
    want = float(np.median(x.numpy()))
    assert OnlineMapper.np_median(x) == pytest.approx(want, rel=1e-7, abs=0)


def test_np_median_of_the_pcd_fixtures():
    from wgsr.online import OnlineMapper
    F = np.load(os.path.join(GOLD, "ref_pcd.npz"))
    for ci in (0, 1):
        d = torch.from_numpy(F[f"c{ci}_depth"])
        assert OnlineMapper.np_median(d) == pytest.approx(float(F[f"c{ci}_np_median"]), rel=1e-7, abs=0)
        if d.numel() % 2 == 0:   # the case torch.median gets wrong
            assert float(d.median()) != pytest.approx(float(F[f"c{ci}_np_median"]), rel=1e-9, abs=0)


def _qmul(q1, q2):
    w1, x1, y1, z1 = q1.unbind(-1)
    w2, x2, y2, z2 = q2.unbind(-1)
    return torch.stack((w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2, w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2,
                        w1 * y2 + y1 * w2 + z1 * x2 - x1 * z2, w1 * z2 + z1 * w2 + x1 * y2 - y1 * x2), -1)


def test_rigid_deformation_host_restatement():
    """deform_transform's (T, q) applied in torch reproduce the reference's
    rigid calls row by row (the device kernel runs the same formulas)."""
    from wgsr.store import deform_transform
    F = np.load(os.path.join(GOLD, "ref_deform.npz"))
    kf_id = F["s0_kf_id"]
    for ci in range(int(F["ncalls"])):
        if str(F[f"c{ci}_method"]) != "rigid":
            continue
        before, after = f"s{ci}", f"s{ci + 1}"
        T, q = deform_transform(torch.from_numpy(F[f"c{ci}_w2c"]), torch.from_numpy(F[f"c{ci}_w2c_old"]))
        rows = kf_id == int(F[f"c{ci}_kf"])
        if not rows.any():
            for k in ("xyz", "rotation", "m_xyz", "m_rotation"):
                assert np.array_equal(F[f"{before}_{k}"], F[f"{after}_{k}"])
            continue
        p = torch.from_numpy(F[f"{before}_xyz"][rows])
        want = torch.from_numpy(F[f"{after}_xyz"][rows])
        got = (T @ torch.cat([p, torch.ones(p.shape[0], 1)], 1).T).T[:, :3]
        assert (got - want).abs().max() <= 2e-6 * max(1.0, float(want.abs().max()))
        r = torch.nn.functional.normalize(torch.from_numpy(F[f"{before}_rotation"]))
        want_r = torch.from_numpy(F[f"{after}_rotation"])
        assert (r[~rows] - want_r[~rows]).abs().max() <= 1e-6    # every other row is normalised
        got_r = _qmul(q.expand(int(rows.sum()), 4), r[rows])
        assert (got_r - want_r[rows]).abs().max() <= 2e-6
        assert not F[f"{after}_m_xyz"].any() and not F[f"{after}_m_rotation"].any()
        assert np.array_equal(F[f"{after}_m_scaling"], F[f"{before}_m_scaling"])


def test_view_draw_matches_generator_choice():
    """map_opt_online's per-iteration view pick restates numpy's
    Generator.choice(n, p=prob) as its inverse-CDF draw (one random() per
    call): the same indices from the same generator state."""
    prob = np.array([0.05, 0.3, 0.1, 0.25, 0.2, 0.1])
    prob /= prob.sum()
    r1, r2 = np.random.default_rng(11), np.random.default_rng(11)
    cdf = prob.cumsum()
    cdf /= cdf[-1]
    a = [int(r1.choice(len(prob), p=prob)) for _ in range(20000)]
    b = [int(cdf.searchsorted(r2.random(), side="right")) for _ in range(20000)]
    assert a == b
