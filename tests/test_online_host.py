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


def test_np_median_nan_and_zero_maps():
    """Degenerate depth maps: np.median is NaN as soon as one value is NaN
    (torch.sort puts NaN last, so the middle values alone would not say so),
    and an all-zero map gives 0."""
    from wgsr.online import OnlineMapper
    g = torch.Generator().manual_seed(7)
    for shape, nan_at in (((6, 8), [(0, 0)]), ((5, 7), [(4, 6), (2, 3)]), ((1, 1), [(0, 0)])):
        x = torch.rand(shape, generator=g) * 3
        x[0, :] = 0.0
        for ij in nan_at:
            x[ij] = float("nan")
        assert np.isnan(np.median(x.numpy()))
        assert np.isnan(OnlineMapper.np_median(x))
    z = torch.zeros(4, 6)
    assert OnlineMapper.np_median(z) == float(np.median(z.numpy())) == 0.0


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


def test_batched_deform_transform_matches_per_frame():
    """update_mapping_points forms every frame's (T, q) in one batched pass:
    within an ulp of the reference's per-frame formation."""
    from wgsr.store import deform_transform
    F = np.load(os.path.join(GOLD, "ref_deform.npz"))
    n = int(F["ncalls"])
    W = torch.stack([torch.from_numpy(F[f"c{i}_w2c"]) for i in range(n)])
    Wo = torch.stack([torch.from_numpy(F[f"c{i}_w2c_old"]) for i in range(n)])
    T, q = deform_transform(W, Wo)
    for i in range(n):
        t1, q1 = deform_transform(W[i], Wo[i])
        assert (T[i] - t1).abs().max() <= 2.5e-7 * max(1.0, float(t1.abs().max()))
        assert (q[i] - q1).abs().max() <= 2.5e-7


def _ref_eviction(cams, cur, window):
    """mapper.py:680-704 step for step (per-pair getWorld2View2 and fp32 4x4
    inverses) on (R, T) pairs."""
    from wgsr.camera import get_world2view2
    N = 2
    kf0_wc = torch.linalg.inv(get_world2view2(*cams[cur]))
    inv_dist = []
    for i in range(N, len(window)):
        ki_cw = get_world2view2(*cams[window[i]])
        d = []
        for j in range(N, len(window)):
            if i == j:
                continue
            t = ki_cw @ torch.linalg.inv(get_world2view2(*cams[window[j]]))
            d.append(1.0 / (torch.norm(t[0:3, 3]) + 1e-6).item())
        inv_dist.append(torch.sqrt(torch.norm((ki_cw @ kf0_wc)[0:3, 3])).item() * sum(d))
    return window[N + int(np.argmax(inv_dist))], inv_dist


@pytest.mark.parametrize("seed", range(6))
def test_window_eviction_matches_reference_loop(seed):
    """_add_to_window's batched inverse-distance eviction picks the keyframe
    the reference's double loop picks (random trajectories, windows of 4-12)."""
    from wgsr.online import Keyframe, OnlineMapper
    g = torch.Generator().manual_seed(seed)
    n = 4 + 2 * seed
    m = OnlineMapper(sh_degree=0, feature_dim=64, device="cpu", config={"window_size": n - 1})
    cams = {}
    for k in range(n + 1):
        a = torch.randn(3, generator=g) * 0.2
        K = torch.tensor([[0.0, -a[2], a[1]], [a[2], 0.0, -a[0]], [-a[1], a[0], 0.0]])
        R = torch.linalg.matrix_exp(K)
        T = torch.randn(3, generator=g) * (0.5 + k * 0.1)
        cams[k] = (R, T)
        m.keyframes[k] = Keyframe(k, R, T, 50.0, 50.0, 16.0, 12.0, torch.rand(3, 24, 32), torch.ones(1, 24, 32),
                                  torch.zeros(2, 2, 64))
    window = list(range(n - 1, -1, -1))
    vis = torch.ones(10, dtype=torch.long)
    m.occ_vis = {k: vis.clone() for k in window}
    got, removed = m._add_to_window(n, vis, list(window))
    want_removed, _ = _ref_eviction(cams, n, [n] + window)
    assert removed == want_removed
    assert got == [k for k in [n] + window if k != want_removed]


def _quat_torch(R):
    """general_utils.rotation_matrix_to_quaternion (general_utils.py:138-162)
    as torch ops (the form wgsr.store restates in numpy)."""
    z = torch.tensor(0.0, dtype=R.dtype)
    q = torch.zeros((R.size(0), 4), dtype=R.dtype)
    q[:, 0] = torch.sqrt(torch.max(z, 1 + R[:, 0, 0] + R[:, 1, 1] + R[:, 2, 2])) / 2
    q[:, 1] = torch.sqrt(torch.max(z, 1 + R[:, 0, 0] - R[:, 1, 1] - R[:, 2, 2])) / 2
    q[:, 2] = torch.sqrt(torch.max(z, 1 - R[:, 0, 0] + R[:, 1, 1] - R[:, 2, 2])) / 2
    q[:, 3] = torch.sqrt(torch.max(z, 1 - R[:, 0, 0] - R[:, 1, 1] + R[:, 2, 2])) / 2
    q[:, 1] *= torch.sign(q[:, 1] * (R[:, 2, 1] - R[:, 1, 2]))
    q[:, 2] *= torch.sign(q[:, 2] * (R[:, 0, 2] - R[:, 2, 0]))
    q[:, 3] *= torch.sign(q[:, 3] * (R[:, 1, 0] - R[:, 0, 1]))
    return q


def test_quaternion_numpy_form_bit_identical():
    from wgsr.store import rotation_matrix_to_quaternion
    g = torch.Generator().manual_seed(5)
    Rs = []
    for _ in range(200):
        a = torch.randn(3, generator=g) * 2.0
        K = torch.tensor([[0.0, -a[2], a[1]], [a[2], 0.0, -a[0]], [-a[1], a[0], 0.0]])
        M = torch.eye(4)
        M[:3, :3] = torch.linalg.matrix_exp(K)
        Rs.append(M)
    Rs.append(torch.eye(4))                                   # zero differences: q_i zeroed by sign(0)
    Rs.append(torch.diag(torch.tensor([1.0, -1.0, -1.0, 1.0])))  # 180 degrees about x
    R = torch.stack(Rs)
    assert torch.equal(rotation_matrix_to_quaternion(R), _quat_torch(R))
    Rd = R.double()
    assert torch.equal(rotation_matrix_to_quaternion(Rd), _quat_torch(Rd))
