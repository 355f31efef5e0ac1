"""GPU parity of the configs[4]-shaped mapper loop against fixtures produced
by EXECUTING the reference's own mapper code (tests/golden/
make_online_fixtures.py):

* ``wgsr.tracking.compute_grad_mask``  vs Camera.compute_grad_mask
  (camera_utils.py:157-180)                              ref_grad_mask.npz
* ``OnlineMapper.keyframe_points``     vs create_pcd_from_image(_and_depth)
  (gaussian_model.py:108-226), incl. np.median's point size  ref_pcd.npz
* ``GaussianStore.update_mapping_points`` vs Mapper._update_mapping_points
  (mapper.py:431-558), rigid and depth branches, one call per keyframe and
  all keyframes in one pass                              ref_deform.npz
* ``OnlineMapper.map_opt_online``      vs Mapper.map_opt_online
  (mapper.py:1049-1232), four iterations through both loss modes, the DINO
  term, densify_and_prune, reset_opacity_nonvisible, the Adam steps and the
  occlusion-aware visibility                             ref_map_opt_online.npz

The rasteriser inside the reference run is the float64 restatement (the
upstream CUDA source is absent), so image-level numbers carry the fp32-vs-
fp64 rounding; tolerances are written at each check.
"""
import functools
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(name):
    return np.load(os.path.join(GOLD, name))


def _t(a, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(a))
    return (t if dtype is None else t.to(dtype)).to(DEV)


def _rel(a, b):
    a = torch.as_tensor(a).detach().double().cpu()
    b = torch.as_tensor(b).detach().double().cpu()
    return float((a - b).abs().sum() / b.abs().sum().clamp_min(1e-30))


# ---------------------------------------------------------------------------
@pytest.mark.parametrize("ci", [0, 1, 2])
def test_grad_mask_matches_reference(ci):
    """Scharr taps sum in another order than conv2d: a pixel sitting on its
    block's median threshold may flip (<= 1e-3 of the block pixels); pixels
    outside the 32 x 32 block grid keep the raw intensity (rel 1e-5)."""
    from wgsr.tracking import compute_grad_mask
    F = _load("ref_grad_mask.npz")
    img = _t(F[f"c{ci}_image_u8"]).float() / 255.0
    want = torch.from_numpy(F[f"c{ci}_grad_mask"])
    got = compute_grad_mask(img, float(F["edge_threshold"])).cpu()
    H, W = img.shape[-2:]
    bh, bw = H // 32, W // 32
    inside = torch.zeros(1, H, W, dtype=torch.bool)
    inside[:, :32 * bh, :32 * bw] = True
    assert got.shape == want.shape
    assert ((got != want) & inside).float().mean().item() <= 1e-3
    assert set(torch.unique(got[inside]).tolist()) <= {0.0, 1.0}
    if (~inside).any():
        assert _rel(got[~inside], want[~inside]) <= 1e-5


# ---------------------------------------------------------------------------
@pytest.mark.parametrize("ci", [0, 1])
def test_keyframe_points_match_reference(ci):
    """Positions rel 1e-6 (Open3D's double back-projection, then fp32),
    colours exact (SH within one ulp), scales rel 1e-6 (distCUDA2 bit-exact, log/sqrt of one
    ulp), rotations and opacities exact; the adaptive point size follows
    np.median (mean of the two middle values)."""
    from wgsr.online import Keyframe, OnlineMapper
    F = _load("ref_pcd.npz")
    k = f"c{ci}_"
    fx, fy, cx, cy = (float(v) for v in F[k + "intr"])
    img = _t(F[k + "image"])
    depth = _t(F[k + "depth"])[None]
    H, W = img.shape[-2:]
    ea, eb = (float(v) for v in F[k + "exposure"])
    kf = Keyframe(ci, torch.from_numpy(F[k + "R"]), torch.from_numpy(F[k + "T"]), fx, fy, cx, cy, img, depth,
                  torch.zeros(2, 2, 64, device=DEV), exposure_a=torch.tensor([ea], device=DEV),
                  exposure_b=torch.tensor([eb], device=DEV))
    m = OnlineMapper(sh_degree=0, feature_dim=64, device=DEV)
    assert abs(m.np_median(depth[0]) - float(F[k + "np_median"])) <= 1e-7 * abs(float(F[k + "np_median"]))
    # the kept-count rule: int((1 / ds) * n) of the valid pixels
    init = bool(F[k + "init"])
    ds = int(F["pcd_downsample_init"] if init else F["pcd_downsample"])
    n_valid = int(((depth > 0) & (depth < 100.0)).sum())
    assert int((1.0 / ds) * n_valid) == F[k + "kept"].shape[0]
    xyz, feats, scales, rots, opac = m.keyframe_points(kf, init, keep=F[k + "kept"])
    torch.cuda.synchronize()
    ref_feats = torch.from_numpy(F[k + "features"]).transpose(1, 2)  # reference [n, 3, M] -> [n, M, 3]
    assert xyz.shape == F[k + "xyz"].shape
    assert _rel(xyz, F[k + "xyz"]) <= 1e-6
    assert (xyz.cpu() - torch.from_numpy(F[k + "xyz"])).abs().max() <= 1e-5
    # RGB2SH divides by C0: torch on the device multiplies by its reciprocal
    # (a CPU-scalar divisor), the fixture ran on the CPU: one ulp apart
    assert (feats.cpu() - ref_feats).abs().max() <= 2e-7 * ref_feats.abs().max()
    assert _rel(scales, F[k + "scales"]) <= 1e-6
    assert torch.equal(rots.cpu(), torch.from_numpy(F[k + "rots"]))
    assert torch.equal(opac.cpu(), torch.from_numpy(F[k + "opacities"]))


# ---------------------------------------------------------------------------
def _store_from(F, tag, P):
    from wgsr.store import GaussianStore
    feats = np.concatenate([F[f"{tag}_f_dc"], F[f"{tag}_f_rest"]], axis=1)
    st = GaussianStore(_t(F[f"{tag}_xyz"]), _t(feats), _t(F[f"{tag}_opacity"]), _t(F[f"{tag}_scaling"]),
                       _t(F[f"{tag}_rotation"]), capacity=P, kf_id=torch.from_numpy(F[f"{tag}_kf_id"]).int())
    for name, ref in (("xyz", "xyz"), ("features", "f_dc"), ("opacity", "opacity"), ("scaling", "scaling"),
                      ("rotation", "rotation")):
        st.exp_avg(name).copy_(_t(F[f"{tag}_m_{ref}"]).reshape(st.exp_avg(name).shape))
        st.exp_avg_sq(name).copy_(_t(F[f"{tag}_v_{ref}"]).reshape(st.exp_avg_sq(name).shape))
    return st


def _boundary_rows(F, ci, xyz_before):
    """Rows of a depth-branch call whose projected pixel coordinate lies within
    1e-3 of an integer: fp32 rounding may move their depth lookup by a pixel."""
    if str(F[f"c{ci}_method"]) != "depth":
        return np.zeros(xyz_before.shape[0], bool)
    w = F[f"c{ci}_w2c_old"].astype(np.float64)
    K = F["K"].astype(np.float64)
    pc = (w[:3, :3] @ xyz_before.astype(np.float64).T + w[:3, 3:4])
    pix = K @ pc
    u, v = pix[0] / pix[2], pix[1] / pix[2]
    return (np.abs(u - np.round(u)) < 1e-3) | (np.abs(v - np.round(v)) < 1e-3)


def _check_deform(st, F, tag, skip_rows=None, tol=2e-6):
    keep = np.ones(F[f"{tag}_xyz"].shape[0], bool) if skip_rows is None else ~skip_rows
    for name, ref in (("xyz", "xyz"), ("rotation", "rotation"), ("scaling", "scaling")):
        got = st.param(name).cpu().numpy()[keep]
        want = F[f"{tag}_{ref}"][keep]
        assert np.abs(got - want).max() <= tol * max(1.0, np.abs(want).max()), (tag, name)
        for mom in ("m", "v"):
            g = (st.exp_avg(name) if mom == "m" else st.exp_avg_sq(name)).cpu().numpy()
            w_ = F[f"{tag}_{mom}_{ref}"]
            if not np.any(w_):
                assert not np.any(g), (tag, name, mom, "moments must be zeroed")
            else:
                assert np.array_equal(g, w_), (tag, name, mom, "moments must be kept")
    # untouched groups
    for name, ref in (("opacity", "opacity"),):
        assert np.array_equal(st.param(name).cpu().numpy(), F[f"{tag}_{ref}"])


def test_deformation_matches_reference_call_by_call():
    """Each of the reference's calls (rigid, depth-rescale, a keyframe without
    rows = no-op, a large rotation) against its snapshot: positions /
    rotations / scales within 2e-6 of the largest magnitude (two fp32 4x4
    products in another summation order), moments exactly zeroed or kept."""
    F = _load("ref_deform.npz")
    P = int(F["P"])
    st = _store_from(F, "s0", P)
    K = torch.from_numpy(F["K"])
    for ci in range(int(F["ncalls"])):
        before = st.param("xyz").cpu().numpy().copy()
        fr = {"kf_id": int(F[f"c{ci}_kf"]), "w2c": torch.from_numpy(F[f"c{ci}_w2c"]),
              "w2c_old": torch.from_numpy(F[f"c{ci}_w2c_old"]), "method": str(F[f"c{ci}_method"])}
        if fr["method"] == "depth":
            fr["depth"], fr["depth_old"] = _t(F[f"c{ci}_depth"]), _t(F[f"c{ci}_depth_old"])
        st.update_mapping_points([fr], K)
        torch.cuda.synchronize()
        skip = _boundary_rows(F, ci, before) & (F["s0_kf_id"] == fr["kf_id"])
        assert skip.mean() < 0.02
        _check_deform(st, F, f"s{ci + 1}", skip)
        if skip.any():  # re-sync the boundary rows to the reference for the next call
            for name in ("xyz", "rotation", "scaling"):
                st.param(name)[torch.from_numpy(skip).to(DEV)] = _t(F[f"s{ci + 1}_{name}"][skip])


def test_deformation_batched_equals_sequence():
    """All keyframes of the fixture in ONE update_mapping_points call give the
    reference's sequential result (a row belongs to one keyframe; only the
    repeated normalisation rounds differently)."""
    F = _load("ref_deform.npz")
    P = int(F["P"])
    n = int(F["ncalls"])
    st = _store_from(F, "s0", P)
    frames = []
    for ci in range(n):
        fr = {"kf_id": int(F[f"c{ci}_kf"]), "w2c": torch.from_numpy(F[f"c{ci}_w2c"]),
              "w2c_old": torch.from_numpy(F[f"c{ci}_w2c_old"]), "method": str(F[f"c{ci}_method"])}
        if fr["method"] == "depth":
            fr["depth"], fr["depth_old"] = _t(F[f"c{ci}_depth"]), _t(F[f"c{ci}_depth_old"])
        frames.append(fr)
    before = F["s0_xyz"]
    skip = np.zeros(P, bool)
    for ci in range(n):
        skip |= _boundary_rows(F, ci, before) & (F["s0_kf_id"] == int(F[f"c{ci}_kf"]))
    st.update_mapping_points(frames, torch.from_numpy(F["K"]))
    torch.cuda.synchronize()
    _check_deform(st, F, f"s{n}", skip, tol=4e-6)


def test_deformation_without_rows_is_a_no_op():
    F = _load("ref_deform.npz")
    P = int(F["P"])
    st = _store_from(F, "s0", P)
    snap = {k: st.param(k).clone() for k in ("xyz", "rotation", "scaling")}
    m0 = st.exp_avg("xyz").clone()
    st.update_mapping_points([{"kf_id": 7, "w2c": torch.eye(4), "w2c_old": 2 * torch.eye(4) - torch.eye(4) * 0.5}])
    torch.cuda.synchronize()
    for k, v in snap.items():
        assert torch.equal(st.param(k), v)   # not even the rotation normalisation
    assert torch.equal(st.exp_avg("xyz"), m0)


# ---------------------------------------------------------------------------
class _Scripted:
    """Stands in for OnlineMapper.rng: returns the fixture's view picks and
    records the probability vectors map_opt_online passes."""

    def __init__(self, picks):
        self.picks = list(picks)
        self.p = []

    def choice(self, n, p=None):
        self.p.append(np.asarray(p, np.float64).copy())
        return self.picks[len(self.p) - 1]


def _online_from_fixture(F):
    from wgsr.mapping import MappingStep
    from wgsr.online import Keyframe, OnlineMapper
    C = int(F["C"])
    m = OnlineMapper(sh_degree=0, feature_dim=C, device=DEV, config={"gaussian_reset": 501}, seed=0)
    m.net.load_state_dict({k[len("mlp_before_"):]: torch.from_numpy(F[k]) for k in F.files
                           if k.startswith("mlp_before_")})
    fx, fy, cx, cy = (float(F[k]) for k in ("fx", "fy", "cx", "cy"))
    for k in range(5):
        ea, eb = (float(v) for v in F[f"kf{k}_exposure_before"])
        kf = Keyframe(k, torch.from_numpy(F[f"kf{k}_R"]), torch.from_numpy(F[f"kf{k}_T"]), fx, fy, cx, cy,
                      _t(F[f"kf{k}_image"]), _t(F[f"kf{k}_depth"])[None], _t(F[f"kf{k}_features"]),
                      exposure_a=torch.tensor([ea], device=DEV), exposure_b=torch.tensor([eb], device=DEV))
        m.keyframes[k] = kf
    lr = {g: float(F[f"before_lr_{g}"]) for g in ("xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation")}
    for g in ("f_dc", "f_rest", "opacity", "scaling", "rotation"):   # the config's rates (gaussian_model.py:276-307)
        assert abs(lr[g] - m.lr[g]) <= 1e-12 * lr[g], g
    P = F["before_xyz"].shape[0]
    ms = MappingStep(_t(F["before_xyz"]), _t(F["before_f_dc"]), _t(F["before_f_rest"]), _t(F["before_opacity"]),
                     _t(F["before_scaling"]), _t(F["before_rotation"]), 0, lr=lr, capacity=2 * P)
    st = ms.store
    st.kf_id.copy_(torch.from_numpy(F["before_kf_id"]).int())
    for name, ref in (("xyz", "xyz"), ("features", "f_dc"), ("opacity", "opacity"), ("scaling", "scaling"),
                      ("rotation", "rotation")):
        st.exp_avg(name).copy_(_t(F[f"before_m_{ref}"]).reshape(st.exp_avg(name).shape))
        st.exp_avg_sq(name).copy_(_t(F[f"before_v_{ref}"]).reshape(st.exp_avg_sq(name).shape))
        ms.steps[name] = int(F[f"before_step_{ref}"])
    st.stat("xyz_gradient_accum").copy_(_t(F["before_accum"]))
    st.stat("denom").copy_(_t(F["before_denom"]))
    st.stat("max_radii2D").copy_(_t(F["before_max_radii2D"]))
    m.ms = ms
    m.window = [int(v) for v in F["window"]]
    m._new_exposure_optimizer()
    m.iteration_count = 497
    m.iterations_after_densify_or_reset = 18
    # the reference's random draws
    m.rng = _Scripted(F["picks"])
    offs = np.concatenate([[0], np.cumsum(F["dino_perm_lens"])])
    perms = [F["dino_perms"][offs[i]:offs[i + 1]] for i in range(len(offs) - 1)]
    m._perm = lambda n: _t(perms.pop(0)).long()
    seeds = [int(s) for s in F["mlp_seeds"]]
    m.net.seed_source = lambda: seeds.pop(0)
    ms.densify_and_prune = functools.partial(ms.densify_and_prune, z=_t(F["z"]))
    losses = []
    fbu = ms.forward_backward_uncertainty

    def rec(*a, **k):
        s = torch.exp(ms.scaling)
        iso = 10.0 * (s - s.mean(dim=1, keepdim=True)).abs().mean()
        out = fbu(*a, **k)
        losses.append(float(out["loss"]) - float(iso))
        return out

    ms.forward_backward_uncertainty = rec
    return m, losses, perms, seeds


def test_map_opt_online_matches_reference():
    F = _load("ref_map_opt_online.npz")
    m, losses, perms, seeds = _online_from_fixture(F)
    split = m.map_opt_online([int(v) for v in F["window"]], 4)
    torch.cuda.synchronize()
    ms, st = m.ms, m.ms.store
    # draws consumed exactly as the reference drew them
    assert not perms and not seeds
    np.testing.assert_allclose(np.stack(m.rng.p), F["probs"], rtol=1e-12)
    assert bool(split) == bool(F["split"])
    assert m.iteration_count == int(F["iteration_count"])
    assert m.iterations_after_densify_or_reset == int(F["iterations_after"])
    # the loss of each iteration (fp32 render vs the fp64 restatement)
    np.testing.assert_allclose(losses, F["losses"], rtol=2e-4)
    # densify / prune / reset: identical rows
    assert st.P == F["after_xyz"].shape[0]
    assert np.array_equal(st.kf_id.cpu().numpy(), F["after_kf_id"])
    lr = {g: float(F[f"before_lr_{g}"]) for g in ("xyz", "f_dc", "opacity", "scaling", "rotation")}
    for name, ref, lr_g in (("xyz", "xyz", lr["xyz"]), ("features", "f_dc", lr["f_dc"]),
                            ("opacity", "opacity", lr["opacity"]), ("scaling", "scaling", lr["scaling"]),
                            ("rotation", "rotation", lr["rotation"])):
        got = st.param(name).cpu().numpy().reshape(F[f"after_{ref}"].shape)
        want = F[f"after_{ref}"]
        d = np.abs(got - want)
        # Adam moves a parameter by ~lr per step: the difference must be a
        # small fraction of that; a fresh row's first step is lr * sign(g),
        # so a gradient within rounding of 0 may flip (few elements)
        assert d.mean() <= 0.01 * lr_g, (name, d.mean(), lr_g)
        assert (d > 0.1 * lr_g + 1e-6 * np.abs(want)).mean() <= 5e-3, name
        for mom, tol in (("m", 2e-3), ("v", 5e-3)):
            g = (st.exp_avg(name) if mom == "m" else st.exp_avg_sq(name)).cpu().numpy().reshape(want.shape)
            assert _rel(g, F[f"after_{mom}_{ref}"]) <= tol, (name, mom)
        assert ms.steps[name] == int(F[f"after_step_{ref}"]), name
    assert abs(ms.lr["xyz"] - float(F["after_lr_xyz"])) <= 1e-9 * float(F["after_lr_xyz"])
    # statistics after the densify reset and the last iteration
    assert torch.equal(st.stat("denom").cpu(), torch.from_numpy(F["after_denom"]))
    assert torch.equal(st.stat("max_radii2D").cpu(), torch.from_numpy(F["after_max_radii2D"]))
    assert _rel(st.stat("xyz_gradient_accum"), F["after_accum"]) <= 1e-3
    # exposures (window keyframes moved, the others kept) and the MLP
    for k in range(5):
        got = torch.cat([m.keyframes[k].exposure_a, m.keyframes[k].exposure_b]).cpu().numpy()
        want, before = F[f"kf{k}_exposure_after"], F[f"kf{k}_exposure_before"]
        assert np.abs(got - want).max() <= 1e-3 * 0.01 + 1e-7, k
        assert np.array_equal(want == before, got == before), k
    for n_, p_ in m.net.state_dict().items():
        want = F["mlp_after_" + n_]
        d = np.abs(p_.cpu().numpy() - want)
        assert d.mean() <= 0.02 * 4e-4 and (d > 0.2 * 4e-4).mean() <= 5e-3, n_
    # occlusion-aware visibility of the window after the last iteration
    for k in (int(v) for v in F["window"]):
        got = m.occ_vis[k].cpu().numpy()
        lo, hi = F[f"occ_{k}_lo"], F[f"occ_{k}_hi"]
        assert np.all(got >= lo) and np.all(got <= hi), k
