"""GPU parity of the mapper's other loops against fixtures produced by
EXECUTING the reference's own mapper code (tests/golden/
make_online_fixtures.py, VERDICT r4 "Next round" item 1):

* ``OnlineMapper.initialize_map_opt``  vs Mapper.initialize_map_opt
  (mapper.py:922-1047): a densify at the first iteration, reset_opacity at
  iteration_count == init_gaussian_reset, the strided DINO term, no exposure
  step, the occlusion-aware visibility               ref_init_map_opt.npz
* ``OnlineMapper.final_refine``        vs Mapper.final_refine
  (mapper.py:1234-1372): across the frozen-uncertainty / DINO switch at 200,
  densification statistics untouched                 ref_final_refine.npz
* ``OnlineMapper.refine_pose_non_key_frame`` (wgsr.tracking.PoseRefine) vs
  Mapper.refine_pose_non_key_frame (mapper.py:810-917): the tracking
  uncertainty, the pose after 1 / 5 iterations and at convergence
                                                      ref_refine_pose.npz
* ``OnlineMapper.insert_keyframe``     vs one pass of Mapper.run's
  per-keyframe body (mapper.py:184-266): visibility render, _add_to_window
  (overlap removal AND distance eviction), extend_from_pcd_seq, a fresh
  exposure Adam, map_opt_online with a densify, the extra iteration
                                                      ref_run_body.npz

The rasteriser inside the reference run is the float64 restatement (the
upstream CUDA source is absent), so image-level numbers carry the fp32-vs-
fp64 rounding; tolerances are written at each check.  Random draws (view
picks, DINO permutations, dropout seeds, split noise, the point subset) are
the reference run's own, fed through the instance's stand-ins.
"""
import functools
import os

import numpy as np
import pytest
import torch

from test_gpu_online_ref import _Scripted

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
GROUPS = (("xyz", "xyz"), ("features", "f_dc"), ("opacity", "opacity"), ("scaling", "scaling"),
          ("rotation", "rotation"))


def _load(name):
    return np.load(os.path.join(GOLD, name))


def _t(a, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(a))
    return (t if dtype is None else t.to(dtype)).to(DEV)


def _rel(a, b):
    a = torch.as_tensor(a).detach().double().cpu()
    b = torch.as_tensor(b).detach().double().cpu()
    return float((a - b).abs().sum() / b.abs().sum().clamp_min(1e-30))


def _keyframe(F, k):
    from wgsr.online import Keyframe
    fx, cx, cy = (float(F[n]) for n in ("fx", "cx", "cy"))
    ea, eb = (float(v) for v in F[f"kf{k}_exposure_before"])
    return Keyframe(k, torch.from_numpy(F[f"kf{k}_R"]), torch.from_numpy(F[f"kf{k}_T"]), fx, fx, cx, cy,
                    _t(F[f"kf{k}_image"]), _t(F[f"kf{k}_depth"])[None], _t(F[f"kf{k}_features"]),
                    exposure_a=torch.tensor([ea], device=DEV), exposure_b=torch.tensor([eb], device=DEV))


def _mapping_step(F, tag, cap_mult=2, stats=True):
    from wgsr.mapping import MappingStep
    lr = {g: float(F[f"{tag}_lr_{g}"]) for g in ("xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation")}
    P = F[f"{tag}_xyz"].shape[0]
    ms = MappingStep(_t(F[f"{tag}_xyz"]), _t(F[f"{tag}_f_dc"]), _t(F[f"{tag}_f_rest"]), _t(F[f"{tag}_opacity"]),
                     _t(F[f"{tag}_scaling"]), _t(F[f"{tag}_rotation"]), 0, lr=lr, capacity=cap_mult * P)
    st = ms.store
    st.kf_id.copy_(torch.from_numpy(F[f"{tag}_kf_id"]).int())
    for name, ref in GROUPS:
        st.exp_avg(name).copy_(_t(F[f"{tag}_m_{ref}"]).reshape(st.exp_avg(name).shape))
        st.exp_avg_sq(name).copy_(_t(F[f"{tag}_v_{ref}"]).reshape(st.exp_avg_sq(name).shape))
        ms.steps[name] = int(F[f"{tag}_step_{ref}"])
    if stats:
        st.stat("xyz_gradient_accum").copy_(_t(F[f"{tag}_accum"]))
        st.stat("denom").copy_(_t(F[f"{tag}_denom"]))
        st.stat("max_radii2D").copy_(_t(F[f"{tag}_max_radii2D"]))
    return ms


def _mapper(F, nkf, window, it_count, it_after, config=None):
    """An OnlineMapper in the fixture's "before" state with the reference
    run's draws scripted in."""
    from wgsr.online import OnlineMapper
    m = OnlineMapper(sh_degree=0, feature_dim=int(F["C"]), device=DEV, config=config, seed=0)
    m.net.load_state_dict({k[len("mlp_before_"):]: torch.from_numpy(F[k]) for k in F.files
                           if k.startswith("mlp_before_")})
    for k in range(nkf):
        m.keyframes[k] = _keyframe(F, k)
    ms = _mapping_step(F, "before")
    for g in ("f_dc", "f_rest", "opacity", "scaling", "rotation"):   # the config's rates (gaussian_model.py:276-307)
        assert abs(ms.lr[g] - m.lr[g]) <= 1e-12 * ms.lr[g], g
    m.ms = ms
    m.window = list(window)
    m._new_exposure_optimizer()
    m.iteration_count, m.iterations_after_densify_or_reset = it_count, it_after
    m.rng = _Scripted(F["picks"])
    lens = F["dino_perm_lens"] if "dino_perm_lens" in F.files else np.zeros(0, np.int64)
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    perms = [F["dino_perms"][offs[i]:offs[i + 1]] for i in range(len(lens))]
    m._perm = lambda n: _t(perms.pop(0)).long()
    seeds = [int(s) for s in F["mlp_seeds"]]
    m.net.seed_source = lambda: seeds.pop(0)
    if "z" in F.files:
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


def _check_state(m, F, nkf, stats="after", accum_tol=1e-3):
    """Parameters, Adam moments / steps, learning rate, statistics, exposures
    and the MLP against the fixture's "after" snapshot."""
    ms, st = m.ms, m.ms.store
    assert st.P == F["after_xyz"].shape[0]
    assert np.array_equal(st.kf_id.cpu().numpy(), F["after_kf_id"])
    for name, ref in GROUPS:
        lr_g = float(F[f"before_lr_{ref}"])
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
    assert m.iteration_count == int(F["after_iteration_count"])
    assert m.iterations_after_densify_or_reset == int(F["after_iterations_after"])
    if stats == "after":
        assert torch.equal(st.stat("denom").cpu(), torch.from_numpy(F["after_denom"]))
        assert torch.equal(st.stat("max_radii2D").cpu(), torch.from_numpy(F["after_max_radii2D"]))
        assert _rel(st.stat("xyz_gradient_accum"), F["after_accum"]) <= accum_tol
    elif stats == "unchanged":
        for n in ("xyz_gradient_accum", "denom", "max_radii2D"):
            ref = {"xyz_gradient_accum": "accum"}.get(n, n)
            assert torch.equal(st.stat(n).cpu(), torch.from_numpy(F[f"before_{ref}"])), n
            assert np.array_equal(F[f"before_{ref}"], F[f"after_{ref}"]), n
    for k in range(nkf):
        got = torch.cat([m.keyframes[k].exposure_a, m.keyframes[k].exposure_b]).cpu().numpy()
        want, before = F[f"after_kf{k}_exposure"], F[f"kf{k}_exposure_before"]
        assert np.abs(got - want).max() <= 1e-3 * 0.01 + 1e-7, k
        assert np.array_equal(want == before, got == before), k
    for n_, p_ in m.net.state_dict().items():
        want = F["after_mlp_" + n_]
        d = np.abs(p_.cpu().numpy() - want)
        assert d.mean() <= 0.02 * 4e-4 and (d > 0.2 * 4e-4).mean() <= 5e-3, n_


def _check_occ(m, F, kfs):
    """n_touched > 0 of each keyframe's last render: only Gaussians whose
    contribution sits within 1e-5 of the 0.5 threshold may differ."""
    for k in kfs:
        got = m.occ_vis[k].cpu().numpy()
        lo, hi = F[f"occ_{k}_lo"], F[f"occ_{k}_hi"]
        assert got.shape == lo.shape, k
        assert np.all(got >= lo) and np.all(got <= hi), k


# ---------------------------------------------------------------------------
def test_initialize_map_opt_matches_reference():
    F = _load("ref_init_map_opt.npz")
    cfg = {"init_gaussian_update": int(F["init_gaussian_update"]), "init_gaussian_reset": int(F["init_gaussian_reset"])}
    m, losses, perms, seeds = _mapper(F, int(F["nkf"]), [int(v) for v in F["window"]], 0, 0, cfg)
    assert int(F["n_densify"]) == 1
    m.initialize_map_opt(int(F["init_itr_num"]))
    torch.cuda.synchronize()
    assert not perms and not seeds
    assert all(p is None or not np.asarray(p).shape for p in m.rng.p)   # uniform draws (no p)
    np.testing.assert_allclose(losses, F["losses"], rtol=2e-4)
    assert [e[1] for e in m.events] == ["densify", "reset_opacity"]
    _check_state(m, F, int(F["nkf"]))
    # the initialisation loss has no exposure term: nothing stepped
    for k in range(int(F["nkf"])):
        assert m.kopt_steps.get(k, 0) == 0
    _check_occ(m, F, sorted(set(int(v) for v in F["picks"])))


def test_final_refine_matches_reference():
    F = _load("ref_final_refine.npz")
    m, losses, perms, seeds = _mapper(F, int(F["nkf"]), [int(v) for v in F["window"]], 2000, 197)
    m.final_refine(iters=3)
    torch.cuda.synchronize()
    assert not perms and not seeds
    assert len(F["dino_perm_lens"]) == 1          # the DINO term only at iterations_after == 200
    np.testing.assert_allclose(losses, F["losses"], rtol=2e-4)
    _check_state(m, F, int(F["nkf"]), stats="unchanged")


def test_refine_pose_non_key_frame_matches_reference():
    """The tracking uncertainty (the MLP with the reference run's dropout
    draw, clip, bilinear resize, bias rescale) within 1e-5 relative; the pose
    after 1 and 5 iterations within 2e-5 / 1e-4 (fp32 render vs the fp64
    restatement); the converged pose within 1e-4 of the reference's and the
    iteration count within 3 (the |tau| < 1e-4 test on a rounded tau)."""
    from wgsr.online import OnlineMapper
    F = _load("ref_refine_pose.npz")
    H, W = int(F["H"]), int(F["W"])
    fx, cx, cy = (float(F[n]) for n in ("fx", "cx", "cy"))
    m = OnlineMapper(sh_degree=0, feature_dim=int(F["C"]), device=DEV, seed=0)
    m.net.load_state_dict({k[len("mlp_"):]: torch.from_numpy(F[k]) for k in F.files if k.startswith("mlp_")
                           and not k.startswith("mlp_seeds")})
    m.ms = _mapping_step(F, "model", stats=False)
    seed = int(F["mlp_seeds"][0])
    assert len(F["mlp_seeds"]) == 1
    m.net.seed_source = lambda: seed
    feats, img = _t(F["features"]), _t(F["image"])
    unc = m.tracking_uncertainty(feats, H, W)
    assert _rel(unc, F["uncertainty"]) <= 1e-5
    poses = F["poses"]
    w2c0 = torch.from_numpy(F["w2c_init"])
    # early iterations track the reference's trajectory closely; later ones
    # drift apart by the accumulated fp32-vs-fp64 rounding of 10s of Adam
    # steps (a few 1e-4 of a 1e-2 initial offset)
    dev_n = {}
    for n, tol in ((1, 2e-5), (5, 1e-4), (20, 1e-3)):
        w2c, it = m.refine_pose_non_key_frame(w2c0, img, fx, fx, cx, cy, features=feats, iters=n)
        assert it == n
        dev_n[n] = float(np.abs(w2c.numpy() - poses[n - 1][:16].reshape(4, 4)).max())
    w2c, it = m.refine_pose_non_key_frame(w2c0, img, fx, fx, cx, cy, features=feats)
    n_ref = poses.shape[0]
    dev_n["final"] = float(np.abs(w2c.numpy() - F["w2c_refined"]).max())
    print("pose deviation from the reference trajectory:", dev_n, "iterations", it, "vs", n_ref)
    assert dev_n[1] <= 2e-5 and dev_n[5] <= 1e-4 and dev_n[20] <= 1e-3, dev_n
    assert abs(it - n_ref) <= max(3, n_ref // 5), (it, n_ref)
    assert dev_n["final"] <= 1e-3, dev_n
    # both converge to the true pose equally well
    err = lambda a: np.abs(a[:3, 3] - F["w2c_true"][:3, 3]).max()  # noqa: E731
    assert err(w2c.numpy()) <= 1.5 * err(F["w2c_refined"]) + 5e-4
    assert err(w2c.numpy()) < 0.5 * err(F["w2c_init"])


def test_insert_keyframe_matches_reference_run_body():
    F = _load("ref_run_body.npz")
    nkf = int(F["nkf"])
    new = int(F["new_kf"])
    cfg = {"window_size": int(F["window_size"]), "mapping_itr_num": int(F["mapping_itr_num"])}
    m, losses, perms, seeds = _mapper(F, new, [int(v) for v in F["window_before"]], 498, 40, cfg)
    m.occ_vis = {int(k[len("occ_before_"):]): _t(F[k]).long() for k in F.files if k.startswith("occ_before_")}
    kf = _keyframe(F, new)
    # the visibility of the new keyframe (the first render of the body)
    vis = m.visibility(kf).cpu().numpy()
    assert np.all(vis >= F["vis_new_lo"]) and np.all(vis <= F["vis_new_hi"])
    added = m.insert_keyframe(kf, keep=F["kept"])
    torch.cuda.synchronize()
    assert added == F["kept"].shape[0]
    assert m.window == [int(v) for v in F["window_after"]] == [int(v) for v in F["current_window"]]
    assert m.last_removed == int(F["removed"])
    assert not perms and not seeds
    np.testing.assert_allclose(np.stack(m.rng.p), F["probs"][:len(m.rng.p)], rtol=1e-12)
    assert len(m.rng.p) == len(F["losses"])
    np.testing.assert_allclose(losses, F["losses"], rtol=2e-4)
    assert [e[1] for e in m.events] == ["densify"] * int(F["n_densify"])
    _check_state(m, F, nkf)
    _check_occ(m, F, m.window)


def test_add_to_window_rejects_missing_visibility():
    """A window keyframe without an occlusion-aware visibility is an error (the
    reference indexes the dict and raises), not a silently skipped candidate."""
    F = _load("ref_run_body.npz")
    new = int(F["new_kf"])
    m, *_ = _mapper(F, new, [int(v) for v in F["window_before"]], 498, 40, {"window_size": 3})
    m.occ_vis = {int(k[len("occ_before_"):]): _t(F[k]).long() for k in F.files if k.startswith("occ_before_")}
    m.keyframes[new] = _keyframe(F, new)
    vis = _t(F["vis_new_lo"]).long()
    del m.occ_vis[3]
    with pytest.raises(RuntimeError, match="keyframe 3"):
        m._add_to_window(new, vis, list(m.window))
    m.occ_vis[3] = vis[:-1]          # a stale length
    with pytest.raises(RuntimeError):
        m._add_to_window(new, vis, list(m.window))
