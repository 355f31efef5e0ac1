"""GPU parity of densification on the device (wgsr.store.GaussianStore,
csrc/densify.hip) against fixtures produced by the
reference's OWN GaussianModel code (tests/golden/make_densify_fixtures.py:
densify_and_prune with its clone / split / postfix / prune steps,
reset_opacity_nonvisible, prune_points, reset_opacity, with torch.optim.Adam
state), fed the same split noise z.

Tolerances: row counts, row order, kept Adam moments, zero moments of new
rows, keyframe ids, observation counts and statistics exact; features,
opacity and rotation copies exact; split xyz (R(q) (z s) + xyz: the
reference's bmm vs three rounded products) and split scaling (log(exp(s) /
1.6): a division on the fixture's CPU, a reciprocal multiply on the GPU as
torch's CUDA kernel does) rel 1e-6; opacity resets (sigmoid / log on another
math library) rel 1e-6.
"""
import os

import numpy as np
import pytest
import torch

from _util import GOLDEN

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
GROUPS = ("xyz", "features", "opacity", "scaling", "rotation")


def _z():
    return np.load(os.path.join(GOLDEN, "ref_densify.npz"))


def _store_from(z, tag, capacity=None):
    from wgsr.store import GaussianStore
    t = lambda k: torch.from_numpy(z[f"{tag}_{k}"]).to(DEV)  # noqa: E731
    feat = torch.cat([t("f_dc"), t("f_rest")], 1)
    st = GaussianStore(t("xyz"), feat, t("opacity"), t("scaling"), t("rotation"), capacity=capacity,
                       kf_id=t("kf_id"), n_obs=t("n_obs"))
    for name, ref in (("xyz", "xyz"), ("opacity", "opacity"), ("scaling", "scaling"), ("rotation", "rotation")):
        st.exp_avg(name).copy_(t("m_" + ref))
        st.exp_avg_sq(name).copy_(t("v_" + ref))
    st.exp_avg("features").copy_(torch.cat([t("m_f_dc"), t("m_f_rest")], 1))
    st.exp_avg_sq("features").copy_(torch.cat([t("v_f_dc"), t("v_f_rest")], 1))
    st.stat("xyz_gradient_accum").copy_(t("accum"))
    st.stat("denom").copy_(t("denom"))
    st.stat("max_radii2D").copy_(t("max_radii2D"))
    return st


def _check(st, z, tag, approx=(), rtol=1e-6):
    c = lambda x: x.detach().cpu().numpy()  # noqa: E731
    P = z[f"{tag}_xyz"].shape[0]
    assert st.P == P, (st.P, P)
    got = {"xyz": c(st.param("xyz")), "f_dc": c(st.param("features")[:, :1]), "f_rest": c(st.param("features")[:, 1:]),
           "opacity": c(st.param("opacity")), "scaling": c(st.param("scaling")), "rotation": c(st.param("rotation"))}
    for name in ("xyz", "opacity", "scaling", "rotation"):
        got["m_" + name], got["v_" + name] = c(st.exp_avg(name)), c(st.exp_avg_sq(name))
    got["m_f_dc"], got["m_f_rest"] = c(st.exp_avg("features")[:, :1]), c(st.exp_avg("features")[:, 1:])
    got["v_f_dc"], got["v_f_rest"] = c(st.exp_avg_sq("features")[:, :1]), c(st.exp_avg_sq("features")[:, 1:])
    got["accum"], got["denom"] = c(st.stat("xyz_gradient_accum")), c(st.stat("denom"))
    got["max_radii2D"], got["kf_id"], got["n_obs"] = c(st.stat("max_radii2D")), c(st.kf_id), c(st.n_obs)
    for k, v in got.items():
        ref = z[f"{tag}_{k}"]
        if k in approx:
            np.testing.assert_allclose(v, ref, rtol=rtol, atol=1e-7, err_msg=f"{tag} {k}")
        else:
            np.testing.assert_array_equal(v, ref, err_msg=f"{tag} {k}")


@pytest.mark.parametrize("capacity", [None, 4096])
def test_densify_and_prune_matches_reference(capacity):
    """capacity None: the banks grow during the densify (P 700 -> 700 +
    clones + 2 x splits before the prune); 4096: no re-allocation."""
    z = _z()
    st = _store_from(z, "before", capacity)
    banks = [b["xyz"].data_ptr() for b in st.banks]
    out = st.densify_and_prune(float(z["param_max_grad"]), float(z["param_min_opacity"]), float(z["param_extent"]),
                               float(z["param_max_screen_size"]), float(z["param_percent_dense"]),
                               z=torch.from_numpy(z["z"]))
    torch.cuda.synchronize()
    assert out["split_selected"] == z["z"].shape[0] // 2
    _check(st, z, "after", approx=("xyz", "scaling"))
    if capacity:
        assert sorted(b["xyz"].data_ptr() for b in st.banks) == sorted(banks)  # no re-allocation


def test_reset_prune_reset_match_reference():
    z = _z()
    st = _store_from(z, "after")
    f1, f2 = (torch.from_numpy(z[k]).to(DEV) for k in ("reset_filter1", "reset_filter2"))
    st.reset_opacity_nonvisible([f1, f2])
    torch.cuda.synchronize()
    _check(st, z, "reset", approx=("opacity",))
    st = _store_from(z, "preprune")
    st.prune_points(torch.from_numpy(z["prune_mask"]).to(DEV))
    torch.cuda.synchronize()
    _check(st, z, "pruned")
    st.reset_opacity()
    torch.cuda.synchronize()
    _check(st, z, "reset_all", approx=("opacity",))


def test_append_keeps_rows_and_zeroes_new_moments_and_stats():
    """densification_postfix for a keyframe insert (extend_from_pcd): rows
    after the last one, zero moments, every row's statistics reset; growing
    past the capacity keeps the current rows."""
    from wgsr.store import GaussianStore
    g = torch.Generator().manual_seed(3)
    P, M = 100, 4
    r = lambda *s: torch.randn(*s, generator=g).to(DEV)  # noqa: E731
    st = GaussianStore(r(P, 3), r(P, M, 3), r(P, 1), r(P, 3), r(P, 4), capacity=120)
    st.exp_avg("xyz").copy_(r(P, 3))
    st.stat("denom").fill_(2.0)
    before = st.param("xyz").clone(), st.exp_avg("xyz").clone()
    new = (r(50, 3), r(50, M, 3), r(50, 1), r(50, 3), r(50, 4))
    st.append(*new, kf_id=torch.full((50,), 7, dtype=torch.int32))
    assert st.P == 150 and st.capacity >= 150
    assert torch.equal(st.param("xyz")[:P], before[0]) and torch.equal(st.exp_avg("xyz")[:P], before[1])
    assert torch.equal(st.param("xyz")[P:], new[0]) and torch.equal(st.param("features")[P:], new[1])
    assert not st.exp_avg("xyz")[P:].any() and not st.exp_avg_sq("rotation")[P:].any()
    assert not st.stat("denom").any()
    assert (st.kf_id[P:] == 7).all()


def test_mapping_step_skips_replaced_groups_like_torch_adam():
    """After a densify every parameter is a new nn.Parameter without a
    gradient, so the reference's optimizer.step() skips all groups (and their
    step counts); after reset_opacity_nonvisible only the opacity group."""
    from wgsr.mapping import MappingStep
    from wgsr.scene import make_scene
    sc = make_scene(500, 64, 48, 1, seed=2)
    ms = MappingStep(sc.means3D.to(DEV), sc.shs[:, :1].to(DEV), sc.shs[:, 1:].to(DEV),
                     torch.logit(sc.opacities).to(DEV), torch.log(sc.scales).to(DEV), sc.rotations.to(DEV), 1)
    for v in ms.grad.values():
        v.normal_()
    ms.optimizer_step()
    assert ms.steps == {g: 1 for g in GROUPS}
    op = ms.opacity.clone()
    ms.reset_opacity_nonvisible([torch.zeros(ms.P, dtype=torch.bool, device=DEV)])
    ms.optimizer_step()
    assert ms.steps["opacity"] == 1 and ms.steps["xyz"] == 2
    assert not torch.equal(ms.opacity, op) and (ms.exp_avg["opacity"] == 0).all()
    ms.store.stat("denom").fill_(1.0)
    ms.store.stat("xyz_gradient_accum").fill_(1.0)
    ms.densify_and_prune(2e-4, 0.0, 10.0, None)
    xyz = ms.xyz.clone()
    ms.optimizer_step()
    assert ms.steps == {"xyz": 2, "features": 2, "opacity": 1, "scaling": 2, "rotation": 2}
    assert torch.equal(ms.xyz, xyz)
