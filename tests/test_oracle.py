"""CPU tests of the oracle itself (no GPU).

* The restated helpers reproduce the reference's own helper outputs
  (tests/golden/ref_helpers.npz, generated from /root/reference).
* The fp32 CPU restatement (oracle/cpu_raster.cpp) matches the float64
  autograd oracle (oracle/dense.py) on every golden scene.
* The pose gradient equals a finite difference of the reference's pose update
  new_w2c = SE3_exp([rho, theta]) @ w2c (src/utils/pose_utils.py:81-98).
* The CPU distCUDA2 matches float64 brute force.

Tolerances: images rel-L1 <= 1e-4; radii / n_touched /
num_rendered exact; gradients rel-L1 <= 1e-4, pose (summed over P) <= 1e-3.
"""
import math
import os

import numpy as np
import pytest
import torch

from _util import GOLDEN, GRAD_KEYS, load_scene, rel_l1, scene_names
from oracle import cpu_oracle, dense
from wgsr import camera as wcam
from wgsr.scene import make_scene, make_upstream_grads

IMG_TOL = 1e-4
GRAD_TOL = 1e-4
TAU_TOL = 1e-3


def test_restated_helpers_match_reference_outputs():
    z = np.load(os.path.join(GOLDEN, "ref_helpers.npz"))
    for c, ref in zip(z["proj_in"], z["proj_out"]):
        np.testing.assert_array_equal(wcam.get_projection_matrix2(*c).numpy(), ref)
    for R, t, ref in zip(z["w2v_R"], z["w2v_t"], z["w2v_out"]):
        np.testing.assert_array_equal(
            wcam.get_world2view2(torch.from_numpy(R), torch.from_numpy(t)).numpy(), ref)
    for (f, p), ref in zip(z["fov_in"], z["fov_out"]):
        assert wcam.focal2fov(f, p) == ref
    for tau, ref in zip(z["se3_in"], z["se3_out"]):
        np.testing.assert_allclose(dense.se3_exp(torch.from_numpy(tau)).numpy(), ref, rtol=0, atol=1e-12)
        np.testing.assert_allclose(wcam.se3_exp(torch.from_numpy(tau)).numpy(), ref, rtol=0, atol=1e-12)
    sh = torch.from_numpy(z["sh_coeffs"])
    dirs = torch.from_numpy(z["sh_dirs"])
    for deg in range(4):
        np.testing.assert_allclose(dense.eval_sh(deg, sh, dirs).numpy(), z[f"sh_out_deg{deg}"],
                                   rtol=0, atol=1e-12)
    assert float(z["sh_C0"]) == dense.SH_C0


def _cpu_run(inputs, settings, grads):
    cr = cpu_oracle.CpuRaster(**inputs, **settings)
    g = cr.backward(*grads)
    return cr, g


@pytest.mark.parametrize("name", scene_names())
def test_cpu_restatement_matches_dense_oracle(name):
    inputs, settings, expect, grads = load_scene(name)
    cr, g = _cpu_run(inputs, settings, grads)
    assert cr.num_rendered == expect["num_rendered"]
    np.testing.assert_array_equal(cr.radii, expect["radii"])
    np.testing.assert_array_equal(cr.n_touched, expect["n_touched"])
    for k in ("color", "depth", "opacity"):
        assert rel_l1(getattr(cr, k), expect[k]) <= IMG_TOL, k
    for k in GRAD_KEYS:
        if k in expect:
            got = g[k]
            if k == "dL_dsh":
                got = got[:, : expect[k].shape[1]]
            assert rel_l1(got, expect[k]) <= GRAD_TOL, (k, rel_l1(got, expect[k]))
    assert rel_l1(g["dL_dtau"].sum(0), expect["dL_dtau"]) <= TAU_TOL


def test_pose_gradient_is_left_perturbation_of_reference_update():
    """dL/dtau from the oracle == finite difference through SE3_exp(tau) @ w2c."""
    W, H = 48, 32
    sc = make_scene(60, W, H, 1, seed=9)
    gc, gd = make_upstream_grads(W, H, seed=10)
    cam = wcam.synthetic_camera(W, H, 2)
    base = dict(H=H, W=W, bg=torch.tensor([0.1, 0.1, 0.1]), scale_modifier=1.0, sh_degree=1)
    inputs = dict(means3D=sc.means3D, opacities=sc.opacities, shs=sc.shs, scales=sc.scales,
                  rotations=sc.rotations)

    def fields(c):
        f = c.raster_fields()
        return dict(tanfovx=f["tanfovx"], tanfovy=f["tanfovy"], viewmatrix=f["viewmatrix"],
                    projmatrix=f["projmatrix"], projmatrix_raw=f["projmatrix_raw"],
                    campos=f["campos"])

    res = dense.dense_forward_backward(inputs, {**base, **fields(cam)}, gc, gd)

    def loss_at(tau):
        # reference pose update (pose_utils.py:81-98) in float64
        T = torch.eye(4, dtype=torch.float64)
        T[:3, :3] = cam.R.double()
        T[:3, 3] = cam.T.double()
        T2 = wcam.se3_exp(tau) @ T
        Vrm = T2.T  # world_view_transform (row-vector storage)
        Prm = cam.projection_matrix.double()
        st = dict(base, tanfovx=fields(cam)["tanfovx"], tanfovy=fields(cam)["tanfovy"],
                  viewmatrix=Vrm, projmatrix=Vrm @ Prm, projmatrix_raw=Prm,
                  campos=fields(cam)["campos"].double())
        z = torch.zeros(6, dtype=torch.float64)
        out = dense.rasterize_dense(
            inputs["means3D"].double(), torch.zeros(60, 3, dtype=torch.float64),
            inputs["opacities"].double(), inputs["shs"].double(), None, inputs["scales"].double(),
            inputs["rotations"].double(), None, z, **st)
        return float((out["color"] * gc.double()).sum() + (out["depth"] * gd.double()).sum())

    eps = 1e-6
    fd = []
    for k in range(6):
        e = torch.zeros(6, dtype=torch.float64)
        e[k] = eps
        fd.append((loss_at(e) - loss_at(-e)) / (2 * eps))
    fd = np.array(fd)
    np.testing.assert_allclose(res["dL_dtau"].numpy(), fd, rtol=2e-4, atol=1e-3 * np.abs(fd).max())


def test_knn_oracle_matches_brute_force():
    z = np.load(os.path.join(GOLDEN, "knn_cases.npz"))
    for k in z.files:
        if not k.startswith("pts_"):
            continue
        tag = k[4:]
        pts, ref = z[k], z["ref_" + tag]
        got = cpu_oracle.dist_knn(pts)
        if pts.shape[0] < 4:
            # missing neighbours stay FLT_MAX: P <= 2 overflows to inf,
            # P == 3 gives FLT_MAX / 3
            np.testing.assert_array_equal(got, ref.astype(np.float32), err_msg=tag)
            continue
        np.testing.assert_allclose(got, ref, rtol=1e-6, atol=0, err_msg=tag)


def test_config0_cpu_plumbing_10k_640x480():
    """BASELINE.json configs[0]: 10k Gaussians, 640x480, SH0, single view
    fwd+bwd on the CPU rasteriser, checked against the float64 oracle."""
    W, H = 640, 480
    sc = make_scene(10_000, W, H, 0, seed=0)
    gc, gd = make_upstream_grads(W, H, seed=1)
    f = wcam.synthetic_camera(W, H, 0).raster_fields()
    settings = dict(H=H, W=W, tanfovx=f["tanfovx"], tanfovy=f["tanfovy"],
                    bg=torch.zeros(3), scale_modifier=1.0, viewmatrix=f["viewmatrix"],
                    projmatrix=f["projmatrix"], projmatrix_raw=f["projmatrix_raw"], sh_degree=0,
                    campos=f["campos"])
    inputs = dict(means3D=sc.means3D, opacities=sc.opacities, shs=sc.shs, scales=sc.scales,
                  rotations=sc.rotations)
    ref = dense.dense_forward_backward(inputs, settings, gc, gd)
    cr, g = _cpu_run(inputs, settings, (gc, gd))
    assert cr.num_rendered == ref["num_rendered"]
    assert (cr.radii != ref["radii"].numpy()).sum() == 0
    for k in ("color", "depth", "opacity"):
        assert rel_l1(getattr(cr, k), ref[k].numpy()) <= IMG_TOL
    for k in ("dL_dmeans3D", "dL_dmeans2D", "dL_dopacity", "dL_dscales", "dL_drotations"):
        assert rel_l1(g[k], ref[k].numpy()) <= GRAD_TOL, k
    assert rel_l1(g["dL_dtau"].sum(0), ref["dL_dtau"].numpy()) <= TAU_TOL


def test_n_touched_firm_soft_band_is_consistent():
    """The CPU restatement's n_touched classification (cpu_raster.cpp): its
    own count lies in [firm, firm + soft], equals firm wherever no decision is
    soft, and only a small fraction of Gaussians carry a soft decision; on the
    golden scenes (dense float64 oracle) every firm count matches too."""
    W, H = 320, 240
    sc = make_scene(8000, W, H, 3, seed=9)
    f = wcam.synthetic_camera(W, H, 1).raster_fields()
    cr = cpu_oracle.CpuRaster(means3D=sc.means3D, opacities=sc.opacities, shs=sc.shs, scales=sc.scales,
                              rotations=sc.rotations, H=H, W=W, tanfovx=f["tanfovx"], tanfovy=f["tanfovy"],
                              bg=np.zeros(3, np.float32), scale_modifier=1.0, viewmatrix=f["viewmatrix"],
                              projmatrix=f["projmatrix"], projmatrix_raw=f["projmatrix_raw"], sh_degree=3,
                              campos=f["campos"])
    n, firm, soft = cr.n_touched, cr.n_touched_firm, cr.n_touched_soft
    assert np.all((n >= firm) & (n <= firm + soft))
    np.testing.assert_array_equal(n[soft == 0], firm[soft == 0])
    assert np.count_nonzero(soft) <= 0.02 * len(n) and n.sum() > 0
    for name in scene_names():
        inputs, settings, expect, grads = load_scene(name)
        c = cpu_oracle.CpuRaster(**inputs, **settings)
        clear = c.n_touched_soft == 0
        np.testing.assert_array_equal(c.n_touched_firm[clear], expect["n_touched"][clear])
