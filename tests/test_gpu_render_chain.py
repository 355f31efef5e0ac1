"""GPU parity of the whole caller chain against fixtures produced by the
reference's OWN render() + GaussianModel + Camera (tests/golden/
make_render_fixtures.py, executed in the build container with the float64
oracle standing in for the absent CUDA rasteriser).

The raw GaussianModel parameters of each fixture go through
* ``wgsr.render.render_model`` (the reference render() restated: torch
  activations, python covariance / SH colour branches) into the drop-in
  ``diff_gaussian_rasterization`` package (HIP library through the C ABI),
  autograd backward to the raw parameters and the pose deltas;
* ``wgsr.mapping.MappingStep`` (fused activation kernels, the rasteriser
  writing straight into the gradient storage) for the cases without the
  python-side branches.

Tolerances (north_star: <= 1e-4 rel L1): images rel-L1 1e-4; radii and
visibility exact; n_touched exact for every Gaussian whose oracle count does
not move when the T > 0.5 threshold moves by 1e-5, and inside that band for
the others; raw-parameter and means2D gradients rel-L1 1e-4; pose deltas
(sums over every Gaussian) rel-L1 1e-3.
"""
import types

import numpy as np
import pytest
import torch

from _util import rel_l1
from test_render_chain import CASES, camera, load, params

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
IMG_TOL, GRAD_TOL, TAU_TOL = 1e-4, 1e-4, 1e-3


def check_n_touched(got, z):
    exp, lo, hi = z["out_n_touched"], z["out_n_touched_lo"], z["out_n_touched_hi"]
    firm = lo == hi
    np.testing.assert_array_equal(got[firm], exp[firm])
    assert np.all((got[~firm] >= lo[~firm]) & (got[~firm] <= hi[~firm]))


@pytest.mark.parametrize("name", CASES)
def test_render_model_matches_reference_chain(name):
    from wgsr.render import DeviceCamera, render_model
    z = load(name)
    pc, raw = params(z, requires_grad=True, device=DEV)
    cam = DeviceCamera.from_pinhole(camera(z), DEV)
    pipe = types.SimpleNamespace(compute_cov3D_python=bool(z["compute_cov3D_python"]),
                                 convert_SHs_python=bool(z["convert_SHs_python"]))
    pkg = render_model(cam, pc, pipe, torch.from_numpy(z["bg"]).to(DEV), scaling_modifier=float(z["scaling_modifier"]))
    loss = (pkg["render"] * torch.from_numpy(z["grad_color"]).to(DEV)).sum() + \
        (pkg["depth"] * torch.from_numpy(z["grad_depth"]).to(DEV)).sum()
    loss.backward()
    torch.cuda.synchronize()
    for k in ("render", "depth", "opacity"):
        r = rel_l1(pkg[k].detach().cpu().numpy(), z["out_" + k])
        assert r <= IMG_TOL, (k, r)
    np.testing.assert_array_equal(pkg["radii"].cpu().numpy(), z["out_radii"])
    np.testing.assert_array_equal(pkg["visibility_filter"].cpu().numpy(), z["out_visibility_filter"])
    check_n_touched(pkg["n_touched"].cpu().numpy(), z)
    for k, t in raw.items():
        g = t.grad if t.grad is not None else torch.zeros_like(t)
        r = rel_l1(g.cpu().numpy(), z["g_" + k])
        assert r <= GRAD_TOL, (k, r)
    r = rel_l1(pkg["viewspace_points"].grad.cpu().numpy(), z["g_viewspace_points"])
    assert r <= GRAD_TOL, ("viewspace_points", r)
    for k in ("cam_rot_delta", "cam_trans_delta"):
        r = rel_l1(getattr(cam, k).grad.cpu().numpy(), z["g_" + k])
        assert r <= TAU_TOL, (k, r)


@pytest.mark.parametrize("name", [c for c in CASES if "pyprecomp" not in c])
def test_mapping_step_matches_reference_chain(name):
    from wgsr.mapping import MappingStep
    z = load(name)
    _, raw = params(z, device=DEV)
    ms = MappingStep(raw["xyz"], raw["features_dc"], raw["features_rest"], raw["opacity"], raw["scaling"],
                     raw["rotation"], sh_degree=int(z["active_sh_degree"]))
    f = camera(z).raster_fields()
    cam = {k: (v.to(DEV) if torch.is_tensor(v) else v) for k, v in f.items()}
    H, W = int(z["H"]), int(z["W"])
    bg = torch.from_numpy(z["bg"]).to(DEV)
    fwd = ms._render(cam, H, W, bg)
    _, tau = ms._backward(cam, bg, fwd, torch.from_numpy(z["grad_color"]).to(DEV),
                          torch.from_numpy(z["grad_depth"]).to(DEV), 0.0)
    torch.cuda.synchronize()
    assert rel_l1(fwd[1].cpu().numpy(), z["out_render"]) <= IMG_TOL
    np.testing.assert_array_equal(fwd[2].cpu().numpy(), z["out_radii"])
    check_n_touched(fwd[8].cpu().numpy(), z)
    feat = np.concatenate([z["g_features_dc"], z["g_features_rest"]], axis=1)
    for mine, ref in ((ms.grad["xyz"], z["g_xyz"]), (ms.grad["features"], feat), (ms.grad["opacity"], z["g_opacity"]),
                      (ms.grad["scaling"], z["g_scaling"]), (ms.grad["rotation"], z["g_rotation"])):
        r = rel_l1(mine.cpu().numpy(), ref)
        assert r <= GRAD_TOL, r
    t = tau.cpu().numpy()
    assert rel_l1(t[:3], z["g_cam_trans_delta"]) <= TAU_TOL
    assert rel_l1(t[3:], z["g_cam_rot_delta"]) <= TAU_TOL
