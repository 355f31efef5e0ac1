"""CPU tests of the caller chain around the rasteriser, pinned by fixtures the
reference's OWN code produced (tests/golden/make_render_fixtures.py executes
gaussian_renderer.render(), GaussianModel's activations, Camera and
general_utils in the build container; no GPU needed here).

* ``wgsr.render.build_rotation`` / ``build_scaling_rotation`` /
  ``strip_symmetric`` equal general_utils.py:97-186's outputs.
* ``wgsr.camera.PinholeCamera`` produces the camera fields render() handed the
  rasteriser (viewmatrix, projmatrix, projmatrix_raw, campos, tangents).
* ``wgsr.render.render_model`` hands the rasteriser the same tensors as the
  reference render() (activations, python covariance / SH colours branches).
* With the same float64 oracle standing in for the rasteriser, the gradients
  autograd delivers through ``render_model`` to the raw parameters and to the
  pose deltas equal the ones the reference chain delivered.

Tolerances: camera fields and activated inputs rel 1e-6 / atol 1e-7 (fp32
ops in another order), gradients rel-L1 1e-6 (same float64 oracle, float32
activations).
"""
import glob
import os
import types

import numpy as np
import pytest
import torch

from _util import GOLDEN, rel_l1

CASES = sorted(os.path.basename(p)[11:-4] for p in glob.glob(os.path.join(GOLDEN, "ref_render_*.npz")))


def load(name):
    return np.load(os.path.join(GOLDEN, f"ref_render_{name}.npz"))


def test_fixtures_present():
    assert set(CASES) >= {"sh0_128x96", "sh3_pose_96x72", "pyprecomp_64x48"}


def test_general_utils_match_reference():
    from wgsr.render import build_rotation, build_scaling_rotation, strip_symmetric
    z = np.load(os.path.join(GOLDEN, "ref_general_utils.npz"))
    r, s = torch.from_numpy(z["r"]), torch.from_numpy(z["s"])
    np.testing.assert_allclose(build_rotation(r).numpy(), z["build_rotation"], rtol=0, atol=1e-7)
    L = build_scaling_rotation(s, r)
    np.testing.assert_allclose(L.numpy(), z["build_scaling_rotation"], rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(strip_symmetric(L @ L.transpose(1, 2)).numpy(), z["strip_symmetric"],
                               rtol=1e-6, atol=1e-7)


def camera(z):
    from wgsr.camera import PinholeCamera
    return PinholeCamera(R=torch.from_numpy(z["R"]), T=torch.from_numpy(z["T"]), fx=float(z["fx"]),
                         fy=float(z["fx"]), cx=float(z["cx"]), cy=float(z["cy"]), W=int(z["W"]), H=int(z["H"]))


def params(z, requires_grad=False, device="cpu"):
    from wgsr.render import GaussianParams
    t = {k: torch.from_numpy(z["raw_" + k]).to(device).requires_grad_(requires_grad)
         for k in ("xyz", "features_dc", "features_rest", "opacity", "scaling", "rotation")}
    return GaussianParams(t["xyz"], t["features_dc"], t["features_rest"], t["opacity"], t["scaling"], t["rotation"],
                          int(z["max_sh_degree"]), int(z["active_sh_degree"])), t


@pytest.mark.parametrize("name", CASES)
def test_camera_fields_match_reference(name):
    z = load(name)
    cam = camera(z)
    f = cam.raster_fields()
    assert f["image_height"] == int(z["set_image_height"]) and f["image_width"] == int(z["set_image_width"])
    assert cam.FoVx == float(z["FoVx"]) and cam.FoVy == float(z["FoVy"])
    assert f["tanfovx"] == float(z["set_tanfovx"]) and f["tanfovy"] == float(z["set_tanfovy"])
    for k in ("viewmatrix", "projmatrix", "projmatrix_raw", "campos"):
        np.testing.assert_allclose(f[k].numpy(), z["set_" + k], rtol=1e-6, atol=1e-7, err_msg=k)


class _Recorder(torch.nn.Module):
    """Stands in for GaussianRasterizer: records the call, returns zeros."""
    calls: list = []

    def __init__(self, raster_settings):
        super().__init__()
        self.raster_settings = raster_settings

    def forward(self, **kw):
        _Recorder.calls.append(dict(kw, settings=self.raster_settings))
        s = self.raster_settings
        P = kw["means3D"].shape[0]
        H, W = s.image_height, s.image_width
        z = torch.zeros
        return z(3, H, W), z(P, dtype=torch.int32), z(1, H, W), z(1, H, W), z(P, dtype=torch.int32)


def _device_camera(z, cam):
    from wgsr.render import DeviceCamera
    return DeviceCamera.from_pinhole(cam, "cpu")


@pytest.mark.parametrize("name", CASES)
def test_render_model_hands_over_reference_tensors(name, monkeypatch):
    import wgsr.render as R
    z = load(name)
    monkeypatch.setattr(R, "GaussianRasterizer", _Recorder)
    _Recorder.calls = []
    pc, _ = params(z)
    pipe = types.SimpleNamespace(compute_cov3D_python=bool(z["compute_cov3D_python"]),
                                 convert_SHs_python=bool(z["convert_SHs_python"]))
    R.render_model(_device_camera(z, camera(z)), pc, pipe, torch.from_numpy(z["bg"]),
                   scaling_modifier=float(z["scaling_modifier"]))
    (call,) = _Recorder.calls
    s = call["settings"]
    assert s.sh_degree == int(z["set_sh_degree"]) and s.scale_modifier == float(z["set_scale_modifier"])
    assert s.prefiltered == bool(z["set_prefiltered"]) and s.debug == bool(z["set_debug"])
    np.testing.assert_array_equal(s.bg.numpy(), z["set_bg"])
    for k in ("means3D", "opacities", "shs", "colors_precomp", "scales", "rotations", "cov3D_precomp"):
        got = call.get(k)
        if "in_" + k not in z.files:
            assert got is None, k
            continue
        np.testing.assert_allclose(got.detach().numpy(), z["in_" + k], rtol=1e-6, atol=1e-7, err_msg=k)
    assert call["theta"].shape == (3,) and call["rho"].shape == (3,)


class _DenseRasterizer(torch.nn.Module):
    """The float64 oracle as the rasteriser -- the same stand-in the fixture
    script put under the reference's render()."""

    def __init__(self, raster_settings):
        super().__init__()
        self.s = raster_settings

    def forward(self, means3D, means2D, opacities, shs=None, colors_precomp=None, scales=None, rotations=None,
                cov3D_precomp=None, theta=None, rho=None):
        from oracle import dense
        s = self.s
        d = lambda x: None if x is None else x.double()  # noqa: E731
        out = dense.rasterize_dense(
            d(means3D), d(means2D), d(opacities), d(shs), d(colors_precomp), d(scales), d(rotations),
            d(cov3D_precomp), torch.cat([rho, theta]).double(), H=s.image_height, W=s.image_width,
            tanfovx=s.tanfovx, tanfovy=s.tanfovy, bg=s.bg, scale_modifier=s.scale_modifier,
            viewmatrix=s.viewmatrix, projmatrix=s.projmatrix, projmatrix_raw=s.projmatrix_raw,
            sh_degree=s.sh_degree, campos=s.campos)
        return (out["color"].float(), out["radii"], out["depth"].float(), out["opacity"].detach().float(),
                out["n_touched"])


@pytest.mark.parametrize("name", CASES)
def test_render_model_gradients_match_reference_chain(name, monkeypatch):
    import wgsr.render as R
    z = load(name)
    monkeypatch.setattr(R, "GaussianRasterizer", _DenseRasterizer)
    pc, raw = params(z, requires_grad=True)
    cam = _device_camera(z, camera(z))
    pipe = types.SimpleNamespace(compute_cov3D_python=bool(z["compute_cov3D_python"]),
                                 convert_SHs_python=bool(z["convert_SHs_python"]))
    pkg = R.render_model(cam, pc, pipe, torch.from_numpy(z["bg"]), scaling_modifier=float(z["scaling_modifier"]))
    for k in ("render", "depth", "opacity"):
        assert rel_l1(pkg[k].detach().numpy(), z["out_" + k]) <= 1e-6, k
    np.testing.assert_array_equal(pkg["radii"].numpy(), z["out_radii"])
    np.testing.assert_array_equal(pkg["visibility_filter"].numpy(), z["out_visibility_filter"])
    loss = (pkg["render"] * torch.from_numpy(z["grad_color"])).sum() + \
        (pkg["depth"] * torch.from_numpy(z["grad_depth"])).sum()
    loss.backward()
    for k, t in raw.items():
        g = t.grad if t.grad is not None else torch.zeros_like(t)
        assert rel_l1(g.numpy(), z["g_" + k]) <= 1e-6, (k, rel_l1(g.numpy(), z["g_" + k]))
    assert rel_l1(pkg["viewspace_points"].grad.numpy(), z["g_viewspace_points"]) <= 1e-6
    assert rel_l1(cam.cam_rot_delta.grad.numpy(), z["g_cam_rot_delta"]) <= 1e-6
    assert rel_l1(cam.cam_trans_delta.grad.numpy(), z["g_cam_trans_delta"]) <= 1e-6
