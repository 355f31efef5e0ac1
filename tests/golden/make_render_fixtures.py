"""Generate tests/golden/ref_render_*.npz and ref_general_utils.npz by EXECUTING
the reference's own caller chain in the build container (/root/reference
exists only here; the fixtures travel, the reference does not).

What runs unchanged from the reference:

* ``render()``  -- thirdparty/gaussian_splatting/gaussian_renderer/__init__.py:24-153
  (dummy means2D with retain_grad, tangents from FoV, the 13 settings fields,
  the pipe.compute_cov3D_python / convert_SHs_python branches, the keyword
  call into the rasteriser with theta=cam_rot_delta, rho=cam_trans_delta, the
  result dict);
* ``GaussianModel`` -- thirdparty/gaussian_splatting/scene/gaussian_model.py:35-106
  (raw ``_xyz/_features_dc/_features_rest/_opacity/_scaling/_rotation`` and the
  activations exp / sigmoid / normalize / cat, ``get_covariance`` through
  ``build_scaling_rotation`` + ``strip_symmetric``);
* ``Camera`` -- src/utils/camera_utils.py:23-151 (world_view_transform,
  full_proj_transform, camera_center, cam_rot_delta/cam_trans_delta
  parameters, ``update_RT``) with the projection matrix built as
  mapper.py:111-121 does;
* ``build_rotation`` / ``build_scaling_rotation`` / ``strip_symmetric``
  (thirdparty/gaussian_splatting/utils/general_utils.py:97-186).

Stand-ins (nothing of them reaches a recorded value):

* ``open3d``, ``plyfile``, ``simple_knn``, ``cv2`` -- absent here, imported by
  gaussian_model.py / loss_utils.py but not used by the functions above:
  empty modules in ``sys.modules``;
* ``device="cuda"`` / ``.cuda()`` in the reference code -> CPU (no GPU here):
  a ``TorchFunctionMode`` rewrites the device argument;
* ``diff_gaussian_rasterization`` -> a RECORDING fake whose forward is the
  float64 restatement ``oracle/dense.py`` (autograd provides its backward).
  The upstream CUDA rasteriser is absent (empty submodule), so the
  rasteriser's own numbers stay oracle numbers; what this pins is everything
  AROUND it: the exact tensors ``render()`` hands over, and how the gradients
  the rasteriser returns flow back through the reference's activations to the
  raw parameters and to the camera's pose deltas.

Loss: ``(render * gc).sum() + (depth * gd).sum()`` with seeded gc, gd.

Usage:  python tests/golden/make_render_fixtures.py
"""
from __future__ import annotations

import math
import os
import sys
import types
from collections import namedtuple

import numpy as np
import torch
from torch.overrides import TorchFunctionMode

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, "..", ".."))
REF = "/root/reference"


class CudaToCpu(TorchFunctionMode):
    """device='cuda...' -> 'cpu', Tensor.cuda() -> identity."""

    def __torch_function__(self, func, types_, args=(), kwargs=None):
        kwargs = dict(kwargs or {})
        d = kwargs.get("device")
        if d is not None and str(d).startswith("cuda"):
            kwargs["device"] = "cpu"
        if func is torch.Tensor.cuda:
            return args[0]
        return func(*args, **kwargs)


RECORD: list = []

_FIELDS = ("image_height", "image_width", "tanfovx", "tanfovy", "bg", "scale_modifier", "viewmatrix",
           "projmatrix", "projmatrix_raw", "sh_degree", "campos", "prefiltered", "debug")


def _fake_rasterizer_module():
    sys.path.insert(0, REPO)
    from oracle import dense

    m = types.ModuleType("diff_gaussian_rasterization")
    m.GaussianRasterizationSettings = namedtuple("GaussianRasterizationSettings", _FIELDS)

    class GaussianRasterizer(torch.nn.Module):
        def __init__(self, raster_settings):
            super().__init__()
            self.raster_settings = raster_settings

        def forward(self, means3D, means2D, opacities, shs=None, colors_precomp=None, scales=None,
                    rotations=None, cov3D_precomp=None, theta=None, rho=None):
            s = self.raster_settings
            d = lambda x: None if x is None else x.double()  # noqa: E731
            tau = torch.cat([rho, theta]).double()
            out = dense.rasterize_dense(
                d(means3D), d(means2D), d(opacities), d(shs), d(colors_precomp), d(scales), d(rotations),
                d(cov3D_precomp), tau, H=s.image_height, W=s.image_width, tanfovx=s.tanfovx,
                tanfovy=s.tanfovy, bg=s.bg, scale_modifier=s.scale_modifier, viewmatrix=s.viewmatrix,
                projmatrix=s.projmatrix, projmatrix_raw=s.projmatrix_raw, sh_degree=s.sh_degree,
                campos=s.campos)
            band = {}
            with torch.no_grad():   # n_touched with the 0.5 threshold moved by -/+ 1e-5
                for tag, th in (("hi", 0.5 - 1e-5), ("lo", 0.5 + 1e-5)):
                    band[tag] = dense.rasterize_dense(
                        d(means3D), d(means2D), d(opacities), d(shs), d(colors_precomp), d(scales), d(rotations),
                        d(cov3D_precomp), tau, H=s.image_height, W=s.image_width, tanfovx=s.tanfovx,
                        tanfovy=s.tanfovy, bg=s.bg, scale_modifier=s.scale_modifier, viewmatrix=s.viewmatrix,
                        projmatrix=s.projmatrix, projmatrix_raw=s.projmatrix_raw, sh_degree=s.sh_degree,
                        campos=s.campos, touch_threshold=th)["n_touched"]
            RECORD.append(dict(n_touched_lo=band["lo"], n_touched_hi=band["hi"], settings=s, means3D=means3D, means2D=means2D, opacities=opacities, shs=shs,
                               colors_precomp=colors_precomp, scales=scales, rotations=rotations,
                               cov3D_precomp=cov3D_precomp, num_rendered=out["num_rendered"]))
            # upstream returns float32; the opacity image's gradient is not
            # propagated upstream: detached here
            return (out["color"].float(), out["radii"], out["depth"].float(),
                    out["opacity"].detach().float(), out["n_touched"])

    m.GaussianRasterizer = GaussianRasterizer
    return m


def _install_stubs():
    sys.modules["diff_gaussian_rasterization"] = _fake_rasterizer_module()
    for name in ("open3d", "cv2"):
        sys.modules.setdefault(name, types.ModuleType(name))
    ply = types.ModuleType("plyfile")
    ply.PlyData = ply.PlyElement = None
    sys.modules.setdefault("plyfile", ply)
    sk = types.ModuleType("simple_knn")
    skc = types.ModuleType("simple_knn._C")

    def _no_knn(*a, **k):
        raise RuntimeError("distCUDA2 is not part of this fixture")
    skc.distCUDA2 = _no_knn
    sk._C = skc
    sys.modules.setdefault("simple_knn", sk)
    sys.modules.setdefault("simple_knn._C", skc)
    sys.path.insert(0, REF)


def _rot(axis, deg):
    a = torch.tensor(axis, dtype=torch.float64)
    a = a / a.norm()
    th = math.radians(deg)
    K = torch.tensor([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]], dtype=torch.float64)
    return (torch.eye(3, dtype=torch.float64) + math.sin(th) * K + (1 - math.cos(th)) * K @ K).float()


def _case(name, *, P, W, H, fx, max_sh, active_sh, R, T, bg, seed, cov_python=False, shs_python=False,
          scaling_modifier=1.0):
    from src.utils.camera_utils import Camera
    from thirdparty.gaussian_splatting.gaussian_renderer import render
    from thirdparty.gaussian_splatting.scene.gaussian_model import GaussianModel
    from thirdparty.gaussian_splatting.utils.graphics_utils import focal2fov, getProjectionMatrix2

    g = torch.Generator().manual_seed(seed)
    cx, cy = W / 2.0, H / 2.0            # centred principal point
    # Gaussians in the camera frame (BASELINE.md distribution), then to world
    tanx, tany = W / (2.0 * fx), H / (2.0 * fx)
    z = 2.0 + 6.0 * torch.rand(P, generator=g)
    u = torch.rand(P, generator=g) * 2 - 1
    v = torch.rand(P, generator=g) * 2 - 1
    pc = torch.stack([u * z * tanx * 1.1, v * z * tany * 1.1, z], 1)
    xyz = ((pc - T[None]) @ R).contiguous()          # p_w = R^T (p_c - T), row form
    log_s = math.log(0.01) + (math.log(0.08) - math.log(0.01)) * torch.rand(P, 3, generator=g)
    q = torch.randn(P, 4, generator=g)
    q = q * (0.5 + 1.5 * torch.rand(P, 1, generator=g))               # NOT unit: normalize() is pinned
    op = 0.05 + 0.9 * torch.rand(P, 1, generator=g)
    logit = torch.log(op / (1 - op))
    M = (max_sh + 1) ** 2
    feat = torch.randn(P, M, 3, generator=g) * 0.1
    feat[:, 0] = torch.randn(P, 3, generator=g) * 0.5
    gc = torch.randn(3, H, W, generator=g)
    gd = torch.randn(1, H, W, generator=g)

    with CudaToCpu():
        gm = GaussianModel(max_sh)
        gm.active_sh_degree = active_sh
        gm._xyz = torch.nn.Parameter(xyz.clone())
        gm._features_dc = torch.nn.Parameter(feat[:, :1].clone().contiguous())
        gm._features_rest = torch.nn.Parameter(feat[:, 1:].clone().contiguous())
        gm._opacity = torch.nn.Parameter(logit.clone())
        gm._scaling = torch.nn.Parameter(log_s.clone())
        gm._rotation = torch.nn.Parameter(q.clone())
        proj = getProjectionMatrix2(znear=0.01, zfar=100.0, fx=fx, fy=fx, cx=cx, cy=cy, W=W, H=H).transpose(0, 1)
        cam = Camera(0, None, None, torch.eye(4), proj, fx, fx, cx, cy, focal2fov(fx, W), focal2fov(fx, H),
                     H, W, device="cpu")
        cam.update_RT(R, T)
        pipe = types.SimpleNamespace(compute_cov3D_python=cov_python, convert_SHs_python=shs_python)
        RECORD.clear()
        pkg = render(cam, gm, pipe, torch.tensor(bg, dtype=torch.float32), scaling_modifier=scaling_modifier)
        loss = (pkg["render"] * gc).sum() + (pkg["depth"] * gd).sum()
        loss.backward()
    rec = RECORD[0]
    s = rec["settings"]
    f = lambda t: t.detach().float().numpy()  # noqa: E731
    out = dict(
        P=np.array(P), W=np.array(W), H=np.array(H), fx=np.array(fx), cx=np.array(cx), cy=np.array(cy),
        R=R.numpy(), T=T.numpy(), FoVx=np.array(cam.FoVx), FoVy=np.array(cam.FoVy), bg=np.array(bg, np.float32),
        max_sh_degree=np.array(max_sh), active_sh_degree=np.array(active_sh),
        compute_cov3D_python=np.array(cov_python), convert_SHs_python=np.array(shs_python),
        scaling_modifier=np.array(scaling_modifier),
        raw_xyz=f(gm._xyz), raw_features_dc=f(gm._features_dc), raw_features_rest=f(gm._features_rest),
        raw_opacity=f(gm._opacity), raw_scaling=f(gm._scaling), raw_rotation=f(gm._rotation),
        grad_color=gc.numpy(), grad_depth=gd.numpy(),
        # what render() handed the rasteriser
        set_image_height=np.array(s.image_height), set_image_width=np.array(s.image_width),
        set_tanfovx=np.array(s.tanfovx), set_tanfovy=np.array(s.tanfovy), set_bg=f(s.bg),
        set_scale_modifier=np.array(s.scale_modifier), set_viewmatrix=f(s.viewmatrix),
        set_projmatrix=f(s.projmatrix), set_projmatrix_raw=f(s.projmatrix_raw),
        set_sh_degree=np.array(s.sh_degree), set_campos=f(s.campos),
        set_prefiltered=np.array(s.prefiltered), set_debug=np.array(s.debug),
        num_rendered=np.array(rec["num_rendered"]),
        # result dict
        out_render=f(pkg["render"]), out_depth=f(pkg["depth"]), out_opacity=f(pkg["opacity"]),
        out_radii=pkg["radii"].numpy(), out_visibility_filter=pkg["visibility_filter"].numpy(),
        out_n_touched=pkg["n_touched"].numpy(),
        # n_touched counts T > 0.5 after blending: Gaussians whose count moves
        # when that threshold moves by 1e-5 are the only ones allowed to differ
        out_n_touched_lo=rec["n_touched_lo"].numpy(), out_n_touched_hi=rec["n_touched_hi"].numpy(),
        # gradients autograd delivers through the reference chain
        g_xyz=f(gm._xyz.grad), g_features_dc=f(gm._features_dc.grad),
        g_features_rest=f(gm._features_rest.grad) if gm._features_rest.grad is not None
        else np.zeros(tuple(gm._features_rest.shape), np.float32),
        g_opacity=f(gm._opacity.grad), g_scaling=f(gm._scaling.grad), g_rotation=f(gm._rotation.grad),
        g_cam_rot_delta=f(cam.cam_rot_delta.grad), g_cam_trans_delta=f(cam.cam_trans_delta.grad),
        g_viewspace_points=f(pkg["viewspace_points"].grad),
    )
    for k in ("means3D", "opacities", "shs", "colors_precomp", "scales", "rotations", "cov3D_precomp"):
        if rec[k] is not None:
            out["in_" + k] = f(rec[k])
    path = os.path.join(HERE, f"ref_render_{name}.npz")
    np.savez_compressed(path, **out)
    print(f"{os.path.basename(path)}: P={P} {W}x{H} N={rec['num_rendered']} "
          f"visible={int(pkg['visibility_filter'].sum())} {os.path.getsize(path) / 1e3:.0f} kB")


def general_utils_cases():
    from thirdparty.gaussian_splatting.utils import general_utils as gu
    g = torch.Generator().manual_seed(77)
    r = torch.randn(64, 4, generator=g) * (0.3 + 2 * torch.rand(64, 1, generator=g))
    s = torch.exp(torch.randn(64, 3, generator=g))
    with CudaToCpu():
        R = gu.build_rotation(r)
        L = gu.build_scaling_rotation(s, r)
        sym = gu.strip_symmetric(L @ L.transpose(1, 2))
    np.savez_compressed(os.path.join(HERE, "ref_general_utils.npz"), r=r.numpy(), s=s.numpy(),
                        build_rotation=R.numpy(), build_scaling_rotation=L.numpy(), strip_symmetric=sym.numpy())
    print("ref_general_utils.npz written")


def main():
    torch.set_num_threads(8)
    _install_stubs()
    general_utils_cases()
    # SH0 at the TUM operating point scaled down 4x (512x384 -> 128x96, fx = 517.3 / 4),
    # identity pose, black background (mapper.py:83-86)
    _case("sh0_128x96", P=1500, W=128, H=96, fx=517.3 / 4, max_sh=0, active_sh=0,
          R=torch.eye(3), T=torch.zeros(3), bg=[0.0, 0.0, 0.0], seed=101)
    # SH3 with a non-identity keyframe pose and a coloured background
    _case("sh3_pose_96x72", P=900, W=96, H=72, fx=0.9 * 96, max_sh=3, active_sh=3,
          R=_rot([0.3, 1.0, -0.2], 7.0), T=torch.tensor([0.12, -0.05, 0.3]), bg=[0.1, 0.2, 0.3], seed=102)
    # the python-side branches: cov3D from get_covariance, colours from eval_sh
    # (active degree 1 of max 2), scale modifier
    _case("pyprecomp_64x48", P=400, W=64, H=48, fx=0.9 * 64, max_sh=2, active_sh=1,
          R=_rot([1.0, 0.0, 0.4], -5.0), T=torch.tensor([-0.1, 0.04, 0.0]), bg=[0.3, 0.0, 0.6], seed=103,
          cov_python=True, shs_python=True, scaling_modifier=0.7)


if __name__ == "__main__":
    main()
