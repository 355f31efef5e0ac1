"""Generate the golden fixtures under tests/golden/ (run in the build container).

Two kinds of vectors are written:

1. ``ref_helpers.npz`` - inputs and outputs of the reference's OWN importable
   helpers (imported from /root/reference, which exists only in the build
   container): ``getProjectionMatrix2``/``getWorld2View2``/``focal2fov``
   (thirdparty/gaussian_splatting/utils/graphics_utils.py:33-101),
   ``SE3_exp`` (src/utils/pose_utils.py:66-78) and ``eval_sh``
   (thirdparty/gaussian_splatting/utils/sh_utils.py:54-119).  These are the
   "true-reference" components that pin the restatements in
   wildgs-slam-blackwell_amd/python/wgsr/camera.py and oracle/dense.py.

2. ``scene_*.npz`` - synthetic Gaussian scenes + camera settings with the
   float64 autograd oracle's (oracle/dense.py) forward outputs and gradients,
   and ``knn_cases.npz`` with float64 brute-force distCUDA2 answers.

The reference CUDA rasteriser itself is absent from the snapshot (empty
submodule, .gitmodules:7-9), so these scene vectors are oracle outputs, not
reference-binary outputs: parity with the binary is unpinned.

Usage:  python tests/golden/make_fixtures.py
"""
from __future__ import annotations

import math
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(REPO, "wildgs-slam-blackwell_amd", "python"))
sys.path.insert(0, REPO)

from oracle import dense  # noqa: E402
from wgsr import camera as wcam  # noqa: E402
from wgsr.scene import make_scene, make_upstream_grads, make_points  # noqa: E402

REF = "/root/reference"


def ref_helpers():
    sys.path.insert(0, REF)
    from thirdparty.gaussian_splatting.utils import graphics_utils as gu
    from thirdparty.gaussian_splatting.utils import sh_utils as su
    from src.utils import pose_utils as pu

    out = {}
    g = torch.Generator().manual_seed(7)
    # projection matrices
    cams = np.array([[0.01, 100.0, 320, 240, 576, 576, 640, 480],
                     [0.01, 100.0, 960, 540, 1728, 1728, 1920, 1080],
                     [0.01, 100.0, 250.3, 190.1, 517.3, 516.5, 512, 384]], np.float64)
    out["proj_in"] = cams
    out["proj_out"] = np.stack([gu.getProjectionMatrix2(*c).numpy() for c in cams])
    mine = np.stack([wcam.get_projection_matrix2(*c).numpy() for c in cams])
    assert np.array_equal(mine, out["proj_out"]), "getProjectionMatrix2 restatement differs"
    # world2view
    Rs, ts, w2v = [], [], []
    for k in range(4):
        q = torch.randn(4, generator=g)
        q = q / q.norm()
        R = dense.quat_to_rot(q[None].double())[0].float()
        t = torch.randn(3, generator=g)
        Rs.append(R.numpy()); ts.append(t.numpy())
        w2v.append(gu.getWorld2View2(R, t).numpy())
        assert torch.equal(wcam.get_world2view2(R, t), gu.getWorld2View2(R, t))
    out["w2v_R"], out["w2v_t"], out["w2v_out"] = np.stack(Rs), np.stack(ts), np.stack(w2v)
    # focal2fov
    f_in = np.array([[576.0, 640], [1728.0, 1920], [517.3, 512]])
    out["fov_in"] = f_in
    out["fov_out"] = np.array([gu.focal2fov(f, p) for f, p in f_in])
    assert all(wcam.focal2fov(f, p) == gu.focal2fov(f, p) for f, p in f_in)
    # SE3_exp
    taus = [torch.zeros(6, dtype=torch.float64)]
    for k in range(5):
        taus.append(torch.randn(6, generator=g, dtype=torch.float64) * (10.0 ** -k))
    out["se3_in"] = np.stack([t.numpy() for t in taus])
    out["se3_out"] = np.stack([pu.SE3_exp(t).numpy() for t in taus])
    for t, ref in zip(taus, out["se3_out"]):
        assert np.allclose(dense.se3_exp(t).numpy(), ref, rtol=0, atol=1e-12)
        assert np.allclose(wcam.se3_exp(t).numpy(), ref, rtol=0, atol=1e-12)
    # eval_sh (reference layout [..., 3, K])
    dirs = torch.randn(64, 3, generator=g, dtype=torch.float64)
    dirs = dirs / dirs.norm(dim=1, keepdim=True)
    sh = torch.randn(64, 16, 3, generator=g, dtype=torch.float64)
    out["sh_dirs"], out["sh_coeffs"] = dirs.numpy(), sh.numpy()
    for deg in range(4):
        ref = su.eval_sh(deg, sh.transpose(1, 2), dirs)
        out[f"sh_out_deg{deg}"] = ref.numpy()
        assert torch.allclose(dense.eval_sh(deg, sh, dirs), ref, rtol=0, atol=1e-12)
    out["sh_C0"] = np.array(su.C0)
    np.savez_compressed(os.path.join(HERE, "ref_helpers.npz"), **out)
    print("ref_helpers.npz: reference helpers match the restatements")


def settings_for(cam: wcam.PinholeCamera, bg, sh_degree, scale_modifier=1.0):
    f = cam.raster_fields()
    return dict(H=cam.H, W=cam.W, tanfovx=f["tanfovx"], tanfovy=f["tanfovy"],
                bg=torch.tensor(bg, dtype=torch.float32), scale_modifier=scale_modifier,
                viewmatrix=f["viewmatrix"], projmatrix=f["projmatrix"],
                projmatrix_raw=f["projmatrix_raw"], sh_degree=sh_degree, campos=f["campos"])


def write_case(name, inputs: dict, settings: dict, grad_color, grad_depth):
    res = dense.dense_forward_backward(inputs, settings, grad_color, grad_depth)
    arr = {}
    for k, v in inputs.items():
        if v is not None:
            arr["in_" + k] = v.detach().float().numpy()
    for k, v in settings.items():
        arr["set_" + k] = v.numpy() if torch.is_tensor(v) else np.array(v)
    arr["grad_color"] = grad_color.numpy()
    arr["grad_depth"] = grad_depth.numpy()
    for k in ("color", "depth", "opacity"):
        arr["out_" + k] = res[k].float().numpy()
    arr["out_radii"] = res["radii"].numpy()
    arr["out_n_touched"] = res["n_touched"].numpy()
    arr["out_num_rendered"] = np.array(res["num_rendered"])
    for k, v in res.items():
        if k.startswith("dL_") and v is not None:
            arr[k] = v.float().numpy()
    path = os.path.join(HERE, f"scene_{name}.npz")
    np.savez_compressed(path, **arr)
    print(f"{os.path.basename(path)}: P={inputs['means3D'].shape[0]} N={res['num_rendered']} "
          f"{os.path.getsize(path) / 1e3:.0f} kB")


def scene_cases():
    # main parity scenes (BASELINE.md synthetic distribution, reduced size)
    W, H = 160, 120
    sc = make_scene(2000, W, H, 0, seed=0)
    gc, gd = make_upstream_grads(W, H, seed=1)
    write_case("sh0_p2000_160x120",
               dict(means3D=sc.means3D, opacities=sc.opacities, shs=sc.shs, scales=sc.scales,
                    rotations=sc.rotations),
               settings_for(wcam.synthetic_camera(W, H, 0), [0.0, 0.0, 0.0], 0), gc, gd)

    W, H = 128, 96
    sc = make_scene(800, W, H, 3, seed=3)
    gc, gd = make_upstream_grads(W, H, seed=4)
    cam = wcam.synthetic_camera(W, H, 3)
    write_case("sh3_pose_p800_128x96",
               dict(means3D=sc.means3D, opacities=sc.opacities, shs=sc.shs, scales=sc.scales,
                    rotations=sc.rotations),
               settings_for(cam, [0.1, 0.2, 0.3], 3), gc, gd)

    # edge cases: W/H not multiples of 16 everywhere
    W, H = 40, 27
    g = torch.Generator().manual_seed(11)
    sc = make_scene(64, W, H, 1, seed=12)
    m = sc.means3D.clone()
    m[0] = torch.tensor([0.0, 0.0, 0.15])       # z <= 0.2: culled
    m[1] = torch.tensor([0.1, 0.0, -1.0])       # behind the camera
    m[2] = torch.tensor([0.0, 0.0, 0.2])        # exactly at the near plane: culled
    m[3] = torch.tensor([3.0, 0.0, 3.0])        # |x/z| = 1 > 1.3 tanfovx -> clamp (off-screen)
    m[4] = torch.tensor([0.0, 0.0, 1.5])        # huge Gaussian in front
    s = sc.scales.clone()
    s[4] = torch.tensor([0.5, 0.4, 0.3])
    s[3] = torch.tensor([1.5, 1.5, 1.5])       # big enough to reach the image from outside
    sh = sc.shs.clone()
    sh[5:10, 0, :] = -3.0                       # negative colour -> clamp flags
    gc, gd = make_upstream_grads(W, H, seed=13)
    write_case("edge_mixed_40x27",
               dict(means3D=m, opacities=sc.opacities, shs=sh, scales=s, rotations=sc.rotations),
               settings_for(wcam.synthetic_camera(W, H, 0), [0.3, 0.0, 0.7], 1), gc, gd)

    W, H = 33, 17
    sc = make_scene(1, W, H, 0, seed=21)
    gc, gd = make_upstream_grads(W, H, seed=22)
    write_case("edge_p1_33x17",
               dict(means3D=sc.means3D, opacities=sc.opacities, shs=sc.shs, scales=sc.scales * 4,
                    rotations=sc.rotations),
               settings_for(wcam.synthetic_camera(W, H, 0), [0.5, 0.5, 0.5], 0), gc, gd)

    sc = make_scene(16, W, H, 0, seed=23)
    m = sc.means3D.clone()
    m[:, 2] = -m[:, 2]                          # all behind the camera
    write_case("edge_allculled_33x17",
               dict(means3D=m, opacities=sc.opacities, shs=sc.shs, scales=sc.scales,
                    rotations=sc.rotations),
               settings_for(wcam.synthetic_camera(W, H, 0), [0.2, 0.4, 0.6], 0), gc, gd)

    W, H = 48, 40
    sc = make_scene(150, W, H, 2, seed=31)
    gc, gd = make_upstream_grads(W, H, seed=32)
    write_case("edge_scalemod_48x40",
               dict(means3D=sc.means3D, opacities=sc.opacities, shs=sc.shs, scales=sc.scales * 3,
                    rotations=sc.rotations),
               settings_for(wcam.synthetic_camera(W, H, 2), [0.0, 0.1, 0.0], 2, scale_modifier=0.5),
               gc, gd)

    # precomputed colours + precomputed covariance
    sc = make_scene(150, W, H, 0, seed=41)
    colors = torch.rand(150, 3, generator=g)
    R = dense.quat_to_rot(sc.rotations.double())
    S = torch.diag_embed(sc.scales.double() ** 2)
    Sig = R @ S @ R.transpose(1, 2)
    cov6 = torch.stack([Sig[:, 0, 0], Sig[:, 0, 1], Sig[:, 0, 2], Sig[:, 1, 1], Sig[:, 1, 2],
                        Sig[:, 2, 2]], dim=1).float()
    write_case("edge_precomp_48x40",
               dict(means3D=sc.means3D, opacities=sc.opacities, colors_precomp=colors,
                    cov3D_precomp=cov6),
               settings_for(wcam.synthetic_camera(W, H, 1), [0.0, 0.0, 0.0], 0), gc, gd)

    # dense, nearly opaque crowd -> early termination (T < 1e-4) everywhere
    sc = make_scene(600, W, H, 0, seed=51, opacity_range=(0.85, 0.95),
                    log_scale_range=(math.log(0.05), math.log(0.12)))
    write_case("edge_saturate_48x40",
               dict(means3D=sc.means3D, opacities=sc.opacities, shs=sc.shs, scales=sc.scales,
                    rotations=sc.rotations),
               settings_for(wcam.synthetic_camera(W, H, 0), [1.0, 1.0, 1.0], 0), gc, gd)


def knn_brute(pts: np.ndarray) -> np.ndarray:
    """Mean of the 3 smallest squared distances to other points (float64)."""
    P = pts.shape[0]
    p = pts.astype(np.float64)
    out = np.empty(P, np.float64)
    for s in range(0, P, 1024):
        d = ((p[s:s + 1024, None, :] - p[None, :, :]) ** 2).sum(-1)
        idx = np.arange(s, min(P, s + 1024))
        d[np.arange(len(idx)), idx] = np.inf
        d = np.where(np.isinf(d), np.finfo(np.float32).max, d)
        k = min(3, P)
        best = np.sort(d, axis=1)[:, :k] if P > 1 else np.full((len(idx), 0), 0.0)
        pad = np.full((len(idx), 3 - best.shape[1]), np.finfo(np.float32).max)
        best = np.concatenate([best, pad], axis=1)
        with np.errstate(over="ignore"):
            out[s:s + 1024] = best.astype(np.float32).sum(1, dtype=np.float32) / np.float32(3.0)
    return out


def knn_cases():
    arr = {}
    sizes = [1, 2, 3, 4, 7, 100, 1000, 5000]
    for i, P in enumerate(sizes):
        pts = make_points(P, seed=100 + i).numpy()
        arr[f"pts_{P}"] = pts
        arr[f"ref_{P}"] = knn_brute(pts)
    # a clustered cloud (like a back-projected depth map)
    g = torch.Generator().manual_seed(5)
    uv = torch.rand(3000, 2, generator=g)
    z = 1.0 + 0.2 * torch.sin(6 * uv[:, 0]) + 0.001 * torch.randn(3000, generator=g)
    pts = torch.stack([(uv[:, 0] - 0.5) * z, (uv[:, 1] - 0.5) * z, z], 1).float().numpy()
    arr["pts_surface"] = pts
    arr["ref_surface"] = knn_brute(pts)
    np.savez_compressed(os.path.join(HERE, "knn_cases.npz"), **arr)
    print("knn_cases.npz written")


if __name__ == "__main__":
    torch.set_num_threads(8)
    if os.path.isdir(REF):
        ref_helpers()
    else:
        print("reference not present: keeping the committed ref_helpers.npz")
    scene_cases()
    knn_cases()
