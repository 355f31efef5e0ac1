"""GPU parity of the pose-refinement loss (wgsr.tracking; SURVEY.md 8(f) row
f2, tracking half): against the reference's own get_loss_tracking outputs
(tests/golden/track_cases.npz), against oracle/tracking.py at 480 x 640 with
and without uncertainty, Camera.compute_grad_mask against the restatement,
and one refinement iteration through the rasteriser (pose / exposure
gradients) against the reference torch composition.

Tolerances: loss rel 1e-5; image / opacity gradients rel-L1 1e-5 (a sign
flips only where the masked residual is exactly 0); exposure and pose
gradients rel 1e-3 (sums over every pixel / Gaussian); grad mask: the
Scharr taps sum in a different order than the conv2d of the restatement, so
a pixel whose intensity sits on its block's threshold may flip -- at most
1e-3 of the pixels, and the median thresholds themselves agree.
"""
import os
import types

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import tracking as ot

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIX = np.load(os.path.join(ROOT, "tests", "golden", "track_cases.npz"))
CASES = sorted({k.split("_")[0] for k in FIX.files})


def _rel(a, b):
    a, b = a.detach().double().cpu(), torch.as_tensor(b).detach().double().cpu()
    return float((a - b).abs().sum() / b.abs().sum().clamp_min(1e-30))


@pytest.mark.parametrize("k", CASES)
def test_matches_reference_fixtures(k):
    from wgsr.tracking import tracking_loss
    c = {n[len(k) + 1:]: FIX[n] for n in FIX.files if n.startswith(k + "_")}
    t = {n: torch.from_numpy(np.ascontiguousarray(c[n])).to(DEV) for n in ("gt", "ren", "opa", "gm", "ea", "eb")}
    r, o, a, b = (t[n].clone().requires_grad_(True) for n in ("ren", "opa", "ea", "eb"))
    unc = torch.from_numpy(c["unc"]).to(DEV) if "unc" in c else None
    loss = tracking_loss(r, o, t["gt"], a, b, t["gm"], unc)
    loss.backward()
    torch.cuda.synchronize()
    assert abs(float(loss) - float(c["loss"])) <= 1e-5 * abs(float(c["loss"]))
    assert _rel(r.grad, c["g_ren"]) <= 1e-5
    assert _rel(o.grad, c["g_opa"]) <= 1e-5
    assert _rel(a.grad, c["g_ea"]) <= 1e-3
    assert _rel(b.grad, c["g_eb"]) <= 1e-3


def _frame(H, W, seed):
    g = torch.Generator().manual_seed(seed)
    gt = torch.rand(3, H, W, generator=g)
    gt[:, :10, :30] = 0.0
    ren = (gt + 0.1 * torch.randn(3, H, W, generator=g)).clamp(0, 1)
    opa = torch.rand(1, H, W, generator=g)
    unc = torch.rand(H, W, generator=g) * 2.5 + 0.05
    ea, eb = 0.05 * torch.randn(1, generator=g), 0.02 * torch.randn(1, generator=g)
    return [x.to(DEV) for x in (gt, ren, opa, unc, ea, eb)]


@pytest.mark.parametrize("with_unc", [True, False])
def test_matches_oracle_480x640(with_unc):
    from wgsr.tracking import compute_grad_mask, tracking_loss
    gt, ren, opa, unc, ea, eb = _frame(480, 640, 3)
    gm = compute_grad_mask(gt, 4)
    u = unc if with_unc else None
    res = {}
    for who in ("oracle", "hip"):
        r, o, a, b = (x.clone().requires_grad_(True) for x in (ren, opa, ea, eb))
        fn = ot.loss_tracking if who == "oracle" else tracking_loss
        loss = fn(r, o, gt, a, b, gm, u)
        loss.backward()
        res[who] = (float(loss), r.grad, o.grad, a.grad, b.grad)
    torch.cuda.synchronize()
    lo, *go = res["oracle"]
    lh, *gh = res["hip"]
    assert abs(lh - lo) <= 1e-5 * abs(lo)
    for x, y, tol in zip(gh, go, (1e-5, 1e-5, 1e-3, 1e-3)):
        assert _rel(x, y) <= tol


@pytest.mark.parametrize("H,W", [(480, 640), (384, 512), (1080, 1920), (250, 333)])
def test_grad_mask_matches_restatement(H, W):
    from wgsr.tracking import compute_grad_mask
    g = torch.Generator().manual_seed(H)
    # an 8-bit photo-like image: smooth shading, edges, flat dark patches
    yy, xx = torch.meshgrid(torch.linspace(0, 1, H), torch.linspace(0, 1, W), indexing="ij")
    base = 0.5 + 0.3 * torch.sin(9 * xx) * torch.cos(7 * yy)
    img = torch.stack([base, base * 0.8, base * 0.6]) + 0.05 * torch.rand(3, H, W, generator=g)
    img[:, H // 3: H // 2, W // 4: W // 3] = 0.003
    img = (img.clamp(0, 1) * 255).round() / 255
    img = img.to(DEV)
    got = compute_grad_mask(img, 4)
    want = ot.compute_grad_mask(img, 4)
    torch.cuda.synchronize()
    bh, bw = H // 32, W // 32
    inside = torch.zeros(1, H, W, dtype=torch.bool, device=DEV)
    inside[:, :32 * bh, :32 * bw] = True
    mism = ((got != want) & inside).float().mean().item()
    assert mism <= 1e-3
    if (~inside).any():
        assert _rel(got[~inside], want[~inside]) <= 1e-5


def test_refinement_iteration_pose_gradients():
    """render -> get_loss_tracking -> backward: the keyframe's pose and
    exposure gradients match the reference composition (same rasteriser,
    oracle loss)."""
    from wgsr.camera import synthetic_camera
    from wgsr.render import DeviceCamera, render
    from wgsr.scene import make_scene
    from wgsr.tracking import compute_grad_mask, get_loss_tracking
    P, W, H = 3000, 128, 96
    sc = make_scene(P, W, H, 3, seed=5)
    g = torch.Generator().manual_seed(6)
    gt = torch.rand(3, H, W, generator=g).to(DEV)
    unc = (torch.rand(H, W, generator=g) * 2 + 0.05).to(DEV)
    gm = compute_grad_mask(gt, 4)
    out = {}
    for who in ("oracle", "hip"):
        cam = DeviceCamera.from_pinhole(synthetic_camera(W, H, 1), DEV)
        a = torch.tensor([0.1], device=DEV, requires_grad=True)
        b = torch.tensor([-0.02], device=DEV, requires_grad=True)
        pkg = render(cam, sc.means3D.to(DEV), sc.opacities.to(DEV), sc.scales.to(DEV), sc.rotations.to(DEV),
                     sc.shs.to(DEV), 3, torch.zeros(3, device=DEV))
        if who == "oracle":
            loss = ot.loss_tracking(pkg["render"], pkg["opacity"], gt, a, b, gm, unc)
        else:
            vp = types.SimpleNamespace(original_image=gt, grad_mask=gm, exposure_a=a, exposure_b=b)
            loss = get_loss_tracking({"Training": {"rgb_boundary_threshold": 0.01}}, pkg["render"], pkg["depth"],
                                     pkg["opacity"], vp, uncertainty=unc)
        loss.backward()
        out[who] = (float(loss), cam.cam_rot_delta.grad.clone(), cam.cam_trans_delta.grad.clone(), a.grad, b.grad)
    torch.cuda.synchronize()
    assert abs(out["hip"][0] - out["oracle"][0]) <= 1e-5 * abs(out["oracle"][0])
    for x, y in zip(out["hip"][1:], out["oracle"][1:]):
        assert _rel(x, y) <= 1e-3


def test_grad_mask_tiny_and_blockless_images():
    """Images smaller than the 32 x 32 block grid keep the raw intensity
    everywhere (the reference's blocks are empty slices)."""
    from wgsr.tracking import compute_grad_mask
    for H, W in ((20, 40), (33, 31), (2, 2)):
        img = torch.rand(3, H, W, generator=torch.Generator().manual_seed(H * W)).to(DEV)
        got = compute_grad_mask(img, 4)
        want = ot.compute_grad_mask(img, 4)
        torch.cuda.synchronize()
        assert got.shape == (1, H, W)
        torch.testing.assert_close(got, want, rtol=1e-5, atol=1e-6)  # tap-order rounding of ~0 sums


def _reference_refine(sc, deg, bg, cam_p, gt, gm, unc, ea0, eb0, iters, lr=(0.003, 0.001, 0.01), thr=1e-4):
    """mapper.py:856-911 in torch: render (autograd rasteriser), the oracle
    tracking loss, torch.optim.Adam over the four groups, update_pose with the
    restated SE3_exp (pose_utils.py:30-98)."""
    from wgsr.camera import PinholeCamera, se3_exp
    from wgsr.render import DeviceCamera, render
    R, T = cam_p.R.clone(), cam_p.T.clone()
    rot = torch.zeros(3, device=DEV, requires_grad=True)
    trans = torch.zeros(3, device=DEV, requires_grad=True)
    a = ea0.clone().requires_grad_(True)
    b = eb0.clone().requires_grad_(True)
    opt = torch.optim.Adam([{"params": [rot], "lr": lr[0]}, {"params": [trans], "lr": lr[1]},
                            {"params": [a], "lr": lr[2]}, {"params": [b], "lr": lr[2]}])
    it = 0
    for it in range(1, iters + 1):
        pc = PinholeCamera(R=R, T=T, fx=cam_p.fx, fy=cam_p.fy, cx=cam_p.cx, cy=cam_p.cy, W=cam_p.W, H=cam_p.H)
        cam = DeviceCamera.from_pinhole(pc, DEV)
        cam.cam_rot_delta, cam.cam_trans_delta = rot, trans
        pkg = render(cam, sc.means3D.to(DEV), sc.opacities.to(DEV), sc.scales.to(DEV), sc.rotations.to(DEV),
                     sc.shs.to(DEV), deg, bg)
        opt.zero_grad()
        ot.loss_tracking(pkg["render"], pkg["opacity"], gt, a, b, gm, unc).backward()
        opt.step()
        with torch.no_grad():
            tau = torch.cat([trans, rot]).cpu()
            w2c = torch.eye(4)
            w2c[:3, :3], w2c[:3, 3] = R, T
            new = se3_exp(tau) @ w2c
            R, T = new[:3, :3].clone(), new[:3, 3].clone()
            rot.zero_()
            trans.zero_()
            if float(tau.norm()) < thr:
                break
    return R, T, a.detach(), b.detach(), it


@pytest.mark.parametrize("iters", [1, 6])
def test_pose_refine_matches_reference_loop(iters):
    """wgsr.tracking.PoseRefine (device Adam + SE3 update + camera in one
    launch per iteration) vs the reference loop from a perturbed pose."""
    import math
    from wgsr.camera import synthetic_camera
    from wgsr.render import render, DeviceCamera
    from wgsr.scene import make_scene
    from wgsr.tracking import PoseRefine, compute_grad_mask
    P, W, H, deg = 4000, 160, 120, 2
    sc = make_scene(P, W, H, deg, seed=21)
    bg = torch.zeros(3, device=DEV)
    true_cam = synthetic_camera(W, H, 0)
    with torch.no_grad():  # the target: the scene rendered from the true pose
        gt = render(DeviceCamera.from_pinhole(true_cam, DEV), sc.means3D.to(DEV), sc.opacities.to(DEV),
                    sc.scales.to(DEV), sc.rotations.to(DEV), sc.shs.to(DEV), deg, bg)["render"].detach()
    start = synthetic_camera(W, H, 1)  # 2 degrees and 5 cm off
    gm = compute_grad_mask(gt, 4)
    unc = (torch.rand(H, W, generator=torch.Generator().manual_seed(3)) * 2 + 0.05).to(DEV)
    ea0, eb0 = torch.tensor([0.02], device=DEV), torch.tensor([-0.01], device=DEV)
    Rr, Tr, ar, br, itr = _reference_refine(sc, deg, bg, start, gt, gm, unc, ea0, eb0, iters)
    pr = PoseRefine(sc.means3D.to(DEV), sc.opacities.to(DEV), sc.scales.to(DEV), sc.rotations.to(DEV),
                    sc.shs.to(DEV), deg, bg, start.projection_matrix.to(DEV), H, W, start.FoVx, start.FoVy)
    R, T, a, b, it = pr.refine(start.R, start.T, ea0, eb0, gt, gm, unc, iters=iters)
    torch.cuda.synchronize()
    assert it == itr
    assert float((R.cpu() - Rr).abs().max()) <= 1e-5 * max(1, iters)
    assert float((T.cpu() - Tr).abs().max()) <= 1e-5 * max(1, iters)
    assert abs(float(a) - float(ar)) <= 1e-5 * max(1, iters)
    assert abs(float(b) - float(br)) <= 1e-5 * max(1, iters)
    # the refinement moved the pose (toward the truth)
    assert float((R.cpu() - start.R).abs().max()) > 1e-4 and not math.isnan(float(R.sum()))
