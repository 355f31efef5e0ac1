#!/usr/bin/env python
"""The mapper's pose refinement on the MI355X path.

Times, against the reference's own torch formulation (restated below from
src/utils/slam_utils.py:10-82 and src/utils/camera_utils.py:157-180):

* ``compute_grad_mask`` per keyframe (a Python loop of 1024 block medians in
  the reference) vs wgsr.tracking.compute_grad_mask (two launches);
* the tracking loss forward + backward vs wgsr.tracking.tracking_loss (one
  pass);
* one whole refinement iteration (mapper.py:884-906: render -> loss ->
  backward -> Adam over rot/trans/exposure) with each loss, same rasteriser;
* the whole refinement loop with the reference's per-iteration Camera
  matrices and update_pose vs wgsr.tracking.PoseRefine.

Synthetic scene/targets (BASELINE.md distribution); device time per call.
"""
import argparse
import json
import math
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "wildgs-slam-blackwell_amd", "python"))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def ref_grad_mask(img, edge_threshold=4):
    dev = img.device
    gray = img.mean(dim=0, keepdim=True)
    conv_y = torch.tensor([[3, 0, -3], [10, 0, -10], [3, 0, -3]], dtype=torch.float32, device=dev)
    conv_x = torch.tensor([[3, 10, 3], [0, 0, 0], [-3, -10, -3]], dtype=torch.float32, device=dev)
    norm = 1.0 / torch.abs(conv_y).sum()
    p = F.pad(gray, (1, 1, 1, 1), mode="reflect")[None]
    gv = norm * F.conv2d(p, conv_x.view(1, 1, 3, 3))
    gh = norm * F.conv2d(p, conv_y.view(1, 1, 3, 3))
    ones = torch.ones((1, 1, 3, 3), device=dev)
    pm = (torch.abs(p) > 0.01).float()
    mv = F.conv2d(pm, ones)[0] == torch.sum(ones)
    mh = F.conv2d(pm, ones)[0] == torch.sum(ones)
    inten = torch.sqrt((gv[0] * mv) ** 2 + (gh[0] * mh) ** 2)
    _, h, w = img.shape
    for r in range(32):
        for c in range(32):
            block = inten[:, r * int(h / 32):(r + 1) * int(h / 32), c * int(w / 32):(c + 1) * int(w / 32)]
            th = block.median()
            block[block > (th * edge_threshold)] = 1
            block[block <= (th * edge_threshold)] = 0
    return inten


def ref_loss(image, opacity, gt, a, b, gm, unc):
    image_ab = torch.exp(a) * image + b
    _, h, w = gt.shape
    m = (gt.sum(dim=0) > 0.01).view(1, h, w) * gm
    l1 = opacity * torch.abs(image_ab * m - gt * m)
    weights = 0.5 / (unc.unsqueeze(0)) ** 2
    weights = torch.where(weights < 0.1, 0.0, weights)
    l1 *= weights
    return l1.mean()


def timed(fn, iters, warmup=3):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, default=100_000)
    ap.add_argument("--width", type=int, default=512)
    ap.add_argument("--height", type=int, default=384)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from wgsr.camera import synthetic_camera
    from wgsr.render import DeviceCamera, render
    from wgsr.scene import make_scene
    from wgsr.tracking import compute_grad_mask, tracking_loss
    dev = torch.device("cuda:0")
    P, W, H = a.P, a.width, a.height
    g = torch.Generator().manual_seed(1)
    gt = torch.rand(3, H, W, generator=g).to(dev)
    unc = (torch.rand(H, W, generator=g) * 2 + 0.05).to(dev)
    out = {"workload": f"pose refinement, {P} Gaussians, {W}x{H}, SH3"}
    out["grad_mask_ms_reference_torch"] = timed(lambda: ref_grad_mask(gt), 3, 1)
    out["grad_mask_ms_hip"] = timed(lambda: compute_grad_mask(gt), a.iters)
    gm = compute_grad_mask(gt)
    ren = torch.rand(3, H, W, generator=g).to(dev).requires_grad_(True)
    opa = torch.rand(1, H, W, generator=g).to(dev).requires_grad_(True)
    ea = torch.zeros(1, device=dev, requires_grad=True)
    eb = torch.zeros(1, device=dev, requires_grad=True)
    out["loss_fwd_bwd_ms_reference_torch"] = timed(lambda: ref_loss(ren, opa, gt, ea, eb, gm, unc).backward(),
                                                   a.iters)
    out["loss_fwd_bwd_ms_hip"] = timed(lambda: tracking_loss(ren, opa, gt, ea, eb, gm, unc).backward(), a.iters)
    sc = make_scene(P, W, H, 3, seed=0)
    means, opac, scales, rots, shs = (x.to(dev) for x in (sc.means3D, sc.opacities, sc.scales, sc.rotations,
                                                           sc.shs))
    bg = torch.zeros(3, device=dev)

    def refine(loss_fn):
        cam = DeviceCamera.from_pinhole(synthetic_camera(W, H, 0), dev)
        xa = torch.zeros(1, device=dev, requires_grad=True)
        xb = torch.zeros(1, device=dev, requires_grad=True)
        opt = torch.optim.Adam([{"params": [cam.cam_rot_delta], "lr": 0.003},
                                {"params": [cam.cam_trans_delta], "lr": 0.001},
                                {"params": [xa], "lr": 0.01}, {"params": [xb], "lr": 0.01}])

        def it():
            pkg = render(cam, means, opac, scales, rots, shs, 3, bg)
            opt.zero_grad()
            loss_fn(pkg["render"], pkg["opacity"], gt, xa, xb, gm, unc).backward()
            opt.step()
        return timed(it, a.iters)

    out["refine_iter_ms_reference_loss"] = refine(ref_loss)
    out["refine_iter_ms_hip_loss"] = refine(tracking_loss)

    # the whole refinement loop as mapper.py:884-906 runs it, including the
    # Camera properties recomputed on the device each iteration
    # (getWorld2View2's two 4x4 inversions, camera_utils.py:137-151) and
    # update_pose (pose_utils.py:81-98), vs wgsr.tracking.PoseRefine
    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
    from wgsr.tracking import PoseRefine
    cam0 = synthetic_camera(W, H, 0)
    Pt = cam0.projection_matrix.to(dev)
    tanx, tany = math.tan(cam0.FoVx * 0.5), math.tan(cam0.FoVy * 0.5)

    def w2v(R, T):
        Rt = torch.zeros((4, 4), device=dev)
        Rt[:3, :3] = R
        Rt[:3, 3] = T
        Rt[3, 3] = 1.0
        return torch.linalg.inv(torch.linalg.inv(Rt))

    def skew(x):
        m = torch.zeros(3, 3, device=dev)
        m[0, 1], m[0, 2], m[1, 0], m[1, 2], m[2, 0], m[2, 1] = -x[2], x[1], x[2], -x[0], -x[1], x[0]
        return m

    def se3(tau):
        rho, theta = tau[:3], tau[3:]
        Wm = skew(theta)
        W2 = Wm @ Wm
        ang = torch.norm(theta)
        I = torch.eye(3, device=dev)
        if ang < 1e-5:
            Rx, Vx = I + Wm + 0.5 * W2, I + 0.5 * Wm + (1.0 / 6.0) * W2
        else:
            Rx = I + (torch.sin(ang) / ang) * Wm + ((1 - torch.cos(ang)) / (ang ** 2)) * W2
            Vx = I + Wm * ((1.0 - torch.cos(ang)) / (ang ** 2)) + W2 * ((ang - torch.sin(ang)) / (ang ** 3))
        Tm = torch.eye(4, device=dev)
        Tm[:3, :3] = Rx
        Tm[:3, 3] = Vx @ rho
        return Tm

    def ref_loop(n):
        R, T = cam0.R.to(dev).clone(), cam0.T.to(dev).clone()
        rot = torch.zeros(3, device=dev, requires_grad=True)
        trans = torch.zeros(3, device=dev, requires_grad=True)
        xa = torch.zeros(1, device=dev, requires_grad=True)
        xb = torch.zeros(1, device=dev, requires_grad=True)
        opt = torch.optim.Adam([{"params": [rot], "lr": 0.003}, {"params": [trans], "lr": 0.001},
                                {"params": [xa], "lr": 0.01}, {"params": [xb], "lr": 0.01}])
        for _ in range(n):
            wv = w2v(R, T).transpose(0, 1)
            full = w2v(R, T).transpose(0, 1).unsqueeze(0).bmm(Pt.unsqueeze(0)).squeeze(0)
            center = w2v(R, T).transpose(0, 1).inverse()[3, :3]
            st = GaussianRasterizationSettings(H, W, tanx, tany, bg, 1.0, wv, full, Pt, 3, center, False, False)
            m2d = torch.zeros_like(means, requires_grad=True) + 0
            img, _, _, op, _ = GaussianRasterizer(st)(means3D=means, means2D=m2d, shs=shs, colors_precomp=None,
                                                      opacities=opac, scales=scales, rotations=rots,
                                                      cov3D_precomp=None, theta=rot, rho=trans)
            opt.zero_grad()
            ref_loss(img, op, gt, xa, xb, gm, unc).backward()
            opt.step()
            with torch.no_grad():
                tau = torch.cat([trans, rot], axis=0)
                w2c = torch.eye(4, device=dev)
                w2c[0:3, 0:3], w2c[0:3, 3] = R, T
                new = se3(tau) @ w2c
                R, T = new[0:3, 0:3], new[0:3, 3]
                converged = tau.norm() < 0.0
                rot.data.fill_(0)
                trans.data.fill_(0)
                if converged:
                    break

    pr = PoseRefine(means, opac, scales, rots, shs, 3, bg, Pt, H, W, cam0.FoVx, cam0.FoVy)
    z = torch.zeros(1, device=dev)
    n = a.iters
    out["refine_loop_ms_per_iter_reference"] = timed(lambda: ref_loop(n), 2, 1) / n
    out["refine_loop_ms_per_iter_pose_refine"] = timed(
        lambda: pr.refine(cam0.R, cam0.T, z, z, gt, gm, unc, iters=n, converged_threshold=0.0), 2, 1) / n
    out["note"] = ("same rasteriser everywhere; refine_iter_*: render + loss + backward + Adam only; "
                   "refine_loop_*: the whole mapper.py:884-906 iteration incl. the Camera matrices and update_pose; "
                   "reference = slam_utils / camera_utils / pose_utils torch ops restated")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
