#!/usr/bin/env python
"""The mapper's pose refinement on the MI355X path.

Times, against the reference's own torch formulation (restated below from
src/utils/slam_utils.py:10-82 and src/utils/camera_utils.py:157-180):

* ``compute_grad_mask`` per keyframe (a Python loop of 1024 block medians in
  the reference) vs wgsr.tracking.compute_grad_mask (two launches);
* the tracking loss forward + backward vs wgsr.tracking.tracking_loss (one
  pass);
* one whole refinement iteration (mapper.py:884-906: render -> loss ->
  backward -> Adam over rot/trans/exposure) with each loss, same rasteriser.

Synthetic scene/targets (BASELINE.md distribution); device time per call.
"""
import argparse
import json
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
    out["note"] = ("same rasteriser in both refinement loops (update_pose's SE3 step is caller-side torch in both "
                   "and not included); reference = slam_utils / camera_utils torch ops restated")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
