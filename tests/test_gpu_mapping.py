"""GPU parity of the fused mapping iteration (wgsr.mapping.MappingStep;
SURVEY.md 8(f) f1 + f2) against the reference's torch composition.

Reference side, as src/mapper.py:1083-1219 runs it (non-uncertainty branch):
GaussianModel activations (sigmoid / exp / F.normalize / cat), render()
through the autograd rasteriser, get_loss_mapping_rgbd (slam_utils.py:
107-143) with loss_utils' conv2d SSIM restated below, 10 x isotropic loss,
autograd backward, the densification statistics with boolean indexing, and
torch.optim.Adam over the six groups.  Tolerances: loss rel 1e-5; raw
parameter gradients rel-L1 1e-4 (the 1e-4 rasteriser contract; fp32
reduction order differs); exposure / pose gradients rel 1e-3 (sums over
every pixel / Gaussian); statistics exact (radii, counts) or rel 1e-5; the
Adam step on identical gradients to rtol 1e-5 / atol 1e-7 (as
tests/test_gpu_optim.py: torch's foreach kernels round differently).
"""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")
P, W, H, DEG = 3000, 128, 96, 3
ALPHA, LAM, TH = 0.95, 0.2, 0.01


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().sum() / b.abs().sum().clamp_min(1e-30))


def _window(ws, C):
    g = torch.tensor([math.exp(-((x - ws // 2) ** 2) / float(2 * 1.5 ** 2)) for x in range(ws)])
    g = g / g.sum()
    return (g[:, None] @ g[None, :]).expand(C, 1, ws, ws).contiguous().to(DEV)


def _torch_ssim(img1, img2, ws=11):
    """loss_utils.ssim (loss_utils.py:61-99) with size_average."""
    img1, img2 = img1.unsqueeze(0), img2.unsqueeze(0)
    w = _window(ws, 3)
    mu1 = F.conv2d(img1, w, padding=ws // 2, groups=3)
    mu2 = F.conv2d(img2, w, padding=ws // 2, groups=3)
    mu1_sq, mu2_sq, mu1_mu2 = mu1.pow(2), mu2.pow(2), mu1 * mu2
    s11 = F.conv2d(img1 * img1, w, padding=ws // 2, groups=3) - mu1_sq
    s22 = F.conv2d(img2 * img2, w, padding=ws // 2, groups=3) - mu2_sq
    s12 = F.conv2d(img1 * img2, w, padding=ws // 2, groups=3) - mu1_mu2
    return (((2 * mu1_mu2 + 1e-4) * (2 * s12 + 9e-4)) / ((mu1_sq + mu2_sq + 1e-4) * (s11 + s22 + 9e-4))).mean()


def _setup(seed=3):
    from wgsr.camera import synthetic_camera
    from wgsr.scene import make_scene
    sc = make_scene(P, W, H, DEG, seed=seed)
    g = torch.Generator().manual_seed(seed + 1)
    gt_image = torch.rand(3, H, W, generator=g)
    gt_image[:, :8] = 0.0                      # below the rgb boundary threshold
    gt_depth = 2 + 6 * torch.rand(1, H, W, generator=g)
    gt_depth[:, :, :10] = 0.0                  # invalid depth
    raw = dict(xyz=sc.means3D, f_dc=sc.shs[:, :1], f_rest=sc.shs[:, 1:],
               opacity=torch.log(sc.opacities / (1 - sc.opacities)), scaling=torch.log(sc.scales),
               rotation=sc.rotations * 1.7)   # un-normalised raw quaternions
    return synthetic_camera(W, H, 0), raw, gt_image.to(DEV), gt_depth.to(DEV)


def _reference(cam_p, raw, gt_image, gt_depth, ea, eb):
    from wgsr.render import DeviceCamera, render
    cam = DeviceCamera.from_pinhole(cam_p, DEV)
    leaf = {k: v.to(DEV).clone().contiguous().requires_grad_(True) for k, v in raw.items()}
    a = ea.clone().requires_grad_(True)
    b = eb.clone().requires_grad_(True)
    pkg = render(cam, leaf["xyz"], torch.sigmoid(leaf["opacity"]), torch.exp(leaf["scaling"]),
                 F.normalize(leaf["rotation"]), torch.cat((leaf["f_dc"], leaf["f_rest"]), dim=1), DEG,
                 torch.zeros(3, device=DEV))
    image, depth = pkg["render"], pkg["depth"]
    image_ab = torch.exp(a) * image + b
    ssim_loss = 1.0 - _torch_ssim(image_ab, gt_image)
    m = (gt_image.sum(dim=0) > TH).view(1, H, W)
    l1_rgb = torch.abs(image_ab * m - gt_image * m)
    loss = (1.0 - LAM) * l1_rgb + LAM * ssim_loss
    dm = (gt_depth > 0.01).view(*depth.shape)
    l1_depth = torch.abs(depth * dm - gt_depth * dm)
    lm = ALPHA * loss.mean() + (1 - ALPHA) * l1_depth.mean()
    scaling = torch.exp(leaf["scaling"])
    lm = lm + 10 * torch.abs(scaling - scaling.mean(dim=1).view(-1, 1)).mean()
    lm.backward()
    vis, radii = pkg["visibility_filter"], pkg["radii"]
    max_r = torch.zeros(P, device=DEV)
    acc = torch.zeros(P, 1, device=DEV)
    den = torch.zeros(P, 1, device=DEV)
    max_r[vis] = torch.max(max_r[vis], radii[vis].float())
    acc[vis] += torch.norm(pkg["viewspace_points"].grad[vis, :2], dim=-1, keepdim=True)
    den[vis] += 1
    return dict(loss=lm.detach(), leaf=leaf, a=a, b=b, cam=cam, stats=(max_r, acc, den), radii=radii)


def _fused(cam_p, raw, gt_image, gt_depth, ea, eb):
    from wgsr.mapping import MappingStep
    ms = MappingStep(raw["xyz"].to(DEV), raw["f_dc"].to(DEV), raw["f_rest"].to(DEV), raw["opacity"].to(DEV),
                     raw["scaling"].to(DEV), raw["rotation"].to(DEV), DEG)
    f = cam_p.raster_fields()
    cam = {k: (v.to(DEV) if torch.is_tensor(v) else v) for k, v in f.items()}
    out = ms.forward_backward(cam, gt_image, gt_depth, ea, eb, torch.zeros(3, device=DEV), alpha=ALPHA,
                              lambda_dssim=LAM, rgb_threshold=TH)
    torch.cuda.synchronize()
    return ms, out


@pytest.mark.parametrize("expo", [(0.0, 0.0), (0.15, -0.05)])
def test_fused_mapping_iteration_matches_torch_composition(expo):
    cam_p, raw, gt_image, gt_depth = _setup()
    ea = torch.tensor([expo[0]], device=DEV)
    eb = torch.tensor([expo[1]], device=DEV)
    ref = _reference(cam_p, raw, gt_image, gt_depth, ea, eb)
    ms, out = _fused(cam_p, raw, gt_image, gt_depth, ea, eb)
    assert abs(float(out["loss"]) - float(ref["loss"])) <= 1e-5 * abs(float(ref["loss"]))
    lf = ref["leaf"]
    assert _rel(ms.grad["xyz"], lf["xyz"].grad) <= 1e-4
    assert _rel(ms.grad["features"][:, :1], lf["f_dc"].grad) <= 1e-4
    assert _rel(ms.grad["features"][:, 1:], lf["f_rest"].grad) <= 1e-4
    assert _rel(ms.grad["opacity"], lf["opacity"].grad) <= 1e-4
    assert _rel(ms.grad["scaling"], lf["scaling"].grad) <= 1e-4
    assert _rel(ms.grad["rotation"], lf["rotation"].grad) <= 1e-4
    assert _rel(out["dexposure_a"], ref["a"].grad) <= 1e-3
    assert _rel(out["dexposure_b"], ref["b"].grad) <= 1e-3
    assert _rel(out["dtheta"], ref["cam"].cam_rot_delta.grad) <= 1e-3
    assert _rel(out["drho"], ref["cam"].cam_trans_delta.grad) <= 1e-3
    max_r, acc, den = ref["stats"]
    assert torch.equal(out["radii"], ref["radii"])
    assert torch.equal(ms.max_radii2D, max_r)
    assert torch.equal(ms.denom, den)
    assert _rel(ms.xyz_gradient_accum, acc) <= 1e-5


def test_fused_adam_step_matches_torch_adam_groups():
    """Two iterations of ms.optimizer_step() vs torch.optim.Adam over the six
    reference groups fed the same gradients (f_dc / f_rest: the split)."""
    from wgsr.mapping import DEFAULT_LR
    cam_p, raw, gt_image, gt_depth = _setup(seed=9)
    z = torch.zeros(1, device=DEV)
    ms, _ = _fused(cam_p, raw, gt_image, gt_depth, z, z)
    prm = {"xyz": ms.xyz.clone(), "f_dc": ms.f_dc.clone().contiguous(), "f_rest": ms.f_rest.clone().contiguous(),
           "opacity": ms.opacity.clone(), "scaling": ms.scaling.clone(), "rotation": ms.rotation.clone()}
    prm = {k: torch.nn.Parameter(v) for k, v in prm.items()}
    opt = torch.optim.Adam([{"params": [prm[k]], "lr": DEFAULT_LR[k], "name": k} for k in prm], lr=0.0,
                           eps=1e-15)
    for it in range(2):
        if it:
            for v in ms.grad.values():  # a second, different gradient
                v.mul_(-0.5).add_(1e-3)
        grads = {"xyz": ms.grad["xyz"], "f_dc": ms.grad["features"][:, :1], "f_rest": ms.grad["features"][:, 1:],
                 "opacity": ms.grad["opacity"], "scaling": ms.grad["scaling"], "rotation": ms.grad["rotation"]}
        for k, p in prm.items():
            p.grad = grads[k].clone().contiguous()
        opt.step()
        ms.optimizer_step()
        torch.cuda.synchronize()
        got = {"xyz": ms.xyz, "f_dc": ms.f_dc, "f_rest": ms.f_rest, "opacity": ms.opacity, "scaling": ms.scaling,
               "rotation": ms.rotation}
        for k, p in prm.items():
            torch.testing.assert_close(got[k], p.detach(), rtol=1e-5, atol=1e-7, msg=lambda m, k=k: f"{it} {k}: {m}")
