"""GPU parity of the uncertainty-aware mapping loss (wgsr.uncertainty, the
reference's default mapping loss) and of the mapping
iteration built on it (wgsr.mapping.MappingStep.forward_backward_uncertainty).

* against the reference's own outputs (tests/golden/uncer_cases.npz, made by
  tests/golden/make_uncer_fixtures.py from slam_utils.get_loss_mapping_uncertainty);
* against oracle/uncertainty.py (the torch restatement, run on the GPU with
  the same inputs) on a 540 x 960 frame;
* the whole iteration against the reference torch composition: render()
  through the autograd rasteriser, the oracle loss, 10 x isotropic loss, and
  autograd into the raw parameters, the exposures and an uncertainty MLP.

Tolerances: loss rel 1e-5; image / depth / uncertainty gradients rel-L1 1e-4
(fp32 reduction order and interpolation rounding differ: a weight may land
on the other side of the w < 0.1 cut); exposure gradients (sums over every
pixel) rel 1e-3; raw Gaussian parameter gradients rel-L1 1e-4 as in
tests/test_gpu_mapping.py.
"""
import os
import types

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import uncertainty as ou

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIX = np.load(os.path.join(ROOT, "tests", "golden", "uncer_cases.npz"))
CASES = sorted({k.split("_")[0] for k in FIX.files})


def _rel(a, b):
    a, b = a.detach().double().cpu(), torch.as_tensor(b).detach().double().cpu()
    return float((a - b).abs().sum() / b.abs().sum().clamp_min(1e-30))


def _leaves(c):
    t = {n: torch.from_numpy(np.ascontiguousarray(c[n])).to(DEV) for n in
         ("gt", "ren", "ref", "dep", "opa", "unc", "ea", "eb")}
    for n in ("ren", "dep", "unc", "ea", "eb"):
        t[n] = t[n].clone().requires_grad_(True)
    return t


@pytest.mark.parametrize("k", CASES)
def test_matches_reference_fixtures(k):
    from wgsr.uncertainty import mapping_loss_uncertainty
    c = {n[len(k) + 1:]: FIX[n] for n in FIX.files if n.startswith(k + "_")}
    tf, sf, init, freeze = (float(v) for v in c["meta"])
    t = _leaves(c)
    loss = mapping_loss_uncertainty(t["ren"], t["dep"], t["opa"], t["gt"], t["ref"], t["ea"], t["eb"], t["unc"], tf,
                                    sf, ou.DEFAULT_CONFIG, bool(init), bool(freeze))
    loss.backward()
    torch.cuda.synchronize()
    assert abs(float(loss) - float(c["loss"])) <= 1e-5 * abs(float(c["loss"]))
    assert _rel(t["ren"].grad, c["g_ren"]) <= 1e-4
    assert _rel(t["dep"].grad, c["g_dep"]) <= 1e-4
    if freeze:
        assert t["unc"].grad is None
    else:
        assert _rel(t["unc"].grad, c["g_unc"]) <= 1e-4
    if init:
        assert t["ea"].grad is None and t["eb"].grad is None
    else:
        assert _rel(t["ea"].grad, c["g_ea"]) <= 1e-3
        assert _rel(t["eb"].grad, c["g_eb"]) <= 1e-3


def _frame(H, W, h, w, seed):
    g = torch.Generator().manual_seed(seed)
    gt = torch.rand(3, H, W, generator=g)
    gt[:, :20, :40] = 0.0
    ren = (gt + 0.1 * torch.randn(3, H, W, generator=g)).clamp(0, 1)
    ref = 1.0 + 3.0 * torch.rand(1, H, W, generator=g)
    ref[:, 100:130, 200:300] = 0.0
    ref[:, -40:, -60:] = 90.0
    dep = ref + 1.5 * torch.randn(1, H, W, generator=g)
    opa = torch.rand(1, H, W, generator=g) * 0.3 + 0.7
    unc = torch.rand(h, w, generator=g) * 2.5
    unc[0, :5] = 0.05
    ea = 0.05 * torch.randn(1, generator=g)
    eb = 0.02 * torch.randn(1, generator=g)
    return [x.to(DEV) for x in (gt, ren, ref, dep, opa, unc, ea, eb)]


@pytest.mark.parametrize("tf,sf", [(0.3, 0.3), (0.9, 0.1)])
def test_matches_oracle_540x960(tf, sf):
    from wgsr.uncertainty import mapping_loss_uncertainty
    gt, ren, ref, dep, opa, unc, ea, eb = _frame(540, 960, 38, 68, seed=int(10 * tf))
    ins = {}
    outs = {}
    for who in ("oracle", "hip"):
        r, d, u, a, b = (x.clone().requires_grad_(True) for x in (ren, dep, unc, ea, eb))
        if who == "oracle":
            loss = ou.loss_mapping_uncertainty(ou.DEFAULT_CONFIG, r, d, gt, ref, a, b, opa, u, tf, sf)
        else:
            loss = mapping_loss_uncertainty(r, d, opa, gt, ref, a, b, u, tf, sf, ou.DEFAULT_CONFIG)
        loss.backward()
        ins[who] = (r, d, u, a, b)
        outs[who] = float(loss)
    torch.cuda.synchronize()
    assert abs(outs["hip"] - outs["oracle"]) <= 1e-5 * abs(outs["oracle"])
    (r0, d0, u0, a0, b0), (r1, d1, u1, a1, b1) = ins["oracle"], ins["hip"]
    assert _rel(r1.grad, r0.grad) <= 1e-4
    assert _rel(d1.grad, d0.grad) <= 1e-4
    assert _rel(u1.grad, u0.grad) <= 1e-4
    assert _rel(a1.grad, a0.grad) <= 1e-3
    assert _rel(b1.grad, b0.grad) <= 1e-3


def test_drop_in_signature_and_mlp_gradient():
    """wgsr.uncertainty.get_loss_mapping_uncertainty with the reference's
    arguments (viewpoint, network) -> (uncertainty, loss); the gradient
    reaches the network's parameters and the exposures."""
    from wgsr.uncertainty import get_loss_mapping_uncertainty
    H, W, h, w = 96, 128, 7, 9
    gt, ren, ref, dep, opa, _, ea, eb = _frame(H, W, h, w, seed=5)
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.ReLU(), torch.nn.Linear(16, 1),
                              torch.nn.Softplus()).to(DEV)
    feats = torch.randn(h, w, 8, device=DEV)
    mlp = lambda f: net(f.view(-1, 8)).view(h, w)  # noqa: E731
    a, b = ea.clone().requires_grad_(True), eb.clone().requires_grad_(True)
    vp = types.SimpleNamespace(original_image=gt, depth=ref[0].cpu().numpy(), exposure_a=a, exposure_b=b,
                               features=feats)
    r = ren.clone().requires_grad_(True)
    unc, loss = get_loss_mapping_uncertainty(ou.DEFAULT_CONFIG, r, dep, vp, opa, mlp, 0.3, 0.3)
    loss.backward()
    got = [p.grad.clone() for p in net.parameters()] + [a.grad.clone(), b.grad.clone(), r.grad.clone()]
    for p in net.parameters():
        p.grad = None
    a2, b2, r2 = a.detach().clone().requires_grad_(True), b.detach().clone().requires_grad_(True), \
        ren.clone().requires_grad_(True)
    u2 = mlp(feats)
    loss2 = ou.loss_mapping_uncertainty(ou.DEFAULT_CONFIG, r2, dep, gt, ref, a2, b2, opa, u2, 0.3, 0.3)
    loss2.backward()
    want = [p.grad for p in net.parameters()] + [a2.grad, b2.grad, r2.grad]
    assert unc.shape == (h, w)
    assert abs(float(loss) - float(loss2)) <= 1e-5 * abs(float(loss2))
    for g1, g0 in zip(got, want):
        assert _rel(g1, g0) <= 1e-3


@pytest.mark.parametrize("mode", ["map_opt_online", "final_refine", "initialize"])
def test_mapping_iteration_uncertainty_matches_torch_composition(mode):
    """MappingStep.forward_backward_uncertainty against the mapper's own call
    of each of its three call sites: map_opt_online passes the exposure-corrected
    render into the loss, which corrects it again (mapper.py:1127-1129,
    slam_utils.py:179-181); final_refine passes the raw render
    (mapper.py:1298-1306); initialize_map_opt uses initialization=True
    (mapper.py:974-984)."""
    from wgsr.camera import synthetic_camera
    from wgsr.mapping import MappingStep
    from wgsr.render import DeviceCamera, render
    from wgsr.scene import make_scene
    P, W, H, DEG, h, w = 3000, 128, 96, 3, 7, 9
    sc = make_scene(P, W, H, DEG, seed=3)
    g = torch.Generator().manual_seed(4)
    gt = torch.rand(3, H, W, generator=g).to(DEV)
    ref = (2 + 6 * torch.rand(1, H, W, generator=g)).to(DEV)
    unc0 = (torch.rand(h, w, generator=g) * 2.0 + 0.05).to(DEV)
    ea, eb = torch.tensor([0.1], device=DEV), torch.tensor([-0.03], device=DEV)
    raw = dict(xyz=sc.means3D, f_dc=sc.shs[:, :1], f_rest=sc.shs[:, 1:],
               opacity=torch.log(sc.opacities / (1 - sc.opacities)), scaling=torch.log(sc.scales),
               rotation=sc.rotations * 1.7)
    cam_p = synthetic_camera(W, H, 0)
    # reference composition
    cam = DeviceCamera.from_pinhole(cam_p, DEV)
    leaf = {k: v.to(DEV).clone().contiguous().requires_grad_(True) for k, v in raw.items()}
    a, b = ea.clone().requires_grad_(True), eb.clone().requires_grad_(True)
    u_ref = unc0.clone().requires_grad_(True)
    pkg = render(cam, leaf["xyz"], torch.sigmoid(leaf["opacity"]), torch.exp(leaf["scaling"]),
                 F.normalize(leaf["rotation"]), torch.cat((leaf["f_dc"], leaf["f_rest"]), dim=1), DEG,
                 torch.zeros(3, device=DEV))
    img = pkg["render"]
    if mode == "map_opt_online":
        img = torch.exp(a) * img + b  # mapper.py:1129
    lm = ou.loss_mapping_uncertainty(ou.DEFAULT_CONFIG, img, pkg["depth"], gt, ref, a, b, pkg["opacity"],
                                     u_ref, 0.3, 0.3, initialization=(mode == "initialize"))
    scaling = torch.exp(leaf["scaling"])
    lm = lm + 10 * torch.abs(scaling - scaling.mean(dim=1).view(-1, 1)).mean()
    lm.backward()
    # fused iteration
    ms = MappingStep(raw["xyz"].to(DEV), raw["f_dc"].to(DEV), raw["f_rest"].to(DEV), raw["opacity"].to(DEV),
                     raw["scaling"].to(DEV), raw["rotation"].to(DEV), DEG)
    f = cam_p.raster_fields()
    camd = {k: (v.to(DEV) if torch.is_tensor(v) else v) for k, v in f.items()}
    u = unc0.clone().requires_grad_(True)
    out = ms.forward_backward_uncertainty(camd, gt, ref, ea, eb, torch.zeros(3, device=DEV), u, 0.3, 0.3,
                                          config=ou.DEFAULT_CONFIG, initialization=(mode == "initialize"),
                                          pre_exposed=(mode == "map_opt_online"))
    torch.cuda.synchronize()
    assert abs(float(out["loss"]) - float(lm)) <= 1e-5 * abs(float(lm))
    assert _rel(ms.grad["xyz"], leaf["xyz"].grad) <= 1e-4
    assert _rel(ms.grad["features"][:, :1], leaf["f_dc"].grad) <= 1e-4
    assert _rel(ms.grad["features"][:, 1:], leaf["f_rest"].grad) <= 1e-4
    assert _rel(ms.grad["opacity"], leaf["opacity"].grad) <= 1e-4
    assert _rel(ms.grad["scaling"], leaf["scaling"].grad) <= 1e-4
    assert _rel(ms.grad["rotation"], leaf["rotation"].grad) <= 1e-4
    assert _rel(u.grad, u_ref.grad) <= 1e-4
    if mode == "initialize":
        assert a.grad is None and b.grad is None
    else:
        assert _rel(out["dexposure_a"], a.grad) <= 1e-3
        assert _rel(out["dexposure_b"], b.grad) <= 1e-3
    assert _rel(out["dtheta"], cam.cam_rot_delta.grad) <= 1e-3
    assert _rel(out["drho"], cam.cam_trans_delta.grad) <= 1e-3


def test_rejects_cpu_and_bad_shapes():
    from wgsr.uncertainty import mapping_loss_uncertainty
    gt, ren, ref, dep, opa, unc, ea, eb = _frame(64, 80, 5, 6, seed=1)
    with pytest.raises(RuntimeError):
        mapping_loss_uncertainty(ren.cpu(), dep.cpu(), opa.cpu(), gt.cpu(), ref.cpu(), ea.cpu(), eb.cpu(), unc.cpu(),
                                 0.3, 0.3)
    with pytest.raises(ValueError):
        mapping_loss_uncertainty(ren, dep, opa, gt, ref, ea, eb, unc[:2], 0.3, 0.3)
    with pytest.raises(NotImplementedError):
        mapping_loss_uncertainty(ren, dep, opa, gt, ref, ea, eb, unc, 0.3, 0.3, {"full_resolution": True})


def test_smallest_maps_and_initialization_mode():
    """h, w = 3 (the reflect padding's minimum), an image not a multiple of
    the feature grid, and the initialization branch (no exposure term)."""
    from wgsr.uncertainty import mapping_loss_uncertainty
    gt, ren, ref, dep, opa, unc, ea, eb = _frame(45, 61, 3, 3, seed=9)
    for init in (False, True):
        ins = {}
        for who in ("oracle", "hip"):
            r, d, u = (x.clone().requires_grad_(True) for x in (ren, dep, unc))
            if who == "oracle":
                loss = ou.loss_mapping_uncertainty(ou.DEFAULT_CONFIG, r, d, gt, ref, ea, eb, opa, u, 0.5, 0.5,
                                                   initialization=init)
            else:
                loss = mapping_loss_uncertainty(r, d, opa, gt, ref, ea, eb, u, 0.5, 0.5, ou.DEFAULT_CONFIG,
                                                initialization=init)
            loss.backward()
            ins[who] = (float(loss), r.grad, d.grad, u.grad)
        torch.cuda.synchronize()
        assert abs(ins["hip"][0] - ins["oracle"][0]) <= 1e-5 * abs(ins["oracle"][0])
        for x, y in zip(ins["hip"][1:], ins["oracle"][1:]):
            assert _rel(x, y) <= 1e-4
