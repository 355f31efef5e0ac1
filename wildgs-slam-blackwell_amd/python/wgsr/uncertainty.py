"""The uncertainty-aware mapping loss on the gfx950 path.

``get_loss_mapping_uncertainty`` is a drop-in for the reference's
src/utils/slam_utils.py:146-258 (same signature and return value), the loss
WildGS-SLAM's mapper runs by default (uncertainty_params.activate,
configs/wildgs_slam.yaml:64-77; mapper.py:1120-1138): exposure correction,
the uncertainty-weighted rgb L1 + SSIM and depth L1, and the uncertainty
loss of compute_mapping_loss_components (src/utils/dyn_uncertainty/
mapping_utils.py:206-323).  The returned loss is differentiable with respect
to the rendered image and depth, the viewpoint's exposure_a / exposure_b and
the uncertainty network's output (hence its parameters), like the
reference's.

Per call: two full-resolution kernels (csrc/uncertainty.hip), the fused SSIM
forward/backward and SSIM components (csrc/ssim.hip) and two
feature-resolution kernels, plus one ``torch.median`` of the reference depth
(pass ``median_depth`` to reuse it: it is constant per keyframe).  The
uncertainty MLP itself stays a torch module (hipBLASLt GEMMs).

``loss_forward`` / ``loss_backward`` are the same computation without
autograd (wgsr.mapping.MappingStep drives them directly).  No fallback:
without libwgsr.so, or on CPU tensors, these raise.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import torch

from . import _lib

# configs/wildgs_slam.yaml mapping section (Training, opt_params, uncertainty_params)
DEFAULTS = {"alpha": 0.5, "rgb_boundary_threshold": 0.01, "ssim_loss": True, "lambda_dssim": 0.2,
            "ssim_window_size": 7, "ssim_median_filter_size": 5, "opacity_th_for_uncer_loss": 0.9,
            "ssim_mult": 0.5, "uncer_depth_mult": 0.2}


def bias_factor(x: float, s: float) -> float:
    """compute_bias_factor (mapping_utils.py:44-57)."""
    return x / (1 + (1 - x) * (1 / s - 2))


def flatten_config(config) -> dict:
    """The reference's mapping config dict -> the flat parameter set (DEFAULTS
    for what it does not name; Training.alpha defaults to 0.95 as in
    slam_utils.py:186 when Training is given without it)."""
    c = dict(DEFAULTS)
    if config:
        if "Training" in config:
            tr = config["Training"]
            c["alpha"] = tr.get("alpha", 0.95)
            for k in ("rgb_boundary_threshold", "ssim_loss"):
                if k in tr:
                    c[k] = tr[k]
        if "lambda_dssim" in config.get("opt_params", {}):
            c["lambda_dssim"] = config["opt_params"]["lambda_dssim"]
        for k, v in config.get("uncertainty_params", {}).items():
            if k in c:
                c[k] = v
        if config.get("full_resolution", False):
            raise NotImplementedError("uncertainty mapping loss: full_resolution mapping is not supported")
    if int(c["ssim_median_filter_size"]) != 5:
        raise NotImplementedError("uncertainty mapping loss: ssim_median_filter_size must be 5")
    if int(c["ssim_window_size"]) not in (3, 5, 7, 9, 11):
        raise ValueError("uncertainty mapping loss: ssim_window_size must be one of 3, 5, 7, 9, 11")
    return c


def _blocks(n):
    return max(1, int(_lib.load().wgsr_uncer_blocks(int(n))))


@dataclass
class LossState:
    """What the backward needs from the forward."""

    prm: _lib.UncerParams
    cfg: dict
    image: torch.Tensor
    image_ab: torch.Tensor
    gt: torch.Tensor
    depth: torch.Tensor
    ref: torch.Tensor
    ea: torch.Tensor
    eb: torch.Tensor
    unc: torch.Tensor
    med: torch.Tensor
    sums: torch.Tensor           # [3]: sum w rgb-L1, sum w, sum re-weighted depth L1
    ssim_dmap: torch.Tensor | None
    d_unc: torch.Tensor          # dL/d(uncertainty) for dL/dloss = 1 (zeros when frozen)
    uncertainty_loss: torch.Tensor
    ssim_scale: torch.Tensor     # [3] the SSIM backward's dL/dS for dL/dloss = 1


def _check(t, who):
    if not t.is_cuda or t.dtype != torch.float32:
        raise RuntimeError(f"{who}: fp32 device tensors only (the HIP path has no CPU fallback)")


def loss_forward(image, depth, opacity, gt, ref_depth, exposure_a, exposure_b, uncertainty, train_frac: float,
                 ssim_frac: float, cfg: dict, initialization: bool = False, freeze_uncertainty_loss: bool = False,
                 median_depth=None, extra=None, pre_exposed: bool = False):
    """-> (loss 0-d device tensor, LossState).  image/gt [3,H,W], depth /
    ref_depth / opacity [1,H,W] (or [H,W]), uncertainty [h,w].  ``extra``:
    optional (partials [n] device tensor, weight) added to the loss as
    weight * sum(partials) in the same epilogue launch (MappingStep's
    isotropic term).  ``pre_exposed``: ``image`` is the raw render and the
    loss is the one map_opt_online computes, which passes
    ``exp(a) * image + b`` into get_loss_mapping_uncertainty (mapper.py:
    1127-1129), where the exposure is applied again (slam_utils.py:179-181);
    the returned image / exposure gradients chain through both applications.
    Ignored with ``initialization``."""
    L = _lib.load()
    H, W = gt.shape[-2], gt.shape[-1]
    if uncertainty.dim() != 2:
        raise ValueError("uncertainty mapping loss: the uncertainty map must be [h, w]")
    h, w = uncertainty.shape
    if h <= 2 or w <= 2:
        raise ValueError("uncertainty mapping loss: the uncertainty map needs h, w > 2 (reflect padding)")
    if image.shape != gt.shape or image.shape[0] != 3:
        raise ValueError("uncertainty mapping loss: image and gt must both be [3, H, W]")
    for t, n in ((depth, "depth"), (ref_depth, "ref_depth"), (opacity, "opacity")):
        if t.numel() != H * W:
            raise ValueError(f"uncertainty mapping loss: {n} must have H x W elements (full_resolution unsupported)")
    for t in (image, depth, opacity, gt, ref_depth, uncertainty):
        _check(t, "uncertainty mapping loss")
    dev = image.device
    HW, hw = H * W, h * w
    st = _lib.stream_handle(dev)
    p = _lib.ptr
    image = image.detach().contiguous()
    depth = depth.detach().contiguous()
    opacity = opacity.detach().contiguous()
    gt = gt.detach().contiguous()
    ref = ref_depth.detach().contiguous()
    z = torch.zeros(1, device=dev) if initialization else None  # (no fill launch otherwise)
    ea = z if initialization else exposure_a.detach().to(torch.float32).reshape(1).contiguous()
    eb = z if initialization else exposure_b.detach().to(torch.float32).reshape(1).contiguous()
    unc = uncertainty.detach().contiguous()
    med = (ref.median() if median_depth is None else torch.as_tensor(median_depth, device=dev)).to(
        torch.float32).reshape(1).contiguous()
    prm = _lib.UncerParams(H, W, h, w, cfg["rgb_boundary_threshold"], 1.0 + bias_factor(train_frac, 0.8),
                           100.0 + 900.0 * bias_factor(ssim_frac, 0.8), cfg["opacity_th_for_uncer_loss"],
                           cfg["uncer_depth_mult"], int(bool(initialization)),
                           int(bool(pre_exposed) and not initialization))
    image_ab = torch.empty_like(image)
    lpart = torch.empty(_blocks(HW), 3, device=dev)
    comps = [torch.empty(1, H, W, device=dev) for _ in range(3)]
    small = [torch.empty(h, w, device=dev) for _ in range(3)]
    upart = torch.empty(_blocks(hw), device=dev)
    uloss = torch.empty(h, w, device=dev)
    d_unc = torch.empty(h, w, device=dev)
    ssim_dmap = ssim_mean = None
    with torch.cuda.device(dev):
        _lib.check(L.wgsr_uncer_loss_forward(ctypes.byref(prm), p(image), p(gt), p(depth), p(ref), p(ea), p(eb),
                                             p(unc), p(med), p(image_ab), p(lpart), st))
        if cfg["ssim_loss"]:
            # (tile partials only: the epilogue launch below reduces them)
            ssim_dmap = torch.empty(3 * 3 * HW, device=dev)
            ssim_part = torch.empty(3 * int(L.wgsr_ssim_tiles(H, W)), device=dev)
            ssim_mean = torch.empty((), device=dev)
            _lib.check(L.wgsr_ssim_forward_partials(p(image_ab), p(gt), 3, H, W, 11, p(ssim_dmap), p(ssim_part), st))
        # compute_ssim_components(gt_img, rendered_img) at full resolution, then
        # the feature-resolution maps of the uncertainty loss
        _lib.check(L.wgsr_ssim_components(p(gt), p(image_ab), 1, 3, H, W, int(cfg["ssim_window_size"]),
                                          *[p(c) for c in comps], st))
        _lib.check(L.wgsr_uncer_small_maps(ctypes.byref(prm), p(opacity), p(depth), p(ref), p(med),
                                           *[p(c) for c in comps], *[p(s) for s in small], st))
        gscale = 0.0 if freeze_uncertainty_loss else cfg["ssim_mult"] / hw
        _lib.check(L.wgsr_uncer_loss_small(ctypes.byref(prm), p(unc), *[p(s) for s in small], float(gscale),
                                           p(uloss), p(upart), p(d_unc), st))
    loss = torch.empty((), device=dev)
    sums = torch.empty(3, device=dev)
    ssim_scale = torch.empty(3, device=dev)
    ex, exw = (None, 0.0) if extra is None else (extra[0].contiguous(), float(extra[1]))
    with torch.cuda.device(dev):
        if cfg["ssim_loss"]:
            _lib.check(L.wgsr_uncer_loss_combine_ssim(ctypes.byref(prm), p(lpart), p(upart), p(ssim_part),
                                                      p(ssim_mean), p(ex), 0 if ex is None else ex.numel(), exw,
                                                      float(cfg["alpha"]), float(cfg["lambda_dssim"]),
                                                      float(cfg["ssim_mult"]), p(loss), p(sums), p(ssim_scale), st))
        else:
            _lib.check(L.wgsr_uncer_loss_combine(ctypes.byref(prm), p(lpart), p(upart), p(ssim_mean), p(ex),
                                                 0 if ex is None else ex.numel(), exw, float(cfg["alpha"]),
                                                 float(cfg["lambda_dssim"]), float(cfg["ssim_mult"]),
                                                 int(bool(cfg["ssim_loss"])), p(loss), p(sums), p(ssim_scale), st))
    state = LossState(prm, cfg, image, image_ab, gt, depth, ref, ea, eb, unc, med, sums, ssim_dmap, d_unc, uloss,
                      ssim_scale)
    return loss, state


def loss_backward(s: LossState, loss_grad=None, exposure_partials: bool = False):
    """-> (dL/dimage [3,H,W], dL/ddepth [1,H,W], dL/dexposure_a [1],
    dL/dexposure_b [1], dL/duncertainty [h,w]) for dL/dloss = loss_grad
    (0-d device tensor; None = 1).  ``exposure_partials``: the exposure
    gradient as its per-block (a, b) partial sums [n, 2] in place of
    dL/dexposure_a, and None for dL/dexposure_b (no summing launch)."""
    L = _lib.load()
    dev = s.image.device
    st = _lib.stream_handle(dev)
    p = _lib.ptr
    H, W = s.prm.H, s.prm.W
    HW = H * W
    alpha, lam = s.cfg["alpha"], s.cfg["lambda_dssim"]
    lg = None if loss_grad is None else loss_grad.detach().to(torch.float32).reshape(1).contiguous()
    d_image = torch.empty_like(s.image)
    d_depth = torch.empty(1, H, W, device=dev)
    epart = torch.empty(_blocks(HW), 2, device=dev)
    ssim_grad = None
    with torch.cuda.device(dev):
        if s.cfg["ssim_loss"]:
            # dL/dS per pixel = -alpha lambda (sum w) / HW / (3 HW) (x dL/dloss)
            scale = s.ssim_scale if lg is None else (s.ssim_scale * lg[0]).contiguous()
            ssim_grad = torch.empty_like(s.image_ab)
            _lib.check(L.wgsr_ssim_backward(p(s.image_ab), p(s.gt), 3, H, W, 11, p(s.ssim_dmap), p(scale),
                                            p(ssim_grad), st))
        w_rgb = alpha * ((1.0 - lam) if s.cfg["ssim_loss"] else 1.0) / (3 * HW)
        _lib.check(L.wgsr_uncer_loss_backward(ctypes.byref(s.prm), p(s.image), p(s.image_ab), p(s.gt), p(s.depth),
                                              p(s.ref), p(s.ea), p(s.eb), p(s.unc), p(s.med), float(w_rgb),
                                              float((1.0 - alpha) / HW), p(lg), p(ssim_grad), p(d_image), p(d_depth),
                                              p(epart), st))
    d_unc = s.d_unc if lg is None else s.d_unc * lg[0]
    if exposure_partials:
        if s.prm.initialization:
            epart.zero_()
        return d_image, d_depth, epart, None, d_unc
    esum = epart.sum(0)
    if s.prm.initialization:
        esum = torch.zeros_like(esum)
    return d_image, d_depth, esum[0:1], esum[1:2], d_unc


class _UncerLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, image, depth, exposure_a, exposure_b, uncertainty, opacity, gt, ref_depth, train_frac, ssim_frac,
                cfg, initialization, freeze, median_depth):
        loss, state = loss_forward(image, depth, opacity, gt, ref_depth, exposure_a, exposure_b, uncertainty,
                                   train_frac, ssim_frac, cfg, initialization, freeze, median_depth)
        ctx.state = state
        ctx.shapes = (image.shape, depth.shape, exposure_a.shape if exposure_a is not None else None,
                      exposure_b.shape if exposure_b is not None else None)
        ctx.freeze = freeze
        return loss

    @staticmethod
    def backward(ctx, grad):
        d_image, d_depth, d_a, d_b, d_unc = loss_backward(ctx.state, grad)
        ish, dsh, ash, bsh = ctx.shapes
        init = bool(ctx.state.prm.initialization)  # no exposure term: no exposure gradient (not zeros)
        ga = d_a.view(ash) if ash is not None and ctx.needs_input_grad[2] and not init else None
        gb = d_b.view(bsh) if bsh is not None and ctx.needs_input_grad[3] and not init else None
        gu = None if ctx.freeze or not ctx.needs_input_grad[4] else d_unc
        ctx.state = None
        return (d_image.view(ish), d_depth.view(dsh), ga, gb, gu) + (None,) * 9


def mapping_loss_uncertainty(rendered_img, rendered_depth, opacity, gt_img, ref_depth, exposure_a, exposure_b,
                             uncertainty, train_frac: float, ssim_frac: float, config=None,
                             initialization: bool = False, freeze_uncertainty_loss: bool = False, median_depth=None):
    """Differentiable total loss of get_loss_mapping_uncertainty from plain
    tensors (exposure_a / exposure_b: the viewpoint's [1] parameters)."""
    cfg = flatten_config(config)
    return _UncerLoss.apply(rendered_img, rendered_depth, exposure_a, exposure_b, uncertainty, opacity, gt_img,
                            ref_depth, float(train_frac), float(ssim_frac), cfg, bool(initialization),
                            bool(freeze_uncertainty_loss), median_depth)


def get_loss_mapping_uncertainty(config, rendered_img, rendered_depth, viewpoint, opacity, uncertainty_network,
                                 train_frac: float, ssim_frac: float, initialization: bool = False,
                                 freeze_uncertainty_loss: bool = False):
    """Drop-in for src/utils/slam_utils.py:146-258: -> (uncertainty, total_loss)."""
    gt_img = viewpoint.original_image.cuda()
    dev = rendered_img.device
    ref_depth = torch.from_numpy(viewpoint.depth).to(dtype=torch.float32, device=dev)[None]
    features = viewpoint.features.to(device=dev)
    uncertainty = uncertainty_network(features)
    _, h, w = gt_img.shape
    loss = mapping_loss_uncertainty(rendered_img, rendered_depth, opacity.view(1, h, w), gt_img, ref_depth,
                                    viewpoint.exposure_a, viewpoint.exposure_b, uncertainty, train_frac, ssim_frac,
                                    config, initialization, freeze_uncertainty_loss)
    return uncertainty, loss


# ---- DINO feature-similarity regulariser (mapping_utils.py:325-389) --------
DINO_TOP_K = 128
DINO_SIMILARITY_THRESHOLD = 0.75
DINO_EPS = float(torch.finfo(torch.float32).eps)


def dino_reg_raw(u, feat, want_loss: bool = True):
    """wgsr_dino_reg (csrc/dino.hip) on u [N], feat [N, C] (device, fp32,
    contiguous): -> (loss 0-d, d loss / d u [N]), no autograd; without
    ``want_loss`` the loss launch is skipped and None returned for it."""
    L = _lib.load()
    N, C = feat.shape
    dev = feat.device
    fn = torch.empty(N, C, device=dev)
    sim = torch.empty(N, N, device=dev)
    row_var = torch.empty(N, device=dev)
    grad_u = torch.empty(N, device=dev)
    loss = torch.empty((), device=dev) if want_loss else None
    pt = _lib.ptr
    with torch.cuda.device(dev):
        _lib.check(L.wgsr_dino_reg(pt(u), pt(feat), N, C, DINO_TOP_K, DINO_SIMILARITY_THRESHOLD, DINO_EPS,
                                   pt(fn), pt(sim), pt(row_var), pt(grad_u), pt(loss), _lib.stream_handle(dev)))
    return loss, grad_u


class _DinoReg(torch.autograd.Function):
    """wgsr_dino_reg (csrc/dino.hip): the whole regulariser in four launches;
    d loss / d u is produced by the forward and scaled in the backward."""

    @staticmethod
    def forward(ctx, u, feat):
        loss, grad_u = dino_reg_raw(u, feat)
        ctx.save_for_backward(grad_u)
        return loss

    @staticmethod
    def backward(ctx, g):
        (grad_u,) = ctx.saved_tensors
        return grad_u * g, None


def dino_regularization_loss(uncertainty, features):
    """compute_dino_regularization_loss (mapping_utils.py:332-389): the mean
    over samples of the variance of the uncertainty over each sample's (up
    to) 128 most similar features with cosine similarity > 0.75 (NeRF-on-the-
    Go eqs. 2-3).  ``uncertainty`` [.., 1] or a list of tensors, ``features``
    [.., C] (or a list) with the same sample count; differentiable in the
    uncertainty.  Device tensors run the HIP kernels (csrc/dino.hip; fails
    loudly without the library); CPU tensors run the torch restatement with
    the reference's own arithmetic (the CPU parity tests' path)."""
    unc = torch.stack(uncertainty) if isinstance(uncertainty, (list, tuple)) else uncertainty
    feat = torch.stack(features) if isinstance(features, (list, tuple)) else features
    C = feat.shape[-1]
    u = unc.reshape(-1, 1)
    if u.shape[0] != feat.numel() // C:
        raise ValueError("Uncertainty and feature buffers must have same number of samples"
                         + f"but got {u.shape[0]} and {feat.numel() // C}")
    if feat.is_cuda:
        if feat.dtype != torch.float32 or unc.dtype != torch.float32:
            raise RuntimeError("dino_regularization_loss: fp32 device tensors only (the HIP path has no fallback)")
        return _DinoReg.apply(u.reshape(-1).contiguous(), feat.detach().contiguous().view(-1, C))
    fn = torch.nn.functional.normalize(feat.contiguous().view(-1, C), p=2, dim=-1)
    sim = fn @ fn.T
    k = min(DINO_TOP_K, sim.shape[-1])
    top, idx = torch.topk(sim, k=k, dim=-1)
    mask = (top > DINO_SIMILARITY_THRESHOLD).float()
    nb = u[idx] * mask.unsqueeze(-1)
    cnt = mask.sum(dim=-1, keepdim=True) + DINO_EPS
    mean = nb.sum(dim=1) / cnt
    var = (((nb - mean.unsqueeze(-1)) ** 2) * mask.unsqueeze(-1)).sum(dim=1) / cnt
    return var.mean()
