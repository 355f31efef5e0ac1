"""The mapper's pose-refinement loss on the gfx950 path (SURVEY.md 8(f) row f2,
tracking half).

WildGS-SLAM refines a keyframe's pose with 100 iterations of render ->
``get_loss_tracking`` -> backward -> Adam over (cam_rot_delta,
cam_trans_delta, exposure_a, exposure_b) (src/mapper.py:856-911); the loss
needs the keyframe's ``Camera.grad_mask`` (camera_utils.py:157-180).

* ``get_loss_tracking(config, image, depth, opacity, viewpoint, monocular=True,
  uncertainty=None)`` -- drop-in for src/utils/slam_utils.py:47-82: one HIP
  pass computes the loss and every gradient (the weights of this L1 do not
  depend on the parameters); the autograd backward only rescales them.  The
  opacity gradient is returned like the reference's (the rasteriser drops
  it: upstream ignores dL/dopacity-image).
* ``compute_grad_mask(original_image, edge_threshold)`` -- Camera.
  compute_grad_mask's mask (two launches instead of ~3000).

No fallback: without libwgsr.so, or on CPU tensors, these raise.
"""
from __future__ import annotations

import torch

from . import _lib


def _check(t, who):
    if not t.is_cuda or t.dtype != torch.float32:
        raise RuntimeError(f"{who}: fp32 device tensors only (the HIP path has no CPU fallback)")


def compute_grad_mask(original_image: torch.Tensor, edge_threshold: float = 4.0) -> torch.Tensor:
    """[3, H, W] image -> grad_mask [1, H, W] (Camera.compute_grad_mask)."""
    _check(original_image, "compute_grad_mask")
    if original_image.dim() != 3 or original_image.shape[0] != 3:
        raise ValueError("compute_grad_mask: expected a [3, H, W] image")
    img = original_image.contiguous()
    H, W = img.shape[1], img.shape[2]
    out = torch.empty(1, H, W, device=img.device)
    L = _lib.load()
    with torch.cuda.device(img.device):
        _lib.check(L.wgsr_grad_mask(H, W, img.data_ptr(), float(edge_threshold), out.data_ptr(),
                                    _lib.stream_handle(img.device)))
    return out


class _TrackLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, image, opacity, exposure_a, exposure_b, gt, grad_mask, uncertainty, rgb_threshold):
        for t in (image, opacity, gt):
            _check(t, "get_loss_tracking")
        H, W = gt.shape[-2], gt.shape[-1]
        HW = H * W
        if image.shape != gt.shape or image.shape[0] != 3 or opacity.numel() != HW:
            raise ValueError("get_loss_tracking: image / gt must be [3, H, W] and opacity [1, H, W]")
        dev = image.device
        img = image.detach().contiguous()
        op = opacity.detach().contiguous()
        gtc = gt.detach().contiguous()
        gm = None if grad_mask is None else grad_mask.detach().to(torch.float32).contiguous()
        un = None if uncertainty is None else uncertainty.detach().to(torch.float32).contiguous()
        for t, n in ((gm, "grad_mask"), (un, "uncertainty")):
            if t is not None and t.numel() != HW:
                raise ValueError(f"get_loss_tracking: {n} must have H x W elements")
        ea = exposure_a.detach().to(torch.float32).reshape(1).contiguous()
        eb = exposure_b.detach().to(torch.float32).reshape(1).contiguous()
        L = _lib.load()
        nb = max(1, int(L.wgsr_track_blocks(HW)))
        part = torch.empty(nb, 3, device=dev)
        d_img = torch.empty_like(img)
        d_op = torch.empty_like(op)
        p = _lib.ptr
        with torch.cuda.device(dev):
            _lib.check(L.wgsr_tracking_loss(H, W, p(img), p(gtc), p(op), p(gm), p(un), p(ea), p(eb),
                                            float(rgb_threshold), p(d_img), p(d_op), p(part),
                                            _lib.stream_handle(dev)))
        sums = part.sum(0)
        ctx.save_for_backward(d_img, d_op, sums)
        ctx.shapes = (image.shape, opacity.shape, exposure_a.shape, exposure_b.shape)
        return sums[0] / (3 * HW)

    @staticmethod
    def backward(ctx, grad):
        d_img, d_op, sums = ctx.saved_tensors
        ish, osh, ash, bsh = ctx.shapes
        g = grad.detach()
        return ((d_img * g).view(ish), (d_op * g).view(osh), (sums[1:2] * g).view(ash), (sums[2:3] * g).view(bsh),
                None, None, None, None)


def tracking_loss(image, opacity, gt_image, exposure_a, exposure_b, grad_mask=None, uncertainty=None,
                  rgb_threshold: float = 0.01):
    """get_loss_tracking_rgb on the exposure-corrected image, from plain tensors."""
    return _TrackLoss.apply(image, opacity, exposure_a, exposure_b, gt_image, grad_mask, uncertainty,
                            float(rgb_threshold))


def get_loss_tracking(config, image, depth, opacity, viewpoint, monocular: bool = True, uncertainty=None):
    """Drop-in for src/utils/slam_utils.py:47-54 (-> get_loss_tracking_rgb)."""
    if not monocular:
        raise NotImplementedError("Only implemented monocular, not rgbd for uncertainty-aware tracking")
    gt = viewpoint.original_image.cuda()
    return tracking_loss(image, opacity, gt, viewpoint.exposure_a, viewpoint.exposure_b, viewpoint.grad_mask,
                         uncertainty, config["Training"]["rgb_boundary_threshold"])
