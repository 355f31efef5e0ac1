"""SSIM for the mapping loss on the gfx950 path.

``ssim(img1, img2, window_size=11, size_average=True)`` is a drop-in for
loss_utils.ssim (thirdparty/gaussian_splatting/utils/loss_utils.py:61-101),
the ``1 - ssim(rendered, gt)`` term of get_loss_mapping /
get_loss_mapping_uncertainty (src/utils/slam_utils.py:130, 200): one HIP
launch forward (``wgsr_ssim_forward``) and one backward
(``wgsr_ssim_backward``) instead of 5 depthwise conv2d and ~15 elementwise
kernels each way.  The gradient flows to ``img1`` (the rendered image, as in
every reference call); asking for a gradient of ``img2`` raises.

``ssim_components(img1, img2, window_size=7)`` is
mapping_utils.compute_ssim_components (src/utils/dyn_uncertainty/
mapping_utils.py:99-204): the channel-mean luminance / contrast / structure
maps of the uncertainty loss, forward only (the reference detaches them,
:294), one launch.

No fallback: without libwgsr.so (or on CPU tensors) these raise.
"""
from __future__ import annotations

import torch

from . import _lib

_WINDOWS = (3, 5, 7, 9, 11)


def _planes(img: torch.Tensor):
    if img.dim() < 3:
        raise ValueError("ssim: expected [C, H, W] or [N, C, H, W] images")
    H, W = img.shape[-2], img.shape[-1]
    return img.numel() // (H * W), H, W


def _check(img1: torch.Tensor, img2: torch.Tensor, window_size: int, who: str):
    if img1.shape != img2.shape:
        raise ValueError(f"{who}: image shapes differ ({tuple(img1.shape)} vs {tuple(img2.shape)})")
    if window_size not in _WINDOWS:
        raise ValueError(f"{who}: window_size must be one of {_WINDOWS}")
    for t in (img1, img2):
        if not t.is_cuda or t.dtype != torch.float32:
            raise RuntimeError(f"{who}: fp32 device tensors only (the HIP path has no CPU fallback)")


class _SSIM(torch.autograd.Function):
    @staticmethod
    def forward(ctx, img1, img2, window_size, size_average):
        img1c, img2c = img1.detach().contiguous(), img2.detach().contiguous()
        planes, H, W = _planes(img1c)
        dev = img1c.device
        need_grad = ctx.needs_input_grad[0]
        dmap = torch.empty(3 * planes * H * W, device=dev) if need_grad else None
        plane_mean = torch.empty(planes, device=dev)
        mean = torch.empty((), device=dev)
        L = _lib.load()
        with torch.cuda.device(dev), _lib.AllocRequest(dev):
            _lib.check(L.wgsr_ssim_forward(img1c.data_ptr(), img2c.data_ptr(), planes, H, W, window_size,
                                           dmap.data_ptr() if dmap is not None else None, plane_mean.data_ptr(),
                                           mean.data_ptr(), _lib.ALLOC_SCRATCH, None, _lib.stream_handle(dev)))
        ctx.window_size, ctx.size_average, ctx.shape = window_size, size_average, img1.shape
        if need_grad:
            ctx.save_for_backward(img1c, img2c, dmap)
        if size_average:
            return mean
        N, C = img1.shape[0], planes // img1.shape[0]
        return plane_mean.view(N, C).mean(1)

    @staticmethod
    def backward(ctx, grad):
        img1c, img2c, dmap = ctx.saved_tensors
        planes, H, W = _planes(img1c)
        dev = img1c.device
        grad = grad.detach().to(torch.float32)
        if ctx.size_average:
            scale = (grad / float(planes * H * W)).reshape(1).expand(planes).contiguous()
        else:
            N = ctx.shape[0]
            C = planes // N
            scale = (grad / float(C * H * W)).reshape(N, 1).expand(N, C).reshape(-1).contiguous()
        out = torch.empty_like(img1c)
        L = _lib.load()
        with torch.cuda.device(dev):
            _lib.check(L.wgsr_ssim_backward(img1c.data_ptr(), img2c.data_ptr(), planes, H, W, ctx.window_size,
                                            dmap.data_ptr(), scale.data_ptr(), out.data_ptr(),
                                            _lib.stream_handle(dev)))
        return out.view(ctx.shape), None, None, None


def ssim(img1: torch.Tensor, img2: torch.Tensor, window_size: int = 11, size_average: bool = True) -> torch.Tensor:
    """loss_utils.ssim: mean SSIM (size_average) or per-image mean of a 4-D batch."""
    _check(img1, img2, window_size, "ssim")
    if not size_average and img1.dim() != 4:
        # the reference's ssim_map.mean(1).mean(1).mean(1) needs a batch dim
        raise IndexError("ssim: size_average=False needs [N, C, H, W] images")
    if img2.requires_grad and torch.is_grad_enabled():
        raise NotImplementedError("ssim: no gradient w.r.t. img2 (the reference passes the ground truth there)")
    return _SSIM.apply(img1, img2, window_size, size_average)


@torch.no_grad()
def ssim_components(img1: torch.Tensor, img2: torch.Tensor, window_size: int = 7):
    """mapping_utils.compute_ssim_components: (luminance, contrast, structure),
    each the channel mean; [H, W] for a [C, H, W] image, [N, H, W] for a batch."""
    _check(img1, img2, window_size, "ssim_components")
    if img1.dim() == 3:
        images, C = 1, img1.shape[0]
    elif img1.dim() == 4:
        images, C = img1.shape[0], img1.shape[1]
    else:
        raise ValueError("ssim_components: expected [C, H, W] or [N, C, H, W] images")
    H, W = img1.shape[-2], img1.shape[-1]
    a, b = img1.contiguous(), img2.contiguous()
    dev = a.device
    outs = [torch.empty(images, H, W, device=dev) for _ in range(3)]
    L = _lib.load()
    with torch.cuda.device(dev):
        _lib.check(L.wgsr_ssim_components(a.data_ptr(), b.data_ptr(), images, C, H, W, window_size,
                                          *[o.data_ptr() for o in outs], _lib.stream_handle(dev)))
    if img1.dim() == 3:
        return tuple(o.squeeze() for o in outs)  # the reference's .mean(1).squeeze()
    return tuple(outs)
