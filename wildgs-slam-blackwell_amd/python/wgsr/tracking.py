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


class PoseRefine:
    """The mapper's keyframe pose refinement (src/mapper.py:856-911) on device.

    Per iteration, as the reference: render the keyframe, get_loss_tracking,
    backward, Adam over (cam_rot_delta, cam_trans_delta, exposure_a,
    exposure_b) with their learning rates (config["mapping"]["Training"]["lr"],
    0.01 for the exposures), update_pose (SE3_exp([trans, rot]) @ w2c, deltas
    reset), stop when |tau| < converged_threshold.  The Adam step, the SE(3)
    update and the next iteration's camera matrices are ONE launch
    (``wgsr_pose_step``) instead of ~60 small torch kernels; the Gaussians are
    activated once (they do not change during the refinement).

    Deviation: the reference's backward also accumulates the Gaussians'
    parameter gradients into their ``.grad`` during the refinement (a side
    effect its mapping loop then adds to the first mapping step); here they
    are computed by the rasteriser but not kept.
    """

    def __init__(self, means3D, opacities, scales, rotations, shs, sh_degree: int, bg, projection_matrix, H: int,
                 W: int, FoVx: float, FoVy: float, lr_rot: float = 0.003, lr_trans: float = 0.001,
                 lr_exposure: float = 0.01, betas=(0.9, 0.999), eps: float = 1e-8, rgb_threshold: float = 0.01):
        import math
        for t in (means3D, opacities, scales, rotations, shs):
            _check(t, "PoseRefine")
        self.means, self.opac = means3D.detach().contiguous(), opacities.detach().contiguous()
        self.scales, self.rots = scales.detach().contiguous(), rotations.detach().contiguous()
        self.shs, self.deg = shs.detach().contiguous(), int(sh_degree)
        self.bg = bg.detach().to(torch.float32).contiguous()
        self.praw = projection_matrix.detach().to(torch.float32).contiguous()
        self.H, self.W = int(H), int(W)
        self.tanx, self.tany = math.tan(FoVx * 0.5), math.tan(FoVy * 0.5)
        self.lr = (float(lr_rot), float(lr_trans), float(lr_exposure))
        self.betas, self.eps, self.rgb_threshold = betas, float(eps), float(rgb_threshold)
        dev = self.means.device
        L = _lib.load()
        self.state = torch.zeros(int(L.wgsr_pose_state_floats()), device=dev)
        self.conv = torch.zeros(1, dtype=torch.int32, device=dev)
        self.zero_depth = torch.zeros(1, self.H, self.W, device=dev)
        self.part = torch.empty(max(1, int(L.wgsr_track_blocks(self.H * self.W))), 3, device=dev)
        self.d_img = torch.empty(3, self.H, self.W, device=dev)

    def refine(self, R, T, exposure_a, exposure_b, gt_image, grad_mask, uncertainty=None, iters: int = 100,
               converged_threshold: float = 1e-4):
        """-> (R [3,3], T [3], exposure_a [1], exposure_b [1], iterations run)."""
        from diff_gaussian_rasterization import _C
        L = _lib.load()
        dev = self.means.device
        st = self.state
        st.zero_()
        st[0:9] = R.detach().to(device=dev, dtype=torch.float32).reshape(9)
        st[9:12] = T.detach().to(device=dev, dtype=torch.float32).reshape(3)
        st[12:13] = exposure_a.detach().to(device=dev, dtype=torch.float32).reshape(1)
        st[13:14] = exposure_b.detach().to(device=dev, dtype=torch.float32).reshape(1)
        gt = gt_image.detach().contiguous()
        gm = None if grad_mask is None else grad_mask.detach().to(torch.float32).contiguous()
        un = None if uncertainty is None else uncertainty.detach().to(torch.float32).contiguous()
        p = _lib.ptr
        s = _lib.stream_handle(dev)
        b1, b2 = self.betas
        e = torch.empty(0, device=dev)
        view, proj, campos = st[32:48].view(4, 4), st[48:64].view(4, 4), st[64:67]
        with torch.cuda.device(dev):
            _lib.check(L.wgsr_pose_step(p(st), None, None, 0, p(self.praw), 0.0, 0.0, 0.0, b1, b2, self.eps, 0,
                                        0.0, None, 1, s))
        it = 0
        for it in range(1, iters + 1):
            fwd = _C.rasterize_gaussians(self.bg, self.means, e, self.opac, self.scales, self.rots, 1.0, e, view,
                                         proj, self.praw, self.tanx, self.tany, self.H, self.W, self.shs, self.deg,
                                         campos, False, False)
            nr, image, radii, geom, binning, img, _, opac_img, _ = fwd
            with torch.cuda.device(dev):
                _lib.check(L.wgsr_tracking_loss(self.H, self.W, p(image), p(gt), p(opac_img), p(gm), p(un),
                                                p(st[12:13]), p(st[13:14]), self.rgb_threshold, p(self.d_img), None,
                                                p(self.part), s))
            g = _C.rasterize_gaussians_backward(self.bg, self.means, radii, e, self.scales, self.rots, 1.0, e, view,
                                                proj, self.praw, self.tanx, self.tany, self.d_img, self.zero_depth,
                                                self.shs, self.deg, campos, geom, nr, binning, img, False)
            dtau = g[8].sum(0)
            with torch.cuda.device(dev):
                _lib.check(L.wgsr_pose_step(p(st), p(dtau), p(self.part), self.part.shape[0], p(self.praw),
                                            self.lr[0], self.lr[1], self.lr[2], b1, b2, self.eps, it,
                                            float(converged_threshold), p(self.conv), 0, s))
            if int(self.conv.item()):
                break
        return (st[0:9].view(3, 3).clone(), st[9:12].clone(), st[12:13].clone(), st[13:14].clone(), it)
