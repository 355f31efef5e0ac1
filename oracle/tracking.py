"""ORACLE (test infrastructure only) - the mapper's pose-refinement loss of
SURVEY.md 8(f) row f2 (tracking half).  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this module, and only as the checker; the product path (``wgsr.tracking``
over libwgsr.so) never imports it.

Torch restatements (CPU or GPU, fp32, autograd):

* ``loss_tracking`` -- get_loss_tracking / get_loss_tracking_rgb
  (src/utils/slam_utils.py:47-82).  Pinned: tests/golden/make_track_fixtures.py
  runs the reference's own get_loss_tracking on CPU (stand-in viewpoint whose
  ``original_image.cuda()`` returns the CPU tensor) and commits inputs, loss
  and gradients in tests/golden/track_cases.npz.
* ``compute_grad_mask`` -- Camera.compute_grad_mask (src/utils/camera_utils.py:
  157-180) with slam_utils.image_gradient / image_gradient_mask (:10-44).
  The reference builds its Scharr kernels with ``device="cuda"`` and cannot
  run in the CPU-only build container, so this restatement is NOT pinned by a
  reference run ("parity unpinned" for the grad mask): it follows the cited
  lines literally, including the two sequential masked assignments.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def image_gradient(image):
    """slam_utils.image_gradient (:10-27): Scharr, reflect padding, / 32."""
    c = image.shape[0]
    conv_y = torch.tensor([[3, 0, -3], [10, 0, -10], [3, 0, -3]], dtype=torch.float32, device=image.device)
    conv_x = torch.tensor([[3, 10, 3], [0, 0, 0], [-3, -10, -3]], dtype=torch.float32, device=image.device)
    normalizer = 1.0 / torch.abs(conv_y).sum()
    p_img = F.pad(image, (1, 1, 1, 1), mode="reflect")[None]
    img_grad_v = normalizer * F.conv2d(p_img, conv_x.view(1, 1, 3, 3).repeat(c, 1, 1, 1), groups=c)
    img_grad_h = normalizer * F.conv2d(p_img, conv_y.view(1, 1, 3, 3).repeat(c, 1, 1, 1), groups=c)
    return img_grad_v[0], img_grad_h[0]


def image_gradient_mask(image, eps=0.01):
    """slam_utils.image_gradient_mask (:30-44)."""
    c = image.shape[0]
    conv = torch.ones((1, 1, 3, 3), dtype=torch.float32, device=image.device)
    p_img = F.pad(image, (1, 1, 1, 1), mode="reflect")[None]
    p_img = torch.abs(p_img) > eps
    g = F.conv2d(p_img.float(), conv.repeat(c, 1, 1, 1), groups=c)
    return g[0] == torch.sum(conv), g[0] == torch.sum(conv)


def compute_grad_mask(original_image, edge_threshold=4):
    """Camera.compute_grad_mask (camera_utils.py:157-180) -> [1, H, W]."""
    gray = original_image.mean(dim=0, keepdim=True)
    gv, gh = image_gradient(gray)
    mv, mh = image_gradient_mask(gray)
    gv, gh = gv * mv, gh * mh
    inten = torch.sqrt(gv ** 2 + gh ** 2)
    _, h, w = original_image.shape
    for r in range(32):
        for c in range(32):
            block = inten[:, r * int(h / 32):(r + 1) * int(h / 32), c * int(w / 32):(c + 1) * int(w / 32)]
            th = block.median()
            block[block > (th * edge_threshold)] = 1
            block[block <= (th * edge_threshold)] = 0
    return inten


def loss_tracking(image, opacity, gt_image, exposure_a, exposure_b, grad_mask, uncertainty=None,
                  rgb_boundary_threshold=0.01):
    """get_loss_tracking (monocular) -> get_loss_tracking_rgb (slam_utils.py:47-82)."""
    image_ab = torch.exp(exposure_a) * image + exposure_b
    _, h, w = gt_image.shape
    m = (gt_image.sum(dim=0) > rgb_boundary_threshold).view(1, h, w)
    m = m * grad_mask
    l1 = opacity * torch.abs(image_ab * m - gt_image * m)
    if uncertainty is not None:
        weights = 0.5 / (uncertainty.unsqueeze(0)) ** 2
        weights = torch.where(weights < 0.1, 0.0, weights)
        l1 *= weights
    return l1.mean()
