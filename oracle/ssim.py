"""ORACLE (test infrastructure only) - SSIM restatements for SURVEY.md 8(f)
row f2.  Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this module, and only as the checker; the
product path (``wgsr.loss`` over libwgsr.so) never imports it.

* ``ssim_map_f64`` / ``ssim_f64``: loss_utils.ssim / _ssim
  (thirdparty/gaussian_splatting/utils/loss_utils.py:40-101) in float64
  numpy (zero-padded 'same' correlation with the fp32 window the reference
  builds).
* ``ssim_components_f64``: compute_ssim_components / _ssim
  (src/utils/dyn_uncertainty/mapping_utils.py:60-204) in float64 numpy.
* ``ssim_torch``: the same formula as loss_utils.ssim in torch fp32 with
  F.conv2d, the floating-point reference the HIP gradient is checked
  against (autograd).

Pinning (tests/golden/make_ssim_fixtures.py, run where /root/reference
exists): the window and ``compute_ssim_components`` are the reference's own
importable functions (mapping_utils.py imports without cv2); their outputs
are committed in tests/golden/ssim_cases.npz.  loss_utils.py itself imports
cv2, which this image lacks, so the standard SSIM is pinned through an
identity of the reference's components: on single-channel inputs where no
clip or epsilon is active, luminance * contrast * structure equals the
standard SSIM map exactly (C3 = C2 / 2), and the fixture checks those
conditions hold.
"""
from __future__ import annotations

import math

import numpy as np

C1 = 0.01 ** 2
C2 = 0.03 ** 2
C3 = C2 / 2
EPS32 = float(np.finfo(np.float32).eps)
CLIP = 0.98


def window_1d(ws: int, sigma: float = 1.5) -> np.ndarray:
    """loss_utils.gaussian (:40-47): exp in double, fp32 tensor, divided by its
    fp32 sum (torch's sum of <= 11 floats rounds like the exact sum: checked
    against the reference's windows for every size in tests)."""
    g = np.array([math.exp(-((x - ws // 2) ** 2) / float(2 * sigma ** 2)) for x in range(ws)], np.float32)
    total = np.float32(sum(float(v) for v in g))
    return (g / total).astype(np.float32)


def window_2d(ws: int) -> np.ndarray:
    """create_window (:50-58): outer product in fp32."""
    g = window_1d(ws)
    return (g[:, None] * g[None, :]).astype(np.float32)


def conv_same(plane: np.ndarray, w2d: np.ndarray) -> np.ndarray:
    """F.conv2d(x, w, padding=ws//2) on one [H, W] plane, float64."""
    ws = w2d.shape[0]
    r = ws // 2
    H, W = plane.shape
    p = np.zeros((H + 2 * r, W + 2 * r), np.float64)
    p[r:r + H, r:r + W] = plane
    out = np.zeros((H, W), np.float64)
    for i in range(ws):
        for j in range(ws):
            out += float(w2d[i, j]) * p[i:i + H, j:j + W]
    return out


def _stats(x: np.ndarray, y: np.ndarray, ws: int):
    w = window_2d(ws)
    x = x.astype(np.float64)
    y = y.astype(np.float64)
    mu1, mu2 = conv_same(x, w), conv_same(y, w)
    s11 = conv_same(x * x, w) - mu1 * mu1
    s22 = conv_same(y * y, w) - mu2 * mu2
    s12 = conv_same(x * y, w) - mu1 * mu2
    return mu1, mu2, s11, s22, s12


def ssim_map_f64(img1: np.ndarray, img2: np.ndarray, ws: int = 11) -> np.ndarray:
    """ssim_map of loss_utils._ssim (:72-96) for [..., H, W] planes."""
    lead = img1.shape[:-2]
    a = img1.reshape(-1, *img1.shape[-2:])
    b = img2.reshape(-1, *img2.shape[-2:])
    out = np.empty(a.shape, np.float64)
    for p in range(a.shape[0]):
        mu1, mu2, s11, s22, s12 = _stats(a[p], b[p], ws)
        out[p] = ((2 * mu1 * mu2 + C1) * (2 * s12 + C2)) / ((mu1 ** 2 + mu2 ** 2 + C1) * (s11 + s22 + C2))
    return out.reshape(*lead, *img1.shape[-2:])


def ssim_f64(img1: np.ndarray, img2: np.ndarray, ws: int = 11) -> float:
    """loss_utils.ssim(img1, img2, ws) with size_average=True (:61-99)."""
    return float(ssim_map_f64(img1, img2, ws).mean())


def ssim_components_f64(img1: np.ndarray, img2: np.ndarray, ws: int = 7):
    """mapping_utils.compute_ssim_components (:99-204) for one [C, H, W]
    image: the channel means of luminance, contrast, structure ([H, W])."""
    L, Cn, S = [], [], []
    for c in range(img1.shape[0]):
        mu1, mu2, s11, s22, s12 = _stats(img1[c], img2[c], ws)
        s11 = np.maximum(EPS32, s11)
        s22 = np.maximum(EPS32, s22)
        s12 = np.sign(s12) * np.minimum(np.sqrt(s11 * s22), np.abs(s12))
        L.append((2 * mu1 * mu2 + C1) / (mu1 ** 2 + mu2 ** 2 + C1))
        Cn.append(np.minimum((2 * np.sqrt(s11) * np.sqrt(s22) + C2) / (s11 + s22 + C2), CLIP))
        S.append(np.minimum((s12 + C3) / (np.sqrt(s11) * np.sqrt(s22) + C3), CLIP))
    return np.mean(L, 0), np.mean(Cn, 0), np.mean(S, 0)


def well_conditioned(img1: np.ndarray, img2: np.ndarray, ws: int, min_var: float = 1e-3) -> np.ndarray:
    """[..., H, W] mask of pixels whose window variances (both images, every
    channel) exceed ``min_var``.  Elsewhere E[x^2] - E[x]^2 cancels in fp32 and
    the reference's own fp32 result carries errors of order ulp(E[x^2]) /
    variance, so parity there is checked with a looser bound."""
    a = img1.reshape(-1, *img1.shape[-2:])
    b = img2.reshape(-1, *img2.shape[-2:])
    ok = np.ones(a.shape[-2:], bool)
    for p in range(a.shape[0]):
        _, _, s11, s22, _ = _stats(a[p], b[p], ws)
        ok &= (s11 > min_var) & (s22 > min_var)
    return ok


def ssim_torch(img1, img2, ws: int = 11, size_average: bool = True):
    """loss_utils.ssim restated in torch fp32 (F.conv2d, groups=channels)."""
    import torch
    import torch.nn.functional as F

    channel = img1.size(-3)
    w = torch.from_numpy(window_2d(ws)).to(img1.device)
    w = w.expand(channel, 1, ws, ws).contiguous().type_as(img1)
    mu1 = F.conv2d(img1, w, padding=ws // 2, groups=channel)
    mu2 = F.conv2d(img2, w, padding=ws // 2, groups=channel)
    mu1_sq, mu2_sq, mu1_mu2 = mu1.pow(2), mu2.pow(2), mu1 * mu2
    s11 = F.conv2d(img1 * img1, w, padding=ws // 2, groups=channel) - mu1_sq
    s22 = F.conv2d(img2 * img2, w, padding=ws // 2, groups=channel) - mu2_sq
    s12 = F.conv2d(img1 * img2, w, padding=ws // 2, groups=channel) - mu1_mu2
    m = ((2 * mu1_mu2 + C1) * (2 * s12 + C2)) / ((mu1_sq + mu2_sq + C1) * (s11 + s22 + C2))
    return m.mean() if size_average else m.mean(1).mean(1).mean(1)
