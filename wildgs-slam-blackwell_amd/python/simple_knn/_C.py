"""``simple_knn._C`` on MI355X: ``distCUDA2(points[P,3] float32) -> [P]``, the
mean squared distance to the 3 nearest other points,
computed by libwgsr.so's gfx950 kernels (include/wgsr.h wgsr_dist_cuda2)."""
from __future__ import annotations

import torch

from wgsr import _lib


def distCUDA2(points: torch.Tensor) -> torch.Tensor:
    if points.ndimension() != 2 or points.size(1) != 3:
        raise RuntimeError("points must have dimensions (num_points, 3)")
    L = _lib.load()
    dev = points.device
    if dev.type != "cuda":
        raise RuntimeError(f"points: expected a HIP device tensor, got {dev}")
    P = points.size(0)
    pts = points.contiguous().float()
    out = torch.empty(P, dtype=torch.float32, device=dev)
    if P == 0:
        return out
    with torch.cuda.device(dev), _lib.AllocRequest(dev):
        code = L.wgsr_dist_cuda2(P, pts.data_ptr(), out.data_ptr(), _lib.ALLOC_SCRATCH, None,
                                 _lib.stream_handle(dev))
    _lib.check(code)
    return out
