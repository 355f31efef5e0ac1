#!/usr/bin/env python
"""Host cost of the drop-in _C wrapper calls at TUM scale (100k Gaussians,
512x384, SH0): per-call host time of rasterize_gaussians_backward (its
kernels are queued asynchronously, so this is pure host time) and wall time
of rasterize_gaussians (which waits once for the pair counts), next to the
GPU time of a whole step."""
import json
import os
import sys
import time

import torch

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (os.path.join(_ROOT, "wildgs-slam-blackwell_amd", "python"), _ROOT):
    if _p not in sys.path:
        sys.path.insert(0, _p)

from diff_gaussian_rasterization import _C  # noqa: E402
from wgsr.camera import synthetic_camera
from wgsr.scene import make_scene, make_upstream_grads


def main(P=100_000, W=512, H=384, deg=0, iters=200):
    dev = torch.device("cuda:0")
    sc = make_scene(P, W, H, deg, seed=0)
    gc, gd = (t.to(dev) for t in make_upstream_grads(W, H, seed=1))
    f = synthetic_camera(W, H, 0).raster_fields()
    d = lambda x: x.to(dev).contiguous()  # noqa: E731
    means, opac, scales, rots, shs = d(sc.means3D), d(sc.opacities), d(sc.scales), d(sc.rotations), d(sc.shs)
    bg = torch.zeros(3, device=dev)
    view, proj, praw, campos = d(f["viewmatrix"]), d(f["projmatrix"]), d(f["projmatrix_raw"]), d(f["campos"])
    e = torch.empty(0, device=dev)
    tf, tb, tstep = [], [], []

    def step(rec):
        t0 = time.perf_counter()
        nr, color, radii, geom, binning, img, depth, opacity, nt = _C.rasterize_gaussians(
            bg, means, e, opac, scales, rots, 1.0, e, view, proj, praw, f["tanfovx"], f["tanfovy"], H, W, shs, deg,
            campos, False, False)
        t1 = time.perf_counter()
        _C.rasterize_gaussians_backward(bg, means, radii, e, scales, rots, 1.0, e, view, proj, praw, f["tanfovx"],
                                        f["tanfovy"], gc, gd, shs, deg, campos, geom, nr, binning, img, False)
        t2 = time.perf_counter()
        if rec:
            tf.append(t1 - t0)
            tb.append(t2 - t1)

    for _ in range(20):
        step(False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        step(True)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / iters
    med = lambda v: sorted(v)[len(v) // 2] * 1e6  # noqa: E731
    print(json.dumps({"P": P, "W": W, "H": H, "sh": deg, "step_wall_us": wall * 1e6,
                      "forward_call_us_median": med(tf), "backward_call_us_median": med(tb)}))


if __name__ == "__main__":
    main()
