#!/usr/bin/env python
"""Owner-kernel cost of the view-sharded backward at N ranks, on one GPU.

Renders N views of the configs[2] scene (1M Gaussians, 1080p, SH3), builds
each view's records, and times wgsr_gauss_backward_views over ONE rank's
shard (P/N Gaussians x N views: what every rank runs per step at N GPUs)
against the single-view per-Gaussian backward over all P (what the
all-reduce exchange runs per rank).  HIP events on the launch stream.
"""
import json
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
for p in (os.path.join(ROOT, "wildgs-slam-blackwell_amd", "python"), ROOT):
    sys.path.insert(0, p)

import torch  # noqa: E402


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--views", type=int, default=8)
    ap.add_argument("--P", type=int, default=1_000_000)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from diff_gaussian_rasterization import _C
    from wgsr import _lib
    from wgsr.camera import synthetic_camera
    from wgsr.dp import GradBuffer, _HipViewKernels
    from wgsr.scene import make_scene, make_upstream_grads
    dev = torch.device("cuda:0")
    W, H, deg, P, V = 1920, 1080, 3, a.P, a.views
    M = (deg + 1) ** 2
    sc = make_scene(P, W, H, deg, seed=0)
    d = lambda x: x.to(dev).contiguous()  # noqa: E731
    means, opac, scales, rots, shs = d(sc.means3D), d(sc.opacities), d(sc.scales), d(sc.rotations), d(sc.shs)
    e = torch.empty(0, device=dev)
    k = _HipViewKernels()
    S = -(-P // V)
    P_pad = S * V
    recs = torch.empty(V, P_pad, 12, device=dev)
    cams = torch.empty(V, 64, device=dev)
    gc, gd = (d(x) for x in make_upstream_grads(W, H, seed=1))
    for v in range(V):
        f = synthetic_camera(W, H, v).raster_fields()
        cam = dict(viewmatrix=d(f["viewmatrix"]), projmatrix=d(f["projmatrix"]),
                   projmatrix_raw=d(f["projmatrix_raw"]), campos=d(f["campos"]), tanfovx=f["tanfovx"],
                   tanfovy=f["tanfovy"], bg=d(torch.zeros(3)))
        out = _C.rasterize_gaussians(cam["bg"], means, e, opac, scales, rots, 1.0, e, cam["viewmatrix"],
                                     cam["projmatrix"], cam["projmatrix_raw"], f["tanfovx"], f["tanfovy"], H, W,
                                     shs, deg, cam["campos"], False, False)
        nr, color, radii, geom, binning, img = out[:6]
        k.records((means, scales, rots, shs, deg, cam, nr, radii, geom, binning, img), gc, gd, P_pad, recs[v])
        k.pack_camera(cam, W, H, cams[v])
        if v == 0:
            keep = (cam, nr, radii, geom, binning, img)
    # shard 0's view-major block, as the all-to-all delivers it
    shard = recs[:, :S].contiguous()
    buf = GradBuffer.allocate(P_pad, M, dev)
    tb = torch.empty(max(1, k.tau_blocks(0, S)), V, 6, device=dev)
    params = (means, scales, rots, shs, deg, 1.0)

    def timeit(fn):
        for _ in range(3):
            fn()
        s, t = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.iters):
            fn()
        t.record()
        torch.cuda.synchronize()
        return s.elapsed_time(t) / a.iters

    t_views = timeit(lambda: k.gauss_views(params, 0, min(S, P), cams, shard, buf.views, tb, None))
    cam, nr, radii, geom, binning, img = keep
    with _lib.StageProfile() as prof:
        for _ in range(a.iters):
            _C.rasterize_gaussians_backward(cam["bg"], means, radii, e, scales, rots, 1.0, e, cam["viewmatrix"],
                                            cam["projmatrix"], cam["projmatrix_raw"], cam["tanfovx"],
                                            cam["tanfovy"], gc, gd, shs, deg, cam["campos"], geom, nr, binning,
                                            img, False, out=buf.views)
        torch.cuda.synchronize()
    gb = prof.stages["gauss_bwd"]
    print(json.dumps({"views": V, "P": P, "shard": S,
                      "owner_kernel_ms (shard x views)": t_views,
                      "gauss_bwd_ms (all P, one view)": gb[0] / max(1, gb[1]),
                      "record_bytes_per_view": P_pad * 48}))


if __name__ == "__main__":
    main()
