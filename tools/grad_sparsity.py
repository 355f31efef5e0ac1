#!/usr/bin/env python
"""How many Gaussians receive gradient per view (SURVEY.md 8(e) exchange sizing).

Renders configs[3]'s views (view k per rank, wgsr.camera.synthetic_camera)
of the bench scene, writes each view's per-Gaussian screen-space records
(k_view_records) and counts Gaussians that are visible (radius > 0), that
receive any gradient (a non-zero record sum), and the union of the latter over
the first n views -- the rows a sparse gradient exchange would have to move.
"""
import argparse
import json
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "wildgs-slam-blackwell_amd", "python"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, default=1_000_000)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--views", type=int, default=8)
    a = ap.parse_args()
    from diff_gaussian_rasterization import _C
    from wgsr.camera import synthetic_camera
    from wgsr.dp import _HipViewKernels
    from wgsr.scene import make_scene, make_upstream_grads
    dev = torch.device("cuda:0")
    P, W, H = a.P, a.width, a.height
    sc = make_scene(P, W, H, 3, seed=0)
    gc, gd = (x.to(dev) for x in make_upstream_grads(W, H, seed=1))
    means, opac, scales, rots, shs = (x.to(dev).contiguous() for x in (sc.means3D, sc.opacities, sc.scales,
                                                                        sc.rotations, sc.shs))
    bg = torch.zeros(3, device=dev)
    e = torch.empty(0, device=dev)
    k = _HipViewKernels()
    rec = torch.empty(P, 12, device=dev)
    union = torch.zeros(P, dtype=torch.bool, device=dev)
    union_vis = torch.zeros(P, dtype=torch.bool, device=dev)
    rows = []
    for v in range(a.views):
        f = synthetic_camera(W, H, view=v).raster_fields()
        cam = {n: (f[n].to(dev) if torch.is_tensor(f[n]) else f[n]) for n in f}
        cam["bg"] = bg
        nr, color, radii, geom, binning, img, depth, opacity, nt = _C.rasterize_gaussians(
            bg, means, e, opac, scales, rots, 1.0, e, cam["viewmatrix"], cam["projmatrix"], cam["projmatrix_raw"],
            cam["tanfovx"], cam["tanfovy"], H, W, shs, 3, cam["campos"], False, False)
        k.records((means, scales, rots, shs, 3, cam, nr, radii, geom, binning, img), gc, gd, P, rec)
        vis = radii > 0
        nz = (rec[:, :10] != 0).any(dim=1)
        union |= nz
        union_vis |= vis
        rows.append({"view": v, "visible": int(vis.sum()), "nonzero_grad": int(nz.sum()),
                     "union_nonzero_so_far": int(union.sum()), "union_visible_so_far": int(union_vis.sum()),
                     "num_rendered": int(nr)})
    print(json.dumps({"P": P, "image": f"{W}x{H}", "views": rows}))


if __name__ == "__main__":
    main()
