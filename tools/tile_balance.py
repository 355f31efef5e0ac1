"""Dump per-tile work of the bench scene (GPU) for load-balance analysis:
list length (range) and the deepest contributor per tile (the backward's
walk length).  Writes gpurun_out/tile_work.npz."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "wildgs-slam-blackwell_amd", "python"))

from diff_gaussian_rasterization import _C  # noqa: E402
from wgsr.camera import synthetic_camera  # noqa: E402
from wgsr.scene import make_scene  # noqa: E402

P, W, H, deg = (int(a) for a in sys.argv[1:5]) if len(sys.argv) >= 5 else (1_000_000, 1920, 1080, 3)
dev = torch.device("cuda")
sc = make_scene(P, W, H, deg, seed=0)
f = synthetic_camera(W, H, view=0).raster_fields()
d = lambda x: x.to(dev).contiguous()  # noqa: E731
e = torch.empty(0, device=dev)
nr, color, radii, geom, binning, img, depth, opac, nt = _C.rasterize_gaussians(
    d(torch.zeros(3)), d(sc.means3D), e, d(sc.opacities), d(sc.scales), d(sc.rotations), 1.0, e,
    d(f["viewmatrix"]), d(f["projmatrix"]), d(f["projmatrix_raw"]), f["tanfovx"], f["tanfovy"], H, W,
    d(sc.shs), deg, d(f["campos"]), False, False)
torch.cuda.synchronize()
gx, gy = (W + 15) // 16, (H + 15) // 16
ntl = gx * gy
b = img.cpu().numpy().view(np.uint8)
a256 = lambda x: (x + 255) // 256 * 256  # noqa: E731
# ImageLayout (csrc/wgsr_common.h): ranges 8 nt, tile_len 4 nt, tile_m 16 nt, ...
ranges = b[:8 * ntl].view(np.uint32).reshape(ntl, 2)
off_m = a256(8 * ntl) + a256(4 * ntl)
m4 = b[off_m:off_m + 16 * ntl].view(np.uint32).reshape(ntl, 4)
m = m4.max(axis=1)
os.makedirs("gpurun_out", exist_ok=True)
np.savez("gpurun_out/tile_work.npz", length=(ranges[:, 1] - ranges[:, 0]).astype(np.int64), m=m.astype(np.int64),
         gx=gx, gy=gy)
print("tiles", ntl, "pairs", int((ranges[:, 1] - ranges[:, 0]).sum()), "m-sum", int(m.sum()))
