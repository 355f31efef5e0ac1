"""Diagnostic: sparsity of the backward's per-(Gaussian, tile) partial records
and tile-list statistics at the bench workload."""
import os
import sys
ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "wildgs-slam-blackwell_amd", "python"))
import torch  # noqa: E402
from diff_gaussian_rasterization import _C  # noqa: E402
from wgsr import _lib  # noqa: E402
from wgsr.camera import synthetic_camera  # noqa: E402
from wgsr.scene import make_scene, make_upstream_grads  # noqa: E402

P, W, H, deg = 1_000_000, 1920, 1080, 3
dev = torch.device("cuda")
sc = make_scene(P, W, H, deg).to(dev)
gc, gd = (x.to(dev) for x in make_upstream_grads(W, H))
f = synthetic_camera(W, H, 0).raster_fields()
d = {k: (v.to(dev) if torch.is_tensor(v) else v) for k, v in f.items()}
e = torch.empty(0, device=dev)
bg = torch.zeros(3, device=dev)
nr, color, radii, geom, binning, img, depth, opac, nt = _C.rasterize_gaussians(
    bg, sc.means3D, e, sc.opacities, sc.scales, sc.rotations, 1.0, e, d["viewmatrix"], d["projmatrix"],
    d["projmatrix_raw"], d["tanfovx"], d["tanfovy"], H, W, sc.shs, deg, d["campos"], False, False)
kept = {}
orig = _lib._make_alloc


class Keep(_lib.AllocRequest):
    def __exit__(self, *exc):
        kept.update(self.buffers)
        return super().__exit__(*exc)


_lib.AllocRequest = Keep
g = _C.rasterize_gaussians_backward(bg, sc.means3D, radii, e, sc.scales, sc.rotations, 1.0, e,
                                    d["viewmatrix"], d["projmatrix"], d["projmatrix_raw"],
                                    d["tanfovx"], d["tanfovy"], gc, gd, sc.shs, deg, d["campos"],
                                    geom, nr, binning, img, False)
torch.cuda.synchronize()
part = kept["scratch"].view(torch.float32).view(nr, 12)
nz = (part[:, :10].abs().sum(1) > 0)
print(f"num_rendered={nr} nonzero_records={int(nz.sum())} frac={float(nz.float().mean()):.3f}")
# tile list length statistics
ntile = ((W + 15) // 16) * ((H + 15) // 16)
ranges = img[: 8 * ntile].view(torch.int32).view(ntile, 2).long()
L = (ranges[:, 1] - ranges[:, 0]).float()
print(f"tiles={ntile} list len mean={L.mean():.1f} median={L.median():.1f} max={L.max():.0f} "
      f"p99={L.quantile(0.99):.0f}")
def a256(x):
    return (x + 255) & ~255
off = a256(8 * ntile) + a256(4 * W * H)
nc = img[off: off + 4 * W * H].view(torch.int32).view(H, W).float()
print(f"n_contrib mean={nc.mean():.1f} max={nc.max():.0f}; visible={int((radii > 0).sum())}")
tiles = nc.new_zeros(0)
