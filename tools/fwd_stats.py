"""Diagnostic: per quadrant wave census of the render forward
(build: VFLAGS="-DWGSR_FWD_STATS=1" tools/build_variant.sh fstats /tmp/empty;
run with WGSR_LIB=.../lib/variants/fstats.so).

Counts, summed over k_render_fwd_dec's quadrant waves: batches walked,
entries in them, survivors of the per-wave ellipse culling, survivor pairs
(the blend loop's iterations before its early exit), batches that kept the
n_touched bookkeeping, and waves that stopped with every pixel done.  With
the kernel's VALU per wave (PMC) this splits the forward into its per-batch
and per-entry parts."""
import ctypes
import json
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "wildgs-slam-blackwell_amd", "python"))
import torch  # noqa: E402
from diff_gaussian_rasterization import _C  # noqa: E402
from wgsr import _lib  # noqa: E402
from wgsr.camera import synthetic_camera  # noqa: E402
from wgsr.scene import make_scene  # noqa: E402


def run(P, W, H, deg):
    dev = torch.device("cuda")
    sc = make_scene(P, W, H, deg).to(dev)
    f = synthetic_camera(W, H, 0).raster_fields()
    d = {k: (v.to(dev) if torch.is_tensor(v) else v) for k, v in f.items()}
    e = torch.empty(0, device=dev)
    bg = torch.zeros(3, device=dev)
    lib = ctypes.CDLL(_lib.LIB_PATH)
    out = (ctypes.c_ulonglong * 8)()

    def fwd():
        return _C.rasterize_gaussians(bg, sc.means3D, e, sc.opacities, sc.scales, sc.rotations, 1.0, e,
                                      d["viewmatrix"], d["projmatrix"], d["projmatrix_raw"], d["tanfovx"],
                                      d["tanfovy"], H, W, sc.shs, deg, d["campos"], False, False)
    fwd()
    torch.cuda.synchronize()
    lib.wgsr_debug_fwd_stats(out)  # clear
    nr = fwd()[0]
    torch.cuda.synchronize()
    assert lib.wgsr_debug_fwd_stats(out) == 0
    v = list(out)
    waves = max(v[0], 1)
    return {"workload": f"{P} Gaussians, {W}x{H}, SH{deg}", "num_rendered": int(nr), "waves": v[0],
            "batches_per_wave": v[1] / waves, "entries_per_wave": v[2] / waves,
            "survivors_per_wave": v[3] / waves, "survivor_pairs_per_wave": v[4] / waves,
            "touch_batches_per_wave": v[5] / waves, "waves_done_early": v[6] / waves,
            "survivor_fraction": v[3] / max(v[2], 1)}


if __name__ == "__main__":
    for cfg in ((1_000_000, 1920, 1080, 3), (100_000, 512, 384, 0)):
        print(json.dumps(run(*cfg)))
