"""Diagnostic: per-entry quadrant histogram of the quad render backward
(build: VFLAGS="-DWGSR_BWD_STATS=1 -DWGSR_BWD_PAIR=0" tools/build_variant.sh
stats /tmp/empty; run with WGSR_LIB=.../lib/variants/stats.so).

For every entry the walk evaluates: the set of 8x8 quadrants its ellipse
reaches (phase 1 runs there) and the set where some pixel took it (phase 2
runs there).  Prints both histograms by pattern at the bench workload."""
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
from wgsr.scene import make_scene, make_upstream_grads  # noqa: E402


def run(P, W, H, deg):
    dev = torch.device("cuda")
    sc = make_scene(P, W, H, deg).to(dev)
    gc, gd = (x.to(dev) for x in make_upstream_grads(W, H))
    f = synthetic_camera(W, H, 0).raster_fields()
    d = {k: (v.to(dev) if torch.is_tensor(v) else v) for k, v in f.items()}
    e = torch.empty(0, device=dev)
    bg = torch.zeros(3, device=dev)
    lib = ctypes.CDLL(_lib.LIB_PATH)
    out = (ctypes.c_ulonglong * 64)()
    nr, color, radii, geom, binning, img, depth, opac, nt = _C.rasterize_gaussians(
        bg, sc.means3D, e, sc.opacities, sc.scales, sc.rotations, 1.0, e, d["viewmatrix"], d["projmatrix"],
        d["projmatrix_raw"], d["tanfovx"], d["tanfovy"], H, W, sc.shs, deg, d["campos"], False, False)
    torch.cuda.synchronize()
    lib.wgsr_debug_bwd_stats(out)  # clear
    _C.rasterize_gaussians_backward(bg, sc.means3D, radii, e, sc.scales, sc.rotations, 1.0, e,
                                    d["viewmatrix"], d["projmatrix"], d["projmatrix_raw"],
                                    d["tanfovx"], d["tanfovy"], gc, gd, sc.shs, deg, d["campos"],
                                    geom, nr, binning, img, False)
    torch.cuda.synchronize()
    assert lib.wgsr_debug_bwd_stats(out) == 0
    reach, p2 = list(out[:16]), list(out[16:32])
    n = sum(reach)
    pop = lambda h: [sum(c for m, c in enumerate(h) if bin(m).count("1") == k) for k in range(5)]  # noqa: E731
    # row-pair classes of the reach mask: bits 0,1 = row pair 0; 2,3 = row pair 1
    def rows(h):
        cls = {"both_full": 0, "one_full_one_half": 0, "both_half": 0, "one_row_full": 0, "one_row_half": 0}
        for m, c in enumerate(h):
            r0, r1 = m & 3, (m >> 2) & 3
            f = [r == 3 for r in (r0, r1) if r]
            if len(f) == 2:
                cls["both_full" if all(f) else ("one_full_one_half" if any(f) else "both_half")] += c
            elif len(f) == 1:
                cls["one_row_full" if f[0] else "one_row_half"] += c
        return cls
    return {"workload": f"{P} Gaussians, {W}x{H}, SH{deg}", "entries": n, "reach_by_mask": reach,
            "p2_by_mask": p2, "reach_popcount": pop(reach), "p2_popcount": pop(p2),
            "quadrant_evals_p1": sum(c * bin(m).count("1") for m, c in enumerate(reach)),
            "quadrant_evals_p2": sum(c * bin(m).count("1") for m, c in enumerate(p2)),
            "hit_entries": n - p2[0], "reach_rows": rows(reach), "p2_rows": rows(p2),
            # log2 bins: [1], [2, 3], [4, 7], ... [128, 256]
            "pixels_per_hit_entry_log2": list(out[32:40]), "lanes_per_p2_eval_log2": list(out[40:48]),
            "p2_lanes": out[48], "p1_evals_without_p2": out[49], "p1_evals_in_all_live_batches": out[50]}


if __name__ == "__main__":
    os.environ["WGSR_BWD_SPLIT_BELOW"] = "0"  # the quad kernel at every size
    for cfg in ((1_000_000, 1920, 1080, 3), (100_000, 512, 384, 0)):
        print(json.dumps(run(*cfg)))
