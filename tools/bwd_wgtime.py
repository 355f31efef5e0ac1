"""Workgroup timeline of k_render_bwd_quad (diagnostic build): how much of the
kernel's span is the tail, where fewer waves run than the GPU holds.
  VFLAGS=-DWGSR_BWD_WGTIME=1 bash tools/build_variant.sh wgtime /tmp/empty
  WGSR_LIB=wildgs-slam-blackwell_amd/lib/variants/wgtime.so python tools/bwd_wgtime.py
Each workgroup (one wave, one tile) stores its s_memrealtime start / end
(100 MHz) and hardware id (WGTIME_DUMP=file.npz: the first measured call's
per-workgroup arrays).  Prints the span, the summed wave time, the
resident-wave profile over the span (in tenths), the time from the last
workgroup start to the end, and the LPT bound max(sum / slots, longest)."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))


def main():
    import __graft_entry__ as ge
    ge._paths()
    from diff_gaussian_rasterization import _C
    from wgsr.camera import synthetic_camera
    from wgsr.scene import make_scene, make_upstream_grads
    lib = ctypes.CDLL(os.environ["WGSR_LIB"])
    fn = lib.wgsr_debug_bwd_wgtime
    fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    dev = torch.device("cuda:0")
    W, H, P, deg = 1920, 1080, 1_000_000, 3
    sc = make_scene(P, W, H, deg, seed=0)
    gc, gd = make_upstream_grads(W, H, seed=1)
    f = synthetic_camera(W, H, 0).raster_fields()
    d = lambda x: x.to(dev)  # noqa: E731
    e = torch.empty(0, device=dev)
    args = [d(sc.means3D), d(sc.opacities), d(sc.scales), d(sc.rotations), d(sc.shs)]
    bg = torch.zeros(3, device=dev)
    ntiles = ((W + 15) // 16) * ((H + 15) // 16)

    def step():
        nr, color, radii, geom, binning, img, depth, opac, nt = _C.rasterize_gaussians(
            bg, args[0], e, args[1], args[2], args[3], 1.0, e, d(f["viewmatrix"]), d(f["projmatrix"]),
            d(f["projmatrix_raw"]), f["tanfovx"], f["tanfovy"], H, W, args[4], deg, d(f["campos"]), False, False)
        _C.rasterize_gaussians_backward(bg, args[0], radii, e, args[2], args[3], 1.0, e, d(f["viewmatrix"]),
                                        d(f["projmatrix"]), d(f["projmatrix_raw"]), f["tanfovx"], f["tanfovy"],
                                        d(gc), d(gd), args[4], deg, d(f["campos"]), geom, nr, binning, img, False)
    res = []
    for rep in range(4):
        step()
        torch.cuda.synchronize()
        buf = (ctypes.c_ulonglong * (3 * ntiles))()
        assert fn(buf, ntiles) == 0
        if rep == 0:
            continue  # warm-up
        a = np.frombuffer(buf, dtype=np.uint64).reshape(ntiles, 3)
        t0 = a[:, 0].astype(np.int64)
        t1 = a[:, 1].astype(np.int64)
        base = t0.min()
        t0, t1 = (t0 - base) * 10, (t1 - base) * 10  # ns (100 MHz)
        dur = t1 - t0
        span = int(t1.max())
        hw = a[:, 2]
        xcc = ((hw >> 32) & 15).astype(np.int64)
        cu = ((hw >> 8) & 15) | (((hw >> 13) & 7) << 4)  # CU id within SE, SE
        slots_seen = len(set(zip(xcc.tolist(), cu.tolist(), ((hw >> 4) & 3).tolist())))
        grid = np.linspace(0, span, 11)
        prof = [int(((t0 <= g) & (t1 > g)).sum()) for g in grid[:-1] + span / 20]
        peak = max(prof)
        total = int(dur.sum())
        per_xcc_end = [int(t1[xcc == x].max()) for x in range(8) if (xcc == x).any()]
        if rep == 1 and os.environ.get("WGTIME_DUMP"):
            np.savez(os.environ["WGTIME_DUMP"], t0=t0, t1=t1, hw=hw.astype(np.int64))
        res.append({
            "span_us": span / 1e3, "sum_wave_us": total / 1e3, "mean_resident": total / span,
            "peak_resident": peak, "resident_profile_tenths": prof,
            "last_start_to_end_us": (span - int(t0.max())) / 1e3,
            "longest_wg_us": int(dur.max()) / 1e3, "median_wg_us": float(np.median(dur)) / 1e3,
            "lpt_bound_us": max(total / peak, int(dur.max())) / 1e3,
            "xcc_end_us": [x / 1e3 for x in per_xcc_end], "simd_slots_seen": slots_seen,
            "tiles": ntiles})
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
