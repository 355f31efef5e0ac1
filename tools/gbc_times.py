"""Phase clocks of k_gauss_bwd_compact (diagnostic build, round 5): where a
workgroup's time goes at 1M / 1080p / SH3.
  VFLAGS=-DWGSR_GBC_TIMES=1 bash tools/build_variant.sh gbctimes /tmp/empty
  WGSR_LIB=wildgs-slam-blackwell_amd/lib/variants/gbctimes.so python tools/gbc_times.py
Prints the mean s_memtime clocks from a workgroup's start to the end of each
phase (flags + list, slot ranges, scan, record sums, per-Gaussian backward),
over the workgroups that had work, plus their mean listed Gaussians / slots."""
import ctypes
import json
import os
import sys

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
    fn = lib.wgsr_debug_gbc_times
    fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
    dev = torch.device("cuda:0")
    W, H, deg = 1920, 1080, 3
    P = int(os.environ.get("GBC_P", "1000000"))
    sc = make_scene(P, W, H, deg, seed=0)
    gc, gd = make_upstream_grads(W, H, seed=1)
    f = synthetic_camera(W, H, 0).raster_fields()
    d = lambda x: x.to(dev)  # noqa: E731
    e = torch.empty(0, device=dev)
    args = [d(sc.means3D), d(sc.opacities), d(sc.scales), d(sc.rotations), d(sc.shs)]
    bg = torch.zeros(3, device=dev)

    def step():
        nr, color, radii, geom, binning, img, depth, opac, nt = _C.rasterize_gaussians(
            bg, args[0], e, args[1], args[2], args[3], 1.0, e, d(f["viewmatrix"]), d(f["projmatrix"]),
            d(f["projmatrix_raw"]), f["tanfovx"], f["tanfovy"], H, W, args[4], deg, d(f["campos"]), False, False)
        _C.rasterize_gaussians_backward(bg, args[0], radii, e, args[2], args[3], 1.0, e, d(f["viewmatrix"]),
                                        d(f["projmatrix"]), d(f["projmatrix_raw"]), f["tanfovx"], f["tanfovy"],
                                        d(gc), d(gd), args[4], deg, d(f["campos"]), geom, nr, binning, img, False)
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * 16)()
    fn(buf)
    n = 5
    for _ in range(n):
        step()
    torch.cuda.synchronize()
    fn(buf)
    v = list(buf)
    wg = max(v[8], 1)
    out = {"P": P, "workgroups_launched_per_call": v[15] / n, "workgroups_with_work_per_call": v[8] / n,
           "listed_per_wg": v[9] / wg, "slots_per_wg": v[10] / wg, "max_slots_one_wg": v[12],
           "max_slots_one_gaussian": v[14], "slowest_wg_clocks_to_record_sums_end": v[11],
           "slowest_wg_clocks_to_end": v[13],
           "clocks_to_end_of": {name: v[k] / wg for k, name in enumerate(
               ("flags_list", "slot_ranges", "scan", "record_sums", "gaussian_backward"))}}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
