#!/usr/bin/env python
"""Summarise rocprofv3 --pmc runs of bench.py per kernel.

HBM bytes follow MI355X_MICROARCH.md "HBM": FETCH_SIZE and WRITE_SIZE are in
KiB; on gfx950 FETCH_SIZE reports half the bytes of wide (16 B/lane)
coalesced reads, so the corrected read bytes are 2 x FETCH_SIZE (reported
next to the raw value; other access widths are uncalibrated).  Counters come
from separate passes (FETCH_SIZE and WRITE_SIZE do not fit one pass).

Per-step figures: each kernel's per-dispatch average times its dispatches per
step (dispatch count over the run / --steps-run, the warmup + timed steps of
the profiled bench.py command); a stage's bytes and VALU instructions are
summed over its kernels.  The config the counters were taken on is recorded
(--config P,W,H,SH) so that bench.py only quotes them for the same workload.

The optional SQ_ACTIVE_INST_VALU / SQ_BUSY_CYCLES pass (pmc_sq2) gives each
kernel's VALU pipe occupancy at the clock it actually ran: SQ_ACTIVE_INST_VALU
counts quad-cycles (4 cycles, the issue slot of one wave64 VALU instruction;
an 8-cycle transcendental or permlane counts 2) summed over waves, and
SQ_BUSY_CYCLES counts SQ clocks summed over the 32 shader engines, so
  clock = SQ_BUSY_CYCLES / 32 / kernel duration,
  valu_busy_frac = 4 x SQ_ACTIVE_INST_VALU / (1024 SIMDs x SQ_BUSY_CYCLES / 32).

usage: python tools/pmc_summary.py gpurun_out out.json --config 1000000,1920,1080,3 --steps-run 7 [--source label] [--suffix _tum]
"""
import csv
import json
import os
import re
import sys
from collections import defaultdict

STAGE_OF = {
    "k_preprocess": "preprocess", "k_duplicate": "duplicate", "k_ranges": "ranges",
    "k_render_fwd": "render_fwd", "k_render_bwd": "render_bwd", "k_gauss_bwd": "gauss_bwd",
    "k_render_fwd_quad": "render_fwd", "k_render_bwd_quad": "render_bwd", "k_sum_partials": "gauss_bwd",
    "k_render_fwd1": "render_fwd", "k_tile_order": "render_bwd",
    "k_scan_reduce": "offsets_scan", "k_scan_bsum": "offsets_scan", "k_scan_down": "offsets_scan",
    "k_scan2_reduce": "offsets_scan", "k_scan2_bsum": "offsets_scan",
    "k_duplicate_bins": "duplicate", "k_bin_bounds": "ranges", "k_expand_bins": "ranges",
    "k_render_bwd_split": "render_bwd", "k_sum_active": "gauss_bwd", "k_gauss_bwd_compact": "gauss_bwd",
    "k_depth_hist": "depth_sort", "k_depth_scatter": "depth_sort",
    "k_bin_depth_sort": "tile_sort",  # (per-bin depth order: small frames)
    "k_preprocess2": "preprocess", "k_preprocess3": "preprocess",
    "k_render_fwd_dec": "render_fwd", "k_render_bwd_seg": "render_bwd",
}


def short(name):
    name = name.replace("wgsr::(anonymous namespace)::", "").replace("void ", "")
    return re.split(r"[(<]", name, maxsplit=1)[0]


N_SE, N_SIMD = 32, 1024  # MI355X: 8 XCDs x 4 shader engines; 256 CUs x 4 SIMDs


def load(path):
    """-> {(kernel, grid): {counter: [values per dispatch], "_ns": [durations]}}"""
    out = defaultdict(lambda: defaultdict(list))
    if not os.path.exists(path):
        return out
    seen = set()
    for r in csv.DictReader(open(path)):
        key = (short(r["Kernel_Name"]), int(r["Grid_Size"]))
        out[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
        did = r.get("Dispatch_Id")
        if did is not None and did not in seen and r.get("Start_Timestamp"):
            seen.add(did)
            out[key]["_ns"].append(float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
    return out


def stage_for(kernel, grid, P_grid):
    if kernel in STAGE_OF:
        return STAGE_OF[kernel]
    if kernel.startswith("k_radix"):
        # depth sort passes run over P keys (grid ~ P/4096 workgroups)
        return "depth_sort" if grid <= P_grid else "tile_sort"
    return None


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("out", nargs="?")
    ap.add_argument("--config", required=True, help="P,W,H,SH of the profiled bench.py run")
    ap.add_argument("--steps-run", type=int, required=True, help="warmup + timed steps of the profiled run")
    ap.add_argument("--source", default="rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE / SQ passes of bench.py")
    ap.add_argument("--suffix", default="", help="directory suffix of the passes (gpu_check.sh SFX)")
    args = ap.parse_args()
    root, out_path, source = args.root, args.out, args.source
    cP, cW, cH, cS = (int(x) for x in args.config.split(","))
    sfx = args.suffix
    fetch = load(os.path.join(root, "pmc_fetch" + sfx, "run_counter_collection.csv"))
    write = load(os.path.join(root, "pmc_write" + sfx, "run_counter_collection.csv"))
    sq = load(os.path.join(root, "pmc_sq" + sfx, "run_counter_collection.csv"))
    sq2 = load(os.path.join(root, "pmc_sq2" + sfx, "run_counter_collection.csv"))
    keys = sorted(set(fetch) | set(write) | set(sq) | set(sq2))
    # grid size of the depth-sort radix kernels: the smallest radix scatter grid
    # (the depth sort's own k_depth_* kernels: then every k_radix_* is the bin sort)
    rg = [g for (k, g) in keys if k == "k_radix_scatter"]
    # (the per-bin schedule has no Gaussian-level sort: every k_radix_* is the bin sort)
    P_grid = 0 if any(k.startswith("k_depth_") or k == "k_bin_depth_sort" for (k, g) in keys) else (min(rg) if rg else 0)
    rows, stages = [], defaultdict(lambda: {"hbm_bytes_per_step": 0.0, "valu_insts_per_step": 0.0,
                                            "launches_per_step": 0.0, "launch_kinds": []})
    hdr = (f"{'kernel':18s} {'grid':>9s} {'FETCH_KB':>10s} {'WRITE_KB':>10s} {'HBM_MB*':>9s} "
           f"{'VALU/wave':>9s} {'VMEM/wave':>9s} {'LDS/wave':>8s} {'wait%':>6s} {'GHz':>5s} {'VALUbusy':>8s}")
    print(hdr)
    for key in keys:
        k, g = key
        avg = lambda d, c: (sum(d[key][c]) / len(d[key][c])) if d[key].get(c) else None  # noqa: E731
        f = avg(fetch, "FETCH_SIZE")
        w = avg(write, "WRITE_SIZE")
        waves = avg(sq, "SQ_WAVES")
        valu = avg(sq, "SQ_INSTS_VALU")
        vrd, vwr = avg(sq, "SQ_INSTS_VMEM_RD"), avg(sq, "SQ_INSTS_VMEM_WR")
        lds = avg(sq, "SQ_INSTS_LDS")
        cyc, wait = avg(sq, "SQ_WAVE_CYCLES"), avg(sq, "SQ_WAIT_ANY")
        hbm = ((2 * f if f is not None else 0) + (w or 0)) * 1024
        act, busy = avg(sq2, "SQ_ACTIVE_INST_VALU"), avg(sq2, "SQ_BUSY_CYCLES")
        dur = avg(sq2, "_ns")
        ghz = (busy / N_SE) / dur if (busy and dur) else None
        vbusy = 4 * act / (N_SIMD * busy / N_SE) if (act and busy) else None
        nd = max(len(d[key].get(c, [])) for d, c in ((fetch, "FETCH_SIZE"), (write, "WRITE_SIZE"),
                                                     (sq, "SQ_WAVES")))
        per_step = nd / args.steps_run
        per = lambda x: (x / waves) if (x is not None and waves) else float("nan")  # noqa: E731
        print(f"{k:18s} {g:9d} {f if f is not None else float('nan'):10.0f} "
              f"{w if w is not None else float('nan'):10.0f} {hbm / 1e6:9.1f} {per(valu):9.0f} "
              f"{per((vrd or 0) + (vwr or 0)):9.1f} {per(lds):8.1f} "
              f"{100 * wait / cyc if (wait and cyc) else float('nan'):6.1f} "
              f"{ghz if ghz else float('nan'):5.2f} {vbusy if vbusy else float('nan'):8.3f}")
        rows.append(dict(kernel=k, grid=g, fetch_kib=f, write_kib=w, hbm_bytes=hbm, waves=waves,
                         valu_per_wave=per(valu), vmem_per_wave=per((vrd or 0) + (vwr or 0)),
                         lds_per_wave=per(lds), wait_frac=(wait / cyc) if (wait and cyc) else None,
                         dispatches_per_step=per_step, clock_ghz=ghz, valu_busy_frac=vbusy,
                         valu_active_quadcycles=act, duration_ns=dur,
                         trans_per_wave=per(avg(sq2, "SQ_INSTS_VALU_TRANS_F32")),
                         salu_per_wave=per(avg(sq2, "SQ_INSTS_SALU"))))
        st = stage_for(k, g, P_grid)
        if st:
            stages[st]["hbm_bytes_per_step"] += hbm * per_step
            stages[st]["launches_per_step"] += per_step
            if valu is not None and waves:
                stages[st]["valu_insts_per_step"] += valu * per_step  # wave-level VALU instructions
            if k not in stages[st]["launch_kinds"]:
                stages[st]["launch_kinds"].append(k)
            if vbusy is not None:
                # the stage's dominant kernel (most VALU quad-cycles) sets its VALU-busy figure
                if act * per_step > stages[st].get("_act", 0.0):
                    stages[st]["_act"] = act * per_step
                    stages[st]["valu_busy_frac"] = vbusy
                    stages[st]["clock_ghz"] = ghz
                    stages[st]["valu_busy_kernel"] = k
    print("* HBM_MB = (2 x FETCH_SIZE + WRITE_SIZE) per dispatch (gfx950 FETCH correction); GHz = SQ_BUSY_CYCLES/32/"
          "duration; VALUbusy = 4 SQ_ACTIVE_INST_VALU / (1024 x SQ_BUSY_CYCLES/32)")
    for st in stages.values():
        st.pop("_act", None)
    if out_path:
        json.dump({"source": source, "config": {"P": cP, "W": cW, "H": cH, "sh": cS},
                   "steps_run": args.steps_run,
                   "note": "kernels: per-dispatch averages; stages: per bench step (every dispatch of the "
                           "stage's kernels in one step)",
                   "kernels": rows, "stages": stages}, open(out_path, "w"), indent=1)


if __name__ == "__main__":
    main()
