#!/usr/bin/env python
"""bench.py -- rasterised Gaussians/s, forward + backward, 1M Gaussians @ 1080p.

BASELINE.json metric: "rasterised Gaussians/s fwd+bwd @1M pts 1080p; PSNR vs ref".

One step = one pass of the hot path over one view: ``_C.rasterize_gaussians``
followed by ``_C.rasterize_gaussians_backward`` for 1M
synthetic Gaussians (BASELINE.md distribution, SH degree 3, pose gradient
always computed) at 1920x1080, all inputs resident in HBM before timing.

* N = 1 (default): BASELINE.json configs[2].  value = P * K / t.
* N > 1 (torchrun, one rank per GPU): configs[3] -- keyframe-view data
  parallelism: rank r renders view r of the same replicated 1M Gaussians and
  every rank ends the step holding the SUM over the N views of the
  per-Gaussian parameter gradients (59 floats each).  Default exchange
  (wgsr.dp.ViewShardedBackward): each view's 12-float screen-space record of
  every Gaussian goes to the Gaussian's owner rank (RCCL all-to-all), owners
  run the camera-side backward of all N views for their 1/N shard, and the
  shards are all-gathered.  Only rows with a non-zero record / gradient
  travel (exactly the same sums: the other rows are zero), ~10 % of the
  Gaussians in this scene; ``--dp-exchange views-dense`` moves every row (71
  instead of 118 floats per Gaussian per rank at N = 8) and ``allreduce`` runs
  the plain RCCL all-reduce.  Weak scaling; value = P * N * K / max_rank(t).

Extra fields: ``roofline`` for the dominant kernel (stage times from HIP
events recorded on the launch stream inside the timed region; algorithmic
bytes from SURVEY.md 8(d)), ``cpu_baseline`` (the fp32 CPU restatement,
oracle/cpu_raster.cpp, on the host cores; rank 0 at N = 1 only) and
``psnr_vs_cpu_db`` (GPU render vs the CPU restatement's render).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (os.path.join(ROOT, "wildgs-slam-blackwell_amd", "python"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "rasterised Gaussians/s fwd+bwd @1M pts 1080p; PSNR vs ref"
HBM_PEAK_GBPS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md)
VALU_PEAK_TFLOPS = 157.3    # fp32 vector peak (MI355X_MICROARCH.md)
# VALU issue peak: 256 CUs x 4 SIMDs x 2.4 GHz / 4 cycles per wave64 instruction
VALU_ISSUE_PEAK = 256 * 4 * 2.4e9 / 4
TILE = 16


def grad_write_bytes(P, M):
    """SURVEY.md 8(d)'s gradient-output write, P (12 + 12 + 12 M + 4 + 12 +
    16 + 24): in this build the render backward streams it as the outputs'
    zero fill and gauss_bwd writes only the ~8 % of rows that got gradient."""
    return P * (12 + 12 + 12 * M + 4 + 12 + 16 + 24)


def byte_model(P, N, W, H, K, M):
    """Algorithmic bytes per stage: SURVEY.md 8(d)'s per-unit figures, the
    same table as DESIGN.md section 3.  The gradient-output write
    (grad_write_bytes) is its own entry, "grad_write"; it is physically
    streamed by the render backward (zero fill), so the roofline reports the
    render backward's fraction both without it (``frac``) and with it
    (``frac_incl_zero_fill``).  N is upstream's num_rendered (rectangle
    pairs), as SURVEY defines it; the build lists fewer pairs (exact tile
    lists) and sorts (Gaussian, bin) pairs -- the counter bytes
    (pass_roofline.counter_bytes) are what it actually moves."""
    npix = W * H
    ntile = ((W + TILE - 1) // TILE) * ((H + TILE - 1) // TILE)
    return {
        "preprocess": P * (44 + 12 * K) + 76 * P,
        "depth_sort": 16 * P,
        "offsets_scan": 8 * P,
        "duplicate": 12 * N,
        "tile_sort": 24 * N,
        "ranges": 8 * N + 8 * ntile,
        "render_fwd": 44 * N + 28 * npix + 4 * P,
        "render_bwd": 48 * N + 24 * npix + 40 * P,
        "gauss_bwd": P * (44 + 12 * K + 24 + 40),
        "grad_write": grad_write_bytes(P, M),
    }


def workload_label(P, W, H, deg, world):
    """BASELINE.json config index of this run's workload, or 'custom'."""
    if world > 1:
        return "configs[3]" if (P, W, H, deg) == (1_000_000, 1920, 1080, 3) else "custom (multi-GPU)"
    return {(1_000_000, 1920, 1080, 3): "configs[2]", (200_000, 1920, 1080, 3): "configs[1]",
            (10_000, 640, 480, 0): "configs[0] (on the GPU)"}.get((P, W, H, deg), "custom")


def n_contrib_sum(img_buffer, W, H):
    """Sum over pixels of n_contrib (pairs walked), from the image state buffer."""
    def a256(x):
        return (x + 255) & ~255
    ntile = ((W + TILE - 1) // TILE) * ((H + TILE - 1) // TILE)
    # ImageLayout (csrc/wgsr_common.h): ranges, tile_len, tile_m, order_bwd,
    # meta, final_T, n_contrib -- each region 256-byte aligned
    off = 0
    for nbytes in (8 * ntile, 4 * ntile, 16 * ntile, 4 * ntile, 16, 4 * W * H):
        off += a256(nbytes)
    nc = img_buffer[off: off + 4 * W * H].view(torch.int32)
    return int(nc.sum().item())


def load_pmc(P, W, H, sh):
    """The committed PMC summary (profiles/pmc_summary*.json) taken on this
    workload, else None: counters are never quoted across configs."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_summary*.json"))):
        try:
            d = json.load(open(path))
        except Exception:
            continue
        if d.get("config") == {"P": P, "W": W, "H": H, "sh": sh}:
            return d
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--P", type=int, default=1_000_000)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--sh", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="CPU baseline sample: repeat the CPU step until this many seconds have passed")
    ap.add_argument("--no-profile", action="store_true", help="skip the stage timers")
    ap.add_argument("--no-knn", action="store_true", help="skip the distCUDA2 measurement (rocprof runs)")
    ap.add_argument("--dp-exchange", choices=("views", "views-dense", "allreduce"), default=None,
                    help="N > 1 gradient exchange: 'views' (default: screen-space records to the "
                         "Gaussians' owners, owner-computed shards all-gathered, only rows with "
                         "non-zero gradient moved; wgsr.dp.ViewShardedBackward), 'views-dense' (the "
                         "same with every row moved) or 'allreduce' (59-float gradient all-reduce). "
                         "Giving it at N = 1 runs that path on one GPU.")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal knobs for the N > 1 code path on a one-GPU box (never used by
    # the driver): WGSR_BENCH_BACKEND=gloo, WGSR_BENCH_SHARE_GPU=1 (all ranks
    # on cuda:0; wgsr.dp stages gloo collectives through host memory)
    backend = os.environ.get("WGSR_BENCH_BACKEND", "nccl")
    if os.environ.get("WGSR_BENCH_SHARE_GPU") == "1":
        local_rank = 0
    ctrl = None
    if world > 1:
        from datetime import timedelta
        # a hung collective ends the run (watchdog timeout -> non-zero exit)
        # instead of holding the node; the gloo control group decides the
        # exchange fallback even when an RCCL collective failed
        tmo = timedelta(seconds=float(os.environ.get("WGSR_BENCH_PG_TIMEOUT", "300")))
        torch.cuda.set_device(local_rank)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank), timeout=tmo)
        else:
            dist.init_process_group(backend, timeout=tmo)
        ctrl = dist.new_group(backend="gloo", timeout=tmo)
    dev = torch.device("cuda", local_rank)

    from diff_gaussian_rasterization import _C
    from wgsr import _lib
    from wgsr.camera import synthetic_camera
    from wgsr.dp import GradBuffer, ViewShardedBackward, allreduce_grads
    from wgsr.scene import make_scene, make_upstream_grads

    P, W, H, deg = args.P, args.width, args.height, args.sh
    M = (deg + 1) ** 2
    scene = make_scene(P, W, H, deg, seed=0)
    gc_cpu, gd_cpu = make_upstream_grads(W, H, seed=1)
    cam = synthetic_camera(W, H, view=rank)  # configs[3]: view k per rank
    f = cam.raster_fields()
    bg_cpu = torch.zeros(3)
    d = lambda x: x.to(dev).contiguous()  # noqa: E731
    means, opac, scales, rots, shs = (d(scene.means3D), d(scene.opacities), d(scene.scales),
                                      d(scene.rotations), d(scene.shs))
    bg, view, proj, praw, campos = (d(bg_cpu), d(f["viewmatrix"]), d(f["projmatrix"]),
                                    d(f["projmatrix_raw"]), d(f["campos"]))
    gc, gd = d(gc_cpu), d(gd_cpu)
    e = torch.empty(0, device=dev)
    tanx, tany = f["tanfovx"], f["tanfovy"]
    gbuf = GradBuffer.allocate(P, M, dev)
    exchange = args.dp_exchange or ("views" if world > 1 else None)
    vsb = (ViewShardedBackward(P, M, dev, sparse=(exchange == "views"))
           if exchange in ("views", "views-dense") else None)
    camd = dict(viewmatrix=view, projmatrix=proj, projmatrix_raw=praw, campos=campos, tanfovx=tanx,
                tanfovy=tany, bg=bg)
    state = {}

    def step():
        nr, color, radii, geom, binning, img, depth, opacity, nt = _C.rasterize_gaussians(
            bg, means, e, opac, scales, rots, 1.0, e, view, proj, praw, tanx, tany, H, W, shs, deg,
            campos, False, False)
        if vsb is not None:
            vsb.backward((means, scales, rots, shs, deg, camd, nr, radii, geom, binning, img), gc, gd)
            state.update(nr=nr, color=color, img=img)
            return
        _C.rasterize_gaussians_backward(
            bg, means, radii, e, scales, rots, 1.0, e, view, proj, praw, tanx, tany, gc, gd, shs,
            deg, campos, geom, nr, binning, img, False, out=gbuf.views)
        if world > 1:
            allreduce_grads(gbuf)
        state.update(nr=nr, color=color, img=img)

    exchange_check = None
    if vsb is not None:
        # the views exchange's summed gradients against the plain backward +
        # RCCL all-reduce of the same views, once before warm-up and timing.  Every rank
        # falls back to the all-reduce exchange if any rank disagrees OR any
        # rank's exchange raised (decided over the gloo control group, which
        # does not depend on RCCL); if the all-reduce itself fails the run
        # exits non-zero.
        err, reason = float("inf"), None
        try:
            nr, color, radii, geom, binning, img, depth, opacity, nt = _C.rasterize_gaussians(
                bg, means, e, opac, scales, rots, 1.0, e, view, proj, praw, tanx, tany, H, W, shs, deg,
                campos, False, False)
            got, _, _ = vsb.backward((means, scales, rots, shs, deg, camd, nr, radii, geom, binning, img), gc, gd)
            ref = GradBuffer.allocate(P, M, dev)
            _C.rasterize_gaussians_backward(
                bg, means, radii, e, scales, rots, 1.0, e, view, proj, praw, tanx, tany, gc, gd, shs,
                deg, campos, geom, nr, binning, img, False, out=ref.views)
            if world > 1:
                allreduce_grads(ref)
            err = 0.0
            for k, v in ref.views.items():
                den = float(v.abs().sum())
                err = max(err, float((got[k] - v).abs().sum()) / max(den, 1e-30))
            del ref
            torch.cuda.synchronize()
        except Exception as ex:  # noqa: BLE001 -- any failure of the exchange: fall back
            reason = f"{type(ex).__name__}: {ex}"[:400]
        ok = torch.tensor([1.0 if (reason is None and err <= 1e-5) else 0.0], dtype=torch.float64)
        if world > 1:
            dist.all_reduce(ok, op=dist.ReduceOp.MIN, group=ctrl)
        exchange_check = {"rel_l1_vs_allreduce": err, "ok": bool(ok.item() > 0.5)}
        if reason is not None:
            exchange_check["error"] = reason
        if not exchange_check["ok"]:
            exchange, vsb = "allreduce", None
            exchange_check["fallback"] = "allreduce"
            try:  # the fallback's own collective must work, else stop here
                allreduce_grads(gbuf)
                torch.cuda.synchronize()
            except Exception as ex:  # noqa: BLE001
                print(json.dumps({"error": f"all-reduce fallback failed: {type(ex).__name__}: {ex}"[:600],
                                  "exchange_check": exchange_check}), file=sys.stderr)
                sys.exit(1)

    # warm-up AFTER the exchange check: an exchange that raises must reach the
    # fallback, not end the run inside an untimed step
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    # per-stage breakdown first, in untimed steps (HIP events around every
    # stage: each pair serialises the stream, ~2-3 us a stage); the timed
    # loop then brackets only the dominant stage, for the roofline's launch
    # duration measured over the timed region itself
    breakdown, dom_stage = None, None
    if not args.no_profile:
        with _lib.StageProfile() as bp:
            for _ in range(min(args.steps, 10)):
                step()
            torch.cuda.synchronize()
        n_bd = min(args.steps, 10)
        breakdown = {k: (v[0] / n_bd, v[1]) for k, v in bp.stages.items() if v[1]}
        cand = {k: v for k, v in breakdown.items() if k != "dist_cuda2"}
        dom_stage = max(cand, key=lambda k: cand[k][0]) if cand else None
    prof = _lib.StageProfile([dom_stage]) if dom_stage else None
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    if prof:
        prof.__enter__()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    if prof:
        prof.__exit__(None, None, None)
    dt = t1 - t0
    if world > 1:
        t = torch.tensor([dt], device=dev if backend == "nccl" else "cpu", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    value = P * world * args.steps / dt
    label = workload_label(P, W, H, deg, world)
    ms_per_step = 1e3 * dt / args.steps
    N = state["nr"]
    out = {
        "metric": METRIC, "value": value, "unit": "Gaussians/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms_per_step,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic", "build": _lib.load().wgsr_version().decode(),
        "config": {
            "workload": (f"{label}: {P} Gaussians, {W}x{H}, SH{deg}, single-view fwd+bwd, pose grad on"
                         if world == 1 else
                         f"{label}: {P} Gaussians x {world} keyframe views (one per GPU), fwd+bwd "
                         "+ the SUM over views of the per-Gaussian gradients on every rank "
                         f"(RCCL, exchange: {exchange})"),
            "gaussians": P, "image": f"{W}x{H}", "sh_degree": deg, "num_rendered": N,
            "views_per_step": world, "parallelism": f"dp{world} (keyframe views)",
            "dp_exchange": exchange or "none",
            "exchange_bytes_per_rank_per_step": (
                0 if world == 1 else
                int(2 * (world - 1) / world * gbuf.flat.numel() * 4) if exchange == "allreduce" else
                vsb.last_exchange["bytes_in"] if vsb.last_exchange is not None else
                int((world - 1) / world * vsb.P_pad * (12 + gbuf.floats_per_gaussian) * 4)),
        },
    }

    if exchange_check is not None:
        out["config"]["exchange_check"] = exchange_check
    if vsb is not None and vsb.last_exchange is not None:
        out["config"]["sparse_exchange"] = {
            "record_rows_in": vsb.last_exchange["record_rows_in"],
            "grad_rows_per_owner": vsb.last_exchange["grad_rows_per_owner"],
            "note": "rows of Gaussians with zero gradient in every view are exactly zero and stay home"}

    if prof:
        model = byte_model(P, N, W, H, M, M)
        # stage times per step from the untimed breakdown steps; the dominant
        # stage's from the timed loop
        out["stages_ms_per_step"] = {k: v[0] for k, v in breakdown.items()}
        out["stages_note"] = ("per-stage device time (HIP events) from untimed steps before the timed loop; "
                              f"the timed loop brackets only {dom_stage}")
        timed = {k: (v[0] * args.steps, v[1] * args.steps // max(1, min(args.steps, 10)))
                 for k, v in breakdown.items() if k in model}
        dom = dom_stage
        td = prof.stages.get(dom, (0.0, 0))
        timed[dom] = td
        ms_avg = td[0] / max(1, td[1])
        achieved = model[dom] / (ms_avg * 1e-3) / 1e9
        pmc = load_pmc(P, W, H, deg) if world == 1 else None
        pst = pmc["stages"] if pmc else {}
        traffic = pst.get(dom, {}).get("hbm_bytes_per_step") if pmc else None
        out["roofline"] = {"kernel": dom, "bound": "hbm", "achieved": achieved,
                           "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBPS,
                           "traffic": traffic, "algorithmic_bytes": model[dom],
                           "avg_launch_ms": ms_avg}
        if dom == "render_bwd":
            # the same launch also streams the gradient outputs' zero fill
            zb = model[dom] + model["grad_write"]
            out["roofline"]["algorithmic_bytes_incl_zero_fill"] = zb
            out["roofline"]["frac_incl_zero_fill"] = zb / (ms_avg * 1e-3) / 1e9 / HBM_PEAK_GBPS
        if traffic is not None:
            out["roofline"]["traffic_source"] = pmc.get("source")
        if pmc:
            # the counters are quoted only with the build they were taken on named
            # (the "src:" digest of wgsr_version())
            src = out["build"].split("src:")[-1]
            out["roofline"]["counters_from_this_build"] = src in str(pmc.get("source", ""))
        # whole fwd+bwd pass against HBM (the north-star roofline) over the
        # timed step; the render kernels' pair arithmetic against the fp32 VALU peak
        total_bytes = sum(model.values())
        pairs = n_contrib_sum(state["img"], W, H)
        out["pass_roofline"] = {
            "algorithmic_bytes": total_bytes,
            "achieved_GBps_step": total_bytes / (ms_per_step * 1e-3) / 1e9,
            "frac_step": total_bytes / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBPS}
        if pmc:
            # what the kernels actually moved (PMC HBM bytes of this workload),
            # per step, beside the algorithmic figure
            cb = {k: v["hbm_bytes_per_step"] for k, v in pst.items() if k in model}
            out["pass_roofline"]["counter_bytes"] = sum(cb.values())
            out["pass_roofline"]["counter_bytes_by_stage"] = cb
            out["pass_roofline"]["frac_step_counter"] = (sum(cb.values()) / (ms_per_step * 1e-3) / 1e9
                                                         / HBM_PEAK_GBPS)
            out["pass_roofline"]["counter_source"] = pmc.get("source")
        rf = timed.get("render_fwd", (0, 1))
        rb = timed.get("render_bwd", (0, 1))
        out["render_valu"] = {
            "pairs_walked": pairs,
            "fwd_TFLOPs": 20 * pairs / (rf[0] / rf[1] * 1e-3) / 1e12 if rf[0] else None,
            "bwd_TFLOPs": 60 * pairs / (rb[0] / rb[1] * 1e-3) / 1e12 if rb[0] else None,
            "peak_TFLOPs": VALU_PEAK_TFLOPS}
        # the render kernels' actual bound: VALU issue.  Wave-level VALU
        # instructions per step (rocprofv3 SQ_INSTS_VALU of THIS workload,
        # profiles/pmc_summary.json) over the live per-step stage time,
        # against 1 wave-instruction / 4 cycles / SIMD.  This is the primary
        # roofline of the two render kernels; their HBM fraction is not.
        issue = {}
        for st in ("render_fwd", "render_bwd"):
            rec = pst.get(st)
            t = timed.get(st)
            if rec and rec.get("valu_insts_per_step") and t and t[0]:
                rate = rec["valu_insts_per_step"] / (t[0] / max(1, args.steps) * 1e-3)
                issue[st] = {"valu_wave_insts_per_step": rec["valu_insts_per_step"],
                             "achieved_Ginst_s": rate / 1e9, "peak_Ginst_s": VALU_ISSUE_PEAK / 1e9,
                             "frac": rate / VALU_ISSUE_PEAK}
        # VALU pipe occupancy measured by the counters (SQ_ACTIVE_INST_VALU
        # quad-cycles incl. 8-cycle ops over SQ_BUSY_CYCLES: at the clock the
        # kernel actually ran, tools/pmc_summary.py)
        for st in ("render_fwd", "render_bwd"):
            rec = pst.get(st)
            if rec and rec.get("valu_busy_frac") is not None:
                issue.setdefault(st, {})
                issue[st]["valu_busy_frac_counters"] = rec["valu_busy_frac"]
                issue[st]["clock_ghz_counters"] = rec.get("clock_ghz")
        if issue:
            out["render_valu_issue"] = issue
            if dom in issue:
                if "frac" in issue[dom]:
                    out["roofline"]["valu_issue_frac"] = issue[dom]["frac"]
                if "valu_busy_frac_counters" in issue[dom]:
                    out["roofline"]["valu_busy_frac"] = issue[dom]["valu_busy_frac_counters"]
                    out["roofline"]["clock_ghz"] = issue[dom]["clock_ghz_counters"]
                vb = issue[dom].get("valu_busy_frac_counters")
                if vb is not None and vb >= 0.85:
                    out["roofline"]["bound"] = "valu"
                what = ("VALU-issue bound" if (vb is not None and vb >= 0.85) else
                        "issue-latency bound at this size (too few waves per SIMD to keep the VALU busy)")
                out["roofline"]["bound_note"] = (
                    f"{dom} is {what}: valu_busy_frac (the VALU pipe's busy share of the kernel's "
                    "SQ clocks, PMC) is its primary roofline; valu_issue_frac = wave-instructions per second "
                    "against 1 per 4 cycles per SIMD at 2.4 GHz; frac is its HBM fraction over SURVEY 8(d)'s "
                    "bytes for the kernel (48N + 24 Npix + 40P), frac_incl_zero_fill adds the gradient "
                    "outputs' zero fill it also streams")

    if rank == 0 and world == 1 and not args.no_knn:
        # simple_knn.distCUDA2 over the scene's points
        # (outside the timed region; device time per call, HIP events)
        from simple_knn._C import distCUDA2
        for _ in range(3):
            d2 = distCUDA2(means)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        for _ in range(10):
            d2 = distCUDA2(means)
        ev1.record()
        torch.cuda.synchronize()
        out["distcuda2"] = {"points": P, "ms_per_call": ev0.elapsed_time(ev1) / 10,
                            "points_per_s": P / (ev0.elapsed_time(ev1) / 10 * 1e-3)}
        if not args.no_cpu_baseline:
            from oracle import cpu_oracle
            t0 = time.perf_counter()
            d2c = cpu_oracle.dist_knn(scene.means3D.numpy())
            tc = time.perf_counter() - t0
            out["distcuda2"]["cpu_baseline_ms"] = 1e3 * tc
            out["distcuda2"]["bitexact_vs_cpu"] = bool(np.array_equal(d2.cpu().numpy(), d2c))

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import cpu_oracle
        threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
        # bounded sample: whole fwd+bwd steps of the same workload until
        # args.cpu_seconds of CPU time have passed (at least one step)
        times = []
        while not times or (sum(times) < args.cpu_seconds and len(times) < 64):
            t0 = time.perf_counter()
            cr = cpu_oracle.CpuRaster(means3D=scene.means3D, opacities=scene.opacities, shs=scene.shs,
                                      scales=scene.scales, rotations=scene.rotations, H=H, W=W,
                                      tanfovx=tanx, tanfovy=tany, bg=bg_cpu, scale_modifier=1.0,
                                      viewmatrix=f["viewmatrix"], projmatrix=f["projmatrix"],
                                      projmatrix_raw=f["projmatrix_raw"], sh_degree=deg,
                                      campos=f["campos"])
            cr.backward(gc_cpu, gd_cpu)
            times.append(time.perf_counter() - t0)
        tc = sum(times) / len(times)
        out["cpu_baseline"] = {
            "value": P / tc, "unit": "Gaussians/s", "cores": threads, "kind": "port",
            "sample": f"{len(times)} full fwd+bwd steps of the same workload ({P} Gaussians, {W}x{H}, SH{deg}) "
                      f"on oracle/cpu_raster.cpp, {sum(times):.1f} s in total, {tc:.2f} s per step (mean)"}
        ref = torch.from_numpy(cr.color)
        mine = state["color"].detach().cpu()
        mse = float(((mine - ref) ** 2).mean())
        out["psnr_vs_cpu_db"] = (20 * math.log10(1.0 / math.sqrt(mse))) if mse > 0 else float("inf")
        out["rel_l1_vs_cpu"] = float((mine - ref).abs().sum() / ref.abs().sum())

    if rank == 0:
        print(json.dumps(out))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
