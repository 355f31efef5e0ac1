#!/usr/bin/env python
"""configs[4]-shaped online mapping run on synthetic keyframes (wgsr.online).

BASELINE.json configs[4] is the TUM fr3/walking_xyz end-to-end mapper loop;
the dataset, droid.pth and the Metric3D / DINOv2 weights are absent offline
(SURVEY.md 8(f) f4), so this runs the same mapper loop -- initialisation,
per-keyframe insertion (distCUDA2 point init), map_opt_online with the
uncertainty-aware loss, the DINO regulariser, densify / prune and the
opacity reset -- on keyframes rendered from a synthetic room at the product
operating point: 512x384, SH degree 0, TUM-like intrinsics.

Ground truth: a dense synthetic room (textured floor, ceiling and walls of
Gaussians) rendered by the same rasteriser from a camera trajectory; depth =
rendered depth / opacity where the opacity exceeds 0.5 (else invalid, 0);
features: a fixed random [h, w, 384] map per keyframe (h, w = H/14, W/14).

Prints one JSON line: ms per mapping iteration (wall clock over
map_opt_online, synchronised), ms per keyframe insertion (visibility render
+ window update + back-projection + distCUDA2 + append), the Gaussian count,
the densify / reset events and the PSNR of the final map's renders against
the keyframes' ground truth.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
for p in (os.path.join(ROOT, "wildgs-slam-blackwell_amd", "python"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402


def room(P, seed=0, dev="cuda"):
    """Gaussians on the inside of a 6 x 3 x 10 m box, textured."""
    g = torch.Generator().manual_seed(seed)
    face = torch.randint(0, 5, (P,), generator=g)
    a, b = torch.rand(P, generator=g), torch.rand(P, generator=g)
    x = torch.empty(P)
    y = torch.empty(P)
    z = torch.empty(P)
    # 0 floor (y = 1.5), 1 ceiling (y = -1.5), 2 back (z = 8), 3 left (x = -3), 4 right (x = 3)
    sel = face == 0
    x[sel], y[sel], z[sel] = -3 + 6 * a[sel], 1.5, -2 + 10 * b[sel]
    sel = face == 1
    x[sel], y[sel], z[sel] = -3 + 6 * a[sel], -1.5, -2 + 10 * b[sel]
    sel = face == 2
    x[sel], y[sel], z[sel] = -3 + 6 * a[sel], -1.5 + 3 * b[sel], 8.0
    sel = face == 3
    x[sel], y[sel], z[sel] = -3.0, -1.5 + 3 * a[sel], -2 + 10 * b[sel]
    sel = face == 4
    x[sel], y[sel], z[sel] = 3.0, -1.5 + 3 * a[sel], -2 + 10 * b[sel]
    xyz = torch.stack([x, y, z], 1)
    u, v = a * 8, b * 8
    col = torch.stack([0.5 + 0.4 * torch.sin(3.1 * u + face), 0.5 + 0.4 * torch.cos(2.3 * v + 2 * face),
                       0.5 + 0.4 * torch.sin(1.7 * (u + v))], 1)
    col = torch.where(((u.floor() + v.floor()) % 2 == 0)[:, None], col, col * 0.6)
    scales = torch.full((P, 3), 0.03)
    rots = torch.zeros(P, 4)
    rots[:, 0] = 1
    opac = torch.full((P, 1), 0.95)
    shs = ((col - 0.5) / 0.28209479177387814)[:, None, :]
    return [t.contiguous().to(dev) for t in (xyz, opac, scales, rots, shs)]


def pose(k):
    ang = math.radians(1.5 * k)
    c, s = math.cos(ang), math.sin(ang)
    R = torch.tensor([[c, 0.0, s], [0.0, 1.0, 0.0], [-s, 0.0, c]])
    T = torch.tensor([-0.08 * k, 0.0, 0.0])
    return R, T


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=512)
    ap.add_argument("--height", type=int, default=384)
    ap.add_argument("--keyframes", type=int, default=12)
    ap.add_argument("--init-keyframes", type=int, default=2)
    ap.add_argument("--init-iters", type=int, default=1050)
    ap.add_argument("--iters", type=int, default=450)
    ap.add_argument("--gt-gaussians", type=int, default=400_000)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--refine-iters", type=int, default=300, help="final_refine iterations after the last keyframe")
    ap.add_argument("--no-deform", action="store_true", help="skip the per-keyframe pose updates / map deformation")
    ap.add_argument("--phases", action="store_true", help="time the insertion / deformation phases (synchronised)")
    ap.add_argument("--dp", action="store_true",
                    help="data-parallel over keyframe views (wgsr.dp_online.DPOnlineMapper): launch with "
                         "torch.distributed.run, one rank per GPU (RCCL); WGSR_BENCH_BACKEND=gloo and "
                         "WGSR_BENCH_SHARE_GPU=1 rehearse it with every rank on cuda:0")
    a = ap.parse_args()
    from diff_gaussian_rasterization import _C
    from wgsr.camera import PinholeCamera
    from wgsr.online import Keyframe, OnlineMapper

    world, rank, local_rank = (int(os.environ.get(k, d)) for k, d in (("WORLD_SIZE", "1"), ("RANK", "0"),
                                                                       ("LOCAL_RANK", "0")))
    if os.environ.get("WGSR_BENCH_SHARE_GPU") == "1":
        local_rank = 0
    if a.dp:
        import torch.distributed as dist
        backend = os.environ.get("WGSR_BENCH_BACKEND", "nccl")
        torch.cuda.set_device(local_rank)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local_rank)
    W, H = a.width, a.height
    fx = fy = 517.3 * W / 512.0
    cx, cy = W / 2.0, H / 2.0
    gt = room(a.gt_gaussians, dev=dev)
    e = torch.empty(0, device=dev)
    kfs = []
    g = torch.Generator().manual_seed(a.seed + 1)
    for k in range(a.keyframes):
        R, T = pose(k)
        f = PinholeCamera(R=R, T=T, fx=fx, fy=fy, cx=cx, cy=cy, W=W, H=H).raster_fields()
        d = {kk: (v.to(dev) if torch.is_tensor(v) else v) for kk, v in f.items()}
        out = _C.rasterize_gaussians(torch.zeros(3, device=dev), gt[0], e, gt[1], gt[2], gt[3], 1.0, e,
                                     d["viewmatrix"], d["projmatrix"], d["projmatrix_raw"], d["tanfovx"],
                                     d["tanfovy"], H, W, gt[4], 0, d["campos"], False, False)
        img, depth, opac = out[1], out[6], out[7]
        dep = torch.where(opac > 0.5, depth / opac.clamp_min(1e-6), torch.zeros_like(depth))
        feats = torch.randn(H // 14, W // 14, 384, generator=g).to(dev)
        kfs.append(Keyframe(k, R, T, fx, fy, cx, cy, img.clamp(0, 1).contiguous(), dep.contiguous(), feats))
    torch.cuda.synchronize()

    if a.dp:
        from wgsr.dp_online import DPOnlineMapper
        m = DPOnlineMapper(sh_degree=0, device=dev, seed=a.seed)
    else:
        m = OnlineMapper(sh_degree=0, device=dev, seed=a.seed)
    t0 = time.perf_counter()
    m.initialize(kfs[:a.init_keyframes], iters=a.init_iters)
    torch.cuda.synchronize()
    t_init = time.perf_counter() - t0
    if a.phases:
        m.phase_ms = {}
    ins_ms, it_ms, its = [], 0.0, 0
    deform_ms, deform_kfs = [], 0

    def nudge(k, scale):
        """a small pose correction of keyframe k (the tracker's BA / loop
        closure moving existing keyframes): rotation about y, translation"""
        kfk = m.keyframes[k]
        ang = math.radians(0.05 * scale)
        c, s_ = math.cos(ang), math.sin(ang)
        dR = torch.tensor([[c, 0.0, s_], [0.0, 1.0, 0.0], [-s_, 0.0, c]])
        w2c = kfk.w2c().clone()
        w2c[:3, :3] = dR @ w2c[:3, :3]
        w2c[:3, 3] += torch.tensor([0.002 * scale, -0.001 * scale, 0.0])
        return w2c

    for n_kf, kf in enumerate(kfs[a.init_keyframes:]):
        torch.cuda.synchronize()
        if not a.no_deform:
            # _update_keyframes_from_frontend before the insertion (mapper.py:194):
            # every existing keyframe's pose moved a little, its Gaussians deformed
            # (the tracker's new poses, formed outside the timed call)
            upd = {k: (nudge(k, 1.0 + 0.1 * n_kf), None) for k in list(m.keyframes)}
            t0 = time.perf_counter()
            moved = m.update_keyframes(upd)
            torch.cuda.synchronize()
            deform_ms.append(1e3 * (time.perf_counter() - t0))
            deform_kfs += moved
        t0 = time.perf_counter()
        m.prepare_keyframe(kf)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        split = m.map_opt_online(m.window, a.iters)
        n = a.iters
        if split:
            m.map_opt_online(m.window, 1)
            n += 1
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        ins_ms.append(1e3 * (t1 - t0))
        it_ms += 1e3 * (t2 - t1)
        its += n
    # final_refine (mapper.py:1234-1372) after the final pose update of every keyframe
    refine_ms = None
    if a.refine_iters > 0:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if not a.no_deform:
            m.update_keyframes({k: (nudge(k, 2.0), None) for k in list(m.keyframes)})
        m.final_refine(a.refine_iters)
        torch.cuda.synchronize()
        refine_ms = 1e3 * (time.perf_counter() - t0) / a.refine_iters
    dp = None
    if a.dp:
        # the slowest rank's loop time; views per second over all ranks
        t = torch.tensor([it_ms], dtype=torch.float64, device=dev if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        it_ms = float(t.item())
        gst = m.graphs.stats if m.graphs is not None else {}
        dp = {"world": world, "backend": dist.get_backend(), "shared_gpu": os.environ.get("WGSR_BENCH_SHARE_GPU") == "1",
              "views_per_s": world * its / max(it_ms * 1e-3, 1e-12),
              "allreduce_ms_per_replay": 1e3 * gst.get("allreduce_s", 0.0) / max(1, gst.get("replays", 0)),
              "allreduce_bytes_per_iteration": 4 * (m.ms.store.grad_flat().numel()
                                                    + (m.graphs.tail.numel() if m.graphs is not None
                                                       and m.graphs.tail is not None else 0)),
              "replica_digest_equal": None}
        dg = m.replica_digest().cpu()
        dp["replica_digest_equal"] = bool((dg == dg[0]).all())
    # PSNR of the final map against every keyframe's ground truth
    ps = []
    for kf in kfs:
        img, _ = m.render_image(kf)
        mse = float(((img.clamp(0, 1) - kf.image) ** 2).mean())
        ps.append(10 * math.log10(1.0 / max(mse, 1e-12)))
    if rank != 0:
        if a.dp:
            dist.barrier()
            dist.destroy_process_group()
        return
    print(json.dumps({
        "dp": dp,
        "workload": f"configs[4]-shaped online mapping: synthetic room, {W}x{H}, SH0, {a.keyframes} keyframes "
                    f"({a.init_keyframes} init x {a.init_iters} its, then {a.iters} its per keyframe)",
        "ms_per_mapping_iteration": it_ms / max(its, 1), "mapping_iterations": its,
        "ms_per_keyframe_insertion": sum(ins_ms) / max(len(ins_ms), 1),
        "ms_per_deformation_call": (sum(deform_ms) / len(deform_ms)) if deform_ms else None,
        "keyframes_deformed_per_call": (deform_kfs / len(deform_ms)) if deform_ms else None,
        "final_refine_iterations": a.refine_iters, "ms_per_final_refine_iteration": refine_ms,
        "init_seconds": t_init, "gaussians_final": m.ms.P,
        "phase_ms_mean": ({k: sum(v) / len(v) for k, v in m.phase_ms.items()} if m.phase_ms is not None else None),
        "phase_ms": ({k: [round(x, 3) for x in v] for k, v in m.phase_ms.items()} if m.phase_ms is not None
                     else None),
        "ms_keyframe_insertion_median": (sorted(ins_ms)[len(ins_ms) // 2] if ins_ms else None),
        "ms_deformation_call_median": (sorted(deform_ms)[len(deform_ms) // 2] if deform_ms else None),
        "ms_keyframe_insertion_each": [round(x, 3) for x in ins_ms],
        "ms_deformation_call_each": [round(x, 3) for x in deform_ms],
        "events": [(i, k, v) for i, k, v in m.events][:40],
        "psnr_db_mean": sum(ps) / len(ps), "psnr_db_per_keyframe": ps,
        "graph": (dict(m.graphs.stats, cap=m.graphs.cap, disabled=m.graphs.disabled) if m.graphs is not None
                  and os.environ.get("WGSR_ONLINE_GRAPH", "1") != "0" else None),
        "note": "uncertainty-aware loss + DINO regulariser + isotropic term, densify/prune, opacity reset, "
                "Adam (Gaussians, exposures, MLP); before every insertion each existing keyframe's pose is "
                "nudged and its Gaussians deformed (update_keyframes, one device pass); final_refine at the "
                "end; wall clock with a device sync per keyframe"}))
    if a.dp:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
