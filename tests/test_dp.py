"""Multi-process (world_size 2, gloo, CPU) tests of the keyframe-view
data-parallel path (wgsr.dp).

Invariant: the all-reduced gradient over V views equals the sum of the V
single-view gradients computed in one process (rel-L1 <= 1e-5).  The per-view
gradients come from the CPU restatement (the renderer itself needs a GPU; the
reduction plumbing does not).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

WORLD = 2
P, W, H, DEG = 300, 64, 48, 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _view_grads(view):
    from oracle import cpu_oracle
    from wgsr.camera import synthetic_camera
    from wgsr.scene import make_scene, make_upstream_grads
    sc = make_scene(P, W, H, DEG, seed=4)
    gc, gd = make_upstream_grads(W, H, seed=5 + view)
    f = synthetic_camera(W, H, view).raster_fields()
    cr = cpu_oracle.CpuRaster(means3D=sc.means3D, opacities=sc.opacities, shs=sc.shs,
                              scales=sc.scales, rotations=sc.rotations, H=H, W=W,
                              tanfovx=f["tanfovx"], tanfovy=f["tanfovy"], bg=torch.zeros(3),
                              scale_modifier=1.0, viewmatrix=f["viewmatrix"],
                              projmatrix=f["projmatrix"], projmatrix_raw=f["projmatrix_raw"],
                              sh_degree=DEG, campos=f["campos"])
    g = cr.backward(gc, gd)
    return {"means3D": g["dL_dmeans3D"], "shs": g["dL_dsh"], "opacities": g["dL_dopacity"],
            "scales": g["dL_dscales"], "rotations": g["dL_drotations"],
            "means2D": g["dL_dmeans2D"], "radii": cr.radii}


def _worker(rank, port, out_dir):
    import sys
    root = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
    for p in (os.path.join(root, "wildgs-slam-blackwell_amd", "python"), root):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    from wgsr.dp import GradBuffer, allreduce_grads, reduce_densification_stats, views_for_rank
    M = (DEG + 1) ** 2
    buf = GradBuffer.allocate(P, M, "cpu")
    buf.flat.zero_()
    for v in views_for_rank(WORLD, rank, WORLD):
        g = _view_grads(v)
        for k in buf.views:
            buf.views[k] += torch.from_numpy(g[k]).reshape(buf.views[k].shape)
    # tiny buckets: exercises the multi-bucket path
    allreduce_grads(buf, bucket_bytes=4096)
    g = _view_grads(rank)
    accum = torch.from_numpy(np.linalg.norm(g["means2D"][:, :2], axis=1)).float()[:, None]
    vis = torch.from_numpy(g["radii"] > 0)
    denom = vis.float()[:, None]
    radii = torch.from_numpy(g["radii"]).float()
    reduce_densification_stats(accum, denom, radii)
    torch.save({"flat": buf.flat, "accum": accum, "denom": denom, "radii": radii},
               os.path.join(out_dir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_allreduced_gradients_equal_sum_of_views(tmp_path):
    port = _free_port()
    mp.spawn(_worker, args=(port, str(tmp_path)), nprocs=WORLD, join=True)
    outs = [torch.load(tmp_path / f"rank{r}.pt", weights_only=True) for r in range(WORLD)]
    from wgsr.dp import GradBuffer
    M = (DEG + 1) ** 2
    ref = GradBuffer.allocate(P, M, "cpu")
    ref.flat.zero_()
    views = [_view_grads(v) for v in range(WORLD)]
    for g in views:
        for k in ref.views:
            ref.views[k] += torch.from_numpy(g[k]).reshape(ref.views[k].shape)
    for o in outs:
        got, exp = o["flat"].double(), ref.flat.double()
        assert float((got - exp).abs().sum() / exp.abs().sum()) <= 1e-5
        assert torch.equal(o["flat"], outs[0]["flat"])  # every rank holds the same result
    acc = sum(torch.from_numpy(np.linalg.norm(g["means2D"][:, :2], axis=1)).float() for g in views)
    assert torch.allclose(outs[0]["accum"][:, 0], acc, rtol=1e-6, atol=0)
    assert torch.equal(outs[0]["denom"][:, 0], sum(torch.from_numpy(g["radii"] > 0).float() for g in views))
    rmax = torch.maximum(*[torch.from_numpy(g["radii"]).float() for g in views])
    assert torch.equal(outs[0]["radii"], rmax)


def test_grad_buffer_layout_is_contiguous_views():
    from wgsr.dp import PARAM_ORDER, GradBuffer
    buf = GradBuffer.allocate(10, 16, "cpu")
    assert buf.floats_per_gaussian == 3 + 48 + 1 + 3 + 4 == 59
    off = 0
    for k in PARAM_ORDER:
        v = buf.views[k]
        assert v.is_contiguous() and v.data_ptr() == buf.flat.data_ptr() + 4 * off
        off += v.numel()
    assert off == buf.flat.numel()


def test_views_for_rank_round_robin():
    from wgsr.dp import views_for_rank
    assert views_for_rank(8, 3, 4) == [3, 7]
    all_views = sorted(v for r in range(3) for v in views_for_rank(8, r, 3))
    assert all_views == list(range(8))
