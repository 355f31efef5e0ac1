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
    # persistent accumulators with earlier steps' totals (identical on every
    # rank, as after a previous reduction): only this step's deltas travel
    prior = torch.arange(P, dtype=torch.float32)[:, None] * 0.5
    acc_total, den_total, rmax_total = prior.clone(), prior.clone() + 3, torch.full((P,), 2.0)
    reduce_densification_stats(accum, denom, radii, acc_total, den_total, rmax_total)
    torch.save({"flat": buf.flat, "accum": accum, "denom": denom, "radii": radii, "acc_total": acc_total,
                "den_total": den_total, "rmax_total": rmax_total},
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
    prior = torch.arange(P, dtype=torch.float32) * 0.5
    for o in outs:  # accumulators = earlier totals + this step's reduced deltas, counted once
        assert torch.allclose(o["acc_total"][:, 0], prior + acc, rtol=1e-6, atol=1e-6)
        assert torch.equal(o["den_total"][:, 0], prior + 3 + outs[0]["denom"][:, 0])
        assert torch.equal(o["rmax_total"], torch.maximum(rmax, torch.full((P,), 2.0)))


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


# ---- view-sharded backward: exchange plumbing (gloo, CPU) ----------------
# The HIP kernels need a GPU (their math is pinned in tests/test_gpu_dp.py);
# here a linear stand-in with the same interface checks that every view's
# records reach the right owner in view order, that the owners' shards are
# gathered into place (ragged P: padding rows), and the pose / statistics
# reductions.  Stand-in: view v's record of Gaussian i is rec(v, i); the
# owner's "backward" of view v scales it by (camera id + 1).
VP, VM = 37, 4


def _mock_rec(view, P_pad):
    i = torch.arange(P_pad, dtype=torch.float32)[:, None]
    k = torch.arange(12, dtype=torch.float32)[None, :]
    r = torch.sin(i * 1.3 + k * 0.7 + view * 2.1)
    r[:, 10] = ((torch.arange(P_pad) + view) % 3).float()  # radius 0 -> not visible
    # visible but no gradient (every pixel saturated before it): an all-zero
    # record apart from the radius -- the rows the sparse exchange skips
    # (views >= 100 have none: their rows must be cleared again afterwards)
    i = torch.arange(P_pad)
    quiet = (((i + view) % 4 == 1) | (i % 4 == 0)) & (view < 100)
    r[quiet, :10] = 0
    r[quiet, 11] = 0
    r[VP:] = 0
    return r


class _MockKernels:
    def pack_camera(self, cam, W, H, out_row):
        out_row.zero_()
        out_row[0] = float(cam["id"])

    def records(self, fwd, dL_dcolor, dL_ddepth, P_pad, out):
        out.copy_(_mock_rec(fwd[5]["id"], P_pad))

    def tau_blocks(self, lo, hi):
        return -(-(hi - lo) // 5) if hi > lo else 0

    def gauss_views(self, params, lo, hi, cams, recs, grads, tau_out, stats_out):
        n = hi - lo
        for name, t in grads.items():
            t[lo:hi] = 0
        if stats_out is not None:
            stats_out.zero_()  # the kernel writes the statistics, it does not accumulate
        for v in range(cams.size(0)):
            r = recs[v, :n]
            s = cams[v, 0] + 1
            vis = r[:, 10] > 0
            w = torch.where(vis, s, torch.zeros(()))[:, None]
            grads["means3D"][lo:hi] += w * r[:, 0:3]
            grads["shs"][lo:hi, 0] += w * r[:, 3:6]
            grads["opacities"][lo:hi] += w * r[:, 6:7]
            grads["scales"][lo:hi] += w * r[:, 7:10]
            grads["rotations"][lo:hi] += w * torch.cat([r[:, 0:3], r[:, 11:12]], 1)
            if tau_out is not None:
                for b in range(tau_out.size(0)):
                    seg = slice(5 * b, min(n, 5 * b + 5))
                    tau_out[b, v] = (w[seg] * r[seg, 0:6]).sum(0)
            if stats_out is not None:
                stats_out[:, 0] += torch.where(vis, r[:, 0:2].norm(dim=1), torch.zeros(()))
                stats_out[:, 1] += vis.float()
                stats_out[:, 2] = torch.maximum(stats_out[:, 2], r[:, 10])


    # sparse exchange stand-ins (csrc/dp_sparse.hip semantics; packed rows
    # in reverse order: the device order is unspecified)
    def grad_row_floats(self, M):
        return 12 + 3 * M

    def mask_words(self, S):
        return (S + 31) // 32

    def summary_block_words(self, world, S):
        return 64 + world + world * self.mask_words(S)

    def sparse_pack_records(self, send, S, counts, packed, nzmask):
        W32 = self.mask_words(S)
        for o in range(send.size(0) // S):
            seg = send[o * S:(o + 1) * S]
            idx = (seg[:, :10] != 0).any(1).nonzero().flatten()
            rows = seg[idx].clone()
            rows[:, 10] = idx.to(torch.int32).view(torch.float32)
            packed[o * S:o * S + idx.numel()] = rows.flip(0)
            counts[o] = idx.numel()
            words = [0] * W32
            for j in idx.tolist():
                words[j // 32] |= 1 << (j % 32)
            nzmask[o * W32:(o + 1) * W32] = torch.tensor([w - (1 << 32) if w >= 1 << 31 else w for w in words],
                                                         dtype=torch.int32)

    def sparse_exchange_summary(self, blocks, world, rank, S, summary, offsets, cams):
        W32 = self.mask_words(S)
        b = blocks.long() & 0xFFFFFFFF
        for o in range(world):
            acc = [0] * W32
            for v in range(world):
                for w in range(W32):
                    acc[w] |= int(b[v, 64 + world + o * W32 + w])
            summary[world * world + o] = sum(bin(a).count("1") for a in acc)
        summary[:world * world] = blocks[:, 64:64 + world].reshape(-1)
        cams.copy_(blocks[:, :64].contiguous().view(torch.float32))
        col = blocks[:, 64 + rank].long()
        offsets[0] = 0
        offsets[1:] = torch.cumsum(col, 0).to(torch.int32)

    def sparse_unpack_records(self, received, offsets, S, keep_radius, recv, mask):
        for v in range(recv.size(0)):
            rows = received[int(offsets[v]):int(offsets[v + 1])]
            idx = rows[:, 10].contiguous().view(torch.int32).long()
            rad = recv[v, idx, 10].clone() if keep_radius else torch.ones(idx.numel())
            recv[v, idx] = rows
            recv[v, idx, 10] = rad
            mask[idx] = 1

    def sparse_fill_radius(self, radii, recv):
        recv[:, 10] = radii

    def sparse_pack_grads(self, grads, lo, hi, mask, count, packed):
        n = hi - lo
        F = self.grad_row_floats(grads["shs"].size(1))
        idx = mask[:n].nonzero().flatten()
        rows = torch.cat([grads["means3D"][lo:hi], grads["shs"][lo:hi].reshape(n, -1), grads["opacities"][lo:hi],
                          grads["scales"][lo:hi], grads["rotations"][lo:hi]], 1)[idx].flip(0)
        out = packed[:idx.numel() * F].view(-1, F)
        out[:, 0] = idx.flip(0).to(torch.int32).view(torch.float32)
        out[:, 1:] = rows
        count[0] = idx.numel()

    def sparse_unpack_grads(self, gathered, block_stride, counts, rank, cap, S, P, grads, clear=False):
        M = grads["shs"].size(1)
        F = self.grad_row_floats(M)
        for r in range(counts.numel()):
            if r == rank:
                continue
            n = min(int(counts[r]), cap)
            rows = gathered[r * block_stride:r * block_stride + n * F].view(n, F)
            i = r * S + rows[:, 0].contiguous().view(torch.int32).long()
            z = 0.0 if clear else 1.0
            grads["means3D"][i] = rows[:, 1:4] * z
            grads["shs"][i] = rows[:, 4:4 + 3 * M].reshape(-1, M, 3) * z
            grads["opacities"][i] = rows[:, 4 + 3 * M:5 + 3 * M] * z
            grads["scales"][i] = rows[:, 5 + 3 * M:8 + 3 * M] * z
            grads["rotations"][i] = rows[:, 8 + 3 * M:12 + 3 * M] * z


def _mock_expected(world):
    P_pad = VP + 5
    out = {"means3D": torch.zeros(VP, 3), "shs": torch.zeros(VP, VM, 3), "opacities": torch.zeros(VP, 1),
           "scales": torch.zeros(VP, 3), "rotations": torch.zeros(VP, 4)}
    taus, st = [], torch.zeros(VP, 3)
    for v in range(world):
        r = _mock_rec(v, P_pad)[:VP]
        vis = r[:, 10] > 0
        w = torch.where(vis, torch.tensor(v + 1.0), torch.zeros(()))[:, None]
        out["means3D"] += w * r[:, 0:3]
        out["shs"][:, 0] += w * r[:, 3:6]
        out["opacities"] += w * r[:, 6:7]
        out["scales"] += w * r[:, 7:10]
        out["rotations"] += w * torch.cat([r[:, 0:3], r[:, 11:12]], 1)
        taus.append((w * r[:, 0:6]).sum(0))
        st[:, 0] += torch.where(vis, r[:, 0:2].norm(dim=1), torch.zeros(()))
        st[:, 1] += vis.float()
        st[:, 2] = torch.maximum(st[:, 2], r[:, 10])
    return out, taus, st


def _vsb_worker(rank, world, port, out_dir, sparse=True):
    import sys
    root = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
    for p in (os.path.join(root, "wildgs-slam-blackwell_amd", "python"), root):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from wgsr.dp import ViewShardedBackward
    vsb = ViewShardedBackward(VP, VM, "cpu", stats=True, kernels=_MockKernels(), sparse=sparse)
    assert vsb.sparse == sparse
    S = -(-VP // world)
    assert vsb.S == S and vsb.P_pad == S * world
    e = torch.zeros(3, 4, 5)
    fwd = (torch.zeros(VP, 3), None, None, None, 0, {"id": rank})
    for step in range(3):  # repeated steps reuse (and must re-zero) the buffers
        # a different view per step: the rows scattered by the previous step
        # must be cleared where this step has none
        fwd = (torch.zeros(VP, 3), None, None, None, 0, {"id": rank if step != 1 else 100 + rank})
        grads, tau, stats = vsb.backward(fwd, e, e[:1])
        if step == 0:
            first = {k: v.clone() for k, v in grads.items()}
    if sparse:
        # rows with a non-zero record only: a quarter of the visible rows stay home
        assert 0 < vsb.last_exchange["record_rows_in"] < (world - 1) * vsb.S
    for k, v in grads.items():  # step 3 = step 1's views again: the same sums
        assert torch.equal(v, first[k]), k
    assert (grads["means3D"][torch.arange(VP) % 4 == 0] == 0).all()  # step 2's extra rows cleared
    torch.save({"grads": {k: v.clone() for k, v in grads.items()}, "tau": tau.clone(), "stats": stats.clone()},
               os.path.join(out_dir, f"vsb{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("sparse", [True, False])
@pytest.mark.parametrize("world", [2, 3])
def test_view_sharded_exchange_routes_records_to_owners(tmp_path, sparse, world):
    mp.spawn(_vsb_worker, args=(world, _free_port(), str(tmp_path), sparse), nprocs=world, join=True)
    exp, taus, st = _mock_expected(world)
    for r in range(world):
        o = torch.load(tmp_path / f"vsb{r}.pt", weights_only=True)
        for k, t in exp.items():
            assert torch.allclose(o["grads"][k], t, rtol=1e-6, atol=1e-6), (r, k)
        assert torch.allclose(o["tau"], taus[r], rtol=1e-5, atol=1e-5)
        assert torch.allclose(o["stats"], st, rtol=1e-6, atol=1e-6)
