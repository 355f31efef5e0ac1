"""GPU parity of the view-sharded data-parallel backward (wgsr.dp,
SURVEY.md 8(e); include/wgsr.h wgsr_rasterize_backward_records /
wgsr_gauss_backward_views).

Invariant: for V views of one Gaussian set, the owner-computed shards summed
over views equal the SUM of the V single-view backwards of
_C.rasterize_gaussians_backward (which tests/test_gpu_raster.py pins to the
oracle): parameter gradients rel-L1 <= 1e-5 (fp32 summation order differs:
the kernel sums dL/dcov3D over views before the linear cov3D -> (scale,
rotation) step), each view's pose gradient rel-L1 <= 1e-4 (a sum over P in a
different order), densification statistics rel <= 1e-6 / exact.
"""
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

P, W, H, DEG, V = 3000, 128, 96, 3, 3


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).abs().sum() / b.abs().sum().clamp_min(1e-30))


def _setup(dev, nviews=V, P_=P):
    from wgsr.camera import synthetic_camera
    from wgsr.scene import make_scene, make_upstream_grads
    sc = make_scene(P_, W, H, DEG, seed=11)
    d = lambda x: x.to(dev).contiguous()  # noqa: E731
    params = dict(means3D=d(sc.means3D), opacities=d(sc.opacities), scales=d(sc.scales),
                  rotations=d(sc.rotations), shs=d(sc.shs))
    views = []
    for v in range(nviews):
        f = synthetic_camera(W, H, v).raster_fields()
        gc, gd = make_upstream_grads(W, H, seed=20 + v)
        cam = dict(viewmatrix=d(f["viewmatrix"]), projmatrix=d(f["projmatrix"]),
                   projmatrix_raw=d(f["projmatrix_raw"]), campos=d(f["campos"]),
                   tanfovx=f["tanfovx"], tanfovy=f["tanfovy"], bg=d(torch.tensor([0.1, 0.2, 0.3])))
        views.append((cam, d(gc), d(gd)))
    return params, views


def _forward(params, cam):
    from diff_gaussian_rasterization import _C
    e = torch.empty(0, device=params["means3D"].device)
    return _C.rasterize_gaussians(
        cam["bg"], params["means3D"], e, params["opacities"], params["scales"], params["rotations"], 1.0, e,
        cam["viewmatrix"], cam["projmatrix"], cam["projmatrix_raw"], cam["tanfovx"], cam["tanfovy"], H, W,
        params["shs"], DEG, cam["campos"], False, False)


def _reference(params, views):
    """Sum over views of the single-view backward + per-view pose gradient
    and densification statistics."""
    from diff_gaussian_rasterization import _C
    e = torch.empty(0, device=params["means3D"].device)
    keys = ("means3D", "shs", "opacities", "scales", "rotations")
    idx = {"means3D": 3, "shs": 5, "opacities": 2, "scales": 6, "rotations": 7}
    tot = {k: torch.zeros_like(params[k] if k != "opacities" else params["opacities"]) for k in keys}
    taus, norm, cnt, rmax = [], 0, 0, 0
    for cam, gc, gd in views:
        nr, color, radii, geom, binning, img, depth, opac, nt = _forward(params, cam)
        g = _C.rasterize_gaussians_backward(
            cam["bg"], params["means3D"], radii, e, params["scales"], params["rotations"], 1.0, e,
            cam["viewmatrix"], cam["projmatrix"], cam["projmatrix_raw"], cam["tanfovx"], cam["tanfovy"], gc,
            gd, params["shs"], DEG, cam["campos"], geom, nr, binning, img, False)
        for k in keys:
            tot[k] += g[idx[k]].view_as(tot[k])
        taus.append(g[8].double().sum(0))
        vis = radii > 0
        norm = norm + torch.where(vis, g[0][:, :2].norm(dim=1), torch.zeros_like(g[0][:, 0]))
        cnt = cnt + vis.float()
        rmax = torch.maximum(torch.as_tensor(rmax, device=radii.device).float(), radii.float())
    return tot, taus, (norm, cnt, rmax)


def _records(params, cam, gc, gd, P_pad):
    from wgsr.dp import _HipViewKernels
    nr, color, radii, geom, binning, img, depth, opac, nt = _forward(params, cam)
    out = torch.empty(P_pad, 12, device=params["means3D"].device)
    _HipViewKernels().records((params["means3D"], params["scales"], params["rotations"], params["shs"], DEG,
                               cam, nr, radii, geom, binning, img), gc, gd, P_pad, out)
    return out


@pytest.mark.parametrize("nshards", [1, 3, 4])
def test_sharded_views_equal_sum_of_single_view_backwards(nshards):
    from wgsr.dp import GradBuffer, _HipViewKernels
    dev = torch.device("cuda:0")
    params, views = _setup(dev)
    ref, taus, (rn, rc, rr) = _reference(params, views)
    k = _HipViewKernels()
    S = -(-P // nshards)
    P_pad = S * nshards
    recs = torch.stack([_records(params, cam, gc, gd, P_pad) for cam, gc, gd in views])  # [V, P_pad, 12]
    cams = torch.zeros(V, 64, device=dev)
    for v, (cam, _, _) in enumerate(views):
        k.pack_camera(cam, W, H, cams[v])
    buf = GradBuffer.allocate(P_pad, (DEG + 1) ** 2, dev)
    buf.flat.fill_(float("nan"))
    stats = torch.zeros(P_pad, 3, device=dev)
    tau = torch.zeros(V, 6, dtype=torch.float64, device=dev)
    for s in range(nshards):
        lo, hi = min(P, s * S), min(P, (s + 1) * S)
        shard = recs[:, s * S:(s + 1) * S].contiguous()  # what the all-to-all delivers to owner s
        nb = k.tau_blocks(lo, hi)
        tb = torch.zeros(max(nb, 1), V, 6, device=dev)
        k.gauss_views((params["means3D"], params["scales"], params["rotations"], params["shs"], DEG, 1.0),
                      lo, hi, cams, shard, buf.views, tb if hi > lo else None, stats[lo:hi])
        tau += tb.double().sum(0)
    torch.cuda.synchronize()
    for name in ("means3D", "shs", "opacities", "scales", "rotations"):
        got = buf.views[name][:P]
        assert torch.isfinite(got).all(), name
        r = _rel(got, ref[name].view_as(got))
        assert r <= 1e-5, (name, r)
    for v in range(V):
        r = _rel(tau[v], taus[v])
        assert r <= 1e-4, (v, r, tau[v], taus[v])
    assert _rel(stats[:P, 0], rn) <= 1e-6
    assert torch.equal(stats[:P, 1], rc)
    assert torch.equal(stats[:P, 2], rr)


def test_records_rows_of_culled_and_padding_are_zero():
    dev = torch.device("cuda:0")
    params, views = _setup(dev, nviews=1)
    cam, gc, gd = views[0]
    rec = _records(params, cam, gc, gd, P + 77)
    nr, color, radii, *_ = _forward(params, cam)
    torch.cuda.synchronize()
    culled = torch.cat([radii <= 0, torch.ones(77, dtype=torch.bool, device=dev)])
    assert culled[:P].any() and (~culled).any()
    assert torch.count_nonzero(rec[culled]) == 0
    assert torch.equal(rec[:P, 10][~culled[:P]], radii[~culled[:P]].float())


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank_main(rank, world, port, out_dir, sparse=True):
    import sys
    root = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
    for p in (os.path.join(root, "wildgs-slam-blackwell_amd", "python"), root):
        sys.path.insert(0, p)
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    # two ranks share the box's one GPU: gloo (device tensors staged through
    # host memory by wgsr.dp); on a node, "nccl" (RCCL) with one GPU per rank
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from wgsr.dp import ViewShardedBackward
    dev = torch.device("cuda:0")
    params, views = _setup(dev, nviews=world, P_=P + 1)  # P + 1: ragged shards
    cam, gc, gd = views[rank]
    nr, color, radii, geom, binning, img, depth, opac, nt = _forward(params, cam)
    vsb = ViewShardedBackward(P + 1, (DEG + 1) ** 2, dev, stats=True, sparse=sparse)
    fwd = (params["means3D"], params["scales"], params["rotations"], params["shs"], DEG, cam, nr, radii, geom,
           binning, img)
    for _ in range(2):  # repeated steps reuse the buffers
        grads, tau, stats = vsb.backward(fwd, gc, gd)
    torch.cuda.synchronize()
    torch.save({"grads": {k: v.cpu() for k, v in grads.items()}, "tau": tau.cpu(), "stats": stats.cpu()},
               os.path.join(out_dir, f"r{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("sparse", [True, False])
def test_two_ranks_gloo_match_sum_of_views(tmp_path, sparse):
    import torch.multiprocessing as mp
    world = 2
    mp.spawn(_rank_main, args=(world, _free_port(), str(tmp_path), sparse), nprocs=world, join=True)
    dev = torch.device("cuda:0")
    params, views = _setup(dev, nviews=world, P_=P + 1)
    ref, taus, (rn, rc, rr) = _reference(params, views)
    outs = [torch.load(tmp_path / f"r{r}.pt", weights_only=True) for r in range(world)]
    for r, o in enumerate(outs):
        for name, g in o["grads"].items():
            assert _rel(g, ref[name].view_as(g)) <= 1e-5, (r, name)
            assert torch.equal(g, outs[0]["grads"][name])
        assert _rel(o["tau"], taus[r]) <= 1e-4
        assert _rel(o["stats"][:, 0], rn) <= 1e-6
        assert torch.equal(o["stats"][:, 1], rc.cpu()) and torch.equal(o["stats"][:, 2], rr.cpu())


@pytest.mark.parametrize("world,S", [(3, 1000), (4, 777), (1, 64)])
def test_sparse_record_and_gradient_round_trip(world, S):
    """csrc/dp_sparse.hip: records packed per owner (+ non-zero row masks),
    the exchange summary of the gathered small blocks (count matrix, union row
    counts, receive offsets, camera table), records scattered back from one
    contiguous all_to_all-shaped buffer equal the dense records of the
    non-zero rows (radius kept or set to 1), the mask is their union, and
    packed gradient rows land at their indices -- and a clear pass puts zeros
    back at exactly those rows."""
    from wgsr.dp import GradBuffer, _HipViewKernels
    dev = torch.device("cuda:0")
    k = _HipViewKernels()
    g = torch.Generator().manual_seed(7)
    P_pad = world * S
    W32 = k.mask_words(S)
    BW = k.summary_block_words(world, S)
    assert W32 == (S + 31) // 32 and BW == 64 + world + world * W32
    views = []
    for v in range(world):
        r = torch.randn(P_pad, 12, generator=g)
        quiet = torch.rand(P_pad, generator=g) < 0.8  # most rows carry no gradient
        r[quiet, :10] = 0
        r[:, 10] = torch.randint(0, 5, (P_pad,), generator=g).float()
        views.append(r.to(dev))
    # every view (= rank) packs; the small blocks are "gathered" by stacking
    blocks = torch.zeros(world, BW, dtype=torch.int32, device=dev)
    packs = []
    for v, r in enumerate(views):
        blocks[v, :64] = (torch.arange(64, device=dev, dtype=torch.float32) + 100 * v).view(torch.int32)
        packed = torch.full((P_pad, 12), float("nan"), device=dev)
        k.sparse_pack_records(r, S, blocks[v, 64:64 + world], packed, blocks[v, 64 + world:])
        packs.append(packed)
        for o in range(world):
            seg = r[o * S:(o + 1) * S]
            assert int(blocks[v, 64 + o]) == int((seg[:, :10] != 0).any(1).sum())
    for owner in range(world):
        summary = torch.zeros(world * world + world, dtype=torch.int32, device=dev)
        offsets = torch.zeros(world + 1, dtype=torch.int32, device=dev)
        cams = torch.zeros(world, 64, device=dev)
        k.sparse_exchange_summary(blocks, world, owner, S, summary, offsets, cams)
        cnt = blocks[:, 64:64 + world].cpu()
        assert torch.equal(summary[:world * world].cpu().view(world, world), cnt)
        assert torch.equal(cams.view(torch.int32), blocks[:, :64])
        assert offsets.tolist() == [0] + torch.cumsum(cnt[:, owner], 0).tolist()
        for o in range(world):
            union = torch.zeros(S, dtype=torch.bool, device=dev)
            for r in views:
                union |= (r[o * S:(o + 1) * S, :10] != 0).any(1)
            assert int(summary[world * world + o]) == int(union.sum())
        # the owner's all_to_all output: view v's rows for this owner, contiguous
        received = torch.cat([packs[v][owner * S:owner * S + int(cnt[v, owner])] for v in range(world)])
        for keep_radius in (False, True):
            dense = torch.zeros(world, S, 12, device=dev)
            if keep_radius:
                k.sparse_fill_radius(torch.stack([r[owner * S:(owner + 1) * S, 10] for r in views]).reshape(-1),
                                     dense.view(-1, 12))
            mask = torch.zeros(S, dtype=torch.uint8, device=dev)
            k.sparse_unpack_records(received, offsets, S, keep_radius, dense, mask)
            union = torch.zeros(S, dtype=torch.bool, device=dev)
            for v, r in enumerate(views):
                seg = r[owner * S:(owner + 1) * S]
                nz = (seg[:, :10] != 0).any(1)
                union |= nz
                exp = torch.where(nz[:, None], seg, torch.zeros_like(seg))
                exp[:, 10] = seg[:, 10] if keep_radius else nz.float()
                assert torch.equal(dense[v], exp), (owner, v, keep_radius)
            assert torch.equal(mask.bool(), union)
    # gradient rows: every owner packs its masked rows into its block's row
    # region (after a `head` of other data), rank 0 unpacks the others
    M = 16
    src = GradBuffer.allocate(P_pad, M, dev)
    src.flat.copy_(torch.randn(src.flat.numel(), generator=g).to(dev))
    F = k.grad_row_floats(M)
    assert F == 12 + 3 * M
    head, cap = 7, S
    blk = head + cap * F
    masks = [(torch.rand(S, generator=g) < 0.3).to(torch.uint8).to(dev) for _ in range(world)]
    counts = torch.zeros(world, dtype=torch.int32, device=dev)
    gathered = torch.full((world, blk), float("nan"), device=dev)
    for r in range(world):
        c = torch.zeros(1, dtype=torch.int32, device=dev)
        k.sparse_pack_grads(src.views, r * S, (r + 1) * S, masks[r], c, gathered[r, head:])
        counts[r] = c[0]
        assert int(c[0]) == int(masks[r].sum())
    dst = GradBuffer.allocate(P_pad, M, dev)
    dst.flat.zero_()
    flat = gathered.view(-1)
    k.sparse_unpack_grads(flat[head:], blk, counts, 0, cap, S, P_pad, dst.views)
    keep = torch.cat([torch.zeros(S, dtype=torch.bool, device=dev)] + [m.bool() for m in masks[1:]])
    for name in src.views:
        exp = src.views[name].clone()
        exp[~keep] = 0
        assert torch.equal(dst.views[name], exp), name
    dst.flat[:3 * S].fill_(5.0)  # rank 0's own shard rows are never touched by the clear
    k.sparse_unpack_grads(flat[head:], blk, counts, 0, cap, S, P_pad, dst.views, clear=True)
    assert torch.equal(dst.views["means3D"][:S], torch.full((S, 3), 5.0, device=dev))
    for name in src.views:
        assert not dst.views[name][S:].any(), name
