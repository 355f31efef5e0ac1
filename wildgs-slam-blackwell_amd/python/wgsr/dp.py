"""Keyframe-view data parallelism over RCCL.

The reference is single-GPU; its mapper renders one keyframe view per
optimiser step (src/mapper.py:1089-1170).  Views are independent given a
replicated Gaussian set, so the natural multi-GPU axis is the VIEW: rank r
renders view r (r + world, ...) with full parameter replicas and the only
exchange is one reduction of the per-Gaussian parameter gradients per step.

* ``GradBuffer`` lays the parameter gradients of one backward out in ONE flat
  fp32 buffer (means3D | SH | opacity | scales | rotations: 59 floats per
  Gaussian at SH degree 3), so the backward writes straight into the
  all-reduce operand -- no pack/unpack copies.
* ``allreduce_grads`` issues SUM all-reduces over that buffer in large
  buckets (xGMI is point-to-point: RCCL's rings are per-link bound, so few,
  large collectives), optionally asynchronously so a caller can overlap them.
* ``reduce_densification_stats`` sums this step's per-view ||dL/dmeans2D||
  contributions and visibility counts and takes the MAX of the screen radii,
  then folds them into the persistent accumulators -- the reference
  accumulates per-view norms (gaussian_model.py:745-749, mapper.py:1177-1183),
  not the norm of the summed gradient, so these cannot ride in the gradient
  sum.

Backend: whatever ``torch.distributed`` was initialised with -- "nccl" is RCCL
on ROCm (over xGMI on one node); the CPU tests use "gloo".
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import torch
import torch.distributed as dist

PARAM_ORDER = ("means3D", "shs", "opacities", "scales", "rotations")


@dataclass
class GradBuffer:
    """Flat gradient storage with per-parameter [P, ...] views."""

    flat: torch.Tensor
    views: dict

    @staticmethod
    def allocate(P: int, M: int, device, dtype=torch.float32) -> "GradBuffer":
        shapes = {"means3D": (P, 3), "shs": (P, M, 3), "opacities": (P, 1), "scales": (P, 3),
                  "rotations": (P, 4)}
        sizes = {k: int(torch.Size(s).numel()) for k, s in shapes.items()}
        flat = torch.empty(sum(sizes.values()), dtype=dtype, device=device)
        views, off = {}, 0
        for k in PARAM_ORDER:
            views[k] = flat[off: off + sizes[k]].view(shapes[k])
            off += sizes[k]
        return GradBuffer(flat, views)

    @property
    def floats_per_gaussian(self) -> int:
        P = self.views["means3D"].shape[0]
        return self.flat.numel() // max(P, 1)


def allreduce_grads(buf: GradBuffer, bucket_bytes: int = 256 << 20, async_op: bool = False,
                    average: bool = False):
    """SUM-all-reduce the flat gradient buffer in buckets of ``bucket_bytes``.

    Returns the list of work handles when ``async_op`` (wait on them before
    reading the gradients), else None.
    """
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return [] if async_op else None
    flat = buf.flat
    per = max(1, bucket_bytes // flat.element_size())
    works = []
    for s in range(0, flat.numel(), per):
        works.append(dist.all_reduce(flat[s: s + per], op=dist.ReduceOp.SUM, async_op=True))
    if average:
        for w in works:
            w.wait()
        flat.div_(dist.get_world_size())
        return [] if async_op else None
    if async_op:
        return works
    for w in works:
        w.wait()
    return None


def reduce_densification_stats(step_grad_norm: torch.Tensor, step_count: torch.Tensor,
                               step_radii: torch.Tensor, xyz_gradient_accum: torch.Tensor | None = None,
                               denom: torch.Tensor | None = None, max_radii2D: torch.Tensor | None = None):
    """Reduce THIS STEP's densification contributions over the ranks' views.

    ``step_grad_norm`` / ``step_count`` / ``step_radii`` must hold only this
    step's per-view contributions (||dL/dmeans2D[:, :2]|| of the visible
    Gaussians, their visibility 0/1 count, their screen radii); they are
    reduced in place (SUM, SUM, MAX).  Passing the persistent accumulators
    here instead would re-add the totals of every earlier step ~world-size
    times, so the accumulators are separate, optional arguments: when given,
    the reduced step values are folded into them the way the reference does
    per view (gaussian_model.py:745-749, mapper.py:1177-1183):
    ``xyz_gradient_accum += step_grad_norm``, ``denom += step_count``,
    ``max_radii2D = max(max_radii2D, step_radii)``.
    """
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(step_grad_norm, op=dist.ReduceOp.SUM)
        dist.all_reduce(step_count, op=dist.ReduceOp.SUM)
        dist.all_reduce(step_radii, op=dist.ReduceOp.MAX)
    if xyz_gradient_accum is not None:
        xyz_gradient_accum += step_grad_norm.view_as(xyz_gradient_accum)
    if denom is not None:
        denom += step_count.view_as(denom)
    if max_radii2D is not None:
        torch.maximum(max_radii2D, step_radii.view_as(max_radii2D).to(max_radii2D.dtype), out=max_radii2D)


def views_for_rank(num_views: int, rank: int, world: int):
    """Round-robin view assignment: rank r renders views r, r + world, ..."""
    return list(range(rank, num_views, world))


# ---------------------------------------------------------------------------
# View-sharded backward: exchange screen-space partials, not gradients.
# ---------------------------------------------------------------------------
# The all-reduce above moves 2 (N-1)/N x 59 floats per Gaussian per rank.  A
# view's parameter gradient is a per-Gaussian function of the camera and of
# ten screen-space partial sums (dL/dmean2D, dL/dconic, dL/dopacity,
# dL/dcolour, dL/ddepth) that the render backward produces.  So each rank
# ships its view's 12-float record of every Gaussian to the Gaussian's OWNER
# (all-to-all, (N-1)/N x 12 floats per Gaussian), each owner runs the
# camera-side backward of all N views for its 1/N shard and sums them in
# registers (one kernel), and the summed shards are all-gathered
# ((N-1)/N x 59 floats) -- every rank ends with the same SUM over views that
# allreduce_grads produces, for 71 instead of 118 floats of traffic per
# Gaussian at N = 8.  The pose gradient of each view is reduced over the
# owners' shards (N x 6 floats), and the densification statistics of all
# views come out of the same kernel.


class _HipViewKernels:
    """The three libwgsr entry points of the view-sharded backward."""

    @staticmethod
    def _raster_args(P, D, M, W, H, means3D, scales, rotations, shs, scale_modifier, cam, keep):
        from diff_gaussian_rasterization import _C
        e = None
        cam = {k: (v.contiguous() if torch.is_tensor(v) else v) for k, v in cam.items()}
        return _C._args(P, D, M, W, H, cam.get("bg", means3D), means3D, e, means3D, scales, rotations, e,
                        shs, cam.get("viewmatrix"), cam.get("projmatrix"), cam.get("projmatrix_raw"),
                        cam.get("campos"), scale_modifier, cam.get("tanfovx", 1.0), cam.get("tanfovy", 1.0),
                        False, False, keep)

    def pack_camera(self, cam, W, H, out_row):
        from wgsr import _lib
        L = _lib.load()
        keep = []
        a = self._raster_args(0, 0, 0, W, H, None, None, None, None, 1.0, cam, keep)
        _lib.check(L.wgsr_pack_view_camera(ctypes.byref(a), out_row.data_ptr(),
                                           _lib.stream_handle(out_row.device)))

    def records(self, fwd, dL_dcolor, dL_ddepth, P_pad, out):
        """fwd: the forward's (means3D, scales, rotations, shs, D, cam dict,
        num_rendered, radii, geom, binning, image).  out: [P_pad, 12]."""
        from wgsr import _lib
        L = _lib.load()
        means3D, scales, rotations, shs, D, cam, nr, radii, geom, binning, image = fwd
        if shs is None or scales is None or rotations is None:
            raise RuntimeError("the view-sharded backward needs SHs, scales and rotations "
                               "(colors_precomp / cov3D_precomp are not supported)")
        P = means3D.size(0)
        M = shs.size(1) if shs is not None else 0
        H, W = dL_dcolor.size(1), dL_dcolor.size(2)
        keep = []
        a = self._raster_args(P, int(D), M, W, H, means3D.contiguous(), scales.contiguous(),
                              rotations.contiguous(), shs.contiguous() if shs is not None else None, 1.0,
                              cam, keep)
        gc, gd = dL_dcolor.contiguous(), dL_ddepth.contiguous()
        p = _lib.ptr
        dev = means3D.device
        with torch.cuda.device(dev), _lib.AllocRequest(dev):
            code = L.wgsr_rasterize_backward_records(
                ctypes.byref(a), p(radii), p(geom), p(binning), p(image), int(nr), gc.data_ptr(),
                gd.data_ptr(), _lib.ALLOC_SCRATCH, None, int(P_pad), out.data_ptr(), _lib.stream_handle(dev))
        _lib.check(code)

    def tau_blocks(self, lo, hi):
        from wgsr import _lib
        return int(_lib.load().wgsr_gauss_backward_views_blocks(int(lo), int(hi)))

    def gauss_views(self, params, lo, hi, cams, recs, grads, tau_out, stats_out):
        """params: (means3D, scales, rotations, shs, D, scale_modifier);
        cams [V, 64]; recs [V, S, 12]; grads: GradBuffer views (rows [lo, hi)
        written); tau_out [blocks, V, 6] or None; stats_out [hi-lo, 3] or None."""
        from wgsr import _lib
        L = _lib.load()
        means3D, scales, rotations, shs, D, scale_modifier = params
        P = means3D.size(0)
        M = shs.size(1) if shs is not None else 0
        keep = []
        a = self._raster_args(P, int(D), M, 1, 1, means3D, scales, rotations, shs, scale_modifier, {}, keep)
        V = cams.size(0)
        dev = means3D.device
        p = _lib.ptr
        code = L.wgsr_gauss_backward_views(
            ctypes.byref(a), int(lo), int(hi), int(V), cams.data_ptr(), recs.data_ptr(),
            int(recs.stride(0)), grads["means3D"].data_ptr(), p(grads["shs"]), grads["opacities"].data_ptr(),
            grads["scales"].data_ptr(), grads["rotations"].data_ptr(), p(tau_out), p(stats_out),
            _lib.stream_handle(dev))
        _lib.check(code)


    # ---- sparse exchange (csrc/dp_sparse.hip) ----
    def grad_row_floats(self, M):
        from wgsr import _lib
        return int(_lib.load().wgsr_sparse_grad_row_floats(int(M)))

    def sparse_pack_records(self, send, S, counts, packed):
        from wgsr import _lib
        _lib.check(_lib.load().wgsr_sparse_pack_records(send.data_ptr(), send.size(0), int(S), counts.data_ptr(),
                                                        packed.data_ptr(), _lib.stream_handle(send.device)))

    def sparse_unpack_records(self, recvp, counts, S, keep_radius, recv, mask):
        from wgsr import _lib
        _lib.check(_lib.load().wgsr_sparse_unpack_records(recvp.data_ptr(), counts.data_ptr(), recv.size(0), int(S),
                                                          int(keep_radius), recv.data_ptr(), mask.data_ptr(),
                                                          _lib.stream_handle(recv.device)))

    def sparse_fill_radius(self, radii, recv):
        from wgsr import _lib
        _lib.check(_lib.load().wgsr_sparse_fill_radius(radii.data_ptr(), radii.numel(), recv.data_ptr(),
                                                       _lib.stream_handle(recv.device)))

    def sparse_pack_grads(self, grads, lo, hi, mask, count, packed):
        from wgsr import _lib
        M = grads["shs"].size(1)
        _lib.check(_lib.load().wgsr_sparse_pack_grads(
            int(lo), int(hi), int(M), mask.data_ptr(), grads["means3D"].data_ptr(), grads["shs"].data_ptr(),
            grads["opacities"].data_ptr(), grads["scales"].data_ptr(), grads["rotations"].data_ptr(),
            count.data_ptr(), packed.data_ptr(), _lib.stream_handle(packed.device)))

    def sparse_unpack_grads(self, gathered, counts, rank, cap, S, P, grads):
        from wgsr import _lib
        M = grads["shs"].size(1)
        _lib.check(_lib.load().wgsr_sparse_unpack_grads(
            gathered.data_ptr(), counts.data_ptr(), counts.numel(), int(rank), int(cap), int(S), int(P), int(M),
            grads["means3D"].data_ptr(), grads["shs"].data_ptr(), grads["opacities"].data_ptr(),
            grads["scales"].data_ptr(), grads["rotations"].data_ptr(), _lib.stream_handle(gathered.device)))


def _gloo_cuda(group):
    """gloo has no device collectives for every op: stage device tensors
    through host memory (test rigs only -- RCCL is the product backend)."""
    return dist.get_backend(group) == "gloo"


def _all_to_all_equal(out, inp, group):
    if _gloo_cuda(group) and inp.is_cuda:
        o = torch.empty_like(out, device="cpu")
        dist.all_to_all_single(o, inp.cpu(), group=group)
        out.copy_(o)
        return None
    return dist.all_to_all_single(out, inp, group=group, async_op=True)


def _all_gather_into(out_flat, inp, group):
    if _gloo_cuda(group) and inp.is_cuda:
        h = torch.empty(out_flat.shape, dtype=out_flat.dtype)
        dist.all_gather_into_tensor(h, inp.cpu(), group=group)
        out_flat.copy_(h)
        return None
    return dist.all_gather_into_tensor(out_flat, inp, group=group, async_op=True)


def _all_gather_inplace(full, rank, group):
    """full [world * S, ...]: rank's block holds its shard; gather the rest."""
    world = dist.get_world_size(group)
    S = full.size(0) // world
    if _gloo_cuda(group) and full.is_cuda:
        h = full.cpu()
        dist.all_gather_into_tensor(h.view(-1), h[rank * S:(rank + 1) * S].reshape(-1).clone(), group=group)
        full.copy_(h)
        return None
    return dist.all_gather_into_tensor(full.view(-1), full[rank * S:(rank + 1) * S].view(-1), group=group,
                                       async_op=True)


def _all_to_all_var(outs, ins, group):
    """outs[v] <- rank v's ins[me]: uneven row blocks, one collective."""
    if dist.get_backend(group) == "gloo":  # test rigs: one alltoallv through host memory
        flat = [t.reshape(t.size(0), -1) for t in ins]
        inp = torch.cat(flat).cpu()
        out = torch.empty((sum(o.size(0) for o in outs),) + tuple(inp.shape[1:]), dtype=inp.dtype)
        dist.all_to_all_single(out, inp, output_split_sizes=[o.size(0) for o in outs],
                               input_split_sizes=[t.size(0) for t in ins], group=group)
        off = 0
        for o in outs:
            n = o.size(0)
            o.copy_(out[off:off + n].view_as(o))
            off += n
        return None
    return dist.all_to_all(outs, ins, group=group, async_op=True)


def _all_gather_many(pairs, group):
    """all_gather_into_tensor of several (out_flat, in_flat) pairs as ONE
    coalesced RCCL group (a single grouped launch, one collective latency)."""
    if any(_gloo_cuda(group) and i.is_cuda for _, i in pairs):
        for o, i in pairs:
            _all_gather_into(o, i, group)
        return None
    try:
        with dist._coalescing_manager(group, async_ops=True) as cm:
            for o, i in pairs:
                dist.all_gather_into_tensor(o, i, group=group)
        return cm
    except (RuntimeError, AttributeError, NotImplementedError):
        # a backend / torch build without the coalesced fast path: every rank
        # takes this branch alike (same code, same backend), so the collectives
        # still pair up -- one gather per buffer
        return _WaitAll([_all_gather_into(o, i, group) for o, i in pairs])


def _all_gather_inplace_many(fulls, rank, group):
    """In-place all-gathers of several [world * S, ...] buffers (each rank's
    block holds its shard) as ONE coalesced collective: RCCL runs the group
    as a single launch, so the small buffers ride along with the SH block
    instead of paying a collective's latency each."""
    world = dist.get_world_size(group)
    pairs = []
    for f in fulls:
        S = f.size(0) // world
        pairs.append((f.view(-1), f[rank * S:(rank + 1) * S].view(-1)))
    return _all_gather_many(pairs, group)


class _WaitAll:
    def __init__(self, works):
        self.works = works

    def wait(self):
        for w in self.works:
            if w is not None:
                w.wait()


class ViewShardedBackward:
    """Keyframe-view data-parallel backward with owner-computes sharding.

    Rank r renders view r (its own forward) and calls ``backward`` with that
    forward's state; every rank returns the SUM over all ranks' views of the
    parameter gradients (``grads``, the same [P, ...] tensors allreduce_grads
    produces), its own view's pose gradient (rho, theta) and, with
    ``stats=True``, the densification statistics summed over the views
    (sum ||dL/dmeans2D[:2]||, visibility count, max radius per Gaussian).

    Gaussians are sharded by index: rank s owns [s S, (s+1) S), S = ceil(P/N).
    """

    def __init__(self, P: int, M: int, device, group=None, stats: bool = False, kernels=None, sparse: bool = True):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.P, self.M = P, M
        self.S = max(1, -(-P // self.world))
        self.P_pad = self.S * self.world
        self.lo = min(P, self.rank * self.S)
        self.hi = min(P, self.lo + self.S)
        self.k = kernels or _HipViewKernels()
        dev = torch.device(device)
        f32 = dict(dtype=torch.float32, device=dev)
        self.buf = GradBuffer.allocate(self.P_pad, M, dev)
        self.buf.flat.zero_()  # padding rows are gathered, never read
        self.grads = {k: v[:P] for k, v in self.buf.views.items()}
        self.send = torch.zeros(self.P_pad, 12, **f32)
        self.recv = torch.empty(self.world, self.S, 12, **f32)
        self.cam_row = torch.zeros(64, **f32)
        self.cams = torch.empty(self.world, 64, **f32)
        nb = self.k.tau_blocks(self.lo, self.hi)
        self.tau_blk = torch.zeros(max(nb, 1), self.world, 6, **f32)
        # per-owner pose-gradient sums [owner, view, 6]: gathered with the
        # gradient shards, summed over owners locally (no separate all-reduce)
        self.tau_own = torch.zeros(self.world, self.world, 6, **f32)
        self.tau = torch.zeros(self.world, 6, **f32)
        self.stats = torch.zeros(self.P_pad, 3, **f32) if stats else None
        # sparse exchange (N > 1): only rows with a non-zero record / gradient
        # travel (csrc/dp_sparse.hip); `last_exchange` reports what moved
        self.sparse = bool(sparse) and self.world > 1
        self.last_exchange = None
        if self.sparse:
            i32 = dict(dtype=torch.int32, device=dev)
            self.F = self.k.grad_row_floats(M)
            self.packed = torch.empty(self.P_pad, 12, **f32)
            self.recvp = torch.empty(self.P_pad, 12, **f32)
            self.mask = torch.zeros(self.S, dtype=torch.uint8, device=dev)
            self.cbuf = torch.zeros(2, self.world, **i32)  # [rows sent to each owner, rows got from each view]
            self.gcount = torch.zeros(1, **i32)
            self.gcounts = torch.zeros(self.world, **i32)
            self.gpack = torch.empty(self.S, self.F, **f32)
            if stats:
                self.rad_send = torch.empty(self.P_pad, **f32)
                self.rad_recv = torch.empty(self.P_pad, **f32)

    def backward(self, fwd, dL_dcolor, dL_ddepth, scale_modifier: float = 1.0):
        """fwd = (means3D, scales, rotations, shs, D, cam, num_rendered, radii,
        geom, binning, image) of this rank's forward; cam is the dict of
        camera tensors/scalars (viewmatrix, projmatrix, projmatrix_raw,
        campos, tanfovx, tanfovy, bg).  -> (grads dict, tau [6] of this
        rank's view, stats [P, 3] or None)."""
        if self.sparse:
            return self._backward_sparse(fwd, dL_dcolor, dL_ddepth, scale_modifier)
        means3D, scales, rotations, shs, D, cam = fwd[:6]
        H, W = dL_dcolor.size(1), dL_dcolor.size(2)
        g = self.group
        # this view's camera row -> every owner (tiny; overlaps the records)
        self.k.pack_camera(cam, W, H, self.cam_row)
        if self.world > 1:
            w_cam = _all_gather_into(self.cams.view(-1), self.cam_row, g)
        else:
            self.cams.copy_(self.cam_row[None])
            w_cam = None
        # this view's screen-space records of every Gaussian -> owners
        self.k.records(fwd, dL_dcolor, dL_ddepth, self.P_pad, self.send)
        if self.world > 1:
            w = _all_to_all_equal(self.recv.view(self.P_pad, 12), self.send, g)
            if w is not None:
                w.wait()
        else:
            self.recv.view(self.P_pad, 12).copy_(self.send)
        if w_cam is not None:
            w_cam.wait()
        # owner: all views of the shard, summed
        st = self.stats[self.lo:self.hi] if self.stats is not None else None
        self.k.gauss_views((means3D, scales, rotations, shs, D, scale_modifier), self.lo, self.hi, self.cams,
                           self.recv, self.buf.views, self.tau_blk if self.hi > self.lo else None, st)
        mine = self.tau_own[self.rank]
        if self.hi > self.lo:
            torch.sum(self.tau_blk, dim=0, out=mine)
        else:
            mine.zero_()
        if self.world > 1:
            fulls = [v.view(self.P_pad, -1) for v in self.buf.views.values()]
            if self.stats is not None:
                fulls.append(self.stats)
            fulls.append(self.tau_own)
            w = _all_gather_inplace_many(fulls, self.rank, g)
            if w is not None:
                w.wait()
        torch.sum(self.tau_own, dim=0, out=self.tau)
        stats = self.stats[:self.P] if self.stats is not None else None
        return self.grads, self.tau[self.rank], stats

    def _backward_sparse(self, fwd, dL_dcolor, dL_ddepth, scale_modifier):
        """The same result as the dense exchange, moving only non-zero rows:
        each view's records with a non-zero partial sum go to their owners
        (uneven all-to-all), and each owner gathers only the gradient rows of
        Gaussians some view gave gradient to (padded to the largest owner's
        count).  Two host reads of row counts per step size the collectives."""
        means3D, scales, rotations, shs, D, cam = fwd[:6]
        H, W = dL_dcolor.size(1), dL_dcolor.size(2)
        g, S, world, rank = self.group, self.S, self.world, self.rank
        self.k.pack_camera(cam, W, H, self.cam_row)
        w_cam = _all_gather_into(self.cams.view(-1), self.cam_row, g)
        self.k.records(fwd, dL_dcolor, dL_ddepth, self.P_pad, self.send)
        cb = self.cbuf
        cb.zero_()
        self.k.sparse_pack_records(self.send, S, cb[0], self.packed)
        w_rad = None
        if self.stats is not None:  # the statistics need every visible Gaussian's radius
            self.rad_send.copy_(self.send[:, 10])
            w_rad = _all_to_all_equal(self.rad_recv, self.rad_send, g)
        w = _all_to_all_equal(cb[1], cb[0], g)
        if w is not None:
            w.wait()
        sent, got = cb.tolist()  # host read 1: the row counts
        ins = [self.packed[o * S:o * S + sent[o]] for o in range(world)]
        outs = [self.recvp[v * S:v * S + got[v]] for v in range(world)]
        w = _all_to_all_var(outs, ins, g)
        self.recv.zero_()
        self.mask.zero_()
        if self.stats is not None:
            if w_rad is not None:
                w_rad.wait()
            self.k.sparse_fill_radius(self.rad_recv, self.recv.view(-1, 12))
        if w is not None:
            w.wait()
        self.k.sparse_unpack_records(self.recvp.view(world, S, 12), cb[1], S, self.stats is not None, self.recv,
                                     self.mask)
        if w_cam is not None:
            w_cam.wait()
        # rows no owner writes stay zero: the sparse gather leaves them alone
        self.buf.flat.zero_()
        st = self.stats[self.lo:self.hi] if self.stats is not None else None
        self.k.gauss_views((means3D, scales, rotations, shs, D, scale_modifier), self.lo, self.hi, self.cams,
                           self.recv, self.buf.views, self.tau_blk if self.hi > self.lo else None, st)
        mine = self.tau_own[rank]
        if self.hi > self.lo:
            torch.sum(self.tau_blk, dim=0, out=mine)
        else:
            mine.zero_()
        self.gcount.zero_()
        self.k.sparse_pack_grads(self.buf.views, self.lo, self.hi, self.mask, self.gcount, self.gpack)
        w = _all_gather_into(self.gcounts, self.gcount, g)
        if w is not None:
            w.wait()
        counts = self.gcounts.tolist()  # host read 2: gradient rows per owner
        cap = max(counts)
        pairs = []
        gathered = None
        if cap > 0:
            gathered = torch.empty(world * cap * self.F, dtype=torch.float32, device=self.gpack.device)
            pairs.append((gathered, self.gpack[:cap].reshape(-1)))
        fulls = ([self.stats] if self.stats is not None else []) + [self.tau_own]
        for f in fulls:
            n = f.size(0) // world
            pairs.append((f.view(-1), f[rank * n:(rank + 1) * n].reshape(-1)))
        w = _all_gather_many(pairs, g)
        if w is not None:
            w.wait()
        if gathered is not None:
            self.k.sparse_unpack_grads(gathered.view(world, cap, self.F), self.gcounts, rank, cap, S, self.P,
                                       self.buf.views)
        torch.sum(self.tau_own, dim=0, out=self.tau)
        others = sum(got) - got[rank]
        self.last_exchange = {
            "record_rows_in": others, "grad_rows_per_owner": counts, "grad_rows_cap": cap,
            "bytes_in": int(others * 48 + (world - 1) * cap * self.F * 4 +
                            ((world - 1) * S * 16 if self.stats is not None else 0) + (world - 1) * world * 24),
        }
        stats = self.stats[:self.P] if self.stats is not None else None
        return self.grads, self.tau[rank], stats
