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
import os
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


def _fault(var: str) -> str:
    """Fault-injection hook for the first multi-GPU run's safety net (bench.py
    exchange check; tests/test_gpu_bench_dp.py): ``$var`` = "raise" |
    "perturb", applied on the ranks listed in WGSR_DP_FAULT_RANKS (comma
    separated; default every rank).  Unset in normal runs."""
    mode = os.environ.get(var, "")
    if not mode:
        return ""
    ranks = os.environ.get("WGSR_DP_FAULT_RANKS", "")
    if ranks and dist.is_initialized() and str(dist.get_rank()) not in ranks.split(","):
        return ""
    return mode


def allreduce_grads(buf: GradBuffer, bucket_bytes: int = 256 << 20, async_op: bool = False,
                    average: bool = False):
    """SUM-all-reduce the flat gradient buffer in buckets of ``bucket_bytes``.

    Returns the list of work handles when ``async_op`` (wait on them before
    reading the gradients), else None.
    """
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return [] if async_op else None
    if _fault("WGSR_DP_FAULT_ALLREDUCE") == "raise":
        raise RuntimeError("WGSR_DP_FAULT_ALLREDUCE=raise: injected all-reduce failure (test hook)")
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

    def mask_words(self, S):
        from wgsr import _lib
        return int(_lib.load().wgsr_sparse_mask_words(int(S)))

    def summary_block_words(self, world, S):
        from wgsr import _lib
        return int(_lib.load().wgsr_sparse_summary_block_words(int(world), int(S)))

    def sparse_pack_records(self, send, S, counts, packed, nzmask):
        from wgsr import _lib
        _lib.check(_lib.load().wgsr_sparse_pack_records(send.data_ptr(), send.size(0), int(S), counts.data_ptr(),
                                                        packed.data_ptr(), _lib.ptr(nzmask),
                                                        _lib.stream_handle(send.device)))

    def sparse_exchange_summary(self, blocks, world, rank, S, summary, offsets, cams):
        from wgsr import _lib
        _lib.check(_lib.load().wgsr_sparse_exchange_summary(blocks.data_ptr(), int(world), int(rank), int(S),
                                                            summary.data_ptr(), offsets.data_ptr(), cams.data_ptr(),
                                                            _lib.stream_handle(blocks.device)))

    def sparse_unpack_records(self, received, offsets, S, keep_radius, recv, mask):
        from wgsr import _lib
        _lib.check(_lib.load().wgsr_sparse_unpack_records(received.data_ptr(), offsets.data_ptr(), recv.size(0),
                                                          int(S), int(keep_radius), recv.data_ptr(), mask.data_ptr(),
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

    def sparse_unpack_grads(self, gathered, block_stride, counts, rank, cap, S, P, grads, clear=False):
        """gathered: flat tensor whose element 0 is owner 0's first packed row;
        owner r's rows start block_stride floats later per owner."""
        from wgsr import _lib
        M = grads["shs"].size(1)
        _lib.check(_lib.load().wgsr_sparse_unpack_grads(
            gathered.data_ptr(), int(block_stride), counts.data_ptr(), counts.numel(), int(rank), int(cap), int(S),
            int(P), int(M), grads["means3D"].data_ptr(), grads["shs"].data_ptr(), grads["opacities"].data_ptr(),
            grads["scales"].data_ptr(), grads["rotations"].data_ptr(), int(bool(clear)),
            _lib.stream_handle(gathered.device)))


# ---- collectives ------------------------------------------------------------
# Exactly two collective shapes carry the exchange on every backend: equal-block
# all_gather_into_tensor and all_to_all_single (equal, or with split sizes in
# rows).  gloo has no device collectives, so on gloo device tensors are staged
# through host memory with the SAME call (test rigs only: RCCL is the product
# backend); the CPU and one-GPU tests therefore run the call shapes the RCCL
# branch runs.

def _staged(group, *ts):
    return dist.get_backend(group) == "gloo" and any(t.is_cuda for t in ts)


def _all_gather_into(out_flat, inp, group, async_op=True):
    """all_gather_into_tensor(out_flat, inp): equal blocks, rank order."""
    if _staged(group, out_flat, inp):
        h = torch.empty(out_flat.shape, dtype=out_flat.dtype)
        dist.all_gather_into_tensor(h, inp.cpu(), group=group)
        out_flat.copy_(h)
        return None
    return dist.all_gather_into_tensor(out_flat, inp, group=group, async_op=async_op)


def _all_to_all(out, inp, group, out_splits=None, in_splits=None, async_op=True):
    """all_to_all_single(out, inp[, output_split_sizes, input_split_sizes])
    (split sizes along dim 0; None = equal blocks)."""
    if _staged(group, out, inp):
        o = torch.empty(out.shape, dtype=out.dtype)
        dist.all_to_all_single(o, inp.cpu(), output_split_sizes=out_splits, input_split_sizes=in_splits,
                               group=group)
        out.copy_(o)
        return None
    return dist.all_to_all_single(out, inp, output_split_sizes=out_splits, input_split_sizes=in_splits, group=group,
                                  async_op=async_op)


def _wait(*works):
    for w in works:
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
            world, S = self.world, self.S
            self.F = self.k.grad_row_floats(M)
            self.BW = self.k.summary_block_words(world, S)
            # this rank's small block: [camera row | rows sent per owner | non-zero row masks]
            self.small = torch.zeros(self.BW, **i32)
            self.small_all = torch.zeros(world, self.BW, **i32)
            self.packed = torch.empty(self.P_pad, 12, **f32)
            self.recvp = torch.empty(self.P_pad, 12, **f32)
            self.mask = torch.zeros(S, dtype=torch.uint8, device=dev)
            self.offsets = torch.zeros(world + 1, **i32)
            self.gcount = torch.zeros(1, **i32)
            # gradient block per rank: [stats S x 3 | tau world x 6 | cap x F packed rows]
            self.st_n = 3 * S if stats else 0
            self.head = self.st_n + 6 * world
            self.gsend = torch.empty(self.head + S * self.F, **f32)
            # two generations (step parity): the next step first clears, on
            # every rank, the rows this step's gather scattered (instead of
            # zeroing the whole gradient buffer)
            self.summary = [torch.zeros(world * world + world, **i32) for _ in range(2)]
            self.gall = [None, None]
            self.gen = 0
            self.prev = None  # (gathered flat, block, counts, cap) of the last step
            if stats:
                self.rad_send = torch.empty(self.P_pad, **f32)
                self.rad_recv = torch.empty(self.P_pad, **f32)

    def backward(self, fwd, dL_dcolor, dL_ddepth, scale_modifier: float = 1.0):
        """fwd = (means3D, scales, rotations, shs, D, cam, num_rendered, radii,
        geom, binning, image) of this rank's forward; cam is the dict of
        camera tensors/scalars (viewmatrix, projmatrix, projmatrix_raw,
        campos, tanfovx, tanfovy, bg).  -> (grads dict, tau [6] of this
        rank's view, stats [P, 3] or None).

        Callers must not write into the gradient rows this rank does not own
        between steps: the sparse exchange clears, at the next step, exactly
        the rows its last gather scattered."""
        fault = _fault("WGSR_DP_FAULT")
        if fault == "raise":
            raise RuntimeError("WGSR_DP_FAULT=raise: injected exchange failure (test hook)")
        if self.sparse:
            out = self._backward_sparse(fwd, dL_dcolor, dL_ddepth, scale_modifier)
        else:
            out = self._backward_dense(fwd, dL_dcolor, dL_ddepth, scale_modifier)
        if fault == "perturb":   # a 1 % error in one gradient tensor
            out[0]["means3D"].mul_(1.01)
        return out

    def _backward_dense(self, fwd, dL_dcolor, dL_ddepth, scale_modifier):
        means3D, scales, rotations, shs, D, cam = fwd[:6]
        H, W = dL_dcolor.size(1), dL_dcolor.size(2)
        g = self.group
        # this view's camera row -> every owner (tiny; overlaps the records)
        self.k.pack_camera(cam, W, H, self.cam_row)
        w_cam = None
        if self.world > 1:
            w_cam = _all_gather_into(self.cams.view(-1), self.cam_row, g)
        else:
            self.cams.copy_(self.cam_row[None])
        # this view's screen-space records of every Gaussian -> owners
        self.k.records(fwd, dL_dcolor, dL_ddepth, self.P_pad, self.send)
        if self.world > 1:
            _wait(_all_to_all(self.recv.view(self.P_pad, 12), self.send, g))
        else:
            self.recv.view(self.P_pad, 12).copy_(self.send)
        _wait(w_cam)
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
            # every buffer's shard gathered in place: one equal-block
            # all_gather_into_tensor each, issued back to back, waited once
            fulls = [v.view(self.P_pad, -1) for v in self.buf.views.values()]
            if self.stats is not None:
                fulls.append(self.stats)
            fulls.append(self.tau_own)
            works = []
            for f in fulls:
                n = f.size(0) // self.world
                works.append(_all_gather_into(f.view(-1), f[self.rank * n:(self.rank + 1) * n].reshape(-1).clone(),
                                              g))
            _wait(*works)
        torch.sum(self.tau_own, dim=0, out=self.tau)
        stats = self.stats[:self.P] if self.stats is not None else None
        return self.grads, self.tau[self.rank], stats

    def _backward_sparse(self, fwd, dL_dcolor, dL_ddepth, scale_modifier):
        """The same result as the dense exchange, moving only non-zero rows.

        Collectives per step: one small equal-block all-gather (camera rows,
        rows sent per owner, non-zero row masks), the records as ONE
        all_to_all_single with split sizes, and ONE equal-block all-gather of
        [statistics | pose sums | packed gradient rows] per owner (padded to
        the largest owner's union count); with statistics also the dense
        radius column (equal all_to_all_single).  ONE host read per step: the
        count matrix and every owner's union row count, both computed on the
        device from the small all-gather (csrc/dp_sparse.hip)."""
        means3D, scales, rotations, shs, D, cam = fwd[:6]
        H, W = dL_dcolor.size(1), dL_dcolor.size(2)
        g, S, world, rank, F = self.group, self.S, self.world, self.rank, self.F
        k = self.k
        small = self.small
        small.zero_()
        self.k.pack_camera(cam, W, H, self.cam_row)
        small[:64].copy_(self.cam_row.view(torch.int32))
        k.records(fwd, dL_dcolor, dL_ddepth, self.P_pad, self.send)
        k.sparse_pack_records(self.send, S, small[64:64 + world], self.packed, small[64 + world:])
        w_rad = None
        if self.stats is not None:  # the statistics need every visible Gaussian's radius
            self.rad_send.copy_(self.send[:, 10])
            w_rad = _all_to_all(self.rad_recv, self.rad_send, g)
        _wait(_all_gather_into(self.small_all.view(-1), small, g))
        p = self.gen & 1
        summary = self.summary[p]
        k.sparse_exchange_summary(self.small_all, world, rank, S, summary, self.offsets, self.cams)
        host = summary.tolist()  # the step's one host read
        cmat = [host[v * world:(v + 1) * world] for v in range(world)]
        union = host[world * world:]
        sent = cmat[rank]
        got = [cmat[v][rank] for v in range(world)]
        cap = max(union)
        # records: this rank's per-owner segments, packed contiguously -> owners
        ins = torch.cat([self.packed[o * S:o * S + sent[o]] for o in range(world)])
        received = self.recvp[:sum(got)]
        w = _all_to_all(received, ins, g, out_splits=got, in_splits=sent)
        self.recv.zero_()
        self.mask.zero_()
        if self.stats is not None:
            _wait(w_rad)
            k.sparse_fill_radius(self.rad_recv, self.recv.view(-1, 12))
        _wait(w)
        k.sparse_unpack_records(received, self.offsets, S, self.stats is not None, self.recv, self.mask)
        # owner: all views of the shard, summed; statistics and pose sums go
        # straight into this rank's gradient block
        blk = self.head + cap * F
        send = self.gsend[:blk]
        st = send[:self.st_n].view(S, 3)[:self.hi - self.lo] if self.stats is not None else None
        tau_mine = send[self.st_n:self.head].view(world, 6)
        k.gauss_views((means3D, scales, rotations, shs, D, scale_modifier), self.lo, self.hi, self.cams,
                      self.recv, self.buf.views, self.tau_blk if self.hi > self.lo else None, st)
        if self.hi > self.lo:
            torch.sum(self.tau_blk, dim=0, out=tau_mine)
        else:
            tau_mine.zero_()
        if self.stats is not None and self.hi - self.lo < S:
            send[:self.st_n].view(S, 3)[self.hi - self.lo:].zero_()
        self.gcount.zero_()
        k.sparse_pack_grads(self.buf.views, self.lo, self.hi, self.mask, self.gcount, send[self.head:])
        gathered = torch.empty(world * blk, dtype=torch.float32, device=send.device)
        _wait(_all_gather_into(gathered, send, g))
        gv = gathered.view(world, blk)
        if self.stats is not None:
            self.stats.view(world, S * 3).copy_(gv[:, :self.st_n])
        self.tau_own.copy_(gv[:, self.st_n:self.head].reshape(world, world, 6))
        counts = summary[world * world:]
        # the rows the previous step scattered from other owners go back to
        # zero (this rank's own shard is rewritten whole by the owner kernel)
        if self.prev is not None:
            pg, pblk, pcounts, pcap = self.prev
            self._unpack_grads(pg, pblk, pcounts, pcap, clear=True)
        self._unpack_grads(gathered, blk, counts, cap, clear=False)
        self.prev = (gathered, blk, counts, cap)
        self.gen += 1
        torch.sum(self.tau_own, dim=0, out=self.tau)
        others = sum(got) - got[rank]
        self.last_exchange = {
            "record_rows_in": others, "grad_rows_per_owner": union, "grad_rows_cap": cap,
            "bytes_in": int(others * 48 + (world - 1) * blk * 4 +
                            ((world - 1) * S * 4 if self.stats is not None else 0) +
                            (world - 1) * self.BW * 4),
        }
        stats = self.stats[:self.P] if self.stats is not None else None
        return self.grads, self.tau[rank], stats

    def _unpack_grads(self, gathered, blk, counts, cap, clear):
        if cap == 0:
            return
        self.k.sparse_unpack_grads(gathered[self.head:], blk, counts, self.rank, cap, self.S, self.P, self.buf.views,
                                   clear=clear)
