"""The online mapper, data-parallel over keyframe views.

The reference maps on one GPU, one keyframe view per optimiser step
(src/mapper.py:1089-1219, 1288-1362).  ``DPOnlineMapper`` runs the same loop
on ``world`` processes (one per GPU, ``torch.distributed``; "nccl" is RCCL
over xGMI) with full replicas of the Gaussians, the uncertainty MLP and the
keyframe exposures:

* every rank makes the SAME random draws (one seed); an iteration draws one
  keyframe per rank and rank r renders draw r -- ``world`` views per step;
* after the backward, ONE SUM all-reduce of a flat buffer holding the
  Gaussians' parameter gradients and the MLP's (``allreduce_flat``), so the
  step's gradient is the sum of the ranks' per-view gradients (8(e) parity:
  "the all-reduced gradient equals the sum of the single-view gradients");
* the densification statistics stay per-rank partial sums and are reduced
  only where they are read, right before a densify (SUM of the per-view
  ||dL/dmean2D|| accumulations and visibility counts, MAX of the screen
  radii): every densify and every keyframe insertion zeroes them on all ranks
  (store.py), and a prune filters the same rows everywhere, so a rank's
  accumulators always hold exactly its own views' contributions until then;
* reset_opacity_nonvisible resets the Gaussians seen by none of the step's
  views (MAX of the visibility masks);
* the keyframes' exposure Adam steps are replayed on every rank from the
  gathered (keyframe, per-block partials) of all ranks, a keyframe drawn by
  several ranks taking one step on the sum (``gather_exposure``);
* initialize_map_opt's occlusion-aware visibility of each drawn keyframe is
  gathered the same way (``gather_rows``).

The steady-state iterations replay captured graphs here too
(``DPIterationGraphs``): the iteration is captured as TWO graphs around the
exchange -- (A) this rank's view up to its gradients, which also packs the MLP
gradient, the overflow word and this rank's exposure partials into one flat
"tail" buffer, then the eager collectives (a SUM all-reduce of the store's
packed gradient rows, ``GaussianStore.grad_flat``, and one of the tail: two
collectives, no copies), then (B) the Adam steps with the all-reduced
overflow word as their skip word; the exposure steps of the step's distinct
keyframes follow eagerly from the summed tail.

Densify's random split samples come from the replicated generator and its
decisions from reduced statistics, Adam is deterministic: the replicas stay
bit-identical (tests/test_gpu_dp_online.py checks it after a run through every
branch).  The optimiser trajectory is NOT the reference's (``world`` views per
step instead of one); as 8(e) states, that is a new configuration.  The
iteration graphs (wgsr.online_graph) are not used here: the all-reduce sits
between the captured backward and the captured Adam step.

Gathers are SUM all-reduces into zeroed [world, ...] buffers, so every
collective here is an all-reduce (RCCL, and gloo on CPU or CUDA tensors).
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

from . import _lib
from .online import OnlineMapper
from .online_graph import IterationGraphs


def _all_reduce(t: torch.Tensor, op, group=None):
    """dist.all_reduce; over gloo a device tensor is staged through the host
    (gloo's device-tensor support varies by type and op)."""
    if t.is_cuda and dist.get_backend(group) == "gloo":
        h = t.cpu()
        dist.all_reduce(h, op=op, group=group)
        t.copy_(h)
        return
    dist.all_reduce(t, op=op, group=group)


def allreduce_grads(store, mlp_params, group=None):
    """SUM-all-reduce the step's gradients: the store's packed gradient rows
    in place (``grad_flat``: one contiguous range, no copy) and the MLP's
    (a few thousand floats, through one small flat buffer)."""
    _all_reduce(store.grad_flat(), dist.ReduceOp.SUM, group)
    allreduce_flat([p.grad for p in mlp_params], group)


def allreduce_flat(tensors, group=None):
    """SUM-all-reduce a list of tensors as ONE flat fp32 buffer (one
    collective: xGMI rings are per-link bound, so one large message beats
    several small ones), results copied back in place."""
    ts = [t for t in tensors if t is not None and t.numel()]
    if not ts:
        return
    flat = torch.cat([t.reshape(-1).to(torch.float32) for t in ts])
    _all_reduce(flat, dist.ReduceOp.SUM, group)
    off = 0
    for t in ts:
        n = t.numel()
        t.copy_(flat[off:off + n].view_as(t))
        off += n


def gather_rows(row: torch.Tensor, group=None) -> torch.Tensor:
    """[world, *row.shape]: every rank's ``row`` in rank order (an all-reduce
    SUM of a zeroed buffer holding this rank's row in its slot)."""
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    buf = torch.zeros((world,) + tuple(row.shape), dtype=row.dtype, device=row.device)
    buf[rank].copy_(row)
    _all_reduce(buf, dist.ReduceOp.SUM, group)
    return buf


def gather_exposure(uid: int, partials: torch.Tensor, group=None):
    """-> [(uid, partials)] over the distinct keyframes the ranks rendered, in
    order of first appearance by rank; a keyframe rendered by several ranks
    gets the concatenation of their partial rows (the step kernel sums every
    row: one Adam step on the summed gradient)."""
    uids = gather_rows(torch.tensor([int(uid)], dtype=torch.int64, device=partials.device), group).view(-1)
    parts = gather_rows(partials.contiguous(), group)
    out = {}
    for r, u in enumerate(uids.tolist()):
        out.setdefault(u, []).append(parts[r])
    return [(u, p[0] if len(p) == 1 else torch.cat(p)) for u, p in out.items()]


class DPOnlineMapper(OnlineMapper):
    """OnlineMapper over ``group``'s ranks (module docstring).  Every rank
    constructs it with the same arguments (seed included) and calls the same
    entry points with the same keyframes."""

    def __init__(self, *args, group=None, **kwargs):
        super().__init__(*args, **kwargs)
        if not dist.is_initialized():
            raise RuntimeError("DPOnlineMapper: torch.distributed is not initialised")
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.graphs = DPIterationGraphs(self) if self.dev.type == "cuda" else None
        self.picks = []

    def _pick(self, draw):
        picks = [draw() for _ in range(self.world)]
        self.picks = picks
        return picks[self.rank]

    def _after_backward(self, out, update: bool, need_vis: bool):
        ms = self.ms
        st = ms.store
        allreduce_grads(st, list(self.net.parameters()), self.group)
        if update:  # the statistics densify_and_prune is about to read
            allreduce_flat([st.stat("xyz_gradient_accum"), st.stat("denom")], self.group)
            _all_reduce(st.stat("max_radii2D"), dist.ReduceOp.MAX, self.group)
        vis = out["radii"] > 0
        if need_vis:
            v = vis.to(torch.int32)
            _all_reduce(v, dist.ReduceOp.MAX, self.group)
            vis = v > 0
        return vis

    def _exposure_step(self, kf, out):
        if "dexposure_partials" not in out:
            raise RuntimeError("DPOnlineMapper: the iteration must return dexposure_partials")
        lr = self.cfg["exposure_lr"]
        for uid, g in gather_exposure(kf.uid, out["dexposure_partials"], self.group):
            if uid not in self.kopt_uids:
                continue
            self.kopt_steps[uid] += 1
            self._exposure_apply(uid, g, self.kopt_steps[uid], lr)

    def _record_occ(self, kf, out):
        uids = gather_rows(torch.tensor([int(kf.uid)], dtype=torch.int64, device=self.dev), self.group).view(-1)
        rows = gather_rows((out["n_touched"] > 0).to(torch.int32), self.group)
        for r, u in enumerate(uids.tolist()):
            self.occ_vis[u] = rows[r].long()

    def replica_digest(self) -> torch.Tensor:
        """float64 [world, 4]: each rank's (sum, sum of squares, weighted sum,
        row count) over its Gaussian parameters, MLP and exposures -- equal
        rows mean bit-identical replicas for every practical purpose."""
        parts = [self.ms.store.param(n).reshape(-1) for n in self.ms.GROUPS]
        parts += [p.detach().reshape(-1) for p in self.net.parameters()]
        parts.append(self.bank.ex.reshape(-1))
        x = torch.cat([t.to(torch.float64) for t in parts])
        w = torch.arange(1, x.numel() + 1, dtype=torch.float64, device=x.device).remainder_(1021.0)
        d = torch.stack([x.sum(), (x * x).sum(), (x * w).sum(), torch.tensor(float(self.ms.P), dtype=torch.float64,
                                                                             device=x.device)])
        return gather_rows(d, self.group)


class DPIterationGraphs(IterationGraphs):
    """IterationGraphs for DPOnlineMapper (module docstring): graph A (this
    rank's view -> gradients + the tail), the two SUM all-reduces, graph B
    (Adam on the summed gradients, skipped when any rank overflowed), then
    the exposure steps of the step's keyframes from the summed partials.

    Every rank takes the same path: whether an iteration replays depends only
    on replicated state, and a capture failure raises instead of falling back
    (an eager iteration on one rank would issue other collectives).  Host
    step counts are not rolled back after an overflow (``rollback`` False):
    the rollback would depend on when each rank's host sees its overflow, and
    the replicas' bias corrections must agree."""

    def __init__(self, mapper):
        super().__init__(mapper)
        self.rollback = False
        self.tail = None
        self.skip_dp = torch.zeros(1, dtype=torch.int32, device=self.dev)
        self.one = torch.ones(1, dtype=torch.int32, device=self.dev)
        self.debug = os.environ.get("WGSR_DP_DEBUG", "0") == "1"
        self.stats.update(allreduce_s=0.0)

    def _capture_body(self, nbc: int, refine: bool):
        m = self.m
        world, rank = m.world, m.rank

        box = {}

        def body_a():
            G, gex, skip = self._body_grads(nbc, refine)
            box["nparts"] = int(gex.shape[0])
            box["nG"] = int(G.numel())  # (wgsr_mlp_grad_floats: may exceed the parameters' count)
            # the tail: MLP gradient | overflow (float) | [world, nparts, 2]
            # exposure partials, this rank's row filled (a gather by SUM);
            # allocated in the graphs' pool, one per captured pair
            ex = torch.zeros(world, box["nparts"] * 2, device=self.dev)
            ex[rank].copy_(gex.reshape(-1))
            box["tail"] = torch.cat([G.reshape(-1), skip.to(torch.float32), ex.reshape(-1)])
            # this rank's overflow bookkeeping (the capacity is per rank): the
            # exposure-step kernel with its own skip word set does only that
            # (sticky[0] += overflow, sticky[1] = max N_rect)
            L = _lib.load()
            p = _lib.ptr
            with torch.cuda.device(self.dev):
                _lib.check(L.wgsr_exposure_step(p(self.m.bank.ex), p(self.i64), p(gex), int(gex.shape[0]),
                                                p(self.f32[self.F_EXPO:self.F_EXPO + 2]), p(skip), p(self.one),
                                                0.9, 0.999, 1e-8, p(self.sticky), p(self.counts), None,
                                                _lib.stream_handle(self.dev)))

        def body_b():
            tail, nG = box["tail"], box["nG"]
            self.skip_dp.copy_((tail[nG:nG + 1] > 0).to(torch.int32))
            self._body_adam(tail[:nG], self.skip_dp)

        ga = self._capture_one(body_a)
        gb = self._capture_one(body_b)
        self.tail = box["tail"]  # (the latest; bench_online reports its size)
        return ga, gb, box["tail"], box["nparts"], box["nG"]

    def _check(self, where, tail):
        """WGSR_DP_DEBUG=1: synchronise and check the step's state (the
        forward's counts, the tail, the store's gradients and parameters,
        the exposure bank); raise with the iteration on the first bad one."""
        m = self.m
        torch.cuda.synchronize(self.dev)
        c = self.counts.tolist()
        st = m.ms.store
        bad = [f"counts {c}"] if (c[0] < 0 or c[0] > (1 << 28)) else []
        bad += [] if bool(torch.isfinite(tail).all()) else ["tail not finite"]
        for n in m.ms.GROUPS:
            bad += [] if bool(torch.isfinite(st.grad(n)).all()) else [f"grad {n} not finite"]
            bad += [] if bool(torch.isfinite(st.param(n)).all()) else [f"param {n} not finite"]
        bad += [] if bool(torch.isfinite(m.bank.ex).all()) else ["exposure bank not finite"]
        if bad:
            raise RuntimeError(f"DPIterationGraphs {where} (iteration {m.iteration_count}, replay "
                               f"{self.stats['replays']}, cap {self.cap}, P {m.ms.P}, slots {self.i64.tolist()}): "
                               f"{'; '.join(bad)}")

    def _capture(self, nbc: int, refine: bool):
        g = super()._capture(nbc, refine)
        if g is None and self.disabled is not None:
            raise RuntimeError(f"DPIterationGraphs: capture failed on rank {self.m.rank}: {self.disabled}")
        return g

    def _fill_exposure(self, kf, f, u):
        pass  # (the exposure steps run after the exchange, _replay)

    def _replay(self, g, kf):
        m = self.m
        ga, gb, tail, nparts, nG = g
        ga.replay()
        dbg = self.debug
        if dbg:
            self._check("after graph A", tail)
        t0 = _time()
        _all_reduce(m.ms.store.grad_flat(), dist.ReduceOp.SUM, m.group)
        _all_reduce(tail, dist.ReduceOp.SUM, m.group)
        self.stats["allreduce_s"] += _time() - t0
        if dbg:
            self._check("after the all-reduces", tail)
        gb.replay()
        if dbg:
            self._check("after graph B", tail)
        # the exposure steps: every keyframe the ranks drew (every rank knows
        # the draws), one step on the sum of its ranks' partials
        uids = [m.stack[c] for c in m.picks]
        ex = tail[nG + 1:].view(m.world, nparts, 2)
        lr = m.cfg["exposure_lr"]
        done = set()
        for r, uid in enumerate(uids):
            if uid in done or uid not in m.kopt_uids:
                continue
            done.add(uid)
            rows = [q for q, v in enumerate(uids) if v == uid]
            g_ex = ex[r] if len(rows) == 1 else ex[rows].reshape(-1, 2)
            m.kopt_steps[uid] += 1
            m._exposure_apply(uid, g_ex, m.kopt_steps[uid], lr, skip=self.skip_dp)


def _time():
    import time
    return time.perf_counter()
