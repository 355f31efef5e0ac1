"""Graph-replayed mapping iterations for ``wgsr.online``.

The reference's mapper (src/mapper.py:1083-1219, 1234-1372) runs each
mapping iteration as ~100 eager kernels with several host synchronisations;
the eager restatement in ``OnlineMapper._iteration`` fuses them to ~35
launches, but one mapping iteration at TUM scale is still bounded by the
host: ~1.8 ms of wall clock for ~0.7 ms of kernels, with the rasteriser's one
host wait (num_rendered) draining the queue every iteration.

Here the steady-state iteration -- no densify / reset, no visibility update,
the DINO term on, the uncertainty loss not frozen -- is captured ONCE per
(map state, neighbour count) as a HIP graph and replayed:

* the keyframe is chosen on the host as before and handed over as a slot
  index: every keyframe's image, depth, features, camera, median depth and
  exposure (+ its Adam moments) live in slot-indexed device banks
  (``KeyframeBank``; the Keyframe objects' tensors are views into them), and
  the graph gathers the chosen slot's rows (one wgsr_gather_rows launch) and
  steps the exposure on its bank row (wgsr_exposure_step);
* the rasteriser runs in capacity mode (wgsr_rasterize_forward_cap): buffers
  sized for ``cap`` pairs, counts on the device, no host wait.  An overflow
  (more pairs than ``cap``) makes the iteration a no-op for every optimiser
  (device skip word) and is seen by the host a few iterations later through a
  pinned flag, which recaptures with a larger capacity;
* everything that changes per step -- the three dropout / sampling seeds,
  every Adam step size and bias correction (Gaussians, MLP, exposure), the
  exposure skip flag, the slot indices -- arrives in one 256-byte block
  copied host->device ahead of the replay (a ring of pinned blocks);
* the uncertainty MLP, the DINO sampling (the first n / reg_stride^4 entries
  of the hash-key permutation, wgsr_random_perm_prefix) and regulariser, and
  all three Adams run without autograd; the MLP's two forwards (keyframe
  features, DINO sample) are one launch and its two backwards one more
  (wgsr.mlp.forward_raw2 / backward_raw2, wgsr.uncertainty.dino_reg_raw,
  wgsr_adam_step_dev).

The eager path draws the same seeds in the same order and uses the same
kernels (the MLP per segment), so a replayed iteration computes what
``_iteration`` computes up to the order of the MLP gradient's sum
(tests/test_gpu_online_graph.py compares them).  Any change of the map's
shape (P, the store's banks, the keyframe banks) invalidates the graphs;
they are recaptured lazily.
"""
from __future__ import annotations

import math
import os
import time

import numpy as np
import torch

from . import _lib
from .mlp import backward_raw, backward_raw2, forward_raw, forward_raw2
from .uncertainty import dino_reg_raw

CAM_FLOATS = 52  # viewmatrix 16 | projmatrix 16 | projmatrix_raw 16 | campos 3 | pad


class KeyframeBank:
    """Slot-indexed device banks of the keyframes' per-view data.

    ``sync(keyframes)`` adopts new keyframes (copies their tensors into a
    slot and rebinds the Keyframe's fields to views of it) and refreshes
    fields a caller replaced (a pose update's new camera tensors, a new
    depth).  The exposure bank ``ex`` [K, 3, 2] = (a, b), Adam exp_avg,
    Adam exp_avg_sq per slot is always kept (the exposure optimiser steps
    through it); the image banks only while every keyframe has the same
    image / feature shape and field of view (``uniform``)."""

    def __init__(self, dev):
        self.dev = torch.device(dev)
        self.cap = 0
        self.slots: dict[int, int] = {}
        self.kfs: dict[int, object] = {}
        self.ex = torch.zeros(0, 3, 2, device=self.dev)
        self.shape = None   # (H, W, h, w, C)
        self.tan = None     # (tanfovx, tanfovy)
        self.uniform = True
        self.image = self.depth = self.feat = self.cam = self.med = None
        self.version = 0

    # -- layout ------------------------------------------------------------
    def _alloc(self, cap):
        old = (self.ex, self.image, self.depth, self.feat, self.cam, self.med)
        n = self.cap
        self.ex = torch.zeros(cap, 3, 2, device=self.dev)
        self.ex[:n].copy_(old[0][:n])
        if self.uniform and self.shape is not None:
            H, W, h, w, C = self.shape
            shapes = ((3, H, W), (1, H, W), (h, w, C), (CAM_FLOATS,), ())
            new = [torch.zeros((cap,) + s, device=self.dev) for s in shapes]
            for t, o in zip(new, old[1:]):
                if o is not None and n:
                    t[:n].copy_(o[:n])
            self.image, self.depth, self.feat, self.cam, self.med = new
        self.cap = cap
        self.version += 1
        for uid, kf in self.kfs.items():
            self._bind(uid, kf)

    def _addr(self, t, slot):
        return t.data_ptr() + slot * t[0].numel() * t.element_size()

    def _stale(self, uid, kf):
        s = self.slots[uid]
        out = []
        base = self._addr(self.ex, s)
        if kf.exposure_a.data_ptr() != base or kf.exposure_b.data_ptr() != base + 4:
            out.append("ex")
        if self.uniform and self.image is not None:
            for name, bank, t in (("image", self.image, kf.image), ("depth", self.depth, kf.depth),
                                  ("feat", self.feat, kf.features), ("med", self.med, kf.median_depth)):
                if not torch.is_tensor(t) or t.data_ptr() != self._addr(bank, s):
                    out.append(name)
            cb = self._addr(self.cam, s)
            if any(kf.cam[k].data_ptr() != cb + 4 * o for k, o in
                   (("viewmatrix", 0), ("projmatrix", 16), ("projmatrix_raw", 32), ("campos", 48))):
                out.append("cam")
        return out

    def _store(self, uid, kf, fields):
        s = self.slots[uid]
        with torch.no_grad():
            if "ex" in fields:
                self.ex[s, 0, 0:1].copy_(kf.exposure_a.detach().reshape(1))
                self.ex[s, 0, 1:2].copy_(kf.exposure_b.detach().reshape(1))
            if not (self.uniform and self.image is not None):
                return
            if "image" in fields:
                self.image[s].copy_(kf.image.reshape(self.image.shape[1:]))
            if "depth" in fields:
                self.depth[s].copy_(kf.depth.reshape(self.depth.shape[1:]))
            if "feat" in fields:
                self.feat[s].copy_(kf.features.reshape(self.feat.shape[1:]))
            if "med" in fields:
                self.med[s].copy_(torch.as_tensor(kf.median_depth, device=self.dev).reshape(()))
            if "cam" in fields:
                c = self.cam[s]
                for k, o, n in (("viewmatrix", 0, 16), ("projmatrix", 16, 16), ("projmatrix_raw", 32, 16),
                                ("campos", 48, 3)):
                    c[o:o + n].copy_(kf.cam[k].reshape(-1))

    def _bind(self, uid, kf):
        s = self.slots[uid]
        kf.exposure_a = self.ex[s, 0, 0:1]
        kf.exposure_b = self.ex[s, 0, 1:2]
        if self.uniform and self.image is not None:
            kf.image = self.image[s]
            kf.depth = self.depth[s]
            kf.features = self.feat[s]
            kf.median_depth = self.med[s]
            c = self.cam[s]
            kf.cam = dict(kf.cam, viewmatrix=c[0:16].view(4, 4), projmatrix=c[16:32].view(4, 4),
                          projmatrix_raw=c[32:48].view(4, 4), campos=c[48:51])

    def _check_shape(self, kf):
        H, W = kf.image.shape[-2:]
        h, w, C = kf.features.shape[-3:]
        shp = (int(H), int(W), int(h), int(w), int(C))
        tan = (float(kf.cam["tanfovx"]), float(kf.cam["tanfovy"]))
        ok = (kf.image.dtype == torch.float32 and kf.features.dtype == torch.float32
              and kf.depth.numel() == H * W and kf.image.device == self.dev)
        if self.shape is None and ok:
            self.shape, self.tan = shp, tan
            return
        if not ok or shp != self.shape or tan != self.tan:
            self.uniform = False  # (graphs off; the exposure bank stays)

    # -- public ------------------------------------------------------------
    def sync(self, keyframes: dict):
        """Adopt new keyframes, refresh replaced fields of adopted ones."""
        for uid, kf in keyframes.items():
            if uid in self.slots and self.kfs.get(uid) is kf:
                st = self._stale(uid, kf)
                if st:
                    self._store(uid, kf, st)
                    self._bind(uid, kf)
        for uid, kf in keyframes.items():
            if self.kfs.get(uid) is kf:
                continue
            if uid not in self.slots:
                was_uniform = self.uniform
                self._check_shape(kf)
                if was_uniform and not self.uniform:
                    self.version += 1  # (graphs off from here on)
                need_images = self.uniform and self.image is None and self.shape is not None
                if len(self.slots) >= self.cap or need_images:
                    # (re)allocates and rebinds the keyframes adopted so far;
                    # this one is bound below, after its data is stored
                    self._alloc(max(16, 2 * self.cap, len(self.slots) + 1))
                self.slots[uid] = len(self.slots)
            with torch.no_grad():
                self.ex[self.slots[uid], 1:].zero_()
            self._store(uid, kf, ("ex", "image", "depth", "feat", "med", "cam"))
            self.kfs[uid] = kf
            self._bind(uid, kf)

    def ex_ptrs(self, uid):
        """(param, exp_avg, exp_avg_sq) device addresses of uid's exposure row."""
        b = self._addr(self.ex, self.slots[uid])
        return b, b + 8, b + 16


class IterationGraphs:
    """The steady-state mapping iteration as replayed HIP graphs (module doc)."""

    NF = 40                       # float words of the per-step block
    F_GAUSS, F_MLP, F_EXPO, F_EXSKIP = 3, 18, 36, 39
    RING = 16
    PEEK = 4  # replays between the host's looks at the overflow words

    def __init__(self, mapper):
        self.m = mapper
        dev = mapper.dev
        self.dev = dev
        self.block = torch.zeros(256, dtype=torch.uint8, device=dev)
        self.f32 = self.block[:160].view(torch.float32)
        self.i32 = self.block[:160].view(torch.int32)
        self.i64 = self.block[160:208].view(torch.int64)
        self.ring = torch.zeros(self.RING, 256, dtype=torch.uint8).pin_memory()
        rn = self.ring.numpy()
        self.ring_f = rn[:, :160].view(np.float32)
        self.ring_u = rn[:, :160].view(np.uint32)
        self.ring_i = rn[:, 160:208].view(np.int64)
        self.ring_ev = [None] * self.RING
        self.slot = 0
        self.counts = torch.zeros(5, dtype=torch.int32, device=dev)
        self.sticky = torch.zeros(2, dtype=torch.int64, device=dev)   # overflowed replays, max N_rect
        self.sticky_host = torch.zeros(2, dtype=torch.int64).pin_memory()
        self.sticky_np = self.sticky_host.numpy()
        # per exposure-bank row: replayed exposure steps the overflow word held
        # back (the host had already counted them in kopt_steps)
        self.slot_skips = torch.zeros(0, dtype=torch.int64, device=dev)
        self.replays_since_account = 0
        self.pending_mx = 0          # largest N_rect of replays already accounted
        self.graphs = {}
        self.key = None
        self.pool = None
        self.stream = None
        self.cap = None
        self.S = None
        self.disabled = None  # reason string once disabled
        self.stats = {"captures": 0, "replays": 0, "overflows": 0, "skipped_iterations": 0, "capture_s": 0.0,
                      "replay_call_s": 0.0, "step_host_s": 0.0}
        # capacity = max(min_cap, cap_scale x the largest recent pair count + cap_margin)
        self.min_cap, self.cap_scale, self.cap_margin = 1 << 16, 2.0, 4096
        # account() rolls the host step counts of overflowed (skipped) replays
        # back; the data-parallel graphs keep them (wgsr.dp_online)
        self.rollback = True

    # -- eligibility -----------------------------------------------------------
    def usable(self) -> bool:
        m = self.m
        if self.disabled is not None or os.environ.get("WGSR_ONLINE_GRAPH", "1") == "0":
            return False
        if m.dev.type != "cuda" or m.ms is None or m.ms.P == 0 or getattr(m.ms, "_skip", None):
            return False
        if m.net.seed_source is not None or "_perm" in m.__dict__:
            return False  # a test feeds the random draws: eager only
        return m.bank.uniform and m.bank.image is not None

    def _map_key(self):
        st = self.m.ms.store
        return (st.P, st.cur, id(st.banks), self.m.bank.version)

    def invalidate(self):
        if self.graphs and self.replays_since_account:
            # (a replay may still be running: its graph, kernel arguments and
            # pool must outlive it)
            torch.cuda.synchronize(self.dev)
        self.graphs = {}
        self.pool = None
        self.S = None

    # -- static state ----------------------------------------------------------
    def _build_static(self):
        m = self.m
        B = m.bank
        H, W, h, w, C = B.shape
        dev = self.dev
        S = type("Static", (), {})()
        S.image4 = torch.zeros(1, 3, H, W, device=dev)
        S.depth4 = torch.zeros(1, 1, H, W, device=dev)
        S.feat4 = torch.zeros(1, h, w, C, device=dev)
        S.cam2 = torch.zeros(1, CAM_FLOATS, device=dev)
        S.med = torch.zeros(1, device=dev)
        S.ex = torch.zeros(2, device=dev)          # the keyframe's exposure (a, b)
        S.nbf = torch.zeros(5, h, w, C, device=dev)
        S.keys = torch.zeros(5 * h * w, dtype=torch.int32, device=dev)
        S.perm = torch.zeros(5 * h * w, dtype=torch.int32, device=dev)
        c = S.cam2[0]
        S.cam = dict(viewmatrix=c[0:16].view(4, 4), projmatrix=c[16:32].view(4, 4), projmatrix_raw=c[32:48].view(4, 4),
                     campos=c[48:51], tanfovx=B.tan[0], tanfovy=B.tan[1], image_height=H, image_width=W)
        # the MLP optimiser's state must exist before a capture bakes its addresses in
        opt = m.uopt
        S.mlp_params = list(m.net.parameters())
        S.mlp_steps = []
        for p in S.mlp_params:
            st = opt.state[p]
            if len(st) == 0:
                st["step"] = torch.tensor(0.0)
                st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            S.mlp_steps.append(st["step"])
        g = opt.param_groups[0]
        S.mlp_lr, S.mlp_betas, S.mlp_eps, S.mlp_wd = g["lr"], g["betas"], g["eps"], g.get("weight_decay", 0.0)
        m.ms.iso_part  # noqa: B018  (allocated outside the capture)
        if self.slot_skips.numel() < B.ex.shape[0]:
            self.slot_skips = torch.zeros(B.ex.shape[0], dtype=torch.int64, device=dev)
        self.S = S

    def _gather_jobs(self, nbc: int):
        """wgsr_gather_rows jobs: the chosen slot's rows into the static
        buffers, the neighbours' features (one launch)."""
        B, S = self.m.bank, self.S
        p = _lib.ptr

        def job(bank, dst, off, n, words=None, stride=None):
            rw = bank[0].numel() if words is None else words
            return _lib.GatherJob(p(bank), p(dst), rw, rw if stride is None else stride, off, n)
        jobs = [job(B.image, S.image4, 0, 1), job(B.depth, S.depth4, 0, 1), job(B.feat, S.feat4, 0, 1),
                job(B.cam, S.cam2, 0, 1), job(B.med, S.med, 0, 1), job(B.ex, S.ex, 0, 1, words=2, stride=6),
                job(B.feat, S.nbf, 1, nbc)]
        return (_lib.GatherJob * len(jobs))(*jobs)

    def _body(self, nbc: int, refine: bool):
        """One mapping iteration's device work (captured; see the module doc)."""
        G, gex, skip = self._body_grads(nbc, refine)
        self._body_exposure(gex, skip)
        self._body_adam(G, skip)

    def _body_grads(self, nbc: int, refine: bool):
        """The iteration up to its gradients: the keyframe's rows gathered, the
        DINO draw, the MLP forwards, the loss and rasteriser forward/backward
        (capacity mode; the Gaussians' gradients into the store) and the MLP
        backward -> (MLP gradient G, exposure partials, overflow word)."""
        m, S = self.m, self.S
        ms, B, c = m.ms, m.bank, m.cfg
        L = _lib.load()
        dev = self.dev
        st = _lib.stream_handle(dev)
        p = _lib.ptr
        H, W, h, w, C = B.shape
        with torch.cuda.device(dev):
            jobs = self._gather_jobs(nbc)
            _lib.check(L.wgsr_gather_rows(jobs, len(jobs), p(self.i64), st))
        # the DINO term's draw: features sampled from the neighbouring
        # keyframes (the first ns entries of the random permutation)
        n = nbc * h * w
        ns = n // (c["reg_stride"] ** 4)
        with torch.cuda.device(dev):
            if n <= int(L.wgsr_random_perm_prefix_max_n()) and ns <= int(L.wgsr_random_perm_prefix_max_k()):
                _lib.check(L.wgsr_random_perm_prefix(n, ns, 0, p(self.i32[1:2]), p(S.perm), st))
                perm = S.perm[:ns]
            elif n <= int(L.wgsr_random_perm_max()):
                _lib.check(L.wgsr_random_perm(n, 0, p(self.i32[1:2]), p(S.keys), p(S.perm), st))
                perm = S.perm[:ns]
            else:  # (large feature maps: the same keys, torch's stable sort)
                _lib.check(L.wgsr_random_keys(n, 0, p(self.i32[1:2]), p(S.keys), st))
                perm = torch.argsort(S.keys[:n], stable=True)[:ns]
        sf = S.nbf[:nbc].view(n, C).index_select(0, perm)
        # the uncertainty MLP on the keyframe's features and on the sample (one
        # launch, each with its own dropout draw), the loss + rasteriser
        # forward/backward (capacity mode), the DINO term, and one MLP backward
        # of both (the DINO gradient scaled by reg_mult: autograd's sum)
        if ns > 0:
            u_all, sv = forward_raw2(m.net, S.feat4.view(h * w, C), sf, self.i32[0:1], self.i32[2:3])
            u, u2 = u_all[:h * w], u_all[h * w:]
        else:
            u, sv = forward_raw(m.net, S.feat4.view(h * w, C), self.i32[0:1])
        out = ms.forward_backward_uncertainty(S.cam, S.image4[0], S.depth4[0], S.ex[0:1], S.ex[1:2], m.bg,
                                              u.view(h, w), c["train_frac_fix"], c["train_frac_fix"],
                                              freeze_uncertainty_loss=False, median_depth=S.med,
                                              pre_exposed=not refine, cap=self.cap, counts=self.counts,
                                              need_tau=False, exposure_partials=True, stats=not refine)
        du = out["uncertainty_grad"].reshape(-1).contiguous()
        if ns > 0:
            _, gu = dino_reg_raw(u2, sf, want_loss=False)
            G = backward_raw2(sv, du, gu, 1.0, float(c["reg_mult"]))
        else:
            G = backward_raw(sv, du)
        return G, out["dexposure_partials"], self.counts[3:4]

    def _body_exposure(self, gex, skip):
        """The keyframe's exposure Adam step on its bank row (skipped unless the
        window optimiser holds it; also the overflow bookkeeping)."""
        L = _lib.load()
        p = _lib.ptr
        with torch.cuda.device(self.dev):
            _lib.check(L.wgsr_exposure_step(p(self.m.bank.ex), p(self.i64), p(gex), int(gex.shape[0]),
                                            p(self.f32[self.F_EXPO:self.F_EXPO + 2]),
                                            p(skip), p(self.i32[self.F_EXSKIP:self.F_EXSKIP + 1]), 0.9, 0.999, 1e-8,
                                            p(self.sticky), p(self.counts), p(self.slot_skips),
                                            _lib.stream_handle(self.dev)))

    def _body_adam(self, G, skip):
        """The Gaussians' and the MLP's Adam (L2 weight decay for the MLP), one
        launch when their betas agree; nothing moves when the skip word is set."""
        m, S = self.m, self.S
        ms = m.ms
        L = _lib.load()
        dev = self.dev
        st = _lib.stream_handle(dev)
        p = _lib.ptr
        ts, off = [], 0
        opt = m.uopt
        for prm in S.mlp_params:
            k = prm.numel()
            sto = opt.state[prm]
            ts.append(_lib.AdamTensor(prm.data_ptr(), G.data_ptr() + 4 * off, sto["exp_avg"].data_ptr(),
                                      sto["exp_avg_sq"].data_ptr(), k, 0.0, 1.0))
            off += k
        # the Gaussians' and the MLP's Adam in one launch (shared betas)
        gts = ms.adam_tensors()
        with torch.cuda.device(dev):
            if tuple(ms.betas) == tuple(S.mlp_betas):
                allt = gts + ts
                _lib.check(L.wgsr_adam_step_dev2((_lib.AdamTensor * len(allt))(*allt), len(gts), len(allt),
                                                 ms.betas[0], ms.betas[1], ms.eps, 0.0,
                                                 p(self.f32[self.F_GAUSS:self.F_GAUSS + 15]), S.mlp_eps, S.mlp_wd,
                                                 p(self.f32[self.F_MLP:self.F_MLP + 18]), p(skip), st))
            else:
                ms.optimizer_step_dev(gts, self.f32[self.F_GAUSS:self.F_GAUSS + 15], skip)
                _lib.check(L.wgsr_adam_step_dev((_lib.AdamTensor * len(ts))(*ts), len(ts), S.mlp_betas[0],
                                                S.mlp_betas[1], S.mlp_eps, S.mlp_wd,
                                                p(self.f32[self.F_MLP:self.F_MLP + 18]), p(skip), st))

    def _capture_one(self, fn):
        """One graph of ``fn``'s device work on the capture stream, in the
        shared pool."""
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(self.stream):
            g.capture_begin(pool=self.pool)
            try:
                fn()
            finally:
                g.capture_end()
        return g

    def _capture_body(self, nbc: int, refine: bool):
        """-> what ``_replay`` launches: the whole iteration as one graph."""
        return self._capture_one(lambda: self._body(nbc, refine))

    def _capture(self, nbc: int, refine: bool):
        t0 = time.perf_counter()
        try:
            return self._capture_timed(nbc, refine)
        finally:
            self.stats["capture_s"] += time.perf_counter() - t0

    def _capture_timed(self, nbc: int, refine: bool):
        if self.S is None:
            self._build_static()
        # (capture_begin / capture_end directly: torch.cuda.graph's context
        # also runs gc.collect() and empty_cache() per capture, tens of ms)
        if self.pool is None:
            self.pool = torch.cuda.graph_pool_handle()
        if self.stream is None:
            self.stream = torch.cuda.Stream(self.dev)
        cur = torch.cuda.current_stream(self.dev)
        self.stream.wait_stream(cur)
        try:
            g = self._capture_body(nbc, refine)
        except Exception as e:  # e.g. a configuration the capacity-mode forward does not cover
            self.disabled = f"{type(e).__name__}: {e}"
            self.invalidate()
            return None
        cur.wait_stream(self.stream)
        self.graphs[(nbc, refine)] = g
        self.stats["captures"] += 1
        return g

    # -- the step ----------------------------------------------------------------
    def _fill_exposure(self, kf, f, u):
        """The per-step block's exposure fields: keyframe ``kf``'s Adam step
        size and bias correction when the window optimiser holds it (its host
        step count advanced), else the skip flag."""
        m = self.m
        if kf.uid in m.kopt_uids:
            m.kopt_steps[kf.uid] += 1
            ne = m.kopt_steps[kf.uid]
            lr = m.cfg["exposure_lr"]
            f[self.F_EXPO:self.F_EXPO + 3] = (lr / (1.0 - 0.9 ** ne), math.sqrt(1.0 - 0.999 ** ne), 0.0)
            u[self.F_EXSKIP] = 0
        else:
            u[self.F_EXSKIP] = 1

    def _replay(self, g, kf):
        """Launch the captured iteration (its per-step block already queued)."""
        g.replay()

    def account(self, consume: bool = False):
        """Settle the overflow bookkeeping of the replays so far: wait for them
        (so no in-flight replay is missed), roll back the step counts of the
        optimiser steps an overflow held back -- the Gaussians' and the MLP's
        by the overflow count, each keyframe's exposure by its row's count in
        ``slot_skips`` -- and zero the device words.  Called before the
        capacity changes and whenever the host is about to reset or read the
        step counts (the end of a map_opt_online / final_refine call, a new
        exposure optimiser).  Returns (overflowed replays, largest N_rect);
        the latter is kept for the next capacity check unless ``consume``."""
        if self.replays_since_account == 0:
            mx = self.pending_mx
            if consume:
                self.pending_mx = 0
            return 0, mx
        torch.cuda.synchronize(self.dev)
        self.replays_since_account = 0
        self.sticky_host.copy_(self.sticky)
        ovf, mx = int(self.sticky_np[0]), max(int(self.sticky_np[1]), self.pending_mx)
        if ovf and not self.rollback:
            self.stats["overflows"] += 1
            self.stats["skipped_iterations"] += ovf
            self.m.events.append((self.m.iteration_count, "capacity_overflow", {"cap": self.cap, "skipped": ovf}))
        elif ovf:
            self.stats["overflows"] += 1
            self.stats["skipped_iterations"] += ovf
            # the skipped steps advanced no moments on the device: undo their counts
            for name in self.m.ms.GROUPS:
                self.m.ms.steps[name] -= ovf
            if self.S is not None:
                for t in self.S.mlp_steps:
                    t -= ovf
            sk = self.slot_skips.cpu().numpy()
            if sk.any():
                by_slot = {s_: u for u, s_ in self.m.bank.slots.items()}
                for s_ in np.nonzero(sk)[0]:
                    uid = by_slot.get(int(s_))
                    if uid in self.m.kopt_steps:
                        self.m.kopt_steps[uid] -= int(sk[s_])
                self.slot_skips.zero_()
            self.m.events.append((self.m.iteration_count, "capacity_overflow", {"cap": self.cap, "skipped": ovf}))
        self.sticky.zero_()
        self.sticky_np[:] = 0
        self.pending_mx = 0 if consume else mx
        return ovf, mx

    def _check_capacity(self, new_generation: bool):
        """The pair capacity: twice the largest upstream num_rendered seen since
        the last check (replays through the pinned copy of the device maximum,
        eager iterations through the mapper's own record) + 4096.  Changed --
        and the graphs recaptured -- after an overflow, when the maximum comes
        within 3/4 of the capacity, or, for a new map state, when it is more
        than twice what is needed (the map shrank after a prune)."""
        ovf, mx = int(self.sticky_np[0]), max(int(self.sticky_np[1]), self.pending_mx)
        if not new_generation and self.cap is not None and not ovf and mx <= 0.75 * self.cap:
            return
        ovf, mx = self.account(consume=True)
        want = max(self.min_cap, int(self.cap_scale * max(mx, int(self.m._max_nr))) + self.cap_margin)
        if ovf and self.cap is not None:
            want = max(want, 2 * self.cap)
        if self.cap is None or ovf or mx > 0.75 * self.cap or want > self.cap or 2 * want < self.cap:
            if self.cap is not None and want != self.cap:
                self.invalidate()
            if want != self.cap:  # (the capacity's history: iteration, old, new, overflows, max N_rect)
                log = self.stats.setdefault("cap_log", [])
                if len(log) < 64:
                    log.append((self.m.iteration_count, self.cap, want, ovf, mx, int(self.m._max_nr)))
            self.cap = want
        self.m._max_nr = 0

    def step(self, kf, neighbours, refine: bool = False) -> bool:
        """Run one steady-state iteration on keyframe ``kf`` as a graph replay;
        False when the graph path does not apply (the caller runs it eagerly)."""
        if not self.usable():
            return False
        t_step = time.perf_counter()
        m = self.m
        nbc = len(neighbours)
        if not 1 <= nbc <= 5:
            return False
        key = self._map_key()
        fresh = key != self.key
        if fresh:
            # settle the replays of the old map state first: account() waits
            # for them (no graph or pool is dropped under an in-flight replay)
            # and rolls the MLP step counts back while S still holds them
            self.account()
            self.invalidate()
            self.key = key
        self._check_capacity(fresh)
        g = self.graphs.get((nbc, refine))
        if g is None:
            g = self._capture(nbc, refine)
            if g is None:
                return False
        S = self.S
        i = self.slot
        self.slot = (i + 1) % self.RING
        ev = self.ring_ev[i]
        if ev is not None:
            ev.synchronize()
        f, u, ix = self.ring_f[i], self.ring_u[i], self.ring_i[i]
        # the seeds in the eager path's order: MLP forward, DINO draw, DINO MLP
        # forward (one batched draw: the same three values as three single ones)
        u[0:3] = torch.randint(0, 2 ** 31 - 1, (3,)).tolist()
        m.ms.adam_scalars(f[self.F_GAUSS:self.F_GAUSS + 15])
        b1, b2 = S.mlp_betas
        n = float(S.mlp_steps[0]) + 1.0
        bc1 = 1.0 - b1 ** n
        bc2s = math.sqrt(1.0 - b2 ** n)
        f[self.F_MLP:self.F_MLP + 18] = np.tile(np.array([S.mlp_lr / bc1, bc2s, S.mlp_lr / bc1], np.float32), 6)
        self._fill_exposure(kf, f, u)
        ix[0] = m.bank.slots[kf.uid]
        for j, k in enumerate(neighbours):
            ix[1 + j] = m.bank.slots[k]
        self.block.copy_(self.ring[i], non_blocking=True)
        if ev is None:
            ev = self.ring_ev[i] = torch.cuda.Event()
        ev.record()
        t_rep = time.perf_counter()
        self._replay(g, kf)
        t_end = time.perf_counter()
        torch._foreach_add_(S.mlp_steps, 1.0)
        self.stats["replays"] += 1
        # the overflow bookkeeping, seen by the host through pinned memory:
        # every PEEK-th replay (a blit kernel per replay cost ~4 us of the
        # ~0.4-0.7 ms iteration); account() reads the device words after its
        # synchronize, so only the early capacity check sees the lag
        if self.stats["replays"] % self.PEEK == 0:
            self.sticky_host.copy_(self.sticky, non_blocking=True)
        self.replays_since_account += 1
        self.stats["replay_call_s"] += t_end - t_rep
        self.stats["step_host_s"] += time.perf_counter() - t_step
        return True
