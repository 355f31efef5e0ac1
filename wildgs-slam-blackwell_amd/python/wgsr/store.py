"""The GaussianModel state in a capacity-preallocated SoA.

The reference grows and shrinks its six parameter tensors and their Adam
moments with ``torch.cat`` / boolean indexing on every keyframe insertion,
densification and prune (thirdparty/gaussian_splatting/scene/gaussian_model.py:
231-269, 526-743): each re-allocates ~18 tensors.  ``GaussianStore`` keeps
them in two preallocated banks of ``capacity`` rows:

* parameters (raw, as ``_xyz``, ``_features_dc|_features_rest`` fused into one
  [C, M, 3] SH storage, ``_opacity``, ``_scaling``, ``_rotation``), their Adam
  moments (``exp_avg`` / ``exp_avg_sq``), keyframe ids and observation counts
  (``unique_kfIDs`` / ``n_obs``) -- per bank;
* gradients, densification statistics (``xyz_gradient_accum``, ``denom``,
  ``max_radii2D``) and activation scratch -- one copy.

A densify / prune reads the current bank and writes the other
(csrc/densify.hip: select + scan + emit, one host read of the four region
sizes); a keyframe insertion writes the new rows after the last one.  Only
when the row count outgrows the capacity are both banks re-allocated
(geometric growth).  Views ``[:P]`` of the current bank are what the
rasteriser and the optimizer see.
"""
from __future__ import annotations

import ctypes
import math

import numpy as np
import torch

from . import _lib

PARAMS = ("xyz", "features", "opacity", "scaling", "rotation")


def inverse_sigmoid(x: torch.Tensor) -> torch.Tensor:
    """general_utils.inverse_sigmoid (general_utils.py:21-22)."""
    return torch.log(x / (1 - x))


def rotation_matrix_to_quaternion(R: torch.Tensor) -> torch.Tensor:
    """general_utils.rotation_matrix_to_quaternion (general_utils.py:138-162),
    op for op in fp32: [B, >=3, >=3] -> [B, 4] (w, x, y, z), including its sign
    rule q_i *= sign(q_i (R_kj - R_jk)) (a zero difference zeroes q_i)."""
    # (the sums, maxima, halvings and signs in numpy on the host tensor's
    # dtype -- the same IEEE operations in the same order -- and each square
    # root by torch on its [n] vector as the reference takes it (torch's CPU
    # sqrt is not always numpy's): bit-identical to the ~20 small torch ops,
    # in a tenth of the host time; tests/test_online_host.py)
    r = R.detach().cpu().numpy()
    one = r.dtype.type(1)
    zero = r.dtype.type(0)
    r00, r11, r22 = r[:, 0, 0], r[:, 1, 1], r[:, 2, 2]
    q = np.empty((r.shape[0], 4), dtype=r.dtype)
    for i, v in enumerate((one + r00 + r11 + r22, one + r00 - r11 - r22, one - r00 + r11 - r22,
                           one - r00 - r11 + r22)):
        q[:, i] = torch.sqrt(torch.from_numpy(np.maximum(zero, v))).numpy() / 2
    q[:, 1] *= np.sign(q[:, 1] * (r[:, 2, 1] - r[:, 1, 2]))
    q[:, 2] *= np.sign(q[:, 2] * (r[:, 0, 2] - r[:, 2, 0]))
    q[:, 3] *= np.sign(q[:, 3] * (r[:, 1, 0] - r[:, 0, 1]))
    return torch.from_numpy(q)


def deform_transform(w2c: torch.Tensor, w2c_old: torch.Tensor):
    """(T, q) of mapper.py:449-460 / 530-545: T = inv(inv(w2c_old) @ w2c),
    q = rotation_matrix_to_quaternion(T), fp32 on the host.  Batched: [n, 4,
    4] poses give [n, 4, 4] / [n, 4]."""
    if w2c.dim() == 3:
        T = torch.linalg.inv(torch.linalg.inv(w2c_old) @ w2c)
        return T, rotation_matrix_to_quaternion(T)
    T = torch.linalg.inv(torch.linalg.inv(w2c_old) @ w2c)
    return T, rotation_matrix_to_quaternion(T.unsqueeze(0))[0]


class GaussianStore:
    def __init__(self, xyz, features, opacity, scaling, rotation, capacity: int | None = None,
                 kf_id=None, n_obs=None, growth: float = 1.5):
        dev = xyz.device
        self.device = dev
        self.P = P = int(xyz.shape[0])
        self.M = int(features.shape[1])
        self.growth = float(growth)
        self.capacity = max(int(capacity or 0), P, 1)
        self.banks = [self._new_bank(self.capacity), self._new_bank(self.capacity)]
        self.cur = 0
        self.single = self._new_single(self.capacity)
        b = self.banks[0]
        for name, t in zip(PARAMS, (xyz, features, opacity, scaling, rotation)):
            b[name][:P].copy_(t.detach().reshape(b[name][:P].shape))
            b["m_" + name][:P].zero_()
            b["v_" + name][:P].zero_()
        b["kf_id"][:P].copy_(kf_id if kf_id is not None else torch.full((P,), -1, dtype=torch.int32))
        b["n_obs"][:P].copy_(n_obs if n_obs is not None else torch.zeros(P, dtype=torch.int32))
        self.zero_stats()

    # ---- storage -------------------------------------------------------------
    def _shape(self, name, n):
        return {"xyz": (n, 3), "features": (n, self.M, 3), "opacity": (n, 1), "scaling": (n, 3),
                "rotation": (n, 4)}[name]

    def _new_bank(self, cap):
        f32 = dict(dtype=torch.float32, device=self.device)
        b = {}
        for name in PARAMS:
            b[name] = torch.empty(self._shape(name, cap), **f32)
            b["m_" + name] = torch.empty(self._shape(name, cap), **f32)
            b["v_" + name] = torch.empty(self._shape(name, cap), **f32)
        b["kf_id"] = torch.empty(cap, dtype=torch.int32, device=self.device)
        b["n_obs"] = torch.empty(cap, dtype=torch.int32, device=self.device)
        return b

    def _grad_widths(self):
        return {"xyz": 3, "features": 3 * self.M, "opacity": 1, "scaling": 3, "rotation": 4}

    def _new_single(self, cap):
        f32 = dict(dtype=torch.float32, device=self.device)
        # the five parameter gradients in ONE flat buffer, packed by the
        # current row count (grad(): group g at P x (widths before g)): per-
        # iteration scratch, so a data-parallel step all-reduces the P rows of
        # every group as one contiguous range (grad_flat())
        s = {"grad_flat": torch.zeros(cap * sum(self._grad_widths().values()) + 64 * len(PARAMS), **f32)}
        s["xyz_gradient_accum"] = torch.zeros(cap, 1, **f32)
        s["denom"] = torch.zeros(cap, 1, **f32)
        s["max_radii2D"] = torch.zeros(cap, **f32)
        s["act_opacity"] = torch.empty(cap, 1, **f32)
        s["act_scales"] = torch.empty(cap, 3, **f32)
        s["act_rotations"] = torch.empty(cap, 4, **f32)
        for k in ("opacity", "scales", "rotations"):
            s["actg_" + k] = torch.empty_like(s["act_" + k])
        return s

    def reserve(self, n: int):
        """Room for n rows (both banks); keeps the current rows, moments and
        statistics.  Growth is geometric, so inserts stay amortised O(1)."""
        if n <= self.capacity:
            return
        cap = max(int(n), int(math.ceil(self.capacity * self.growth)))
        P = self.P
        nb = [self._new_bank(cap), self._new_bank(cap)]
        for k, t in self.banks[self.cur].items():
            nb[0][k][:P].copy_(t[:P])
        ns = self._new_single(cap)
        for k, t in self.single.items():
            if k != "grad_flat":  # (scratch: rewritten by every backward)
                ns[k][:P].copy_(t[:P])
        self.banks, self.single, self.cur, self.capacity = nb, ns, 0, cap

    # ---- views [:P] ---------------------------------------------------------
    def param(self, name):
        return self.banks[self.cur][name][:self.P]

    def exp_avg(self, name):
        return self.banks[self.cur]["m_" + name][:self.P]

    def exp_avg_sq(self, name):
        return self.banks[self.cur]["v_" + name][:self.P]

    def _grad_offsets(self):
        """{group: float offset} in grad_flat for the current P (each group
        256-byte aligned) and the end of the last group."""
        out, off = {}, 0
        for n, w in self._grad_widths().items():
            out[n] = off
            off += (self.P * w + 63) // 64 * 64
        return out, off

    def grad(self, name):
        offs, _ = self._grad_offsets()
        n = self.P * self._grad_widths()[name]
        return self.single["grad_flat"][offs[name]:offs[name] + n].view(self._shape(name, self.P))

    def grad_flat(self):
        """Every group's gradient rows [:P] as one contiguous range
        (grad() views into it; the < 64-float alignment gaps between groups
        are never read)."""
        return self.single["grad_flat"][:self._grad_offsets()[1]]

    def stat(self, name):
        return self.single[name][:self.P]

    def scratch(self, name):
        return self.single[name][:self.P]

    @property
    def kf_id(self):
        return self.banks[self.cur]["kf_id"][:self.P]

    @property
    def n_obs(self):
        return self.banks[self.cur]["n_obs"][:self.P]

    def zero_stats(self):
        """densification_postfix's reset (gaussian_model.py:635-637)."""
        for k in ("xyz_gradient_accum", "denom", "max_radii2D"):
            self.single[k][:self.P].zero_()

    def _bank_struct(self, b):
        bank = self.banks[b]
        s = _lib.GaussianBank()
        for name in PARAMS:
            setattr(s, name, bank[name].data_ptr())
        for k, name in enumerate(PARAMS):
            s.exp_avg[k] = bank["m_" + name].data_ptr()
            s.exp_avg_sq[k] = bank["v_" + name].data_ptr()
        s.kf_id = bank["kf_id"].data_ptr()
        s.n_obs = bank["n_obs"].data_ptr()
        return s

    # ---- reference operations ------------------------------------------------
    def append(self, xyz, features, opacity, scaling, rotation, kf_id=None, n_obs=None):
        """densification_postfix / extend_from_pcd (gaussian_model.py:231-259,
        602-644): new rows after the last one with zero Adam moments; the
        statistics of ALL rows reset to zero."""
        n = int(xyz.shape[0])
        P = self.P
        self.reserve(P + n)
        b = self.banks[self.cur]
        for name, t in zip(PARAMS, (xyz, features, opacity, scaling, rotation)):
            b[name][P:P + n].copy_(t.detach().reshape(self._shape(name, n)))
            b["m_" + name][P:P + n].zero_()
            b["v_" + name][P:P + n].zero_()
        if kf_id is None or isinstance(kf_id, int):   # (one id for every new row: filled on the device)
            b["kf_id"][P:P + n].fill_(-1 if kf_id is None else kf_id)
        else:
            b["kf_id"][P:P + n].copy_(kf_id)
        if n_obs is None:
            b["n_obs"][P:P + n].zero_()
        else:
            b["n_obs"][P:P + n].copy_(n_obs)
        self.P = P + n
        self.zero_stats()

    def _select_emit(self, prune_mask=None, max_grad=0.0, min_opacity=0.0, extent=0.0, max_screen_size=None,
                     percent_dense=0.0, z=None, generator=None):
        L = _lib.load()
        P, dev = self.P, self.device
        nb = int(L.wgsr_densify_blocks(P))
        flags = torch.empty(max(P, 1), dtype=torch.uint8, device=dev)
        bc = torch.empty(4 * (nb + 1), dtype=torch.int32, device=dev)
        st = _lib.stream_handle(dev)
        pm = prune_mask.to(torch.uint8).contiguous() if prune_mask is not None else None
        with torch.cuda.device(dev):
            _lib.check(L.wgsr_densify_select(
                P, _lib.ptr(self.stat("xyz_gradient_accum")), _lib.ptr(self.stat("denom")),
                _lib.ptr(self.param("opacity")), _lib.ptr(self.param("scaling")), _lib.ptr(pm), float(max_grad),
                float(percent_dense * extent), float(min_opacity), float(0.1 * extent),
                int(bool(max_screen_size)), float(max_screen_size or 0.0), flags.data_ptr(), bc.data_ptr(), st))
        Ko, Kc, Ks, Ns = bc[4 * nb:4 * nb + 4].tolist()  # the one host read
        P_new = Ko + Kc + 2 * Ks
        if Ns and z is None:
            z = torch.randn(2 * Ns, 3, device=dev, generator=generator)
        if z is not None:
            z = z.to(device=dev, dtype=torch.float32).contiguous()
            if Ns and z.numel() < 6 * Ns:
                raise ValueError(f"densify: need z of [{2 * Ns}, 3] standard-normal samples, got {tuple(z.shape)}")
        self.reserve(P_new)
        src, dst = self._bank_struct(self.cur), self._bank_struct(self.cur ^ 1)
        with torch.cuda.device(dev):
            _lib.check(L.wgsr_densify_emit(P, self.M, flags.data_ptr(), bc.data_ptr(), _lib.ptr(z),
                                           ctypes.byref(src), ctypes.byref(dst), st))
        self.cur ^= 1
        self.P = P_new
        self.zero_stats()
        return {"kept": Ko, "cloned": Kc, "split_selected": Ns, "split_kept": Ks, "P": P_new}

    def densify_and_prune(self, max_grad, min_opacity, extent, max_screen_size, percent_dense, z=None,
                          generator=None):
        """GaussianModel.densify_and_prune (gaussian_model.py:646-743) in one
        select + scan + emit.  ``z``: the split's standard-normal samples
        [2 Ns, 3] (copy A rows, then copy B; drawn with ``generator`` when
        absent), i.e. the reference's torch.normal(0, stds) = z * stds."""
        return self._select_emit(None, max_grad, min_opacity, extent, max_screen_size, percent_dense, z, generator)

    def prune_points(self, mask):
        """GaussianModel.prune_points (gaussian_model.py:548-564): rows with
        mask set go, the rest keep their order and moments.  (Unlike
        densification_postfix, prune keeps the statistics of the kept rows.)"""
        keep_stats = {k: self.stat(k)[~mask.bool()].clone() for k in ("xyz_gradient_accum", "denom", "max_radii2D")}
        out = self._select_emit(prune_mask=mask)
        for k, v in keep_stats.items():
            self.single[k][:self.P].copy_(v)
        return out

    def reset_opacity(self):
        """GaussianModel.reset_opacity (gaussian_model.py:389-392)."""
        self._reset_opacity(None, self._inv_sigmoid_const(0.01))

    def reset_opacity_nonvisible(self, visibility_filters):
        """GaussianModel.reset_opacity_nonvisible (gaussian_model.py:394-402):
        invisible rows -> inverse_sigmoid(0.4); rows visible in any filter keep
        get_opacity (the activated value, written into the raw tensor as the
        reference does); opacity moments -> 0."""
        vis = None
        for f in visibility_filters:
            f = f.to(device=self.device, dtype=torch.bool)
            vis = f if vis is None else (vis | f)
        self._reset_opacity(vis, self._inv_sigmoid_const(0.4))

    def _inv_sigmoid_const(self, c):
        """inverse_sigmoid(torch.ones_like(opacity) * c), evaluated on the
        device as the reference does (one element: the value is per row)."""
        return float(inverse_sigmoid(torch.ones(1, device=self.device) * c).item())

    def update_mapping_points(self, frames, K=None):
        """Mapper._update_mapping_points (src/mapper.py:431-558) for several
        keyframes in ONE pass over the rows (csrc/deform.hip).

        frames: iterable of dicts with ``kf_id``, ``w2c`` (new world->camera,
        [4, 4]), ``w2c_old`` ([4, 4]) and, for the depth-rescale branch
        (the reference's ``method=None``), ``depth`` / ``depth_old`` ([H, W]
        maps); ``method`` "rigid" (default when no depth is given) or
        "depth".  K: the mapper's 3x3 intrinsics (depth branch).  The 4x4
        transformation and its quaternion are formed on the host in fp32
        exactly as the reference forms them (torch.linalg.inv,
        rotation_matrix_to_quaternion); the per-row work, the normalisation of
        every rotation and the moment resets of replace_tensor_to_optimizer
        run on the device.  Returns the number of frames passed on."""
        L = _lib.load()
        frames = list(frames)
        if self.P == 0 or not frames:
            return 0
        arr = (_lib.DeformFrame * len(frames))()
        seen = set()
        keep = []
        Kc = None if K is None else torch.as_tensor(K, dtype=torch.float32).cpu().reshape(3, 3)
        # every frame's transformation and quaternion in one batched host pass
        W = torch.stack([torch.as_tensor(fr["w2c"], dtype=torch.float32).cpu().reshape(4, 4) for fr in frames])
        Wo = torch.stack([torch.as_tensor(fr["w2c_old"], dtype=torch.float32).cpu().reshape(4, 4) for fr in frames])
        Ts, qs = deform_transform(W, Wo)
        Ts, qs = Ts.reshape(len(frames), 16).tolist(), qs.tolist()
        for j, fr in enumerate(frames):
            k = int(fr["kf_id"])
            if k in seen:
                raise ValueError(f"update_mapping_points: keyframe {k} given twice")
            seen.add(k)
            method = fr.get("method") or ("rigid" if fr.get("depth") is None else "depth")
            w2c_old = Wo[j]
            f = arr[j]
            f.kf_id, f.method = k, (0 if method == "rigid" else 1)
            f.T[:] = Ts[j]
            f.q[:] = qs[j]
            if method != "rigid":
                if Kc is None:
                    raise ValueError("update_mapping_points: the depth branch needs the intrinsics K")
                d = fr["depth"].to(device=self.device, dtype=torch.float32).contiguous()
                d_old = fr["depth_old"].to(device=self.device, dtype=torch.float32).contiguous()
                if d.dim() != 2 or d.shape != d_old.shape:
                    raise ValueError("update_mapping_points: depth / depth_old must be [H, W] maps of one shape")
                keep += [d, d_old]
                f.w2c_old[:] = w2c_old.flatten().tolist()
                f.c2w_old[:] = torch.linalg.inv(w2c_old).flatten().tolist()
                f.K[:] = Kc.flatten().tolist()
                f.H, f.W = int(d.shape[0]), int(d.shape[1])
                f.depth, f.depth_old = d.data_ptr(), d_old.data_ptr()
        nlut = max(seen) + 1 if max(seen) >= 0 else 1
        lut_h = np.full(nlut, -1, dtype=np.int32)
        for j, fr in enumerate(frames):
            if int(fr["kf_id"]) >= 0:
                lut_h[int(fr["kf_id"])] = j
        dev = self.device
        # the frame table and the keyframe -> frame lookup in ONE upload
        fb = bytes(arr)
        off = (len(fb) + 255) & ~255
        blob = np.zeros(off + 4 * nlut, dtype=np.uint8)
        blob[:len(fb)] = np.frombuffer(fb, dtype=np.uint8)
        blob[off:] = lut_h.view(np.uint8)
        blob_d = torch.from_numpy(blob).to(dev)
        flags = torch.empty(2, dtype=torch.int32, device=dev)
        bank = self._bank_struct(self.cur)
        with torch.cuda.device(dev):
            _lib.check(L.wgsr_deform_points(self.P, ctypes.byref(bank), blob_d.data_ptr(), len(frames),
                                            blob_d.data_ptr() + off, nlut, flags.data_ptr(),
                                            _lib.stream_handle(dev)))
        self._deform_keep = (keep, blob_d, flags)  # alive until the next call (stream order)
        return len(frames)

    def _reset_opacity(self, vis, value):
        L = _lib.load()
        v8 = vis.to(torch.uint8).contiguous() if vis is not None else None
        with torch.cuda.device(self.device):
            _lib.check(L.wgsr_reset_opacity(self.P, self.param("opacity").data_ptr(), _lib.ptr(v8), value,
                                            self.exp_avg("opacity").data_ptr(), self.exp_avg_sq("opacity").data_ptr(),
                                            _lib.stream_handle(self.device)))
