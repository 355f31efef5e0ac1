"""WildGS-SLAM's online mapper loop on the gfx950 path (configs[4] shape;
SURVEY.md 8(f) rows f1 + f2 + f4).

What the reference's Mapper does for every keyframe the tracker hands over
(src/mapper.py:153-266), restated on ``wgsr.mapping.MappingStep`` (fused
activations, rasteriser, uncertainty-aware loss, statistics, one-launch
Adam) and ``wgsr.store.GaussianStore`` (capacity-preallocated state,
densification on the device):

``insert_keyframe``
    render from the keyframe pose for its visibility (n_touched > 0,
    mapper.py:198-203), the MonoGS window update (``_add_to_window``,
    mapper.py:648-706), the point insertion of extend_from_pcd_seq
    (gaussian_model.py:108-269: exposure-corrected colour, back-projected
    depth, random 1/downsample subset, RGB2SH, distCUDA2 scales with the
    adaptive point size, identity rotations, opacity inverse_sigmoid(0.5)), a
    fresh exposure Adam over the window (lr 0.01, mapper.py:219-241), then
    ``map_opt_online(window, mapping_itr_num)`` and one extra iteration after
    a densify / reset (mapper.py:256-260).
``map_opt_online``  (mapper.py:1049-1219)
    per iteration: a random window-weighted keyframe (p >= 0.5 for the current
    window), the uncertainty MLP on its features, the uncertainty-aware
    loss on the pre-exposed render + 10 x isotropic loss, backward (loss
    kernels -> rasteriser -> activations, the MLP's gradient from the loss),
    the DINO regulariser on sampled features of the neighbouring keyframes
    once 20 iterations have passed since the last densify / reset, the
    densification statistics, densify_and_prune every
    ``gaussian_update_every`` (offset) iterations, reset_opacity_nonvisible
    every ``gaussian_reset``, the Gaussians' Adam (groups replaced by a
    densify / reset skip it, as torch's Adam skips parameters without a
    gradient), the xyz learning-rate schedule (general_utils.helper), the
    keyframe exposures' and the MLP's Adam.
``initialize``  (initialize_mapper + initialize_map_opt, mapper.py:732-1047)
    the first keyframes inserted with pcd_downsample_init, then
    ``init_itr_num`` iterations with the initialization loss, the strided
    DINO term, densify every ``init_gaussian_update`` and reset_opacity at
    ``init_gaussian_reset``.

``update_keyframes``  (_update_keyframes_from_frontend + _update_mapping_points,
mapper.py:365-558)
    the tracker's new poses / depths of existing keyframes and the map
    deformation of their anchored Gaussians, every keyframe in one device
    pass (``GaussianStore.update_mapping_points``, csrc/deform.hip).
``final_refine``  (mapper.py:1234-1372)
    the end-of-sequence refinement iterations.

Not restated (absent offline or outside the mapping path): the tracker and
its keyframe decisions (the caller supplies keyframes with poses and
depths, and the pose / depth updates), DINO feature extraction (the caller
supplies features), the GUI / printer, fast mode.
Random draws (view choice, point subsets, split noise, dropout) come from
this object's generators, not the reference's global RNG streams.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np
import torch

from .camera import PinholeCamera, focal2fov, get_world2view2
from .mapping import MappingStep

SH_C0 = 0.28209479177387814

# configs/wildgs_slam.yaml (mapping.Training, opt_params, uncertainty_params,
# pcd_downsample*, point_size, adaptive_pointsize); mapper.py:272-299
DEFAULT_CONFIG = {
    "cameras_extent": 6.0, "init_itr_num": 1050, "init_gaussian_update": 100, "init_gaussian_reset": 500,
    "init_gaussian_th": 0.005, "init_gaussian_extent": 30.0, "mapping_itr_num": 450,
    "gaussian_update_every": 1500, "gaussian_update_offset": 500, "gaussian_th": 0.7, "gaussian_extent": 1.0,
    "gaussian_reset": 20001, "size_threshold": 20, "window_size": 10, "kf_cutoff": 0.4,
    "pcd_downsample": 32, "pcd_downsample_init": 16, "point_size": 0.05, "adaptive_pointsize": True,
    "position_lr_init": 0.00016, "position_lr_final": 0.0000016, "position_lr_delay_mult": 0.01,
    "position_lr_max_steps": 30000, "feature_lr": 0.0025, "opacity_lr": 0.05, "scaling_lr": 0.001,
    "rotation_lr": 0.001, "percent_dense": 0.01, "densify_grad_threshold": 0.0002, "spatial_lr_scale": 6.0,
    "train_frac_fix": 0.3, "reg_stride": 2, "reg_mult": 0.5, "uncer_lr": 0.0004, "uncer_weight_decay": 0.00001,
    "exposure_lr": 0.01, "edge_threshold": 4.0, "lr_cam_rot_delta": 0.003, "lr_cam_trans_delta": 0.001,
    "tracking_itr_num": 100,
}


def lr_helper(step, lr_init, lr_final, lr_delay_steps=0, lr_delay_mult=1.0, max_steps=1000000):
    """general_utils.helper (general_utils.py:78-94)."""
    if step < 0 or (lr_init == 0.0 and lr_final == 0.0):
        return 0.0
    if lr_delay_steps > 0:
        delay_rate = lr_delay_mult + (1 - lr_delay_mult) * np.sin(0.5 * np.pi * np.clip(step / lr_delay_steps, 0, 1))
    else:
        delay_rate = 1.0
    t = min(max(step / max_steps, 0.0), 1.0)  # (np.clip's value, without its per-call overhead)
    return float(delay_rate * np.exp(np.log(lr_init) * (1 - t) + np.log(lr_final) * t))


@dataclass
class Keyframe:
    """A keyframe as the mapper keeps it (src/utils/camera_utils.py Camera):
    world->camera pose (R, T), intrinsics, the keyframe colour image [3,H,W],
    its metric depth [1,H,W] and DINO features [h,w,C], all device tensors."""

    uid: int
    R: torch.Tensor
    T: torch.Tensor
    fx: float
    fy: float
    cx: float
    cy: float
    image: torch.Tensor
    depth: torch.Tensor
    features: torch.Tensor
    exposure_a: torch.Tensor = field(default=None)
    exposure_b: torch.Tensor = field(default=None)

    def __post_init__(self):
        dev = self.image.device
        if self.exposure_a is None:
            self.exposure_a = torch.zeros(1, device=dev)
        if self.exposure_b is None:
            self.exposure_b = torch.zeros(1, device=dev)
        H, W = self.image.shape[-2:]
        self.H, self.W = int(H), int(W)
        pc = PinholeCamera(R=self.R.float().cpu(), T=self.T.float().cpu(), fx=self.fx, fy=self.fy, cx=self.cx,
                           cy=self.cy, W=self.W, H=self.H)
        self.cam = {k: (v.to(dev) if torch.is_tensor(v) else v) for k, v in pc.raster_fields().items()}
        self.FoVx, self.FoVy = focal2fov(self.fx, self.W), focal2fov(self.fy, self.H)
        self.median_depth = self.depth.median()  # constant per keyframe (the loss's depth threshold)

    def w2c(self) -> torch.Tensor:
        """[4, 4] fp32 world->camera (mapper.py:387-389)."""
        m = np.eye(4, dtype=np.float32)
        m[:3, :3], m[:3, 3] = self.R.float().cpu().numpy(), self.T.float().cpu().numpy()
        return torch.from_numpy(m)

    def update_RT(self, R, T, upload: bool = True):
        """Camera.update_RT (camera_utils.py:153-155) + the raster fields.
        ``upload=False``: only the pose; the caller forms and uploads the
        raster fields of several keyframes at once
        (OnlineMapper._upload_cameras)."""
        self.R, self.T = torch.as_tensor(R).float().cpu(), torch.as_tensor(T).float().cpu()
        if not upload:
            return
        pc = PinholeCamera(R=self.R, T=self.T, fx=self.fx, fy=self.fy, cx=self.cx, cy=self.cy, W=self.W, H=self.H)
        dev = self.image.device
        self.cam = {k: (v.to(dev) if torch.is_tensor(v) else v) for k, v in pc.raster_fields().items()}

    @property
    def K(self) -> torch.Tensor:
        return torch.tensor([[self.fx, 0.0, self.cx], [0.0, self.fy, self.cy], [0.0, 0.0, 1.0]])


class OnlineMapper:
    def __init__(self, sh_degree: int = 0, feature_dim: int = 384, device="cuda", config: dict | None = None,
                 seed: int = 0):
        from .mlp import UncertaintyMLP
        from .optim import FusedAdam
        self.cfg = dict(DEFAULT_CONFIG, **(config or {}))
        c = self.cfg
        self.dev = torch.device(device)
        self.D = int(sh_degree)
        self.M = (self.D + 1) ** 2
        self.rng = np.random.default_rng(seed)
        self.gen = torch.Generator(device=self.dev).manual_seed(seed)
        torch.manual_seed(seed)
        self.net = UncertaintyMLP(feature_dim).to(self.dev)
        self.uopt = FusedAdam(self.net.parameters(), lr=c["uncer_lr"], weight_decay=c["uncer_weight_decay"])
        s = c["spatial_lr_scale"]
        self.lr_xyz = (c["position_lr_init"] * s, c["position_lr_final"] * s)
        self.lr = {"xyz": self.lr_xyz[0], "f_dc": c["feature_lr"], "f_rest": c["feature_lr"] / 20.0,
                   "opacity": c["opacity_lr"], "scaling": c["scaling_lr"] * s, "rotation": c["rotation_lr"]}
        self.ms = None
        self.keyframes: dict[int, Keyframe] = {}
        self.window: list[int] = []
        self.occ_vis: dict[int, torch.Tensor] = {}
        from .online_graph import IterationGraphs, KeyframeBank
        # every keyframe's per-view data (and its exposure + Adam moments) in
        # slot-indexed device banks; the Keyframe tensors become views
        self.bank = KeyframeBank(self.dev)
        self.kopt_uids: set[int] = set()   # the window's exposure optimiser (mapper.py:219-241)
        self.kopt_steps: dict[int, int] = {}
        self._max_nr = 0                   # largest num_rendered seen (the graphs' first capacity)
        self.graphs = IterationGraphs(self) if self.dev.type == "cuda" else None
        self.iteration_count = 0
        self.iterations_after_densify_or_reset = 0
        self.bg = torch.zeros(3, device=self.dev)
        self.events = []  # (iteration, "densify" | "reset", details)
        self.last_removed = None  # keyframe the last window update dropped
        self.phase_ms = None      # {phase: [ms, ...]} when prepare_keyframe / update_keyframes are timed

    # ---- Gaussians from a keyframe (gaussian_model.py:108-226) ---------------
    @staticmethod
    def np_median(x: torch.Tensor) -> float:
        """np.median of a float32 map (gaussian_model.py:150): the MEAN of the
        two middle values for an even count (torch.median returns the lower
        one), computed in fp32 as numpy does for a float32 array."""
        v = x.reshape(-1).float()
        n = v.numel()
        # one sort for both order statistics (two kthvalue calls took ~0.75 ms
        # each on a 512 x 384 map on the device)
        sv = torch.sort(v).values
        lo = sv[(n - 1) // 2]
        hi = sv[n // 2] if n % 2 == 0 else lo
        # np.median is NaN when any value is (torch sorts NaN last)
        return float(torch.where(torch.isnan(sv[-1]), sv[-1], (lo + hi) / 2).item())

    @torch.no_grad()
    def keyframe_points(self, kf: Keyframe, init: bool, keep=None):
        """create_pcd_from_image + create_pcd_from_image_and_depth
        (gaussian_model.py:108-226) with Open3D's RGBD back-projection: the
        exposure-corrected uint8 colours, every pixel with 0 < depth <
        depth_trunc = 100 in row-major order, x = (u - cx) z / fx and
        y = (v - cy) z / fy in double and moved to the world by
        inverse(W2C) (Open3D computes in double; the reference then casts to
        fp32), a random 1/downsample subset kept IN PIXEL ORDER (Open3D's
        random_down_sample keeps int(ratio * n) points through
        SelectByIndex), RGB2SH, the distCUDA2 scales with the adaptive point
        size min(0.05, point_size * np.median(depth)), identity rotations,
        opacity inverse_sigmoid(0.5).  ``keep``: the subset's indices into the
        valid pixels (tests feed the reference's draw); default: drawn with
        this mapper's generator."""
        from simple_knn._C import distCUDA2
        c = self.cfg
        mark = self._phase("kp_start")
        ds = c["pcd_downsample_init"] if init else c["pcd_downsample"]
        image_ab = torch.clamp(torch.exp(kf.exposure_a) * kf.image + kf.exposure_b, 0.0, 1.0)
        u8 = (image_ab * 255).byte()
        depth = kf.depth[0]
        point_size = c["point_size"]
        valid = (depth > 0) & (depth < 100.0)                          # depth_trunc = 100
        # the median and the valid-pixel count in ONE read-back (np_median's
        # arithmetic; the count sizes the nonzero below without another sync)
        head = [valid.sum().double()]
        if c["adaptive_pointsize"]:
            sv = torch.sort(depth.reshape(-1).float()).values
            N = sv.numel()
            lo = sv[(N - 1) // 2]
            hi = sv[N // 2] if N % 2 == 0 else lo
            # (np.median's NaN when any depth is NaN: torch sorts NaN last)
            head.append(torch.where(torch.isnan(sv[-1]), sv[-1], (lo + hi) / 2).double())
        head = torch.stack(head).tolist()
        n = int(head[0])
        if c["adaptive_pointsize"]:
            point_size = min(0.05, point_size * head[1])
        mark("kp_median_count")
        if keep is None:
            # a uniform int(n / ds)-subset of the valid pixels in pixel order
            # (Open3D's random_down_sample keeps its shuffled prefix sorted):
            # the k smallest of one random key per pixel (invalid pixels keyed
            # above every valid one), marked in a pixel mask and read back in
            # pixel order.  Every kernel's input has the frame's size whatever
            # k is, so the initial keyframes load them all (a top-k / sort of k
            # elements loaded new kernels at the first insertion: 45 ms)
            k = int((1.0 / ds) * n)
            Wd = depth.shape[1]
            HW = depth.numel()
            key = torch.rand(HW, device=self.dev, generator=self.gen)
            key = torch.where(valid.reshape(-1), key, 2.0)
            sel = torch.zeros(HW, dtype=torch.bool, device=self.dev)
            sel[torch.sort(key).indices[:k]] = True
            pix = torch.nonzero_static(sel, size=k).reshape(-1)
            v, u = pix // Wd, pix % Wd
        else:
            # the caller's subset: indices into the valid pixels (row-major)
            v, u = torch.nonzero(valid, as_tuple=True)
            keep = torch.as_tensor(keep, device=self.dev, dtype=torch.long)
            v, u = v[keep], u[keep]
        mark("kp_subset")
        z = depth[v, u].double()
        pc = torch.stack([(u.double() - kf.cx) * z / kf.fx, (v.double() - kf.cy) * z / kf.fy, z,
                          torch.ones_like(z)], 0)
        w2c = get_world2view2(kf.R.float().cpu(), kf.T.float().cpu()).double()   # getWorld2View2 (fp32)
        pose = torch.linalg.inv(w2c).to(self.dev)
        xyz = (pose @ pc)[:3].T.float().contiguous()
        col = (u8[:, v, u].T.double() / 255.0).float()
        feats = torch.zeros(xyz.shape[0], self.M, 3, device=self.dev)
        feats[:, 0] = (col - 0.5) / SH_C0                               # RGB2SH
        mark("kp_points")
        d2 = distCUDA2(xyz)
        mark("kp_knn")
        dist2 = torch.clamp_min(d2, 0.0000001) * point_size
        scales = torch.log(torch.sqrt(dist2))[..., None].repeat(1, 3)
        rots = torch.zeros(xyz.shape[0], 4, device=self.dev)
        rots[:, 0] = 1
        opac = torch.log(torch.full((xyz.shape[0], 1), 0.5, device=self.dev) / (1 - 0.5))  # inverse_sigmoid(0.5)
        mark("kp_rest")
        return xyz, feats, scales, rots, opac

    def _phase(self, first: str):
        """A phase timer for ``self.phase_ms`` (device-synchronised marks);
        a no-op unless phase timing is on."""
        if self.phase_ms is None:
            return lambda name: None
        import time
        tm = self.phase_ms
        torch.cuda.synchronize(self.dev)
        t = [time.perf_counter()]

        def mark(name):
            torch.cuda.synchronize(self.dev)
            t1 = time.perf_counter()
            tm.setdefault(name, []).append(1e3 * (t1 - t[0]))
            t[0] = t1
        return mark

    def _add_points(self, kf: Keyframe, init: bool, keep=None):
        xyz, feats, scales, rots, opac = self.keyframe_points(kf, init, keep=keep)
        if self.ms is None:
            e = lambda *s: torch.empty(*s, device=self.dev)  # noqa: E731
            self.ms = MappingStep(e(0, 3), e(0, 1, 3), e(0, self.M - 1, 3), e(0, 1), e(0, 3), e(0, 4), self.D,
                                  lr=self.lr, capacity=1 << 16)
        mark = self._phase("extend")
        self.ms.extend(xyz, feats, scales, rots, opac, kf_id=kf.uid)
        mark("extend")
        return xyz.shape[0]

    # ---- rendering helpers ---------------------------------------------------
    @torch.no_grad()
    def visibility(self, kf: Keyframe):
        """render(...)["n_touched"] > 0 (mapper.py:198-203, 560-572)."""
        if self.ms is None or self.ms.P == 0:
            return torch.zeros(0, dtype=torch.long, device=self.dev)
        out = self.ms._render(kf.cam, kf.H, kf.W, self.bg)
        return (out[8] > 0).long()

    @torch.no_grad()
    def render_image(self, kf: Keyframe):
        out = self.ms._render(kf.cam, kf.H, kf.W, self.bg)
        return out[1], out[6]

    def _update_occ_aware_visibility(self, window):
        self.occ_vis = {k: self.visibility(self.keyframes[k]) for k in window}

    def _add_to_window(self, cur, cur_vis, window):
        """MonoGS window update (mapper.py:648-706) -> (window, removed uid or
        None).  The overlap ratios (Szymkiewicz-Simpson: |cur & k| / min(|cur|,
        |k|), fp32 as torch's int / int division) of every candidate come from
        one device pass with one read-back; the inverse-distance eviction uses
        fp32 getWorld2View2 poses and fp32 4x4 inverses, as the reference.  A
        window keyframe without an occlusion-aware visibility of the current
        length is an error, as in the reference (a shape mismatch raises)."""
        N_dont_touch = 2
        window = [cur] + window
        removed = None
        cand = window[N_dont_touch:]
        if cand:
            for k in cand:
                o = self.occ_vis.get(k)
                if o is None or o.numel() != cur_vis.numel():
                    raise RuntimeError(f"_add_to_window: keyframe {k} has no occlusion-aware visibility of "
                                       f"{cur_vis.numel()} Gaussians")
            occ = torch.stack([self.occ_vis[k].reshape(-1) for k in cand]).bool()
            cv = cur_vis.reshape(-1).bool()
            counts = torch.cat([(occ & cv).sum(1), occ.sum(1), cv.sum().reshape(1)]).cpu().numpy()
            n = len(cand)
            inter, nk, nc = counts[:n], counts[n:2 * n], counts[2 * n]
            ratio = inter.astype(np.float32) / np.minimum(nc, nk).astype(np.float32)
            to_remove = [k for k, r in zip(cand, ratio) if r <= np.float32(self.cfg["kf_cutoff"])]
            if to_remove:
                window.remove(to_remove[-1])
                removed = to_remove[-1]

        if len(window) > self.cfg["window_size"]:
            # every candidate's getWorld2View2 and its inverse once, the pair
            # products batched (fp32, as the reference's per-pair 4x4 ops;
            # the sums over j in the reference's order, in double)
            ks = [cur] + window[N_dont_touch:]
            cw = torch.stack([get_world2view2(self.keyframes[k].R.float().cpu(), self.keyframes[k].T.float().cpu())
                              for k in ks])
            wc = torch.linalg.inv(cw)
            n = len(ks) - 1
            t_ij = torch.matmul(cw[1:, None], wc[None, 1:])[:, :, 0:3, 3]          # [n, n, 3]: T_CiCj
            inv_ij = (1.0 / (torch.linalg.vector_norm(t_ij, dim=-1) + 1e-6)).tolist()
            k_i = torch.sqrt(torch.linalg.vector_norm(torch.matmul(cw[1:], wc[0])[:, 0:3, 3], dim=-1)).tolist()
            inv_dist = [k_i[i] * sum(inv_ij[i][j] for j in range(n) if j != i) for i in range(n)]
            removed = window[N_dont_touch + int(np.argmax(inv_dist))]
            window.remove(removed)
        return window, removed

    def _perm(self, n: int, k: int | None = None) -> torch.Tensor:
        """The DINO term's feature sampling draw (the reference's
        torch.randperm(n), mapper.py:1155-1157 / 1334-1336): the stable
        ascending order of 31-bit hash keys of a seed drawn from torch's
        host generator (wgsr_random_keys) -- the draw the graph-replayed
        iteration makes on the device from the same seed.  With k: only its
        first k entries (wgsr_random_perm_prefix where it applies)."""
        from . import _lib
        seed = int(torch.randint(0, 2 ** 31 - 1, (1,)).item())
        L = _lib.load()
        if (k is not None and n <= int(L.wgsr_random_perm_prefix_max_n())
                and k <= int(L.wgsr_random_perm_prefix_max_k())):
            perm = torch.empty(max(k, 1), dtype=torch.int32, device=self.dev)
            with torch.cuda.device(self.dev):
                _lib.check(L.wgsr_random_perm_prefix(n, k, seed, None, _lib.ptr(perm), _lib.stream_handle(self.dev)))
            return perm[:k]
        keys = torch.empty(n, dtype=torch.int32, device=self.dev)
        with torch.cuda.device(self.dev):
            if n <= int(L.wgsr_random_perm_max()):  # one-workgroup stable sort (wgsr_random_perm)
                perm = torch.empty(n, dtype=torch.int32, device=self.dev)
                _lib.check(L.wgsr_random_perm(n, seed, None, _lib.ptr(keys), _lib.ptr(perm),
                                              _lib.stream_handle(self.dev)))
                return perm if k is None else perm[:k]
            _lib.check(L.wgsr_random_keys(n, seed, None, _lib.ptr(keys), _lib.stream_handle(self.dev)))
        perm = torch.argsort(keys, stable=True)
        return perm if k is None else perm[:k]

    def _dino_term(self, neighbours, kf):
        """reg_mult * compute_dino_regularization_loss on features sampled from
        the neighbouring keyframes' (stack positions ci-2 .. ci+2) feature maps
        (mapper.py:1141-1164, 1320-1340), and its backward into the MLP."""
        from .uncertainty import dino_regularization_loss
        c = self.cfg
        st = c["reg_stride"]
        buf = torch.stack([self.keyframes[k].features for k in neighbours]).view(-1, kf.features.shape[-1])
        ns = buf.shape[0] // (st ** 4)
        # (a test's fixture draw replaces _perm(n) on the instance: full length)
        perm = self._perm(buf.shape[0])[:ns] if "_perm" in self.__dict__ else self._perm(buf.shape[0], ns)
        sf = buf[perm].unsqueeze(0)
        (c["reg_mult"] * dino_regularization_loss(self.net(sf), sf)).backward()

    def _mlp_pair_ok(self) -> bool:
        """The MLP's two forwards / backwards batched into one launch each
        (the graph-replayed iteration's arithmetic) unless a test feeds the
        random draws."""
        return self.net.seed_source is None and "_perm" not in self.__dict__ and self.dev.type == "cuda"

    def _mlp_pair_loss(self, kf, neighbours, fb):
        """One iteration's uncertainty MLP + loss + DINO term with both MLP
        passes batched (wgsr.mlp.forward_raw2 / backward_raw2), the draws in
        the eager order (the keyframe forward's dropout seed, the sample's
        permutation seed, the sample forward's seed): ``fb(unc)`` runs the
        rasteriser loss on the uncertainty map and returns its dict; the MLP
        gradient (loss + reg_mult x DINO) lands in the parameters' .grad."""
        from .mlp import backward_raw2, forward_raw2
        from .uncertainty import dino_reg_raw
        c = self.cfg
        h, w, C = kf.features.shape
        s1 = int(torch.randint(0, 2 ** 31 - 1, (1,)).item())
        buf = torch.stack([self.keyframes[k].features for k in neighbours]).view(-1, C)
        ns = buf.shape[0] // (c["reg_stride"] ** 4)
        perm = self._perm(buf.shape[0], ns)
        s2 = int(torch.randint(0, 2 ** 31 - 1, (1,)).item())
        sf = buf[perm].contiguous()
        seeds = torch.tensor([s1, s2], dtype=torch.int32).to(self.dev)  # (blocking: a pageable source)
        u_all, sv = forward_raw2(self.net, kf.features.reshape(h * w, C), sf, seeds[0:1], seeds[1:2])
        out = fb(u_all[:h * w].view(h, w))
        _, gu = dino_reg_raw(u_all[h * w:], sf, want_loss=False)
        G = backward_raw2(sv, out["uncertainty_grad"].reshape(-1).contiguous(), gu, 1.0, float(c["reg_mult"]))
        off = 0
        for prm in self.net.parameters():
            k = prm.numel()
            g = G[off:off + k].view_as(prm)
            prm.grad = g if prm.grad is None else prm.grad + g
            off += k
        return out

    # ---- one optimisation iteration ------------------------------------------
    def _iteration(self, kf: Keyframe, neighbours, initialization: bool, update: bool, reset: str | None,
                   occ_window=None):
        c = self.cfg
        ms = self.ms
        self.iteration_count += 1
        self.iterations_after_densify_or_reset += 1
        ea, eb = kf.exposure_a, kf.exposure_b
        if initialization:
            from .uncertainty import dino_regularization_loss
            unc = self.net(kf.features)
            st = c["reg_stride"]
            # the strided DINO term on the SAME uncertainty map the loss uses
            # (mapper.py:986-997): its gradient first, the loss's second
            (c["reg_mult"] * dino_regularization_loss([unc[::st, ::st].unsqueeze(-1)],
                                                      [kf.features[::st, ::st]])).backward(retain_graph=True)
            out = ms.forward_backward_uncertainty(kf.cam, kf.image, kf.depth, ea, eb, self.bg, unc,
                                                  c["train_frac_fix"], c["train_frac_fix"], initialization=True,
                                                  median_depth=kf.median_depth, need_tau=False, exposure_partials=True)
        elif self.iterations_after_densify_or_reset >= 20 and self._mlp_pair_ok():
            out = self._mlp_pair_loss(kf, neighbours, lambda unc: ms.forward_backward_uncertainty(
                kf.cam, kf.image, kf.depth, ea, eb, self.bg, unc, c["train_frac_fix"], c["train_frac_fix"],
                freeze_uncertainty_loss=False, median_depth=kf.median_depth, need_tau=False, exposure_partials=True))
        else:
            unc = self.net(kf.features)
            freeze = self.iterations_after_densify_or_reset < 20
            out = ms.forward_backward_uncertainty(kf.cam, kf.image, kf.depth, ea, eb, self.bg, unc,
                                                  c["train_frac_fix"], c["train_frac_fix"],
                                                  freeze_uncertainty_loss=freeze, median_depth=kf.median_depth,
                                                  need_tau=False, exposure_partials=True)
            if self.iterations_after_densify_or_reset >= 20:
                self._dino_term(neighbours, kf)
        self._max_nr = max(self._max_nr, int(out["num_rendered"]))
        vis = self._after_backward(out, update, reset == "nonvisible")
        if occ_window is not None:  # last iteration of a map_opt_online call (mapper.py:1174-1175)
            self._update_occ_aware_visibility(occ_window)
        if update:
            res = ms.densify_and_prune(c["densify_grad_threshold"],
                                       c["init_gaussian_th"] if initialization else c["gaussian_th"],
                                       c["cameras_extent"] * (c["init_gaussian_extent"] if initialization
                                                              else c["gaussian_extent"]),
                                       None if initialization else c["size_threshold"], c["percent_dense"],
                                       generator=self.gen)
            self.iterations_after_densify_or_reset = 0
            self.events.append((self.iteration_count, "densify", res))
        if reset == "all":
            ms.reset_opacity()
            self.iterations_after_densify_or_reset = 0
            self.events.append((self.iteration_count, "reset_opacity", None))
        elif reset == "nonvisible":
            ms.reset_opacity_nonvisible([vis])
            self.iterations_after_densify_or_reset = 0
            self.events.append((self.iteration_count, "reset_opacity_nonvisible", None))
        ms.optimizer_step()
        ms.lr["xyz"] = lr_helper(self.iteration_count, self.lr_xyz[0], self.lr_xyz[1],
                                 lr_delay_mult=c["position_lr_delay_mult"], max_steps=c["position_lr_max_steps"])
        if not initialization:  # (the initialisation loss has no exposure term: torch's Adam skips it)
            self._exposure_step(kf, out)
        self.uopt.step()
        self.uopt.zero_grad()
        return out

    def _exposure_step(self, kf, out):
        """keyframe_optimizers.step() + zero_grad(set_to_none=True): only the
        rendered keyframe's exposures carry a gradient; others are skipped.
        torch.optim.Adam(lr=exposure_lr) arithmetic (wgsr_adam_step) on the
        keyframe's row of the exposure bank (a, b share one step count: they
        always step together)."""
        if kf.uid not in self.kopt_uids:
            return
        from . import _lib
        self.kopt_steps[kf.uid] += 1
        n = self.kopt_steps[kf.uid]
        lr = self.cfg["exposure_lr"]
        L = _lib.load()
        p = _lib.ptr
        if "dexposure_partials" in out:  # the loss backward's per-block partials, summed in the step (as replays do)
            self._exposure_apply(kf.uid, out["dexposure_partials"], n, lr)
            return
        da, db = out["dexposure_a"], out["dexposure_b"]
        g = da if db.data_ptr() == da.data_ptr() + 4 else torch.cat([da.reshape(1), db.reshape(1)])
        prm, m, v = self.bank.ex_ptrs(kf.uid)
        t = _lib.AdamTensor(prm, g.data_ptr(), m, v, 2, lr / (1.0 - 0.9 ** n), math.sqrt(1.0 - 0.999 ** n))
        with torch.cuda.device(self.dev):
            _lib.check(L.wgsr_adam_step((_lib.AdamTensor * 1)(t), 1, 0.9, 0.999, 1e-8, _lib.stream_handle(self.dev)))

    def _exposure_apply(self, uid, g, n, lr, skip=None):
        """Adam step n of keyframe ``uid``'s exposure row from the loss
        backward's per-block (a, b) partials ``g`` [rows, 2] (summed in the
        step kernel).  ``skip``: an optional device word; set, nothing moves."""
        from . import _lib
        L = _lib.load()
        p = _lib.ptr
        hs = np.zeros(6, dtype=np.float32)
        hs[0], hs[1] = lr / (1.0 - 0.9 ** n), math.sqrt(1.0 - 0.999 ** n)
        hs[2:4].view(np.int64)[0] = self.bank.slots[uid]
        # (a blocking copy: hs is pageable and dies with this call -- an
        # asynchronous copy from it may read the memory after it was reused)
        dv = torch.from_numpy(hs).to(self.dev)
        with torch.cuda.device(self.dev):
            _lib.check(L.wgsr_exposure_step(p(self.bank.ex), p(dv[2:4]), p(g), int(g.shape[0]), p(dv[0:2]),
                                            p(dv[4:5]) if skip is None else p(skip), p(dv[4:5]), 0.9, 0.999, 1e-8,
                                            None, None, None, _lib.stream_handle(self.dev)))

    # ---- hooks of the keyframe-view data-parallel mapper (wgsr.dp_online) ----
    def _pick(self, draw):
        """This process's keyframe draw of one iteration (one draw here;
        DPOnlineMapper draws one per rank and keeps its own)."""
        return draw()

    def _after_backward(self, out, update: bool, need_vis: bool):
        """Between the iteration's backward and its densify / opacity reset /
        optimiser steps: -> the visibility filter of reset_opacity_nonvisible
        (DPOnlineMapper reduces gradients and statistics over the ranks here)."""
        return out["radii"] > 0

    def _record_occ(self, kf, out):
        """initialize_map_opt's occlusion-aware visibility of the rendered
        keyframe (mapper.py:1025-1027)."""
        self.occ_vis[kf.uid] = (out["n_touched"] > 0).long()

    def _settle_replays(self):
        """The graph replays' overflow bookkeeping (IterationGraphs.account)
        before the host resets or reads optimiser step counts."""
        if self.graphs is not None:
            self.graphs.account()

    def _new_exposure_optimizer(self):
        """mapper.py:219-241: a fresh Adam over the window's exposures (not kf
        0): zero moments and step counts on their exposure-bank rows."""
        self._settle_replays()
        self.bank.sync(self.keyframes)
        uids = {k for k in self.window if k != 0 and k in self.keyframes}
        if uids:
            rows = torch.tensor([self.bank.slots[k] for k in sorted(uids)], device=self.dev)
            with torch.no_grad():
                self.bank.ex[rows, 1:] = 0.0
        self.kopt_steps = {k: 0 for k in uids}
        self.kopt_uids = uids

    # ---- the reference's entry points ----------------------------------------
    def initialize(self, keyframes, iters: int | None = None):
        """initialize_mapper + initialize_map_opt (mapper.py:732-1047): the
        keyframes' points (pcd_downsample_init), the window in insertion order,
        the exposure optimiser over every keyframe but 0, the initial
        optimisation, then the window cut to its last window_size keyframes
        (mapper.py:804-805)."""
        self.iteration_count = 0
        self.iterations_after_densify_or_reset = 0
        for kf in keyframes:
            self.keyframes[kf.uid] = kf
            self._add_points(kf, init=True)
            self.window = self.window + [kf.uid]
        self._new_exposure_optimizer()
        self.initialize_map_opt(iters)
        self.window = self.window[-self.cfg["window_size"]:]
        self._warm_deformation()

    def _warm_deformation(self):
        """One no-op pass of the map deformation (a keyframe id no Gaussian
        carries, identity poses) while the mapper initialises: its kernels and
        host ops are loaded here instead of in the first pose update of the
        live loop (~1 ms once)."""
        if self.ms is None or self.ms.P == 0 or not self.keyframes:
            return
        ghost = max(self.keyframes) + 1
        self.ms.store.update_mapping_points([{"kf_id": ghost, "w2c": torch.eye(4), "w2c_old": torch.eye(4),
                                              "method": "rigid"}], self.keyframes[self.window[-1]].K)

    def initialize_map_opt(self, iters: int | None = None):
        """Mapper.initialize_map_opt (mapper.py:922-1047) over the current
        window: per iteration a uniformly drawn keyframe, the initialisation
        loss (no exposure) + the strided DINO term + the isotropic term,
        statistics, densify_and_prune (init_gaussian_th, init_gaussian_extent,
        no size limit) every init_gaussian_update iterations from the first,
        reset_opacity at iteration_count == init_gaussian_reset, the Adams,
        and the keyframe's occlusion-aware visibility (n_touched > 0)."""
        c = self.cfg
        stack = list(self.window)
        self.bank.sync(self.keyframes)
        for it in range(c["init_itr_num"] if iters is None else iters):
            kf = self.keyframes[stack[self._pick(lambda: int(self.rng.choice(len(stack))))]]
            update = it % c["init_gaussian_update"] == 0
            reset = "all" if self.iteration_count + 1 == c["init_gaussian_reset"] else None
            out = self._iteration(kf, [kf.uid], True, update, reset)
            self._record_occ(kf, out)
        self._settle_replays()

    def prepare_keyframe(self, kf: Keyframe, keep=None):
        """The per-keyframe work before the mapping iterations
        (mapper.py:198-241): the visibility render, the window update, the
        keyframe's points, a fresh exposure optimiser -> the number of
        Gaussians added.  With ``self.phase_ms`` a dict, each phase is timed
        (device-synchronised) into it."""
        import time
        tm = self.phase_ms

        def mark(name, t0):
            if tm is None:
                return 0.0
            torch.cuda.synchronize(self.dev)
            t1 = time.perf_counter()
            if name:
                tm.setdefault(name, []).append(1e3 * (t1 - t0))
            return t1
        t = mark(None, 0.0)
        vis = self.visibility(kf)
        t = mark("visibility", t)
        self.keyframes[kf.uid] = kf
        self.bank.sync(self.keyframes)
        t = mark("bank_sync", t)
        self.window, self.last_removed = self._add_to_window(kf.uid, vis, self.window)
        t = mark("add_to_window", t)
        added = self._add_points(kf, init=False, keep=keep)
        t = mark("add_points", t)
        self._new_exposure_optimizer()
        mark("exposure_optimizer", t)
        return added

    def insert_keyframe(self, kf: Keyframe, iters: int | None = None, keep=None):
        """The Mapper's per-keyframe work (mapper.py:184-266) -> the number of
        Gaussians added.  ``keep``: the point subset (keyframe_points)."""
        added = self.prepare_keyframe(kf, keep=keep)
        split = self.map_opt_online(self.window, self.cfg["mapping_itr_num"] if iters is None else iters)
        if split:
            self.map_opt_online(self.window, 1)
        return added

    def update_keyframes(self, updates: dict, deform: bool = True):
        """Mapper._update_keyframes_from_frontend (mapper.py:365-429): the
        tracker's new poses (and, in the reference's ablation without metric
        depth, new depths) of existing keyframes.  ``updates``: {kf uid:
        (w2c [4, 4], depth [1, H, W] or None[, invalid])} -- ``invalid`` is
        get_w2c_and_depth's flag (too few valid frontend depths): the new
        depth is still stored, but the map moves rigidly (mapper.py:413-421).
        A keyframe whose pose is
        unchanged (allclose, atol 1e-6) and that has no new depth is skipped;
        the others get the new pose (and depth) and, with ``deform``
        (mapping.deform_gaussians, default True), their anchored Gaussians
        are moved by ``GaussianStore.update_mapping_points`` -- every
        keyframe in one pass.  As in the reference, the depth-rescale branch
        is handed the keyframe's depth AFTER it was replaced by the new one
        (mapper.py:399-401 then 423-429), so its rescale factor is 1.
        Returns the number of keyframes moved."""
        import time
        tm = self.phase_ms
        if tm is not None:
            torch.cuda.synchronize(self.dev)
            t0 = time.perf_counter()
        frames, moved, new_depth = [], [], False
        for k, upd in updates.items():
            w2c, depth = upd[0], upd[1]
            invalid = bool(upd[2]) if len(upd) > 2 else False
            kf = self.keyframes[k]
            w2c = torch.as_tensor(w2c, dtype=torch.float32).cpu()
            w2c_old = kf.w2c()
            # torch.allclose(w2c_old, w2c, atol=1e-6): |a - b| <= atol + rtol |b|
            # (rtol 1e-5), on the host arrays (a tenth of torch.allclose's time)
            if depth is None:
                a_, b_ = w2c_old.numpy(), w2c.numpy()
                if (np.abs(a_ - b_) <= 1e-6 + 1e-5 * np.abs(b_)).all():
                    continue
            kf.update_RT(w2c[:3, :3], w2c[:3, 3], upload=False)
            moved.append(kf)
            if depth is not None:
                new_depth = True
                kf.depth = depth.to(kf.image.device, torch.float32).reshape(1, kf.H, kf.W).contiguous()
                kf.median_depth = kf.depth.median()
            fr = {"kf_id": k, "w2c": w2c, "w2c_old": w2c_old}
            if depth is not None and not invalid:
                fr.update(method="depth", depth=kf.depth[0], depth_old=kf.depth[0])
            else:
                fr["method"] = "rigid"
            frames.append(fr)
        in_bank = self._upload_cameras(moved)
        if tm is not None:
            torch.cuda.synchronize(self.dev)
            t1 = time.perf_counter()
            tm.setdefault("uk_keyframes", []).append(1e3 * (t1 - t0))
        if deform and frames and self.ms is not None:
            K = self.keyframes[frames[0]["kf_id"]].K
            self.ms.store.update_mapping_points(frames, K)
        if tm is not None:
            torch.cuda.synchronize(self.dev)
            t2 = time.perf_counter()
            tm.setdefault("uk_deform", []).append(1e3 * (t2 - t1))
        if new_depth or not in_bank:
            self.bank.sync(self.keyframes)  # (new depths, or cameras outside the banks)
        if tm is not None:
            torch.cuda.synchronize(self.dev)
            tm.setdefault("uk_bank_sync", []).append(1e3 * (time.perf_counter() - t2))
        return len(frames)

    def _upload_cameras(self, kfs) -> bool:
        """The new raster fields (Keyframe.update_RT(upload=False)) of several
        keyframes in ONE host->device copy, written straight into their rows
        of the keyframe bank when it holds cameras (the Keyframes' fields
        rebound to them); else the Keyframes keep views of the staging copy.
        -> whether every camera went into the bank."""
        from .camera import raster_fields_batched
        from .online_graph import CAM_FLOATS
        if not kfs:
            return True
        groups: dict = {}   # keyframes sharing intrinsics: one batched formation each
        for i, kf in enumerate(kfs):
            groups.setdefault((kf.fx, kf.fy, kf.cx, kf.cy, kf.W, kf.H), []).append(i)
        parts, order = [], []
        for (fx, fy, cx, cy, W, H), idx in groups.items():
            f = raster_fields_batched(torch.stack([kfs[i].R for i in idx]), torch.stack([kfs[i].T for i in idx]),
                                      fx, fy, cx, cy, W, H)
            n = len(idx)
            parts.append(torch.cat([f["viewmatrix"].reshape(n, 16), f["projmatrix"].reshape(n, 16),
                                    f["projmatrix_raw"].reshape(1, 16).expand(n, 16), f["campos"],
                                    torch.zeros(n, CAM_FLOATS - 51)], 1))
            order += idx
        kfs = [kfs[i] for i in order]
        host = parts[0] if len(parts) == 1 else torch.cat(parts)
        b = self.bank
        in_bank = b.uniform and b.cam is not None and all(b.kfs.get(kf.uid) is kf for kf in kfs)
        if in_bank:
            # the keyframes' camera fields are views of their bank rows
            # (KeyframeBank._bind): the new values land under them in place.
            # The bank rows ride in the pad word of the same upload (one copy)
            host[:, CAM_FLOATS - 1] = torch.tensor([float(b.slots[kf.uid]) for kf in kfs])
            dev = host.to(self.dev)
            with torch.no_grad():
                b.cam.index_copy_(0, dev[:, CAM_FLOATS - 1].long(), dev)
            return True
        dev = host.to(self.dev)
        for i, kf in enumerate(kfs):  # (views of the staging copy)
            c = dev[i]
            kf.cam = dict(kf.cam, viewmatrix=c[0:16].view(4, 4), projmatrix=c[16:32].view(4, 4),
                          projmatrix_raw=c[32:48].view(4, 4), campos=c[48:51])
        return False

    def refine_pose_non_key_frame(self, w2c_init, image, fx: float, fy: float, cx: float, cy: float,
                                  features=None, uncertainty_aware: bool = True, iters: int | None = None):
        """Mapper.refine_pose_non_key_frame (mapper.py:810-917): a frame's pose
        refined against the map -> (w2c [4, 4] fp32 on the CPU, iterations run).

        As the reference: with uncertainty-aware tracking, the uncertainty MLP
        on the frame's features (no gradient; its dropout on), clipped at 0.1
        (+1e-3), bilinearly resized to the image, rescaled by 1 +
        bias_factor(train_frac_fix, 0.8) about 0.1; the frame's grad mask
        (Camera.compute_grad_mask); then up to tracking_itr_num iterations of
        render -> get_loss_tracking -> Adam over (cam_rot_delta 0.003,
        cam_trans_delta 0.001, exposure a / b 0.01, from zero) ->
        update_pose, stopping once |tau| < 1e-4 (wgsr.tracking.PoseRefine: the
        Adam step, SE3_exp update and next camera in one launch)."""
        from .camera import get_projection_matrix2
        from .tracking import PoseRefine, compute_grad_mask
        c = self.cfg
        dev = self.dev
        img = image.to(dev, torch.float32).reshape(3, *image.shape[-2:]).contiguous()
        H, W = int(img.shape[-2]), int(img.shape[-1])
        uncer = self.tracking_uncertainty(features, H, W) if uncertainty_aware and features is not None else None
        gm = compute_grad_mask(img, float(c["edge_threshold"]))
        ms = self.ms
        act = ms.activated()
        praw = get_projection_matrix2(0.01, 100.0, cx, cy, fx, fy, W, H).T.contiguous().to(dev)
        pr = PoseRefine(ms.xyz, act["opacity"], act["scales"], act["rotations"], ms.features, self.D, self.bg, praw,
                        H, W, focal2fov(fx, W), focal2fov(fy, H), lr_rot=c["lr_cam_rot_delta"],
                        lr_trans=c["lr_cam_trans_delta"], lr_exposure=0.01)
        w2c = torch.as_tensor(w2c_init, dtype=torch.float32).cpu()
        zero = torch.zeros(1, device=dev)
        R, T, _, _, n = pr.refine(w2c[:3, :3], w2c[:3, 3], zero, zero, img, gm, uncer,
                                  iters=c["tracking_itr_num"] if iters is None else iters)
        out = torch.eye(4)
        out[:3, :3], out[:3, 3] = R.cpu(), T.cpu()
        return out, n

    @torch.no_grad()
    def tracking_uncertainty(self, features, H: int, W: int):
        """The frame's uncertainty for pose refinement (mapper.py:837-849): the
        MLP (dropout on, no gradient), clip(min=0.1) + 1e-3, bilinear resize
        to H x W, (u - 0.1) (1 + bias_factor(train_frac_fix, 0.8)) + 0.1."""
        import torch.nn.functional as F

        from .uncertainty import bias_factor
        u = self.net(features.to(self.dev))
        u = torch.clip(u, min=0.1) + 1e-3
        u = F.interpolate(u.unsqueeze(0).unsqueeze(0), size=(H, W), mode="bilinear").squeeze()
        rate = 1 + 1 * bias_factor(self.cfg["train_frac_fix"], 0.8)
        return ((u - 0.1) * rate + 0.1).contiguous()

    def final_refine(self, iters: int = 26000):
        """Mapper.final_refine (mapper.py:1234-1372): uniform random
        keyframes, the uncertainty-aware loss on the RAW render (the exposure
        applied once), the uncertainty loss frozen for 200 iterations after
        the last densify / reset and the DINO term after them, the isotropic
        term; Adam for the Gaussians (no densification), the last window's
        exposure optimizer and the MLP; no densification statistics (the
        reference never adds them here).  (The reference's preceding
        _update_keyframes_from_frontend is ``update_keyframes``.)"""
        c = self.cfg
        ms = self.ms
        stack = [k for k in self.keyframes]
        self.stack = stack  # (the draws' keyframe list, for the data-parallel graphs)
        self.bank.sync(self.keyframes)
        for _ in range(iters):
            ci = self._pick(lambda: int(self.rng.choice(len(stack))))
            kf = self.keyframes[stack[ci]]
            if (self.graphs is not None and self.iterations_after_densify_or_reset + 1 >= 200
                    and self.graphs.step(kf, [stack[j] for j in range(max(0, ci - 2), min(len(stack), ci + 3))],
                                         refine=True)):
                self.iteration_count += 1
                self.iterations_after_densify_or_reset += 1
                ms.lr["xyz"] = lr_helper(self.iteration_count, self.lr_xyz[0], self.lr_xyz[1],
                                         lr_delay_mult=c["position_lr_delay_mult"],
                                         max_steps=c["position_lr_max_steps"])
                continue
            self.iteration_count += 1
            self.iterations_after_densify_or_reset += 1
            nbrs = [stack[j] for j in range(max(0, ci - 2), min(len(stack), ci + 3))]
            if self.iterations_after_densify_or_reset >= 200 and self._mlp_pair_ok():
                out = self._mlp_pair_loss(kf, nbrs, lambda unc: ms.forward_backward_uncertainty(
                    kf.cam, kf.image, kf.depth, kf.exposure_a, kf.exposure_b, self.bg, unc, c["train_frac_fix"],
                    c["train_frac_fix"], freeze_uncertainty_loss=False, median_depth=kf.median_depth,
                    pre_exposed=False, need_tau=False, exposure_partials=True, stats=False))
                self._max_nr = max(self._max_nr, int(out["num_rendered"]))
            else:
                unc = self.net(kf.features)
                freeze = self.iterations_after_densify_or_reset < 200
                out = ms.forward_backward_uncertainty(kf.cam, kf.image, kf.depth, kf.exposure_a, kf.exposure_b,
                                                      self.bg, unc, c["train_frac_fix"], c["train_frac_fix"],
                                                      freeze_uncertainty_loss=freeze, median_depth=kf.median_depth,
                                                      pre_exposed=False, need_tau=False, exposure_partials=True,
                                                      stats=False)
                self._max_nr = max(self._max_nr, int(out["num_rendered"]))
                if self.iterations_after_densify_or_reset >= 200:
                    self._dino_term(nbrs, kf)
            self._after_backward(out, False, False)
            ms.optimizer_step()
            ms.lr["xyz"] = lr_helper(self.iteration_count, self.lr_xyz[0], self.lr_xyz[1],
                                     lr_delay_mult=c["position_lr_delay_mult"], max_steps=c["position_lr_max_steps"])
            self._exposure_step(kf, out)
            self.uopt.step()
            self.uopt.zero_grad()
        self._settle_replays()

    def map_opt_online(self, window, iters: int = 1):
        """mapper.py:1049-1219."""
        c = self.cfg
        stack = [k for k in self.keyframes]
        cur_prob = 0.5
        n_other = len(stack) - len(window)
        prob = np.full(len(stack), (1 - cur_prob) * iters / n_other if n_other else 0.0)
        if len(window) <= len(stack) / 2.0:
            for i, k in enumerate(stack):
                if k in window:
                    prob[i] = cur_prob * iters / len(window)
        if prob.sum() == 0:
            prob[:] = 1.0
        prob /= prob.sum()
        # rng.choice(len(stack), p=prob) per iteration, restated: numpy's own
        # inverse-CDF draw (the same single random() per call, the same
        # indices) without its per-call checks of p
        # (a test's scripted stand-in for the generator still gets choice())
        cdf = prob.cumsum()
        cdf /= cdf[-1]
        fast = isinstance(self.rng, np.random.Generator)
        split = False
        self.stack = stack
        self.bank.sync(self.keyframes)
        ms = self.ms
        for it in range(iters):
            ci = self._pick(lambda: int(cdf.searchsorted(self.rng.random(), side="right")) if fast
                            else int(self.rng.choice(len(stack), p=prob)))
            kf = self.keyframes[stack[ci]]
            nb = [stack[j] for j in range(max(0, ci - 2), min(len(stack), ci + 3))]
            nxt = self.iteration_count + 1
            update = nxt % c["gaussian_update_every"] == c["gaussian_update_offset"]
            reset = "nonvisible" if (nxt % c["gaussian_reset"] == 0 and not update) else None
            last = it == iters - 1
            # the steady state (no densify / reset / visibility update, the
            # DINO term on) as a graph replay (wgsr.online_graph)
            if (self.graphs is not None and not update and reset is None and not last
                    and self.iterations_after_densify_or_reset + 1 >= 20 and self.graphs.step(kf, nb)):
                self.iteration_count += 1
                self.iterations_after_densify_or_reset += 1
                ms.lr["xyz"] = lr_helper(self.iteration_count, self.lr_xyz[0], self.lr_xyz[1],
                                         lr_delay_mult=c["position_lr_delay_mult"],
                                         max_steps=c["position_lr_max_steps"])
                continue
            self._iteration(kf, nb, False, update, reset, occ_window=window if last else None)
            split = split or update or reset is not None
        self._settle_replays()
        return split
