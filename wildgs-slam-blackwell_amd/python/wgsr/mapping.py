"""One WildGS mapping iteration on the gfx950 path (SURVEY.md 8(f) f1 + f2).

The reference's inner mapping loop (src/mapper.py:1083-1219, the
non-uncertainty branch) runs, per iteration, ~100 small torch kernels around
the rasteriser: GaussianModel's activations and the SH ``torch.cat``
(gaussian_model.py get_*), get_loss_mapping_rgbd (slam_utils.py:107-143:
exposure correction, 0.8 L1 + 0.2 (1 - SSIM) on rgb with the boundary mask,
masked depth L1), ``10 * isotropic_loss.mean()`` (mapper.py:1167-1169), the
autograd backward of all of it, the densification statistics with boolean
indexing (mapper.py:1177-1183, gaussian_model.py:745-749) and
``torch.optim.Adam`` over six parameter groups (gaussian_model.py:309).

``MappingStep`` runs the same iteration as ~15 launches: one activation
kernel, the rasteriser forward, one loss kernel + the fused SSIM, the SSIM
backward, one loss-backward kernel, the rasteriser backward (writing straight
into the parameter-gradient storage), one activation-backward kernel (with
the isotropic term folded in), one statistics kernel and ONE Adam launch.
The SH coefficients live in one [P, M, 3] storage: ``f_dc`` / ``f_rest`` are
views of it (no per-iteration cat, no gradient split), and their different
learning rates ride in one Adam tensor (``wgsr_adam_tensor.split_*``).

Gradients, loss, statistics and Adam arithmetic match the reference's torch
composition (tests/test_gpu_mapping.py).  No fallback: libwgsr.so must load.
"""
from __future__ import annotations

import ctypes
import math

import torch

from . import _lib

# gaussian_model.py:271-309 (training_setup) with opt_params of the configs
DEFAULT_LR = {"xyz": 1.6e-4, "f_dc": 2.5e-3, "f_rest": 2.5e-3 / 20.0, "opacity": 5e-2, "scaling": 5e-3,
              "rotation": 1e-3}


def _blocks(n):
    return int(_lib.load().wgsr_map_blocks(int(n)))


def rasterize_forward_cap(bg, means3D, opacity, scales, rotations, sh, degree: int, cam: dict, H: int, W: int,
                          cap: int, counts):
    """The rasteriser forward in capacity mode (wgsr_rasterize_forward_cap):
    ``_C.rasterize_gaussians``' outputs with no host wait, its buffers sized
    for ``cap`` (Gaussian, tile) pairs and num_rendered = ``cap``; counts
    (int32 [5] device tensor): N_rect, N_exact, N_bin, overflow, min(N_bin,
    cap).  For graph capture (wgsr.online); not an upstream entry point."""
    L = _lib.load()
    dev = means3D.device
    P = int(means3D.shape[0])
    f = dict(dtype=torch.float32, device=dev)
    color = torch.empty(3, H, W, **f)
    depth = torch.empty(1, H, W, **f)
    opac = torch.empty(1, H, W, **f)
    radii = torch.empty(P, dtype=torch.int32, device=dev)
    n_touched = torch.empty(P, dtype=torch.int32, device=dev)
    p = _lib.ptr
    a = _lib.RasterArgs(P=P, D=int(degree), M=int(sh.shape[1]), W=int(W), H=int(H), bg=p(bg), means3D=p(means3D),
                        colors=None, opacities=p(opacity), scales=p(scales), rotations=p(rotations),
                        cov3D_precomp=None, shs=p(sh), viewmatrix=p(cam["viewmatrix"]),
                        projmatrix=p(cam["projmatrix"]), projmatrix_raw=p(cam["projmatrix_raw"]),
                        campos=p(cam["campos"]), scale_modifier=1.0, tan_fovx=float(cam["tanfovx"]),
                        tan_fovy=float(cam["tanfovy"]), prefiltered=0, debug=0)
    with torch.cuda.device(dev), _lib.AllocRequest(dev) as req:
        code = L.wgsr_rasterize_forward_cap(ctypes.byref(a), int(cap), _lib.ALLOC_GEOM, _lib.ALLOC_BINNING,
                                            _lib.ALLOC_IMAGE, None, p(color), p(depth), p(opac),
                                            p(radii) if P else None, p(n_touched) if P else None, p(counts),
                                            _lib.stream_handle(dev))
    _lib.check(code)
    empty = torch.empty(0, dtype=torch.uint8, device=dev)
    b = req.buffers
    return (int(cap), color, radii, b.get("geom", empty), b.get("binning", empty), b.get("image", empty), depth,
            opac, n_touched)


def check_tile_lists(fwd, means3D, cam: dict, H: int, W: int, degree: int, sh, bad):
    """wgsr_check_tile_lists on a forward's state buffers (``fwd``: the
    rasteriser forward's 9-tuple; its num_rendered -- the capacity in
    capacity mode -- sizes the list region): bad tiles, bad ids and bad
    pixels are added to ``bad`` (int32 [3] device tensor).  No host wait."""
    L = _lib.load()
    dev = means3D.device
    p = _lib.ptr
    a = _lib.RasterArgs(P=int(means3D.shape[0]), D=int(degree), M=int(sh.shape[1]), W=int(W), H=int(H),
                        bg=p(means3D), means3D=p(means3D), colors=None, opacities=p(means3D), scales=p(means3D),
                        rotations=p(means3D), cov3D_precomp=None, shs=p(sh), viewmatrix=p(cam["viewmatrix"]),
                        projmatrix=p(cam["projmatrix"]), projmatrix_raw=p(cam["projmatrix_raw"]),
                        campos=p(cam["campos"]), scale_modifier=1.0, tan_fovx=float(cam["tanfovx"]),
                        tan_fovy=float(cam["tanfovy"]), prefiltered=0, debug=0)
    with torch.cuda.device(dev):
        _lib.check(L.wgsr_check_tile_lists(ctypes.byref(a), int(fwd[0]), p(fwd[4]), p(fwd[5]), p(bad),
                                           _lib.stream_handle(dev)))


class MappingStep:
    """GaussianModel state in the fused layout + one-call mapping iterations.

    The state lives in a ``GaussianStore`` (capacity-preallocated banks,
    wgsr/store.py): keyframe insertion (``extend``), ``densify_and_prune`` and
    the opacity resets change the row count without re-allocating, and every
    view below (``xyz``, ``grad``, ``exp_avg`` ...) is re-taken from the
    current bank."""

    GROUPS = ("xyz", "features", "opacity", "scaling", "rotation")

    def __init__(self, xyz, features_dc, features_rest, opacity, scaling, rotation, sh_degree: int,
                 lr: dict | None = None, betas=(0.9, 0.999), eps: float = 1e-15, capacity: int | None = None):
        from .store import GaussianStore
        dev = xyz.device
        f32 = dict(dtype=torch.float32, device=dev)
        P = xyz.shape[0]
        self.D = int(sh_degree)
        features = torch.cat([features_dc, features_rest], dim=1).detach().to(**f32).contiguous()
        self.M = features.shape[1]
        self.store = GaussianStore(xyz.detach().to(**f32), features, opacity.detach().to(**f32).reshape(P, 1),
                                   scaling.detach().to(**f32), rotation.detach().to(**f32), capacity=capacity)
        self.lr = dict(DEFAULT_LR, **(lr or {}))
        self.betas, self.eps = betas, eps
        # torch.optim.Adam keeps a step count per parameter; a group whose
        # parameter was replaced without a gradient (densify, opacity reset)
        # skips its update and its count (f_dc and f_rest always move together)
        self.steps = {g: 0 for g in self.GROUPS}
        self._iso = None
        self.list_check = None  # int32 [3] device tensor: every forward's tile lists checked into it (tests)

    # storage views (current bank, [:P]) --------------------------------------
    @property
    def P(self):
        return self.store.P

    @property
    def step_count(self):
        return self.steps["xyz"]

    @property
    def xyz(self):
        return self.store.param("xyz")

    @property
    def features(self):
        return self.store.param("features")

    @property
    def opacity(self):
        return self.store.param("opacity")

    @property
    def scaling(self):
        return self.store.param("scaling")

    @property
    def rotation(self):
        return self.store.param("rotation")

    @property
    def grad(self):
        return {n: self.store.grad(n) for n in self.GROUPS}

    @property
    def exp_avg(self):
        return {n: self.store.exp_avg(n) for n in self.GROUPS}

    @property
    def exp_avg_sq(self):
        return {n: self.store.exp_avg_sq(n) for n in self.GROUPS}

    @property
    def max_radii2D(self):
        return self.store.stat("max_radii2D")

    @property
    def xyz_gradient_accum(self):
        return self.store.stat("xyz_gradient_accum")

    @property
    def denom(self):
        return self.store.stat("denom")

    @property
    def act(self):
        return {k: self.store.scratch("act_" + k) for k in ("opacity", "scales", "rotations")}

    @property
    def act_grad(self):
        return {k: self.store.scratch("actg_" + k) for k in ("opacity", "scales", "rotations")}

    @property
    def iso_part(self):
        n = max(1, _blocks(self.P))
        if self._iso is None or self._iso.numel() != n:
            self._iso = torch.empty(n, dtype=torch.float32, device=self.store.device)
        return self._iso

    # reference-style views -------------------------------------------------
    @property
    def f_dc(self):
        return self.features[:, :1]

    @property
    def f_rest(self):
        return self.features[:, 1:]

    @property
    def get_opacity(self):
        return torch.sigmoid(self.opacity)

    @property
    def get_scaling(self):
        return torch.exp(self.scaling)

    @property
    def get_rotation(self):
        return torch.nn.functional.normalize(self.rotation)

    # densification (GaussianModel, gaussian_model.py:231-269, 389-402, 646-743)
    def extend(self, xyz, features, scaling, rotation, opacity, kf_id=None):
        """extend_from_pcd (gaussian_model.py:231-259): features [n, M, 3]."""
        self.store.append(xyz, features, opacity, scaling, rotation, kf_id=None if kf_id is None else int(kf_id))

    def densify_and_prune(self, max_grad, min_opacity, extent, max_screen_size, percent_dense=0.01, z=None,
                          generator=None):
        """Every parameter is replaced: the reference's optimizer.step() that
        follows skips them all (their new nn.Parameters carry no gradient)."""
        out = self.store.densify_and_prune(max_grad, min_opacity, extent, max_screen_size, percent_dense, z=z,
                                           generator=generator)
        self._skip = set(self.GROUPS)
        return out

    def reset_opacity_nonvisible(self, visibility_filters):
        self.store.reset_opacity_nonvisible(visibility_filters)
        self._skip = getattr(self, "_skip", set()) | {"opacity"}

    def reset_opacity(self):
        self.store.reset_opacity()
        self._skip = getattr(self, "_skip", set()) | {"opacity"}

    # -----------------------------------------------------------------------
    def activated(self) -> dict:
        """The activated opacity / scales / rotations (get_opacity, get_scaling,
        get_rotation; the activation kernel the render path uses) -> self.act."""
        L = _lib.load()
        dev = self.xyz.device
        p = _lib.ptr
        a = self.act
        with torch.cuda.device(dev):
            _lib.check(L.wgsr_gaussian_activate(self.P, p(self.opacity), p(self.scaling), p(self.rotation),
                                                p(a["opacity"]), p(a["scales"]), p(a["rotations"]),
                                                p(self.iso_part), _lib.stream_handle(dev)))
        return a

    def _render(self, cam: dict, H: int, W: int, bg, cap: int | None = None, counts=None):
        """Activations (+ isotropic partial sums) and the rasteriser forward
        (``cap``: the capacity-mode forward, its counts into ``counts``)."""
        from diff_gaussian_rasterization import _C
        L = _lib.load()
        dev = self.xyz.device
        p = _lib.ptr
        e = torch.empty(0, device=dev)
        a = self.act
        with torch.cuda.device(dev):
            _lib.check(L.wgsr_gaussian_activate(self.P, p(self.opacity), p(self.scaling), p(self.rotation),
                                                p(a["opacity"]), p(a["scales"]), p(a["rotations"]),
                                                p(self.iso_part), _lib.stream_handle(dev)))
        if cap is not None:
            fwd = rasterize_forward_cap(bg, self.xyz, a["opacity"], a["scales"], a["rotations"], self.features,
                                        self.D, cam, H, W, cap, counts)
        else:
            fwd = _C.rasterize_gaussians(
                bg, self.xyz, e, a["opacity"], a["scales"], a["rotations"], 1.0, e, cam["viewmatrix"],
                cam["projmatrix"], cam["projmatrix_raw"], cam["tanfovx"], cam["tanfovy"], H, W, self.features,
                self.D, cam["campos"], False, False)
        if self.list_check is not None:  # (tests: the forward's tile lists checked on the device)
            check_tile_lists(fwd, self.xyz, cam, H, W, self.D, self.features, self.list_check)
        return fwd

    def _backward(self, cam: dict, bg, fwd, d_image, d_depth, w_iso: float, need_tau: bool = True, skip=None,
                  stats: bool = True):
        """Rasteriser backward straight into the gradient storage, activation
        backward (isotropic term folded in), densification statistics.
        ``skip``: a capacity-mode forward's overflow word (counts[3:4]); when
        set on the device the statistics stay unchanged (that iteration has no
        gradient).  ``stats=False``: no densification statistics at all (the
        reference's final_refine, mapper.py:1346-1362, never calls
        add_densification_stats).  -> (dL/dmeans2D, dL/dtau summed over P, or
        None without need_tau)."""
        from diff_gaussian_rasterization import _C
        L = _lib.load()
        dev = self.xyz.device
        p = _lib.ptr
        st = _lib.stream_handle(dev)
        e = torch.empty(0, device=dev)
        a = self.act
        nr, _, radii, geom, binning, img = fwd[:6]
        out = {"means3D": self.grad["xyz"], "shs": self.grad["features"], "opacities": self.act_grad["opacity"],
               "scales": self.act_grad["scales"], "rotations": self.act_grad["rotations"]}
        g = _C.rasterize_gaussians_backward(
            bg, self.xyz, radii, e, a["scales"], a["rotations"], 1.0, e, cam["viewmatrix"], cam["projmatrix"],
            cam["projmatrix_raw"], cam["tanfovx"], cam["tanfovy"], d_image, d_depth, self.features, self.D,
            cam["campos"], geom, nr, binning, img, False, out=out)
        dL_dmeans2D, dL_dtau = g[0], g[8]
        with torch.cuda.device(dev):
            if stats:
                _lib.check(L.wgsr_gaussian_activate_backward_stats(
                    self.P, p(self.opacity), p(self.scaling), p(self.rotation), p(self.act_grad["opacity"]),
                    p(self.act_grad["scales"]), p(self.act_grad["rotations"]), float(w_iso), p(self.grad["opacity"]),
                    p(self.grad["scaling"]), p(self.grad["rotation"]), p(radii), p(dL_dmeans2D), p(self.max_radii2D),
                    p(self.xyz_gradient_accum), p(self.denom), p(skip) if skip is not None else None, st))
            else:
                _lib.check(L.wgsr_gaussian_activate_backward(
                    self.P, p(self.opacity), p(self.scaling), p(self.rotation), p(self.act_grad["opacity"]),
                    p(self.act_grad["scales"]), p(self.act_grad["rotations"]), float(w_iso), p(self.grad["opacity"]),
                    p(self.grad["scaling"]), p(self.grad["rotation"]), st))
        return dL_dmeans2D, (dL_dtau.sum(0) if need_tau else None)

    def forward_backward(self, cam: dict, gt_image, gt_depth, exposure_a, exposure_b, bg,
                         alpha: float = 0.95, lambda_dssim: float = 0.2, rgb_threshold: float = 0.01,
                         iso_weight: float = 10.0):
        """Loss of one view and the gradients of every raw parameter (written
        to ``self.grad``), plus the densification statistics update.

        cam: viewmatrix, projmatrix, projmatrix_raw, campos (device tensors),
        tanfovx, tanfovy (floats).  Returns a dict: ``loss`` (0-d device
        tensor), ``dexposure_a`` / ``dexposure_b`` ([1]), ``dtheta`` / ``drho``
        ([3], the keyframe pose gradient), ``radii``, ``image``, ``depth``."""
        L = _lib.load()
        P, dev = self.P, self.xyz.device
        H, W = gt_image.shape[-2], gt_image.shape[-1]
        HW = H * W
        st = _lib.stream_handle(dev)
        p = _lib.ptr
        fwd = self._render(cam, H, W, bg)
        nr, image, radii, depth = fwd[0], fwd[1], fwd[2], fwd[6]
        gt = gt_image.contiguous()
        gtd = gt_depth.contiguous()
        ea, eb = exposure_a.detach().contiguous(), exposure_b.detach().contiguous()
        nb = max(1, _blocks(HW))
        image_ab = torch.empty_like(image)
        lpart = torch.empty(nb, 2, device=dev)
        ssim_dmap = torch.empty(3 * 3 * HW, device=dev)
        ssim_plane = torch.empty(3, device=dev)
        ssim_mean = torch.empty((), device=dev)
        with torch.cuda.device(dev):
            _lib.check(L.wgsr_mapping_loss_forward(H, W, p(image), p(gt), p(depth), p(gtd), p(ea), p(eb),
                                                   float(rgb_threshold), p(image_ab), p(lpart), st))
            with _lib.AllocRequest(dev):
                _lib.check(L.wgsr_ssim_forward(p(image_ab), p(gt), 3, H, W, 11, p(ssim_dmap), p(ssim_plane),
                                               p(ssim_mean), _lib.ALLOC_SCRATCH, None, st))
        sums = lpart.sum(0)
        w_rgb = alpha * (1.0 - lambda_dssim) / (3 * HW)
        w_depth = (1.0 - alpha) / HW
        w_iso = iso_weight / (3 * P) if P else 0.0
        loss = (w_rgb * sums[0] + alpha * lambda_dssim * (1.0 - ssim_mean) + w_depth * sums[1]
                + w_iso * self.iso_part.sum())
        # backward: SSIM term (dL/dssim = -alpha lambda, size-averaged over 3HW)
        scale = torch.full((3,), -alpha * lambda_dssim / (3 * HW), device=dev)
        ssim_grad = torch.empty_like(image_ab)
        d_image = torch.empty_like(image)
        d_depth = torch.empty_like(depth)
        epart = torch.empty(nb, 2, device=dev)
        with torch.cuda.device(dev):
            _lib.check(L.wgsr_ssim_backward(p(image_ab), p(gt), 3, H, W, 11, p(ssim_dmap), p(scale), p(ssim_grad),
                                            st))
            _lib.check(L.wgsr_mapping_loss_backward(H, W, p(image), p(image_ab), p(gt), p(depth), p(gtd), p(ea),
                                                    float(rgb_threshold), float(w_rgb), float(w_depth),
                                                    p(ssim_grad), p(d_image), p(d_depth), p(epart), st))
        _, tau = self._backward(cam, bg, fwd, d_image, d_depth, w_iso)
        esum = epart.sum(0)
        return {"loss": loss, "dexposure_a": esum[0:1], "dexposure_b": esum[1:2], "drho": tau[:3],
                "dtheta": tau[3:], "radii": radii, "image": image, "depth": depth, "num_rendered": nr}

    def forward_backward_uncertainty(self, cam: dict, gt_image, gt_depth, exposure_a, exposure_b, bg, uncertainty,
                                     train_frac: float, ssim_frac: float, config: dict | None = None,
                                     initialization: bool = False, freeze_uncertainty_loss: bool = False,
                                     median_depth=None, iso_weight: float = 10.0, pre_exposed: bool = True,
                                     cap: int | None = None, counts=None, need_tau: bool = True,
                                     exposure_partials: bool = False, stats: bool = True):
        """The reference's DEFAULT mapping iteration (uncertainty_params.activate):
        get_loss_mapping_uncertainty (slam_utils.py:146-258) + 10 * isotropic
        loss, and their backward.

        Which of the mapper's three call sites is fused is chosen by the flags:

        * ``pre_exposed=True`` (default) -- map_opt_online (mapper.py:1120-1138),
          which passes ``exp(a) * image + b`` into the loss, where the exposure
          correction is applied a second time (slam_utils.py:179-181).  Both
          applications are fused into the loss kernels, and the image and
          exposure gradients chain through both.
        * ``pre_exposed=False`` -- final_refine (mapper.py:1290-1306): the raw
          render goes in and the loss applies the correction once.
        * ``initialization=True`` -- initialize_map_opt (mapper.py:974-984): no
          exposure correction at all (``pre_exposed`` is ignored).

        ``uncertainty`` is the uncertainty MLP's output map [h, w] for this
        view (``uncer_network(viewpoint.features)``, run by the caller); its
        gradient is fed back with ``uncertainty.backward`` (as the reference's
        ``loss.backward()`` reaches the MLP) unless
        ``freeze_uncertainty_loss``.  ``config``: the reference's mapping config
        dict (Training.alpha / rgb_boundary_threshold / ssim_loss,
        opt_params.lambda_dssim, uncertainty_params.*); defaults are
        configs/wildgs_slam.yaml's.  ``median_depth``: optional cached
        ``gt_depth.median()`` (constant per keyframe).  ``full_resolution``
        (depth rendered at another size) is not supported.  ``cap`` /
        ``counts``: the capacity-mode forward (no host wait; graph capture,
        wgsr.online).  ``exposure_partials``: the exposure gradient as the loss
        backward's per-block (a, b) partial sums (``dexposure_partials``
        [n, 2], for wgsr_exposure_step) instead of its sum.  ``stats=False``:
        no densification statistics (final_refine).  Returns the dict of
        ``forward_backward`` plus ``uncertainty_grad`` and ``uncertainty_loss``."""
        from . import uncertainty as U
        cfg = U.flatten_config(config)
        P = self.P
        H, W = gt_image.shape[-2], gt_image.shape[-1]
        fwd = self._render(cam, H, W, bg, cap, counts)
        nr, image, radii, depth, opac_img = fwd[0], fwd[1], fwd[2], fwd[6], fwd[7]
        w_iso = iso_weight / (3 * P) if P else 0.0
        loss, state = U.loss_forward(image, depth, opac_img, gt_image, gt_depth, exposure_a, exposure_b, uncertainty,
                                     train_frac, ssim_frac, cfg, initialization, freeze_uncertainty_loss,
                                     median_depth, extra=(self.iso_part, w_iso), pre_exposed=pre_exposed)
        d_image, d_depth, d_a, d_b, d_unc = U.loss_backward(state, exposure_partials=exposure_partials)
        _, tau = self._backward(cam, bg, fwd, d_image, d_depth, w_iso, need_tau,
                                skip=counts[3:4] if cap is not None else None, stats=stats)
        if uncertainty.requires_grad and not freeze_uncertainty_loss:
            uncertainty.backward(d_unc.to(uncertainty.dtype))
        if exposure_partials:
            return {"loss": loss, "dexposure_partials": d_a, "radii": radii, "image": image, "depth": depth,
                    "n_touched": fwd[8], "num_rendered": nr, "uncertainty_grad": d_unc,
                    "uncertainty_loss": state.uncertainty_loss,
                    "drho": tau[:3] if tau is not None else None, "dtheta": tau[3:] if tau is not None else None}
        return {"loss": loss, "dexposure_a": d_a, "dexposure_b": d_b,
                "drho": tau[:3] if tau is not None else None, "dtheta": tau[3:] if tau is not None else None,
                "radii": radii, "image": image, "depth": depth, "n_touched": fwd[8], "num_rendered": nr,
                "uncertainty_grad": d_unc,
                "uncertainty_loss": state.uncertainty_loss}

    @torch.no_grad()
    def optimizer_step(self, skip=()):
        """torch.optim.Adam(param_groups, lr=0.0, eps=1e-15).step() over the six
        reference groups, ONE launch (f_dc / f_rest as a two-rate split).
        Groups in ``skip`` -- and those whose parameter a densify / opacity
        reset replaced since the last step -- take no update and keep their
        step count, as torch's Adam does for a parameter without a gradient."""
        L = _lib.load()
        skip = set(skip) | getattr(self, "_skip", set())
        self._skip = set()
        b1, b2 = self.betas
        lr = self.lr
        ts = []
        for name, step, tail in (("xyz", lr["xyz"], None), ("features", lr["f_dc"], lr["f_rest"]),
                                 ("opacity", lr["opacity"], None), ("scaling", lr["scaling"], None),
                                 ("rotation", lr["rotation"], None)):
            if name in skip:
                continue
            self.steps[name] += 1
            n = self.steps[name]
            bc1 = 1.0 - b1 ** n
            bc2s = math.sqrt(1.0 - b2 ** n)
            prm = self.store.param(name)
            t = _lib.AdamTensor(prm.data_ptr(), self.store.grad(name).data_ptr(),
                                self.store.exp_avg(name).data_ptr(), self.store.exp_avg_sq(name).data_ptr(),
                                prm.numel(), step / bc1, bc2s)
            if tail is not None:
                t.split_period, t.split_len, t.step_size_tail = 3 * self.M, 3, tail / bc1
            ts.append(t)
        if not ts or self.P == 0:
            return
        arr = (_lib.AdamTensor * len(ts))(*ts)
        dev = self.store.device
        with torch.cuda.device(dev):
            _lib.check(L.wgsr_adam_step(arr, len(ts), b1, b2, self.eps, _lib.stream_handle(dev)))

    def adam_tensors(self):
        """The Gaussian groups as wgsr_adam_tensor rows for wgsr_adam_step_dev
        (3 scalars per group in GROUPS order, from ``adam_scalars``)."""
        ts = []
        for name in self.GROUPS:
            prm = self.store.param(name)
            t = _lib.AdamTensor(prm.data_ptr(), self.store.grad(name).data_ptr(),
                                self.store.exp_avg(name).data_ptr(), self.store.exp_avg_sq(name).data_ptr(),
                                prm.numel(), 0.0, 1.0)
            if name == "features":
                t.split_period, t.split_len = 3 * self.M, 3
            ts.append(t)
        return ts

    def adam_scalars(self, out):
        """optimizer_step's per-group scalars of one step that skips no group,
        into ``out`` (float32 [15]: step_size, sqrt(1 - beta2^n), tail step
        size per group); advances the step counts as optimizer_step does."""
        b1, b2 = self.betas
        lr = self.lr
        for i, (name, step, tail) in enumerate((("xyz", lr["xyz"], lr["xyz"]),
                                                ("features", lr["f_dc"], lr["f_rest"]),
                                                ("opacity", lr["opacity"], lr["opacity"]),
                                                ("scaling", lr["scaling"], lr["scaling"]),
                                                ("rotation", lr["rotation"], lr["rotation"]))):
            self.steps[name] += 1
            n = self.steps[name]
            bc1 = 1.0 - b1 ** n
            out[3 * i] = step / bc1
            out[3 * i + 1] = math.sqrt(1.0 - b2 ** n)
            out[3 * i + 2] = tail / bc1

    @torch.no_grad()
    def optimizer_step_dev(self, tensors, scalars, skip):
        """optimizer_step with the scalars in device memory (``scalars``:
        float32 [15] device tensor, see adam_scalars) and a device skip word
        (a capacity-mode forward's overflow flag): ONE launch whose arguments
        do not change between steps, so it can be captured in a graph."""
        L = _lib.load()
        b1, b2 = self.betas
        arr = (_lib.AdamTensor * len(tensors))(*tensors)
        dev = self.store.device
        with torch.cuda.device(dev):
            _lib.check(L.wgsr_adam_step_dev(arr, len(tensors), b1, b2, self.eps, 0.0, _lib.ptr(scalars),
                                            _lib.ptr(skip), _lib.stream_handle(dev)))

    def step(self, *args, **kwargs):
        """forward_backward + optimizer_step (one reference mapping iteration
        without densify / prune / opacity reset)."""
        out = self.forward_backward(*args, **kwargs)
        self.optimizer_step()
        return out
