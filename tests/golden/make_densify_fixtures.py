"""Generate tests/golden/ref_densify.npz by EXECUTING the reference's own
GaussianModel densification code in the build container (/root/reference
exists only here; the fixture travels, the reference does not).

Runs unchanged (thirdparty/gaussian_splatting/scene/gaussian_model.py):
``training_setup`` (torch.optim.Adam over the six groups, eps 1e-15),
``densify_and_prune`` -> ``densify_and_clone`` / ``densify_and_split`` /
``densification_postfix`` / ``cat_tensors_to_optimizer`` / ``prune_points`` /
``_prune_optimizer``, then ``reset_opacity_nonvisible`` and ``prune_points``
on their own, then ``reset_opacity``.

Stand-ins, as in make_render_fixtures.py: open3d / plyfile / simple_knn /
cv2 modules (imported, unused here); ``device="cuda"`` -> CPU through a
TorchFunctionMode, which also records the split's noise: the reference draws
``torch.normal(mean=0, std=stds)``; the mode returns ``z * stds + 0`` for a
seeded standard-normal ``z`` it stores, so the GPU path can be fed the same
``z``.

Usage:  python tests/golden/make_densify_fixtures.py
"""
from __future__ import annotations

import math
import os
import sys
import types

import numpy as np
import torch
from torch.overrides import TorchFunctionMode

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"

Z_DRAWS: list = []


class CudaToCpuRecordNormal(TorchFunctionMode):
    def __init__(self, gen):
        super().__init__()
        self.gen = gen

    def __torch_function__(self, func, types_, args=(), kwargs=None):
        kwargs = dict(kwargs or {})
        d = kwargs.get("device")
        if d is not None and str(d).startswith("cuda"):
            kwargs["device"] = "cpu"
        if func is torch.Tensor.cuda:
            return args[0]
        if func is torch.normal and "std" in kwargs:
            std, mean = kwargs["std"], kwargs["mean"]
            z = torch.randn(std.shape, generator=self.gen)
            Z_DRAWS.append(z)
            return z * std + mean
        return func(*args, **kwargs)


def _stubs():
    for name in ("open3d", "cv2"):
        sys.modules.setdefault(name, types.ModuleType(name))
    ply = types.ModuleType("plyfile")
    ply.PlyData = ply.PlyElement = None
    sys.modules.setdefault("plyfile", ply)
    sk = types.ModuleType("simple_knn")
    skc = types.ModuleType("simple_knn._C")
    skc.distCUDA2 = None
    sk._C = skc
    sys.modules.setdefault("simple_knn", sk)
    sys.modules.setdefault("simple_knn._C", skc)
    sys.path.insert(0, REF)


NAMES = ("xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation")


def snapshot(gm, tag, out):
    for n, t in zip(NAMES, (gm._xyz, gm._features_dc, gm._features_rest, gm._opacity, gm._scaling, gm._rotation)):
        out[f"{tag}_{n}"] = t.detach().numpy().copy()
    for g in gm.optimizer.param_groups:
        st = gm.optimizer.state.get(g["params"][0], None)
        out[f"{tag}_m_{g['name']}"] = st["exp_avg"].numpy().copy()
        out[f"{tag}_v_{g['name']}"] = st["exp_avg_sq"].numpy().copy()
        out[f"{tag}_step_{g['name']}"] = np.array(float(st["step"]))
    out[f"{tag}_accum"] = gm.xyz_gradient_accum.numpy().copy()
    out[f"{tag}_denom"] = gm.denom.numpy().copy()
    out[f"{tag}_max_radii2D"] = gm.max_radii2D.numpy().copy()
    out[f"{tag}_kf_id"] = gm.unique_kfIDs.numpy().astype(np.int32).copy()
    out[f"{tag}_n_obs"] = gm.n_obs.numpy().astype(np.int32).copy()


def main():
    _stubs()
    from thirdparty.gaussian_splatting.scene.gaussian_model import GaussianModel

    g = torch.Generator().manual_seed(2024)
    P, SH = 700, 1
    M = (SH + 1) ** 2
    out = {}
    with CudaToCpuRecordNormal(g):
        gm = GaussianModel(SH)
        gm.init_lr(1.0)
        xyz = torch.randn(P, 3, generator=g) * 2
        # scales spanning clone (<= 0.01), split (0.01, 0.1] and world-prune (> 0.1)
        log_s = math.log(0.002) + (math.log(0.4) - math.log(0.002)) * torch.rand(P, 3, generator=g)
        q = torch.randn(P, 4, generator=g) * (0.5 + torch.rand(P, 1, generator=g))
        op = torch.randn(P, 1, generator=g) * 2.0
        feat = torch.randn(P, M, 3, generator=g) * 0.3
        rgb = torch.zeros(P, 3, M)
        rgb[:] = feat.transpose(1, 2)
        args = types.SimpleNamespace(percent_dense=0.01, position_lr_init=1.6e-4, position_lr_final=1.6e-6,
                                     position_lr_delay_mult=0.01, position_lr_max_steps=30000, feature_lr=2.5e-3,
                                     opacity_lr=0.05, scaling_lr=1e-3, rotation_lr=1e-3)
        gm.training_setup(args)  # as the Mapper: optimizer first, then the first keyframe's points
        gm.extend_from_pcd(xyz, rgb, log_s, q, op, kf_id=3)
        gm.unique_kfIDs = torch.randint(0, 9, (P,), generator=g).int()
        gm.n_obs = torch.randint(0, 20, (P,), generator=g).int()
        # Adam history: two steps with random gradients (non-zero moments, step 2)
        for _ in range(2):
            for prm in (gm._xyz, gm._features_dc, gm._features_rest, gm._opacity, gm._scaling, gm._rotation):
                prm.grad = torch.randn(prm.shape, generator=g) * 0.01
            gm.optimizer.step()
            gm.optimizer.zero_grad(set_to_none=True)
        # densification statistics: per-row gradient norms around the threshold,
        # some never-visible rows (denom 0 -> NaN -> 0)
        denom = torch.randint(0, 6, (P, 1), generator=g).float()
        gm.denom = denom
        gm.xyz_gradient_accum = denom * torch.exp(math.log(2e-4) + 1.5 * torch.randn(P, 1, generator=g))
        gm.max_radii2D = torch.randint(0, 40, (P,), generator=g).float()
        snapshot(gm, "before", out)
        params = dict(max_grad=2e-4, min_opacity=0.1, extent=1.0, max_screen_size=20)
        gm.densify_and_prune(params["max_grad"], params["min_opacity"], params["extent"],
                             params["max_screen_size"])
        out["z"] = Z_DRAWS[0].numpy() if Z_DRAWS else np.zeros((0, 3), np.float32)
        snapshot(gm, "after", out)
        for k, v in params.items():
            out["param_" + k] = np.array(v)
        out["param_percent_dense"] = np.array(0.01)
        # reset_opacity_nonvisible with two filters, then a standalone prune, then reset_opacity
        P2 = gm.get_xyz.shape[0]
        f1 = torch.rand(P2, generator=g) < 0.3
        f2 = torch.rand(P2, generator=g) < 0.2
        out["reset_filter1"], out["reset_filter2"] = f1.numpy(), f2.numpy()
        gm.reset_opacity_nonvisible([f1, f2])
        snapshot(gm, "reset", out)
        pm = torch.rand(P2, generator=g) < 0.25
        out["prune_mask"] = pm.numpy()
        gm.xyz_gradient_accum = torch.rand(P2, 1, generator=g)
        gm.denom = torch.rand(P2, 1, generator=g)
        gm.max_radii2D = torch.rand(P2, generator=g)
        snapshot(gm, "preprune", out)
        gm.prune_points(pm)
        snapshot(gm, "pruned", out)
        gm.reset_opacity()
        snapshot(gm, "reset_all", out)
    n_sel = out["z"].shape[0] // 2
    print(f"ref_densify.npz: P {P} -> {out['after_xyz'].shape[0]} (split selected {n_sel}) -> prune "
          f"{out['pruned_xyz'].shape[0]}")
    np.savez_compressed(os.path.join(HERE, "ref_densify.npz"), **out)


if __name__ == "__main__":
    main()
