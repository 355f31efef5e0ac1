"""The compiled host wrapper (diff_gaussian_rasterization._native,
csrc_py/wgsr_torch.cpp) against the ctypes bodies of _C.py it replaces: the
same libwgsr calls, so every output is bit-identical, the ``out=`` buffers
are written in place, and argument misuse raises the same RuntimeError
messages."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _inputs(P=20_000, W=320, H=240, deg=3, view=1):
    from wgsr.camera import synthetic_camera
    from wgsr.scene import make_scene, make_upstream_grads
    sc = make_scene(P, W, H, deg, seed=3)
    gc, gd = make_upstream_grads(W, H, seed=4)
    f = synthetic_camera(W, H, view).raster_fields()
    d = lambda x: x.to(DEV).contiguous()  # noqa: E731
    e = torch.empty(0, device=DEV)
    fwd = (d(torch.tensor([0.2, 0.3, 0.4])), d(sc.means3D), e, d(sc.opacities), d(sc.scales), d(sc.rotations), 1.0, e,
           d(f["viewmatrix"]), d(f["projmatrix"]), d(f["projmatrix_raw"]), f["tanfovx"], f["tanfovy"], H, W,
           d(sc.shs), deg, d(f["campos"]), False, False)
    return fwd, d(gc), d(gd)


def _run(C, fwd, gc, gd, out=None):
    r = C.rasterize_gaussians(*fwd)
    (bg, means, _, _, scales, rots, sm, _, view, proj, praw, tx, ty, H, W, shs, deg, campos, _, _) = fwd
    e = torch.empty(0, device=DEV)
    kw = {} if out is None else {"out": out}
    g = C.rasterize_gaussians_backward(bg, means, r[2], e, scales, rots, sm, e, view, proj, praw, tx, ty, gc, gd, shs,
                                       deg, campos, r[3], r[0], r[4], r[5], False, **kw)
    vis = C.mark_visible(means, view, proj)
    torch.cuda.synchronize()
    return r, g, vis


def test_native_wrapper_matches_ctypes_bodies():
    from diff_gaussian_rasterization import _C
    fwd, gc, gd = _inputs()
    try:
        assert _C.use_native(True), "the compiled wrapper is not built (make -C wildgs-slam-blackwell_amd)"
        rn, gn, vn = _run(_C, fwd, gc, gd)
        assert not _C.use_native(False)
        rp, gp, vp = _run(_C, fwd, gc, gd)
    finally:
        _C.use_native(True)
    assert rn[0] == rp[0]
    for i, (a, b) in enumerate(zip(rn[1:], rp[1:])):
        assert a.dtype == b.dtype
        if i == 3:  # binningBuffer: the previous forward's predicted size when that was large enough
            assert a.numel() > 0 and b.numel() > 0
            continue
        assert a.shape == b.shape
        if a.dtype != torch.uint8:  # (state buffers: same sizes; their scratch bytes may differ)
            np.testing.assert_array_equal(a.cpu().numpy(), b.cpu().numpy())
    for a, b in zip(gn, gp):
        np.testing.assert_array_equal(a.cpu().numpy(), b.cpu().numpy())
    np.testing.assert_array_equal(vn.cpu().numpy(), vp.cpu().numpy())


def test_native_wrapper_out_buffers_and_errors():
    from diff_gaussian_rasterization import _C
    assert _C.use_native(True)
    fwd, gc, gd = _inputs(P=5_000, deg=1)
    P, M = fwd[1].shape[0], fwd[15].shape[1]
    out = {"means3D": torch.full((P, 3), 7.0, device=DEV), "shs": torch.full((P, M, 3), 7.0, device=DEV),
           "opacities": torch.full((P, 1), 7.0, device=DEV), "scales": torch.full((P, 3), 7.0, device=DEV),
           "rotations": torch.full((P, 4), 7.0, device=DEV)}
    _, g, _ = _run(_C, fwd, gc, gd, out=out)
    _, g2, _ = _run(_C, fwd, gc, gd)
    for k, i in (("means3D", 3), ("shs", 5), ("opacities", 2), ("scales", 6), ("rotations", 7)):
        assert g[i].data_ptr() == out[k].data_ptr()
        np.testing.assert_array_equal(out[k].cpu().numpy(), g2[i].cpu().numpy())
    # the same messages as the ctypes bodies
    msgs = {}
    for native in (True, False):
        _C.use_native(native)
        got = []
        bad = list(fwd)
        bad[4] = fwd[4].double()
        with pytest.raises(RuntimeError) as ei:
            _C.rasterize_gaussians(*bad)
        got.append(str(ei.value))
        bad = list(fwd)
        bad[5] = fwd[5].cpu()
        with pytest.raises(RuntimeError) as ei:
            _C.rasterize_gaussians(*bad)
        got.append(str(ei.value))
        with pytest.raises(RuntimeError) as ei:
            _C.rasterize_gaussians_backward(*_bwd_args(fwd, gc, gd), out={"means3D": torch.zeros(3, device=DEV)})
        got.append(str(ei.value))
        msgs[native] = got
    _C.use_native(True)
    assert msgs[True] == msgs[False], msgs
    assert "scales: expected torch.float32, got torch.float64" in msgs[True][0]
    assert "rotations: expected a tensor on cuda:0, got cpu" in msgs[True][1]
    assert "out['means3D'] must be a contiguous float32" in msgs[True][2]


def _bwd_args(fwd, gc, gd):
    from diff_gaussian_rasterization import _C
    r = _C.rasterize_gaussians(*fwd)
    (bg, means, _, _, scales, rots, sm, _, view, proj, praw, tx, ty, H, W, shs, deg, campos, _, _) = fwd
    e = torch.empty(0, device=DEV)
    return (bg, means, r[2], e, scales, rots, sm, e, view, proj, praw, tx, ty, gc, gd, shs, deg, campos, r[3], r[0],
            r[4], r[5], False)
