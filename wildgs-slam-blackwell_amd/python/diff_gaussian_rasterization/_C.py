"""``diff_gaussian_rasterization._C`` on MI355X.

Same three functions, argument order and return tuples as the upstream
pybind module (rasterize_points.cu of the diff-gaussian-rasterization-w-pose
submodule, absent from the reference snapshot: .gitmodules:7-9; contract in
SURVEY.md 8(b)), implemented by calls into libwgsr.so's C ABI
(include/wgsr.h).  Tensors must be float32 (int32 radii) on one HIP device.

When the compiled host wrapper ``_native`` (csrc_py/wgsr_torch.cpp, built
in-tree by ``make``) is present, each function hands its arguments to it:
the same checks, messages, allocations and C-ABI calls without the Python
per-call cost.  The bodies below are the reference for that module and the
path taken without it (WGSR_NATIVE_WRAPPER=0 forces them).  Both drive the
libwgsr.so that ``wgsr._lib`` loaded.
"""
from __future__ import annotations

import ctypes
import os

import torch

from wgsr import _lib

try:
    from . import _native as _native_module
except ImportError:  # not built: the ctypes bodies below
    _native_module = None

NUM_CHANNELS = 3
_NATIVE = None  # the bound _native module, False when absent or disabled


def _native():
    global _NATIVE
    if _NATIVE is None:
        n = _native_module if os.environ.get("WGSR_NATIVE_WRAPPER", "1") != "0" else None
        if n is not None:
            L = _lib.load()
            addr = lambda f: ctypes.cast(f, ctypes.c_void_p).value  # noqa: E731
            n.bind(addr(L.wgsr_rasterize_forward), addr(L.wgsr_rasterize_backward), addr(L.wgsr_mark_visible),
                   addr(L.wgsr_last_error))
        _NATIVE = n if n is not None else False
    return _NATIVE


def use_native(on: bool) -> bool:
    """Select the compiled wrapper (True, when built) or the ctypes bodies
    (False); returns whether the compiled one is now in use."""
    global _NATIVE
    os.environ["WGSR_NATIVE_WRAPPER"] = "1" if on else "0"
    _NATIVE = None
    return bool(_native())


def _on(t, dev, dtype, name):
    """Upstream's ``.data<T>()`` raises on a dtype mismatch; a raw pointer
    would not.  Reject anything that is not ``dtype`` on the HIP device
    ``dev`` (a host pointer reaching a kernel faults the GPU)."""
    if t.dtype != dtype:
        raise RuntimeError(f"{name}: expected {dtype}, got {t.dtype}")
    if t.device != dev or t.device.type != "cuda":
        raise RuntimeError(f"{name}: expected a tensor on {dev}, got {t.device}")
    return t.contiguous()


def _f32(t, dev, name):
    if t is None or t.numel() == 0:
        return None
    return _on(t, dev, torch.float32, name)


def _args(P, D, M, W, H, bg, means3D, colors, opacity, scales, rotations, cov3D_precomp, sh,
          viewmatrix, projmatrix, projmatrix_raw, campos, scale_modifier, tan_fovx, tan_fovy,
          prefiltered, debug, keep):
    p = _lib.ptr
    tensors = [bg, means3D, colors, opacity, scales, rotations, cov3D_precomp, sh, viewmatrix,
               projmatrix, projmatrix_raw, campos]
    keep.extend(t for t in tensors if t is not None)
    return _lib.RasterArgs(
        P=P, D=D, M=M, W=W, H=H, bg=p(bg), means3D=p(means3D), colors=p(colors),
        opacities=p(opacity), scales=p(scales), rotations=p(rotations),
        cov3D_precomp=p(cov3D_precomp), shs=p(sh), viewmatrix=p(viewmatrix),
        projmatrix=p(projmatrix), projmatrix_raw=p(projmatrix_raw), campos=p(campos),
        scale_modifier=float(scale_modifier), tan_fovx=float(tan_fovx), tan_fovy=float(tan_fovy),
        prefiltered=int(bool(prefiltered)), debug=int(bool(debug)))


def rasterize_gaussians(background, means3D, colors, opacity, scales, rotations, scale_modifier,
                        cov3D_precomp, viewmatrix, projmatrix, projmatrix_raw, tan_fovx, tan_fovy,
                        image_height, image_width, sh, degree, campos, prefiltered, debug):
    """-> (num_rendered, color[3,H,W], radii[P] int32, geomBuffer, binningBuffer,
    imgBuffer, depth[1,H,W], opacity[1,H,W], n_touched[P] int32)."""
    n = _native()
    if n:
        return n.rasterize_gaussians(background, means3D, colors, opacity, scales, rotations, scale_modifier,
                                     cov3D_precomp, viewmatrix, projmatrix, projmatrix_raw, tan_fovx, tan_fovy,
                                     image_height, image_width, sh, degree, campos, prefiltered, debug)
    if means3D.ndimension() != 2 or means3D.size(1) != 3:
        raise RuntimeError("means3D must have dimensions (num_points, 3)")
    L = _lib.load()
    dev = means3D.device
    P = means3D.size(0)
    H, W = int(image_height), int(image_width)
    fopts = dict(dtype=torch.float32, device=dev)
    out_color = torch.empty(NUM_CHANNELS, H, W, **fopts)
    out_depth = torch.empty(1, H, W, **fopts)
    out_opacity = torch.empty(1, H, W, **fopts)
    radii = torch.empty(P, dtype=torch.int32, device=dev)
    n_touched = torch.empty(P, dtype=torch.int32, device=dev)
    if dev.type != "cuda":
        raise RuntimeError(f"means3D: expected a HIP device tensor, got {dev}")
    shc = _f32(sh, dev, "sh")
    M = shc.size(1) if shc is not None else 0
    keep = []
    a = _args(P, int(degree), M, W, H, _f32(background, dev, "bg"), _f32(means3D, dev, "means3D"),
              _f32(colors, dev, "colors"), _f32(opacity, dev, "opacity"), _f32(scales, dev, "scales"),
              _f32(rotations, dev, "rotations"), _f32(cov3D_precomp, dev, "cov3D_precomp"), shc,
              _f32(viewmatrix, dev, "viewmatrix"), _f32(projmatrix, dev, "projmatrix"),
              _f32(projmatrix_raw, dev, "projmatrix_raw"), _f32(campos, dev, "campos"), scale_modifier,
              tan_fovx, tan_fovy, prefiltered, debug, keep)
    nr = ctypes.c_int64(0)
    with torch.cuda.device(dev), _lib.AllocRequest(dev) as req:
        code = L.wgsr_rasterize_forward(
            ctypes.byref(a), _lib.ALLOC_GEOM, _lib.ALLOC_BINNING, _lib.ALLOC_IMAGE, None,
            out_color.data_ptr(), out_depth.data_ptr(), out_opacity.data_ptr(),
            radii.data_ptr() if P else None, n_touched.data_ptr() if P else None,
            ctypes.byref(nr), _lib.stream_handle(dev))
    _lib.check(code)
    empty = torch.empty(0, dtype=torch.uint8, device=dev)
    b = req.buffers
    return (int(nr.value), out_color, radii, b.get("geom", empty), b.get("binning", empty),
            b.get("image", empty), out_depth, out_opacity, n_touched)


def rasterize_gaussians_backward(background, means3D, radii, colors, scales, rotations,
                                 scale_modifier, cov3D_precomp, viewmatrix, projmatrix,
                                 projmatrix_raw, tan_fovx, tan_fovy, dL_dout_color, dL_dout_depth,
                                 sh, degree, campos, geomBuffer, R, binningBuffer, imageBuffer,
                                 debug, *, out=None):
    """-> (dL_dmeans2D, dL_dcolors, dL_dopacity, dL_dmeans3D, dL_dcov3D, dL_dsh,
    dL_dscales, dL_drotations, dL_dtau[P,6]).

    ``out`` (extension, keyword-only): dict of preallocated contiguous float32
    tensors for "means3D", "shs", "opacities", "scales", "rotations" (e.g. the
    views of a wgsr.dp.GradBuffer) that the kernels write directly."""
    n = _native()
    if n:
        o = out.get if out is not None else (lambda _k: None)
        return n.rasterize_gaussians_backward(
            background, means3D, radii, colors, scales, rotations, scale_modifier, cov3D_precomp, viewmatrix,
            projmatrix, projmatrix_raw, tan_fovx, tan_fovy, dL_dout_color, dL_dout_depth, sh, degree, campos,
            geomBuffer, R, binningBuffer, imageBuffer, debug, o("means3D"), o("shs"), o("opacities"), o("scales"),
            o("rotations"))
    L = _lib.load()
    dev = means3D.device
    P = means3D.size(0)
    H, W = dL_dout_color.size(1), dL_dout_color.size(2)
    if dev.type != "cuda":
        raise RuntimeError(f"means3D: expected a HIP device tensor, got {dev}")
    shc = _f32(sh, dev, "sh")
    M = shc.size(1) if shc is not None else 0
    fopts = dict(dtype=torch.float32, device=dev)
    dL_dmeans2D = torch.empty(P, 3, **fopts)
    dL_dcolors = torch.empty(P, NUM_CHANNELS, **fopts)
    dL_dopacity = torch.empty(P, 1, **fopts)
    dL_dmeans3D = torch.empty(P, 3, **fopts)
    dL_dcov3D = torch.empty(P, 6, **fopts)
    dL_dsh = torch.zeros(P, M, 3, **fopts) if M == 0 else torch.empty(P, M, 3, **fopts)
    dL_dscales = torch.empty(P, 3, **fopts)
    dL_drotations = torch.empty(P, 4, **fopts)
    if out is not None:
        def take(name, default):
            t = out.get(name)
            if t is None:
                return default
            if (t.shape != default.shape or t.dtype != torch.float32 or not t.is_contiguous()
                    or t.device != dev):
                raise RuntimeError(f"out[{name!r}] must be a contiguous float32 {tuple(default.shape)} on {dev}")
            return t
        dL_dmeans3D = take("means3D", dL_dmeans3D)
        dL_dsh = take("shs", dL_dsh)
        dL_dopacity = take("opacities", dL_dopacity)
        dL_dscales = take("scales", dL_dscales)
        dL_drotations = take("rotations", dL_drotations)
    dL_dtau = torch.empty(P, 6, **fopts)
    if P == 0:
        return (dL_dmeans2D, dL_dcolors, dL_dopacity, dL_dmeans3D, dL_dcov3D, dL_dsh, dL_dscales,
                dL_drotations, dL_dtau)
    keep = []
    means = _f32(means3D, dev, "means3D")
    radii = _on(radii, dev, torch.int32, "radii")
    if radii.numel() != P:
        raise RuntimeError(f"radii: expected {P} entries, got {radii.numel()}")
    for buf, name in ((geomBuffer, "geomBuffer"), (binningBuffer, "binningBuffer"), (imageBuffer, "imageBuffer")):
        if buf.numel():
            _on(buf, dev, torch.uint8, name)
    # the backward does not read opacities (they live in the geometry buffer);
    # any valid device pointer satisfies the argument check
    a = _args(P, int(degree), M, W, H, _f32(background, dev, "bg"), means, _f32(colors, dev, "colors"), means,
              _f32(scales, dev, "scales"), _f32(rotations, dev, "rotations"),
              _f32(cov3D_precomp, dev, "cov3D_precomp"), shc, _f32(viewmatrix, dev, "viewmatrix"),
              _f32(projmatrix, dev, "projmatrix"), _f32(projmatrix_raw, dev, "projmatrix_raw"),
              _f32(campos, dev, "campos"), scale_modifier, tan_fovx, tan_fovy, False, debug, keep)
    gc = _on(dL_dout_color, dev, torch.float32, "dL_dout_color")
    gd = _on(dL_dout_depth, dev, torch.float32, "dL_dout_depth")
    p = _lib.ptr
    with torch.cuda.device(dev), _lib.AllocRequest(dev):
        code = L.wgsr_rasterize_backward(
            ctypes.byref(a), radii.data_ptr(), p(geomBuffer), p(binningBuffer), p(imageBuffer),
            int(R), gc.data_ptr(), gd.data_ptr(), _lib.ALLOC_SCRATCH, None,
            dL_dmeans2D.data_ptr(), dL_dcolors.data_ptr(), dL_dopacity.data_ptr(),
            dL_dmeans3D.data_ptr(), dL_dcov3D.data_ptr(), p(dL_dsh), dL_dscales.data_ptr(),
            dL_drotations.data_ptr(), dL_dtau.data_ptr(), _lib.stream_handle(dev))
    _lib.check(code)
    return (dL_dmeans2D, dL_dcolors, dL_dopacity, dL_dmeans3D, dL_dcov3D, dL_dsh, dL_dscales,
            dL_drotations, dL_dtau)


def mark_visible(means3D, viewmatrix, projmatrix):
    """-> bool[P]: view-space depth > 0.2 (upstream checkFrustum)."""
    n = _native()
    if n:
        return n.mark_visible(means3D, viewmatrix, projmatrix)
    L = _lib.load()
    dev = means3D.device
    P = means3D.size(0)
    if dev.type != "cuda":
        raise RuntimeError(f"means3D: expected a HIP device tensor, got {dev}")
    present = torch.empty(P, dtype=torch.bool, device=dev)
    m = _on(means3D, dev, torch.float32, "means3D")
    v = _on(viewmatrix, dev, torch.float32, "viewmatrix")
    pm = _on(projmatrix, dev, torch.float32, "projmatrix")
    with torch.cuda.device(dev):
        code = L.wgsr_mark_visible(P, m.data_ptr(), v.data_ptr(), pm.data_ptr(),
                                   present.data_ptr() if P else None, _lib.stream_handle(dev))
    _lib.check(code)
    return present
