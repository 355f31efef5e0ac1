"""ORACLE (test infrastructure only) - ctypes front-end of the fp32 CPU
restatement in ``oracle/cpu_raster.cpp``.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may use this; the product never does.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libcpu_raster.so")
_lib = None

_f = ctypes.POINTER(ctypes.c_float)
_i = ctypes.POINTER(ctypes.c_int)


def build(force: bool = False) -> str:
    if force or not os.path.exists(_LIB_PATH):
        subprocess.check_call(["make", "-s", "-C", _HERE])
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(_LIB_PATH)
        L.cr_forward.restype = ctypes.c_void_p
        L.cr_forward.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, _f, _f, _f, _f, _f, _f,
                                 ctypes.c_float, _f, _f, _f, _f, ctypes.c_float, ctypes.c_float,
                                 ctypes.c_int, ctypes.c_int, _f, _f, _f, _f, _f, _i, _i,
                                 ctypes.POINTER(ctypes.c_longlong), _i, _i]
        L.cr_backward.restype = None
        L.cr_backward.argtypes = [ctypes.c_void_p] + [_f] * 11
        L.cr_free.restype = None
        L.cr_free.argtypes = [ctypes.c_void_p]
        L.cr_distknn.restype = None
        L.cr_distknn.argtypes = [ctypes.c_int, _f, _f]
        _lib = L
    return _lib


def _p(a):
    if a is None:
        return None
    return a.ctypes.data_as(_f)


def _np(x, dtype=np.float32):
    if x is None:
        return None
    if hasattr(x, "detach"):
        x = x.detach().cpu().numpy()
    x = np.ascontiguousarray(x, dtype=dtype)
    return x if x.size > 0 else None


class CpuRaster:
    """Forward on construction, ``backward()`` on demand; frees on close."""

    def __init__(self, *, means3D, opacities, shs=None, colors_precomp=None, scales=None,
                 rotations=None, cov3D_precomp=None, H, W, tanfovx, tanfovy, bg,
                 scale_modifier, viewmatrix, projmatrix, projmatrix_raw, sh_degree, campos):
        L = lib()
        self._keep = [_np(means3D), _np(opacities), _np(shs), _np(colors_precomp), _np(scales),
                      _np(rotations), _np(cov3D_precomp), _np(bg), _np(viewmatrix),
                      _np(projmatrix), _np(projmatrix_raw), _np(campos)]
        (m, o, sh, col, sc, rot, cov, bgn, vm, pm, pr, cp) = self._keep
        P = m.shape[0]
        M = sh.shape[1] if sh is not None and sh.ndim == 3 else (0 if sh is None else sh.shape[1])
        self.P, self.M, self.H, self.W = P, M, H, W
        self.color = np.zeros((3, H, W), np.float32)
        self.depth = np.zeros((1, H, W), np.float32)
        self.opacity = np.zeros((1, H, W), np.float32)
        self.radii = np.zeros(P, np.int32)
        self.n_touched = np.zeros(P, np.int32)
        # blends whose T > 0.5 decision is clear (firm) or within rounding
        # slack of a threshold (soft), cpu_raster.cpp: any correct count lies
        # in [firm, firm + soft] and equals n_touched where soft == 0
        self.n_touched_firm = np.zeros(P, np.int32)
        self.n_touched_soft = np.zeros(P, np.int32)
        nr = ctypes.c_longlong(0)
        self._h = L.cr_forward(P, int(sh_degree), M, _p(bgn), _p(m), _p(col), _p(o), _p(sc), _p(rot),
                               float(scale_modifier), _p(cov), _p(vm), _p(pm), _p(pr), float(tanfovx),
                               float(tanfovy), int(H), int(W), _p(sh), _p(cp), _p(self.color),
                               _p(self.depth), _p(self.opacity),
                               self.radii.ctypes.data_as(_i), self.n_touched.ctypes.data_as(_i),
                               ctypes.byref(nr), self.n_touched_firm.ctypes.data_as(_i),
                               self.n_touched_soft.ctypes.data_as(_i))
        self.num_rendered = int(nr.value)

    def backward(self, dL_dcolor, dL_ddepth):
        P, M = self.P, self.M
        gc, gd = _np(dL_dcolor), _np(dL_ddepth)
        out = dict(
            dL_dmeans2D=np.zeros((P, 3), np.float32), dL_dcolors=np.zeros((P, 3), np.float32),
            dL_dopacity=np.zeros((P, 1), np.float32), dL_dmeans3D=np.zeros((P, 3), np.float32),
            dL_dcov3D=np.zeros((P, 6), np.float32), dL_dsh=np.zeros((P, max(M, 1), 3), np.float32),
            dL_dscales=np.zeros((P, 3), np.float32), dL_drotations=np.zeros((P, 4), np.float32),
            dL_dtau=np.zeros((P, 6), np.float32))
        lib().cr_backward(self._h, _p(gc), _p(gd), _p(out["dL_dmeans2D"]), _p(out["dL_dcolors"]),
                          _p(out["dL_dopacity"]), _p(out["dL_dmeans3D"]), _p(out["dL_dcov3D"]),
                          _p(out["dL_dsh"]) if M > 0 else None, _p(out["dL_dscales"]),
                          _p(out["dL_drotations"]), _p(out["dL_dtau"]))
        return out

    def close(self):
        if self._h:
            lib().cr_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def dist_knn(points) -> np.ndarray:
    pts = _np(points)
    P = 0 if pts is None else pts.shape[0]
    out = np.zeros(P, np.float32)
    if P:
        lib().cr_distknn(P, _p(pts), _p(out))
    return out
