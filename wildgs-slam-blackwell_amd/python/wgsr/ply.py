"""Gaussian scenes as PLY files.

``save_ply`` / ``load_ply`` mirror GaussianModel.save_ply / load_ply
(thirdparty/gaussian_splatting/scene/gaussian_model.py:338-493), which use
plyfile 0.8.1 (requirements.txt:14; absent from this image):

* file = ASCII header (``ply`` / ``format binary_little_endian 1.0`` /
  ``element vertex P`` / one ``property float <name>`` per attribute /
  ``end_header``, newline-terminated) + P packed little-endian float32
  records in ``construct_list_of_attributes`` order (:338-350): x y z,
  nx ny nz (zeros), f_dc_* and f_rest_* channel-major (the tensors'
  ``transpose(1, 2).flatten(1)``), opacity, scale_*, rot_*.
* loading reads the first element, orders f_rest_* / scale_* / rot* by
  their numeric suffix (:417-455) and rebuilds the tensors exactly as
  :456-489 do (features_dc [P, 1, 3], features_rest [P, K, 3]).

The records are assembled and taken apart on the device
(``wgsr_ply_pack`` / ``wgsr_ply_unpack``, an LDS transpose); the host moves
one contiguous block between the file and HBM.  Binary little- or big-endian
files with any fixed-size scalar property types load (non-float32 columns
are converted to float32 on the host first, as the reference's float64 ->
float32 path rounds them); ASCII PLY is refused.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

from . import _lib

_PLY_TYPES = {
    "char": "i1", "int8": "i1", "uchar": "u1", "uint8": "u1", "short": "i2", "int16": "i2",
    "ushort": "u2", "uint16": "u2", "int": "i4", "int32": "i4", "uint": "u4", "uint32": "u4",
    "float": "f4", "float32": "f4", "double": "f8", "float64": "f8",
}


def attribute_names(n_dc: int = 3, n_rest: int = 45, n_scale: int = 3, n_rot: int = 4):
    """construct_list_of_attributes (gaussian_model.py:338-350)."""
    return (["x", "y", "z", "nx", "ny", "nz"] + [f"f_dc_{i}" for i in range(n_dc)]
            + [f"f_rest_{i}" for i in range(n_rest)] + ["opacity"]
            + [f"scale_{i}" for i in range(n_scale)] + [f"rot_{i}" for i in range(n_rot)])


def header_bytes(names, P: int) -> bytes:
    lines = ["ply", "format binary_little_endian 1.0", f"element vertex {P}"]
    lines += [f"property float {n}" for n in names]
    lines.append("end_header")
    return ("\n".join(lines) + "\n").encode("ascii")


def _sh_cols(t: torch.Tensor, first: int):
    """Record columns of a [P, K, 3] SH tensor (storage k*3 + c) written
    channel-major: column first + c*K + k (``transpose(1, 2).flatten(1)``)."""
    K, C = t.shape[1], t.shape[2]
    return [first + c * K + k for k in range(K) for c in range(C)]


def _column_sets(tensors, cols):
    keep = []  # ctypes arrays must outlive the call
    sets = []
    for t, c in zip(tensors, cols):
        arr = (ctypes.c_int * len(c))(*c)
        keep.append(arr)
        sets.append(_lib.PlyColumnSet(t.data_ptr(), len(c), arr))
    return (_lib.PlyColumnSet * len(sets))(*sets), keep


def _check_device(ts, who):
    for t in ts:
        if not t.is_cuda or t.dtype != torch.float32:
            raise RuntimeError(f"{who}: fp32 device tensors only (the HIP path has no CPU fallback)")


@torch.no_grad()
def save_ply(path: str, xyz, features_dc, features_rest, opacity, scaling, rotation) -> None:
    """GaussianModel.save_ply for tensors as the model holds them:
    xyz [P,3], features_dc [P,1,3], features_rest [P,K,3], opacity [P,1],
    scaling [P,S], rotation [P,R]."""
    ts = [t.detach().contiguous() for t in (xyz, features_dc, features_rest, opacity, scaling, rotation)]
    _check_device(ts, "save_ply")
    xyz, f_dc, f_rest, op, sc, rot = ts
    P = xyz.shape[0]
    n_dc, n_rest = f_dc.shape[1] * f_dc.shape[2], f_rest.shape[1] * f_rest.shape[2]
    names = attribute_names(n_dc, n_rest, sc.shape[1], rot.shape[1])
    ncol = len(names)
    if ncol > _lib.PLY_MAX_COLS:
        raise ValueError(f"save_ply: {ncol} properties exceed {_lib.PLY_MAX_COLS}")
    o_dc = 6
    o_rest = o_dc + n_dc
    o_op = o_rest + n_rest
    o_sc = o_op + 1
    o_rot = o_sc + sc.shape[1]
    cols = [[0, 1, 2], _sh_cols(f_dc, o_dc), _sh_cols(f_rest, o_rest), [o_op],
            list(range(o_sc, o_sc + sc.shape[1])), list(range(o_rot, o_rot + rot.shape[1]))]
    dev = xyz.device
    records = torch.empty((P, ncol), dtype=torch.float32, device=dev)
    if P > 0:
        live = [(t, c) for t, c in zip(ts, cols) if len(c) > 0]  # SH degree 0: no f_rest columns
        sets, _keep = _column_sets([t for t, _ in live], [c for _, c in live])
        L = _lib.load()
        with torch.cuda.device(dev):
            _lib.check(L.wgsr_ply_pack(sets, len(live), P, ncol, records.data_ptr(), _lib.stream_handle(dev)))
    host = torch.empty((P, ncol), dtype=torch.float32, pin_memory=True)
    host.copy_(records)  # synchronous D2H
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    with open(path, "wb") as f:
        f.write(header_bytes(names, P))
        if P > 0:
            f.write(memoryview(host.numpy()).cast("B"))


def read_header(f):
    """Parse a PLY header; returns (format, [(element, count, [(name, dtype)])], body offset)."""
    first = f.readline()
    if first.strip() != b"ply":
        raise ValueError("load_ply: not a PLY file")
    fmt, elements = None, []
    while True:
        line = f.readline()
        if not line:
            raise ValueError("load_ply: header has no end_header")
        words = line.decode("ascii").split()
        if not words or words[0] in ("comment", "obj_info"):
            continue
        if words[0] == "format":
            fmt = words[1]
        elif words[0] == "element":
            elements.append((words[1], int(words[2]), []))
        elif words[0] == "property":
            if words[1] == "list":
                raise ValueError(f"load_ply: list property '{words[-1]}' is not a Gaussian attribute")
            if words[1] not in _PLY_TYPES:
                raise ValueError(f"load_ply: unknown property type '{words[1]}'")
            elements[-1][2].append((words[2], _PLY_TYPES[words[1]]))
        elif words[0] == "end_header":
            return fmt, elements, f.tell()


def _suffix_sorted(names, prefix):
    sel = [n for n in names if n.startswith(prefix)]
    return sorted(sel, key=lambda x: int(x.split("_")[-1]))


@torch.no_grad()
def load_ply(path: str, max_sh_degree: int | None = None, device="cuda"):
    """GaussianModel.load_ply: returns dict(xyz, features_dc, features_rest,
    opacity, scaling, rotation, normals) as fp32 device tensors."""
    dev = torch.device(device)
    if dev.type != "cuda":
        raise RuntimeError("load_ply: device tensors only (the HIP path has no CPU fallback)")
    with open(path, "rb") as f:
        fmt, elements, offset = read_header(f)
    if fmt not in ("binary_little_endian", "binary_big_endian"):
        raise NotImplementedError(f"load_ply: '{fmt}' PLY is not supported (binary only)")
    name, P, props = elements[0]  # the reference reads plydata.elements[0]
    names = [n for n, _ in props]
    ncol = len(names)
    if ncol > _lib.PLY_MAX_COLS:
        raise ValueError(f"load_ply: {ncol} properties exceed {_lib.PLY_MAX_COLS}")
    end = "<" if fmt == "binary_little_endian" else ">"
    if all(t == "f4" for _, t in props) and end == "<":
        body = np.fromfile(path, dtype="<f4", count=P * ncol, offset=offset)
        if body.size != P * ncol:
            raise ValueError("load_ply: file shorter than its header says")
        body = body.reshape(P, ncol)
    else:
        rec = np.fromfile(path, dtype=np.dtype([(n, end + t) for n, t in props]), count=P, offset=offset)
        if rec.shape[0] != P:
            raise ValueError("load_ply: file shorter than its header says")
        body = np.empty((P, ncol), np.float32)
        for j, n in enumerate(names):
            body[:, j] = rec[n].astype(np.float64).astype(np.float32)
    col = {n: j for j, n in enumerate(names)}
    for req in ("x", "y", "z", "opacity", "f_dc_0", "f_dc_1", "f_dc_2"):
        if req not in col:
            raise KeyError(f"load_ply: property '{req}' missing")
    rest = _suffix_sorted(names, "f_rest_")
    if max_sh_degree is not None:
        assert len(rest) == 3 * (max_sh_degree + 1) ** 2 - 3
    K = len(rest) // 3
    scales = _suffix_sorted(names, "scale_")
    rots = _suffix_sorted(names, "rot")
    records = torch.from_numpy(body).to(dev)
    out = {
        "xyz": torch.empty((P, 3), device=dev),
        "features_dc": torch.empty((P, 1, 3), device=dev),
        "features_rest": torch.empty((P, K, 3), device=dev),
        "opacity": torch.empty((P, 1), device=dev),
        "scaling": torch.empty((P, len(scales)), device=dev),
        "rotation": torch.empty((P, len(rots)), device=dev),
    }
    # features_rest[p, k, c] = f_rest_{c*K + k} (gaussian_model.py:427-436, 466-471)
    cols = [[col["x"], col["y"], col["z"]], [col[f"f_dc_{c}"] for c in range(3)],
            [col[rest[c * K + k]] for k in range(K) for c in range(3)], [col["opacity"]],
            [col[n] for n in scales], [col[n] for n in rots]]
    tensors = list(out.values())
    if all(n in col for n in ("nx", "ny", "nz")):
        out["normals"] = torch.empty((P, 3), device=dev)
        tensors.append(out["normals"])
        cols.append([col["nx"], col["ny"], col["nz"]])
    if P > 0:
        live = [(t, c) for t, c in zip(tensors, cols) if len(c) > 0]
        sets, _keep = _column_sets([t for t, _ in live], [c for _, c in live])
        L = _lib.load()
        with torch.cuda.device(dev):
            _lib.check(L.wgsr_ply_unpack(records.data_ptr(), P, ncol, sets, len(live), _lib.stream_handle(dev)))
    return out
