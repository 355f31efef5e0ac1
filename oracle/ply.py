"""ORACLE (test infrastructure only) - GaussianModel.save_ply / load_ply
(thirdparty/gaussian_splatting/scene/gaussian_model.py:338-493) restated in
numpy, with plyfile 0.8.1's binary writer (requirements.txt:14) restated for
the file bytes.  Only ``tests/`` may import this module, as the checker.

plyfile is absent from this image and the reference ships no .ply file, so
the byte layout is pinned to plyfile 0.8.1's published format (header lines
"ply", "format binary_little_endian 1.0", "element vertex N", "property
float <name>"..., "end_header", joined by newlines; body = the structured
array's bytes) rather than to a reference-produced file: parity with
plyfile's own output is unpinned beyond that specification.
"""
from __future__ import annotations

import numpy as np


def construct_list_of_attributes(n_dc, n_rest, n_scale, n_rot):
    """gaussian_model.py:338-350."""
    l = ["x", "y", "z", "nx", "ny", "nz"]
    l += ["f_dc_{}".format(i) for i in range(n_dc)]
    l += ["f_rest_{}".format(i) for i in range(n_rest)]
    l.append("opacity")
    l += ["scale_{}".format(i) for i in range(n_scale)]
    l += ["rot_{}".format(i) for i in range(n_rot)]
    return l


def save_ply_bytes(xyz, f_dc, f_rest, opacity, scale, rotation) -> bytes:
    """gaussian_model.py:352-387 with numpy inputs shaped like the model's
    tensors (f_dc [P,1,3], f_rest [P,K,3]); returns the file's bytes."""
    P = xyz.shape[0]
    normals = np.zeros_like(xyz)
    # torch's transpose(1, 2).flatten(start_dim=1) (well defined for P = 0 too)
    fdc = np.ascontiguousarray(np.transpose(f_dc, (0, 2, 1))).reshape(P, f_dc.shape[1] * f_dc.shape[2])
    frest = np.ascontiguousarray(np.transpose(f_rest, (0, 2, 1))).reshape(P, f_rest.shape[1] * f_rest.shape[2])
    names = construct_list_of_attributes(fdc.shape[1], frest.shape[1], scale.shape[1], rotation.shape[1])
    dtype_full = [(a, "f4") for a in names]
    elements = np.empty(P, dtype=dtype_full)
    attributes = np.concatenate((xyz, normals, fdc, frest, opacity, scale, rotation), axis=1)
    elements[:] = list(map(tuple, attributes))
    header = ["ply", "format binary_little_endian 1.0", f"element vertex {P}"]
    header += [f"property float {n}" for n in names] + ["end_header"]
    return ("\n".join(header) + "\n").encode("ascii") + elements.tobytes()


def load_ply_arrays(elements: np.ndarray, max_sh_degree: int):
    """gaussian_model.py:404-489 on the first element's structured array:
    the float32 arrays the reference turns into its parameters."""
    names = list(elements.dtype.names)
    xyz = np.stack((np.asarray(elements["x"]), np.asarray(elements["y"]), np.asarray(elements["z"])), axis=1)
    opacities = np.asarray(elements["opacity"])[..., np.newaxis]
    features_dc = np.zeros((xyz.shape[0], 3, 1))
    for c in range(3):
        features_dc[:, c, 0] = np.asarray(elements[f"f_dc_{c}"])
    extra = sorted([n for n in names if n.startswith("f_rest_")], key=lambda x: int(x.split("_")[-1]))
    assert len(extra) == 3 * (max_sh_degree + 1) ** 2 - 3
    features_extra = np.zeros((xyz.shape[0], len(extra)))
    for i, n in enumerate(extra):
        features_extra[:, i] = np.asarray(elements[n])
    features_extra = features_extra.reshape((features_extra.shape[0], 3, (max_sh_degree + 1) ** 2 - 1))
    scale_names = sorted([n for n in names if n.startswith("scale_")], key=lambda x: int(x.split("_")[-1]))
    scales = np.zeros((xyz.shape[0], len(scale_names)))
    for i, n in enumerate(scale_names):
        scales[:, i] = np.asarray(elements[n])
    rot_names = sorted([n for n in names if n.startswith("rot")], key=lambda x: int(x.split("_")[-1]))
    rots = np.zeros((xyz.shape[0], len(rot_names)))
    for i, n in enumerate(rot_names):
        rots[:, i] = np.asarray(elements[n])
    f32 = lambda a: np.asarray(a, np.float64).astype(np.float32)  # torch.tensor(..., dtype=torch.float)
    return {
        "xyz": f32(xyz),
        "features_dc": np.ascontiguousarray(np.transpose(f32(features_dc), (0, 2, 1))),
        "features_rest": np.ascontiguousarray(np.transpose(f32(features_extra), (0, 2, 1))),
        "opacity": f32(opacities),
        "scaling": f32(scales),
        "rotation": f32(rots),
    }


def read_first_element(data: bytes):
    """Minimal binary PLY reader (fixed-size scalar properties) for tests."""
    types = {"float": "f4", "double": "f8", "uchar": "u1", "int": "i4", "short": "i2", "ushort": "u2",
             "char": "i1", "uint": "u4", "float32": "f4", "float64": "f8", "uint8": "u1", "int32": "i4"}
    end = data.index(b"end_header\n") + len(b"end_header\n")
    lines = data[:end].decode("ascii").split("\n")
    fmt = [l.split()[1] for l in lines if l.startswith("format")][0]
    bo = "<" if fmt == "binary_little_endian" else ">"
    props, count, seen = [], None, False
    for l in lines:
        w = l.split()
        if not w:
            continue
        if w[0] == "element":
            if seen:
                break
            seen, count = True, int(w[2])
        elif w[0] == "property" and seen:
            props.append((w[2], bo + types[w[1]]))
    return np.frombuffer(data, dtype=np.dtype(props), count=count, offset=end)
