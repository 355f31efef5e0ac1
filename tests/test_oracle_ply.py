"""CPU: the PLY oracle's round trip (oracle/ply.py) and the host-side header
handling of wgsr.ply (no GPU)."""
import io

import numpy as np
import pytest

from oracle import ply as oply


def _scene(P, K=15, seed=0):
    r = np.random.default_rng(seed)
    f = lambda *s: r.standard_normal(s).astype(np.float32)
    return f(P, 3), f(P, 1, 3), f(P, K, 3), f(P, 1), f(P, 3), f(P, 4)


def test_oracle_round_trip_and_layout():
    xyz, dc, rest, op, sc, rot = _scene(37)
    data = oply.save_ply_bytes(xyz, dc, rest, op, sc, rot)
    assert data.startswith(b"ply\nformat binary_little_endian 1.0\nelement vertex 37\nproperty float x\n")
    el = oply.read_first_element(data)
    assert len(data) - data.index(b"end_header\n") - 11 == 37 * 62 * 4
    # channel-major SH columns: f_rest_{c*15 + k} = rest[p, k, c]
    assert el["f_rest_16"][5] == rest[5, 1, 1] and el["f_dc_2"][3] == dc[3, 0, 2]
    assert (el["nx"] == 0).all()
    back = oply.load_ply_arrays(el, 3)
    for k, v in zip(("xyz", "features_dc", "features_rest", "opacity", "scaling", "rotation"),
                    (xyz, dc, rest, op, sc, rot)):
        assert np.array_equal(back[k], v), k


def test_wgsr_header_matches_oracle_header():
    from wgsr import ply
    xyz, dc, rest, op, sc, rot = _scene(5)
    data = oply.save_ply_bytes(xyz, dc, rest, op, sc, rot)
    hdr = ply.header_bytes(ply.attribute_names(), 5)
    assert data[:len(hdr)] == hdr
    fmt, elements, off = ply.read_header(io.BytesIO(data))
    assert fmt == "binary_little_endian" and off == len(hdr)
    assert elements[0][0] == "vertex" and elements[0][1] == 5 and len(elements[0][2]) == 62


def test_wgsr_ply_refuses_cpu_and_ascii(tmp_path):
    import torch
    from wgsr import ply
    t = torch.zeros(2, 3)
    with pytest.raises(RuntimeError):
        ply.save_ply(str(tmp_path / "a.ply"), t, torch.zeros(2, 1, 3), torch.zeros(2, 15, 3), torch.zeros(2, 1), t,
                     torch.zeros(2, 4))
    p = tmp_path / "b.ply"
    p.write_bytes(b"ply\nformat ascii 1.0\nelement vertex 0\nproperty float x\nend_header\n")
    with pytest.raises(RuntimeError):
        ply.load_ply(str(p), device="cpu")
