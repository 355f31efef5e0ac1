"""GPU parity for SURVEY.md 8(f) row f3: wgsr.ply (device pack / unpack)
against the PLY oracle (oracle/ply.py, the reference's save_ply / load_ply
restated).  Bar: bit-exact file bytes and bit-exact loaded tensors."""
import numpy as np
import pytest
import torch

from oracle import ply as oply

pytestmark = pytest.mark.gpu
DEV = "cuda"
KEYS = ("xyz", "features_dc", "features_rest", "opacity", "scaling", "rotation")


def _scene(P, K, seed):
    r = np.random.default_rng(seed)
    f = lambda *s: r.standard_normal(s).astype(np.float32)
    return f(P, 3), f(P, 1, 3), f(P, K, 3), f(P, 1), f(P, 3), f(P, 4)


@pytest.mark.parametrize("P,K", [(0, 15), (1, 15), (63, 15), (65, 3), (1000, 0), (100_003, 15)])
def test_save_bytes_and_load_match_reference(tmp_path, P, K):
    from wgsr import ply
    arrs = _scene(P, K, seed=P + K)
    path = str(tmp_path / "sub" / "point_cloud.ply")
    ply.save_ply(path, *[torch.from_numpy(a).to(DEV) for a in arrs])
    data = open(path, "rb").read()
    assert data == oply.save_ply_bytes(*arrs)
    sh = {15: 3, 3: 1, 0: 0}[K]
    got = ply.load_ply(path, max_sh_degree=sh)
    exp = oply.load_ply_arrays(oply.read_first_element(data), sh)
    for k in KEYS:
        assert got[k].shape == exp[k].shape, k
        assert np.array_equal(got[k].cpu().numpy(), exp[k]), k
    assert (got["normals"] == 0).all()


def test_load_any_property_order_types_and_byte_order(tmp_path):
    """plyfile reads properties by name: shuffled order, double / uchar
    columns, extra properties and big-endian bodies load the same tensors."""
    from wgsr import ply
    P = 777
    arrs = _scene(P, 15, seed=3)
    base = oply.read_first_element(oply.save_ply_bytes(*arrs))
    names = list(base.dtype.names) + ["red"]
    rng = np.random.default_rng(0)
    rng.shuffle(names)
    for bo, fmt in (("<", "binary_little_endian"), (">", "binary_big_endian")):
        types = {n: ("f8" if n.startswith("scale") else "u1" if n == "red" else "f4") for n in names}
        dt = np.dtype([(n, bo + types[n]) for n in names])
        rec = np.empty(P, dt)
        for n in names:
            rec[n] = 7 if n == "red" else base[n]
        ptype = {"f4": "float", "f8": "double", "u1": "uchar"}
        hdr = ["ply", f"format {fmt} 1.0", "comment made by the test", f"element vertex {P}"]
        hdr += [f"property {ptype[types[n]]} {n}" for n in names] + ["end_header"]
        data = ("\n".join(hdr) + "\n").encode() + rec.tobytes()
        path = tmp_path / f"shuffled_{fmt}.ply"
        path.write_bytes(data)
        got = ply.load_ply(str(path), max_sh_degree=3)
        exp = oply.load_ply_arrays(oply.read_first_element(data), 3)
        for k in KEYS:
            assert np.array_equal(got[k].cpu().numpy(), exp[k]), (fmt, k)


def test_one_million_round_trip_bit_exact(tmp_path):
    from wgsr import ply
    g = torch.Generator(device="cpu").manual_seed(1)
    P = 1_000_000
    ts = [torch.randn(s, generator=g).to(DEV) for s in ((P, 3), (P, 1, 3), (P, 15, 3), (P, 1), (P, 3), (P, 4))]
    path = str(tmp_path / "big.ply")
    ply.save_ply(path, *ts)
    got = ply.load_ply(path, max_sh_degree=3)
    for k, t in zip(KEYS, ts):
        assert torch.equal(got[k], t), k
