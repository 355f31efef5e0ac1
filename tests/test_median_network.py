"""The uncertainty loss's 5x5 median (MedianPool2d, mapping_utils.py:306-307)
runs as a 99-comparator selection network (csrc/uncertainty.hip median25).
By the zero-one principle a comparator network selects the median of every
input iff it does so for every input of zeros and ones: all 2^25 of them are
checked here, bit-sliced (each wire a 2^25-bit set, min = AND, max = OR), on
the network parsed from the shipped source."""
import os
import re

import numpy as np

SRC = os.path.join(os.path.dirname(__file__), "..", "wildgs-slam-blackwell_amd", "csrc", "uncertainty.hip")


def _network():
    s = open(SRC).read()
    body = s[s.index("kNet[99][2] = {"):]
    body = body[:body.index("};")]
    pairs = [(int(a), int(b)) for a, b in re.findall(r"\{(\d+), (\d+)\}", body)]
    assert len(pairs) == 99
    return pairs


def test_median25_network_all_zero_one_inputs():
    n = 25
    words = (1 << n) // 64
    idx = np.arange(1 << n, dtype=np.uint32)
    wires = []
    for i in range(n):
        bits = ((idx >> np.uint32(i)) & np.uint32(1)).astype(np.uint8)
        wires.append(np.packbits(bits, bitorder="little").view(np.uint64))
    assert wires[0].size == words
    pc = np.zeros(1 << n, dtype=np.uint8)
    for i in range(n):
        pc += ((idx >> np.uint32(i)) & np.uint32(1)).astype(np.uint8)
    want = np.packbits((pc >= 13).astype(np.uint8), bitorder="little").view(np.uint64)
    del idx, pc
    for a, b in _network():
        lo, hi = wires[a] & wires[b], wires[a] | wires[b]
        wires[a], wires[b] = lo, hi
    assert np.array_equal(wires[12], want)


def test_median25_matches_numpy_on_floats():
    nets = _network()
    rng = np.random.default_rng(0)
    v = rng.normal(size=(20000, 25)).astype(np.float32)
    v[:5000] = np.round(v[:5000])  # many ties
    p = v.copy()
    for a, b in nets:
        lo, hi = np.minimum(p[:, a], p[:, b]), np.maximum(p[:, a], p[:, b])
        p[:, a], p[:, b] = lo, hi
    np.testing.assert_array_equal(p[:, 12], np.sort(v, axis=1)[:, 12])
