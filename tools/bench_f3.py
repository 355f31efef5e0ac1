"""Measure SURVEY.md 8(f) row f3 on the GPU: save_ply / load_ply of a
1M-Gaussian SH3 scene (62 float32 properties per Gaussian, 248 MB body)
through wgsr.ply against the reference's own host path
(gaussian_model.py:352-387 / 404-489: list(map(tuple, ...)) records, per-
column float64 arrays), timed on a 100k-Gaussian sample and scaled.
Files go to $TMPDIR.  Prints one JSON line.
"""
import json
import os
import sys
import tempfile
import time

import numpy as np
import torch

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "wildgs-slam-blackwell_amd", "python"))

from wgsr import ply  # noqa: E402


def ref_save(path, ts):
    """gaussian_model.py:352-387 without plyfile (absent): the same host work."""
    xyz, dc, rest, op, sc, rot = [t.detach().cpu().numpy() for t in ts]
    P = xyz.shape[0]
    fdc = np.ascontiguousarray(dc.transpose(0, 2, 1)).reshape(P, -1)
    frest = np.ascontiguousarray(rest.transpose(0, 2, 1)).reshape(P, -1)
    names = ply.attribute_names(fdc.shape[1], frest.shape[1], sc.shape[1], rot.shape[1])
    el = np.empty(P, dtype=[(n, "f4") for n in names])
    attrs = np.concatenate((xyz, np.zeros_like(xyz), fdc, frest, op, sc, rot), axis=1)
    el[:] = list(map(tuple, attrs))
    with open(path, "wb") as f:
        f.write(ply.header_bytes(names, P))
        f.write(el.tobytes())


def main():
    dev = torch.device("cuda")
    P = 1_000_000
    g = torch.Generator(device="cpu").manual_seed(0)
    ts = [torch.randn(s, generator=g).to(dev) for s in ((P, 3), (P, 1, 3), (P, 15, 3), (P, 1), (P, 3), (P, 4))]
    d = tempfile.mkdtemp(dir=os.environ.get("TMPDIR", "/tmp"))
    path = os.path.join(d, "scene.ply")
    res = {"workload": f"{P} Gaussians, SH3 (62 fp32 properties, {P * 248 / 1e6:.0f} MB body)"}
    ply.save_ply(path, *ts)  # warm
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        ply.save_ply(path, *ts)
    res["save_ms"] = (time.perf_counter() - t0) / 3 * 1e3
    ply.load_ply(path, 3)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        ply.load_ply(path, 3)
    torch.cuda.synchronize()
    res["load_ms"] = (time.perf_counter() - t0) / 3 * 1e3
    n = 100_000
    t0 = time.perf_counter()
    ref_save(os.path.join(d, "ref.ply"), [t[:n] for t in ts])
    res["reference_save_ms_scaled"] = (time.perf_counter() - t0) * 1e3 * P / n
    res["reference_sample"] = f"{n} Gaussians, scaled x{P // n}"
    res["save_speedup"] = res["reference_save_ms_scaled"] / res["save_ms"]
    os.remove(path)
    os.remove(os.path.join(d, "ref.ply"))
    os.rmdir(d)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
