#!/usr/bin/env python
"""simple_knn.distCUDA2 on the MI355X path.

Device time per call (HIP events, median of repeats) for the configs[2]
scene's 1M Gaussian centres and for per-keyframe point clouds of TUM size
(~6k points at downsample 32, ~12k at initialisation; gaussian_model.py:
201-207 calls it once per keyframe).  The CPU comparison lives in bench.py's
``distcuda2`` object (oracle timing is confined there).
"""
import json
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "wildgs-slam-blackwell_amd", "python"))

import torch  # noqa: E402


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    from simple_knn._C import distCUDA2
    from wgsr.scene import make_scene
    dev = torch.device("cuda:0")
    out = {}
    pts = make_scene(1_000_000, 1920, 1080, 0, seed=0).means3D.to(dev).contiguous()
    out["scene_1M_ms"] = timed(lambda: distCUDA2(pts))
    g = torch.Generator().manual_seed(0)
    for n in (6000, 12000, 200_000):
        # a depth-map back-projection: a noisy surface patch
        uv = torch.rand(n, 2, generator=g) * 2 - 1
        z = 2 + 0.3 * torch.sin(3 * uv[:, 0]) + 0.01 * torch.randn(n, generator=g)
        p = torch.stack([uv[:, 0] * z, uv[:, 1] * z * 0.75, z], 1).to(dev).contiguous()
        out[f"surface_{n}_ms"] = timed(lambda p=p: distCUDA2(p))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
