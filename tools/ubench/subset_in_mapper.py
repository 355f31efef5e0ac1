"""The keyframe subset ops timed inside a live mapper (round 5: the subset
phase costs ~1.5 ms in tools/bench_online.py but ~0.1 ms in isolation,
tools/ubench/torch_subset_ops.py).  Builds the bench_online scene with a
short schedule, then times each op of the subset draw (synchronised),
with fresh allocations and with preallocated outputs.
usage: python tools/ubench/subset_in_mapper.py"""
import json
import os
import sys
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.argv = ["bench_online.py", "--keyframes", "4", "--init-iters", "60", "--iters", "40", "--refine-iters", "0"]
import bench_online  # noqa: E402


def main():
    import wgsr.online as online
    captured = {}
    orig = online.OnlineMapper.prepare_keyframe

    def grab(self, kf, keep=None):
        captured["m"], captured["kf"] = self, kf
        return orig(self, kf, keep)
    online.OnlineMapper.prepare_keyframe = grab
    import contextlib
    import io
    with contextlib.redirect_stdout(io.StringIO()):
        bench_online.main()
    m, kf = captured["m"], captured["kf"]
    dev = m.dev
    depth = kf.depth[0]
    valid = (depth > 0) & (depth < 100.0)
    n = int(valid.sum())
    k = n // 32
    res = {"n": n, "k": k, "P": m.ms.P, "mem_reserved_MB": torch.cuda.memory_reserved(dev) / 2**20}

    def t(name, fn, reps=5):
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append(1e3 * (time.perf_counter() - t0))
        res[name] = [round(x, 4) for x in ts]

    t("rand", lambda: torch.rand(depth.numel(), device=dev, generator=m.gen))
    key = torch.rand(depth.numel(), device=dev, generator=m.gen)
    t("where", lambda: torch.where(valid.reshape(-1), key, 2.0))
    kk = torch.where(valid.reshape(-1), key, 2.0)
    t("topk", lambda: torch.topk(kk, k, largest=False, sorted=False))
    idx = torch.topk(kk, k, largest=False, sorted=False).indices
    t("sort_k", lambda: torch.sort(idx))
    t("randperm", lambda: torch.randperm(n, device=dev, generator=m.gen))
    t("nonzero", lambda: torch.nonzero(valid, as_tuple=True))
    buf = torch.empty(depth.numel(), device=dev)
    t("rand_out", lambda: torch.rand(depth.numel(), out=buf, generator=m.gen))
    t("empty_1MB", lambda: torch.empty(1 << 18, device=dev))
    t("keyframe_points", lambda: m.keyframe_points(kf, False))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
