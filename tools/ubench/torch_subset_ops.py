"""Device cost of the torch ops a keyframe's point subset could use (round 5:
OnlineMapper.keyframe_points' subset phase measured 4.6 ms with
nonzero_static).  Each op timed over 20 calls after 3 warm-ups, synchronised.
usage: python tools/ubench/torch_subset_ops.py [H W ds]"""
import json
import sys
import time

import torch


def main():
    H, W, ds = (int(v) for v in sys.argv[1:4]) if len(sys.argv) > 3 else (384, 512, 32)
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    depth = torch.rand(H, W, device=dev, generator=g) * 5
    depth[: H // 7] = 0
    valid = (depth > 0) & (depth < 100.0)
    n = int(valid.sum())
    k = int(n / ds)
    res = {"H": H, "W": W, "n_valid": n, "k": k}

    def t(name, fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            fn()
        torch.cuda.synchronize()
        res[name] = round(1e3 * (time.perf_counter() - t0) / 20, 4)

    t("nonzero", lambda: torch.nonzero(valid, as_tuple=True))
    t("nonzero_static", lambda: torch.nonzero_static(valid, size=n))
    t("randperm", lambda: torch.randperm(n, device=dev, generator=g))
    t("randperm_prefix_sort", lambda: torch.sort(torch.randperm(n, device=dev, generator=g)[:k]).values)
    t("rand_topk_sort", lambda: torch.sort(torch.rand(n, device=dev, generator=g).topk(k, largest=False).indices).values)
    t("sort_depth", lambda: torch.sort(depth.reshape(-1)).values)
    t("cumsum_valid", lambda: torch.cumsum(valid.reshape(-1), 0))
    t("sum_item", lambda: int(valid.sum()))
    t("masked_select", lambda: torch.masked_select(torch.arange(H * W, device=dev), valid.reshape(-1)))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
