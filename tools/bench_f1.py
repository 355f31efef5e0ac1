"""Measure SURVEY.md 8(f) row f1 on the GPU: the fused Adam step and the
fused prune compaction against the reference's torch calls on the same
1M-Gaussian parameter set (gaussian_model.py:271-309 groups; 59 fp32 per
Gaussian: xyz 3, f_dc 3, f_rest 45, opacity 1, scaling 3, rotation 4).

Algorithmic bytes:
  Adam step    28 B per element (read param, grad, exp_avg, exp_avg_sq;
               write param, exp_avg, exp_avg_sq) x 59 P elements
  prune        P (mask) + 2 x kept x 720 B (59 params + 118 moments +
               3 densification stats = 180 fp32 per Gaussian, read + write)
Prints one JSON line.  HBM peak 8 TB/s (MI355X_MICROARCH.md).
"""
import argparse
import json
import os
import sys

import torch
from torch import nn

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "wildgs-slam-blackwell_amd", "python"))

from wgsr.densify import prune_optimizer  # noqa: E402
from wgsr.optim import FusedAdam  # noqa: E402

GROUPS = [("xyz", (3,), 1.6e-4), ("f_dc", (1, 3), 2.5e-3), ("f_rest", (15, 3), 1.25e-4),
          ("opacity", (1,), 5e-2), ("scaling", (3,), 5e-3), ("rotation", (4,), 1e-3)]
HBM_PEAK = 8.0e12


def make_opt(cls, P, dev):
    groups = [{"params": [nn.Parameter(torch.randn((P,) + s, device=dev))], "lr": lr, "name": n}
              for n, s, lr in GROUPS]
    opt = cls(groups, lr=0.0, eps=1e-15)
    for g in opt.param_groups:
        g["params"][0].grad = torch.randn_like(g["params"][0])
    return opt


def time_it(fn, iters, warmup):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e-3


def ref_prune(opt, mask, extra):
    for group in opt.param_groups:  # gaussian_model.py:526-546
        st = opt.state.get(group["params"][0], None)
        st["exp_avg"] = st["exp_avg"][mask]
        st["exp_avg_sq"] = st["exp_avg_sq"][mask]
        del opt.state[group["params"][0]]
        group["params"][0] = nn.Parameter(group["params"][0][mask].requires_grad_(True))
        opt.state[group["params"][0]] = st
    return [t[mask] for t in extra]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, default=1_000_000)
    ap.add_argument("--iters", type=int, default=50)
    args = ap.parse_args()
    dev = torch.device("cuda")
    P = args.P
    elems = P * sum(int(torch.tensor(s).prod()) for _, s, _ in GROUPS)
    res = {"workload": f"{P} Gaussians, reference parameter groups (59 fp32 each)"}
    for name, cls in (("fused", FusedAdam), ("torch", torch.optim.Adam)):
        opt = make_opt(cls, P, dev)
        t = time_it(opt.step, args.iters, 3)
        res[f"adam_{name}_ms"] = t * 1e3
        if name == "fused":
            res["adam_fused_GBps"] = 28 * elems / t / 1e9
            res["adam_fused_frac"] = 28 * elems / t / HBM_PEAK
        del opt
    res["adam_speedup"] = res["adam_torch_ms"] / res["adam_fused_ms"]

    mask = torch.rand(P, device=dev) < 0.9
    kept = int(mask.sum())
    for name in ("fused", "torch"):
        times = []
        for rep in range(5):
            opt = make_opt(torch.optim.Adam, P, dev)
            opt.step()
            extra = [torch.rand(P, 1, device=dev), torch.rand(P, 1, device=dev), torch.rand(P, device=dev)]
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            if name == "fused":
                prune_optimizer(opt, mask, extra)
            else:
                ref_prune(opt, mask, extra)
            e.record()
            torch.cuda.synchronize()
            if rep:
                times.append(s.elapsed_time(e) * 1e-3)
            del opt, extra
        t = sorted(times)[len(times) // 2]
        res[f"prune_{name}_ms"] = t * 1e3
        if name == "fused":
            b = P + 2 * kept * 720
            res["prune_fused_GBps"] = b / t / 1e9
            res["prune_fused_frac"] = b / t / HBM_PEAK
    res["prune_speedup"] = res["prune_torch_ms"] / res["prune_fused_ms"]
    print(json.dumps(res))


if __name__ == "__main__":
    main()
