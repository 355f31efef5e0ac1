"""Keyframe-view data parallelism over RCCL.

The reference is single-GPU; its mapper renders one keyframe view per
optimiser step (src/mapper.py:1089-1170).  Views are independent given a
replicated Gaussian set, so the natural multi-GPU axis is the VIEW: rank r
renders view r (r + world, ...) with full parameter replicas and the only
exchange is one reduction of the per-Gaussian parameter gradients per step.

* ``GradBuffer`` lays the parameter gradients of one backward out in ONE flat
  fp32 buffer (means3D | SH | opacity | scales | rotations: 59 floats per
  Gaussian at SH degree 3), so the backward writes straight into the
  all-reduce operand -- no pack/unpack copies.
* ``allreduce_grads`` issues SUM all-reduces over that buffer in large
  buckets (xGMI is point-to-point: RCCL's rings are per-link bound, so few,
  large collectives), optionally asynchronously so a caller can overlap them.
* ``reduce_densification_stats`` sums the per-view ||dL/dmeans2D|| statistics
  and visibility counts and takes the MAX of the screen radii -- the reference
  accumulates per-view norms (gaussian_model.py:745-749, mapper.py:1177-1183),
  not the norm of the summed gradient, so these cannot ride in the gradient
  sum.

Backend: whatever ``torch.distributed`` was initialised with -- "nccl" is RCCL
on ROCm (over xGMI on one node); the CPU tests use "gloo".
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.distributed as dist

PARAM_ORDER = ("means3D", "shs", "opacities", "scales", "rotations")


@dataclass
class GradBuffer:
    """Flat gradient storage with per-parameter [P, ...] views."""

    flat: torch.Tensor
    views: dict

    @staticmethod
    def allocate(P: int, M: int, device, dtype=torch.float32) -> "GradBuffer":
        shapes = {"means3D": (P, 3), "shs": (P, M, 3), "opacities": (P, 1), "scales": (P, 3),
                  "rotations": (P, 4)}
        sizes = {k: int(torch.Size(s).numel()) for k, s in shapes.items()}
        flat = torch.empty(sum(sizes.values()), dtype=dtype, device=device)
        views, off = {}, 0
        for k in PARAM_ORDER:
            views[k] = flat[off: off + sizes[k]].view(shapes[k])
            off += sizes[k]
        return GradBuffer(flat, views)

    @property
    def floats_per_gaussian(self) -> int:
        P = self.views["means3D"].shape[0]
        return self.flat.numel() // max(P, 1)


def allreduce_grads(buf: GradBuffer, bucket_bytes: int = 256 << 20, async_op: bool = False,
                    average: bool = False):
    """SUM-all-reduce the flat gradient buffer in buckets of ``bucket_bytes``.

    Returns the list of work handles when ``async_op`` (wait on them before
    reading the gradients), else None.
    """
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return [] if async_op else None
    flat = buf.flat
    per = max(1, bucket_bytes // flat.element_size())
    works = []
    for s in range(0, flat.numel(), per):
        works.append(dist.all_reduce(flat[s: s + per], op=dist.ReduceOp.SUM, async_op=True))
    if average:
        for w in works:
            w.wait()
        flat.div_(dist.get_world_size())
        return [] if async_op else None
    if async_op:
        return works
    for w in works:
        w.wait()
    return None


def reduce_densification_stats(grad_norm_accum: torch.Tensor, denom: torch.Tensor,
                               max_radii2D: torch.Tensor):
    """In place: SUM of per-view ||dL/dmeans2D[:, :2]|| accumulations and of
    the visibility counts; MAX of the per-Gaussian screen radii."""
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return
    dist.all_reduce(grad_norm_accum, op=dist.ReduceOp.SUM)
    dist.all_reduce(denom, op=dist.ReduceOp.SUM)
    dist.all_reduce(max_radii2D, op=dist.ReduceOp.MAX)


def views_for_rank(num_views: int, rank: int, world: int):
    """Round-robin view assignment: rank r renders views r, r + world, ..."""
    return list(range(rank, num_views, world))
