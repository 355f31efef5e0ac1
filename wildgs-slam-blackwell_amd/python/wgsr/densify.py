"""Densification bookkeeping on the Gaussian SoA.

``compact_rows(keep, tensors)`` is ``[t[keep] for t in tensors]`` for every
per-Gaussian tensor at once (one scan + one gather launch,
``wgsr_compact_rows``).  ``prune_optimizer`` / ``cat_tensors_to_optimizer``
mirror GaussianModel._prune_optimizer / cat_tensors_to_optimizer
(thirdparty/gaussian_splatting/scene/gaussian_model.py:526-600) for an
optimizer whose groups each hold one named parameter (torch.optim.Adam or
wgsr.optim.FusedAdam): parameters and Adam states are rebuilt exactly as the
reference does, with the pruning gathers fused.
"""
from __future__ import annotations

import torch
from torch import nn

from . import _lib


def compact_rows(keep: torch.Tensor, tensors):
    """Return ``[t[keep] for t in tensors]`` (keep: bool [P]; tensors: [P, ...])."""
    tensors = list(tensors)
    if not tensors:
        return []
    P = keep.shape[0]
    dev = keep.device
    keep_u8 = keep.to(torch.uint8).contiguous()
    kept = int(keep_u8.sum().item())
    outs, descs = [], []
    for t in tensors:
        if t.shape[0] != P or t.device != dev:
            raise ValueError("compact_rows: every tensor needs the mask's row count and device")
        src = t.contiguous()
        out = torch.empty((kept,) + tuple(t.shape[1:]), dtype=t.dtype, device=dev)
        outs.append(out)
        row_bytes = src.element_size() * (src[0].numel() if P > 0 else 0)
        if row_bytes % 4 != 0:
            raise ValueError("compact_rows: rows must be a multiple of 4 bytes")
        descs.append((src, out, row_bytes))
    if P == 0 or kept == 0:
        return outs
    L = _lib.load()
    for i in range(0, len(descs), _lib.COMPACT_MAX_TENSORS):
        chunk = descs[i:i + _lib.COMPACT_MAX_TENSORS]
        arr = (_lib.RowTensor * len(chunk))(*[_lib.RowTensor(s.data_ptr(), o.data_ptr(), rb)
                                              for s, o, rb in chunk])
        with torch.cuda.device(dev), _lib.AllocRequest(dev):
            _lib.check(L.wgsr_compact_rows(keep_u8.data_ptr(), P, arr, len(chunk), _lib.ALLOC_SCRATCH,
                                           None, _lib.stream_handle(dev)))
    return outs


def prune_optimizer(optimizer, keep: torch.Tensor, extra=()):
    """GaussianModel._prune_optimizer with fused gathers.

    Returns ({group name: new nn.Parameter}, [pruned extra tensors])."""
    groups = optimizer.param_groups
    tensors = []
    for group in groups:
        assert len(group["params"]) == 1
        p = group["params"][0]
        tensors.append(p.data)
        st = optimizer.state.get(p, None)
        if st is not None:
            tensors += [st["exp_avg"], st["exp_avg_sq"]]
    extra = list(extra)
    outs = compact_rows(keep, tensors + extra)
    it = iter(outs)
    optimizable = {}
    for group in groups:
        p = group["params"][0]
        new_p = next(it)
        st = optimizer.state.get(p, None)
        if st is not None:
            st["exp_avg"] = next(it)
            st["exp_avg_sq"] = next(it)
            del optimizer.state[p]
        group["params"][0] = nn.Parameter(new_p.requires_grad_(True))
        if st is not None:
            optimizer.state[group["params"][0]] = st
        optimizable[group["name"]] = group["params"][0]
    return optimizable, [next(it) for _ in extra]


def cat_tensors_to_optimizer(optimizer, tensors_dict):
    """GaussianModel.cat_tensors_to_optimizer (new rows get zero Adam moments)."""
    optimizable = {}
    for group in optimizer.param_groups:
        assert len(group["params"]) == 1
        ext = tensors_dict[group["name"]]
        p = group["params"][0]
        st = optimizer.state.get(p, None)
        if st is not None:
            st["exp_avg"] = torch.cat((st["exp_avg"], torch.zeros_like(ext)), dim=0)
            st["exp_avg_sq"] = torch.cat((st["exp_avg_sq"], torch.zeros_like(ext)), dim=0)
            del optimizer.state[p]
        group["params"][0] = nn.Parameter(torch.cat((p, ext), dim=0).requires_grad_(True))
        if st is not None:
            optimizer.state[group["params"][0]] = st
        optimizable[group["name"]] = group["params"][0]
    return optimizable
