"""Fused Adam for the Gaussian parameter groups.

``FusedAdam`` is a drop-in for the reference's optimizer,
``torch.optim.Adam(param_groups, lr=0.0, eps=1e-15)``
(thirdparty/gaussian_splatting/scene/gaussian_model.py:309): same
constructor, same ``param_groups`` (with their ``"name"`` keys and per-group
``lr``, which ``update_learning_rate`` rewrites, :322-336) and the same
per-parameter ``state`` dicts (``"step"``, ``"exp_avg"``, ``"exp_avg_sq"``)
that ``replace_tensor_to_optimizer``, ``_prune_optimizer`` and
``cat_tensors_to_optimizer`` (:495-600) read and rebuild.  ``step()`` updates
every parameter that has a gradient in ONE HIP launch (``wgsr_adam_step``)
instead of torch's ~7 foreach passes.  ``weight_decay`` is torch.optim.Adam's
L2 form (the gradient used is grad + weight_decay * param; ``.grad`` itself
is left untouched, one extra foreach launch) -- the uncertainty MLP's
optimiser uses it (mapper.py:129-133).  Scope as used by the reference: no
amsgrad, no maximize, fp32 CUDA tensors.
"""
from __future__ import annotations

import ctypes
import math

import torch

from . import _lib


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        if weight_decay < 0.0:
            raise ValueError(f"Invalid weight_decay value: {weight_decay}")
        if not 0.0 <= betas[0] < 1.0 or not 0.0 <= betas[1] < 1.0:
            raise ValueError(f"Invalid beta parameters: {betas}")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        batches = {}  # (betas, eps, device) -> [AdamTensor]
        for group in self.param_groups:
            beta1, beta2 = group["betas"]
            wd = group.get("weight_decay", 0.0)
            decayed = {}
            if wd != 0.0:
                live = [p for p in group["params"] if p.grad is not None]
                if live:
                    decayed = dict(zip(map(id, live), torch._foreach_add([p.grad for p in live], live, alpha=wd)))
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.grad.is_sparse:
                    raise RuntimeError("FusedAdam does not support sparse gradients")
                if p.dtype != torch.float32 or not p.is_cuda:
                    raise RuntimeError("FusedAdam: fp32 device parameters only")
                state = self.state[p]
                if len(state) == 0:
                    state["step"] = torch.tensor(0.0)
                    state["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    state["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                step_t = state["step"]
                step_t += 1
                step = float(step_t)
                bc1 = 1.0 - beta1 ** step
                bc2 = 1.0 - beta2 ** step
                grad = decayed.get(id(p), p.grad)
                grad = grad if grad.is_contiguous() else grad.contiguous()
                for t in (p, state["exp_avg"], state["exp_avg_sq"]):
                    if not t.is_contiguous():
                        raise RuntimeError("FusedAdam: parameters and states must be contiguous")
                key = (group["betas"], group["eps"], p.device)
                batches.setdefault(key, []).append(
                    (_lib.AdamTensor(p.data_ptr(), grad.data_ptr(), state["exp_avg"].data_ptr(),
                                     state["exp_avg_sq"].data_ptr(), p.numel(),
                                     group["lr"] / bc1, math.sqrt(bc2)), grad))
        L = _lib.load()
        for (betas, eps, dev), items in batches.items():
            for i in range(0, len(items), _lib.ADAM_MAX_TENSORS):
                chunk = items[i:i + _lib.ADAM_MAX_TENSORS]
                arr = (_lib.AdamTensor * len(chunk))(*[c[0] for c in chunk])
                with torch.cuda.device(dev):
                    _lib.check(L.wgsr_adam_step(arr, len(chunk), betas[0], betas[1], eps,
                                                _lib.stream_handle(dev)))
        return loss
