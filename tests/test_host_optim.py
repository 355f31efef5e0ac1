"""CPU checks of the f1 host logic (no GPU): FusedAdam refuses what the
HIP path cannot do instead of silently falling back, and the densify
helpers validate shapes before launching anything."""
import pytest
import torch
from torch import nn


def test_fused_adam_rejects_negative_weight_decay_and_cpu_params():
    from wgsr.optim import FusedAdam
    p = nn.Parameter(torch.zeros(8))
    with pytest.raises(ValueError):
        FusedAdam([p], weight_decay=-0.1)
    opt = FusedAdam([{"params": [p], "lr": 1e-3, "name": "xyz"}], lr=0.0, eps=1e-15)
    assert opt.param_groups[0]["name"] == "xyz" and opt.defaults["eps"] == 1e-15
    p.grad = torch.ones(8)
    with pytest.raises(RuntimeError, match="device"):
        opt.step()


def test_fused_adam_step_without_grads_is_a_noop():
    from wgsr.optim import FusedAdam
    p = nn.Parameter(torch.zeros(8))
    opt = FusedAdam([p])
    opt.step()  # no gradient anywhere: nothing launched, no state created
    assert len(opt.state) == 0


def test_compact_rows_validates_rows():
    from wgsr.densify import compact_rows
    assert compact_rows(torch.ones(4, dtype=torch.bool), []) == []
    with pytest.raises(ValueError):
        compact_rows(torch.ones(4, dtype=torch.bool), [torch.zeros(5, 3)])
    with pytest.raises(ValueError):
        compact_rows(torch.ones(4, dtype=torch.bool), [torch.zeros(4, 3, dtype=torch.uint8)])
