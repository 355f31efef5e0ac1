"""GPU parity for SURVEY.md 8(f) row f1: the fused Adam step and the fused
densification compaction against the reference's own torch calls.

Reference behaviour checked:
  * ``torch.optim.Adam(groups, lr=0.0, eps=1e-15)`` with one named parameter
    per group and per-group lr (gaussian_model.py:271-309, 322-336).
    Tolerance: params and both moments agree to rtol 1e-5 / atol 1e-7 after
    several steps (the same fp32 operation order as torch's foreach Adam;
    only FMA contraction may differ by an ulp).
  * ``t[mask]`` boolean row selection (prune_points / _prune_optimizer,
    gaussian_model.py:526-564): bit-exact, any dtype, ragged sizes.
  * ``cat_tensors_to_optimizer`` (:566-600): bit-exact.
"""
import pytest
import torch
from torch import nn

pytestmark = pytest.mark.gpu
DEV = "cuda"

# (name, row shape, lr) as in GaussianModel.training_setup
GROUPS = [("xyz", (3,), 1.6e-4), ("f_dc", (1, 3), 2.5e-3), ("f_rest", (15, 3), 1.25e-4),
          ("opacity", (1,), 5e-2), ("scaling", (3,), 5e-3), ("rotation", (4,), 1e-3)]


def _make_params(P, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return {n: torch.randn((P,) + s, generator=g).to(DEV) for n, s, _ in GROUPS}


def _optimizer(cls, tensors):
    groups = [{"params": [nn.Parameter(tensors[n].clone().requires_grad_(True))], "lr": lr, "name": n}
              for n, _, lr in GROUPS]
    return cls(groups, lr=0.0, eps=1e-15)


def _assert_same_state(opt_a, opt_b, rtol=1e-5, atol=1e-7):
    for ga, gb in zip(opt_a.param_groups, opt_b.param_groups):
        pa, pb = ga["params"][0], gb["params"][0]
        torch.testing.assert_close(pa.data, pb.data, rtol=rtol, atol=atol, msg=lambda m, n=ga["name"]: f"{n}: {m}")
        sa, sb = opt_a.state.get(pa), opt_b.state.get(pb)
        assert (sa is None) == (sb is None), ga["name"]
        if sa is None:
            continue
        assert float(sa["step"]) == float(sb["step"])
        for k in ("exp_avg", "exp_avg_sq"):
            torch.testing.assert_close(sa[k], sb[k], rtol=rtol, atol=atol * 1e-3 if k == "exp_avg_sq" else atol,
                                       msg=lambda m, n=f"{ga['name']}.{k}": f"{n}: {m}")


def _step_both(opt_a, opt_b, seed, skip=()):
    g = torch.Generator(device="cpu").manual_seed(seed)
    for ga, gb in zip(opt_a.param_groups, opt_b.param_groups):
        pa, pb = ga["params"][0], gb["params"][0]
        if ga["name"] in skip:
            pa.grad = pb.grad = None
            continue
        grad = torch.randn(pa.shape, generator=g).to(DEV)
        grad[::7] = 0.0  # rows the view did not touch
        pa.grad, pb.grad = grad.clone(), grad.clone()
    opt_a.step()
    opt_b.step()


@pytest.mark.parametrize("P", [1, 1001, 50_003])
def test_fused_adam_matches_torch_adam(P):
    from wgsr.optim import FusedAdam
    t = _make_params(P, seed=P)
    ref, ours = _optimizer(torch.optim.Adam, t), _optimizer(FusedAdam, t)
    for it in range(6):
        # the reference steps only groups with gradients (e.g. a frozen pose)
        _step_both(ref, ours, seed=100 + it, skip=("opacity",) if it < 2 else ())
        # update_learning_rate rewrites the xyz group's lr every iteration
        for o in (ref, ours):
            o.param_groups[0]["lr"] = 1.6e-4 * (0.9 ** it)
    torch.cuda.synchronize()
    _assert_same_state(ref, ours)


def test_fused_adam_weight_decay_matches_torch_adam():
    """The uncertainty MLP's optimiser: torch.optim.Adam(params, lr=4e-4,
    weight_decay=1e-5) (mapper.py:129-133); .grad is left untouched."""
    from wgsr.mlp import UncertaintyMLP
    from wgsr.optim import FusedAdam
    torch.manual_seed(0)
    a, b = UncertaintyMLP(input_dim=128).to(DEV), UncertaintyMLP(input_dim=128).to(DEV)
    b.load_state_dict(a.state_dict())
    ref = torch.optim.Adam(b.parameters(), lr=4e-4, weight_decay=1e-5)
    ours = FusedAdam(a.parameters(), lr=4e-4, weight_decay=1e-5)
    g = torch.Generator(device="cpu").manual_seed(5)
    for it in range(4):
        for pa, pb in zip(a.parameters(), b.parameters()):
            gr = torch.randn(pa.shape, generator=g).to(DEV)
            pa.grad, pb.grad = gr.clone(), gr.clone()
        keep = [pa.grad.clone() for pa in a.parameters()]
        ref.step()
        ours.step()
        for k, pa in zip(keep, a.parameters()):
            assert torch.equal(k, pa.grad)
    for pa, pb in zip(a.parameters(), b.parameters()):
        torch.testing.assert_close(pa.detach(), pb.detach(), rtol=1e-5, atol=1e-7)


def test_fused_adam_unaligned_and_many_tensors():
    """More tensors than one launch holds and storage offsets that rule out
    16-byte vector access (the scalar tail path)."""
    from wgsr.optim import FusedAdam
    g = torch.Generator(device="cpu").manual_seed(3)
    base = [torch.randn(4 * k + 3, generator=g).to(DEV) for k in range(1, 21)]
    views_a = [nn.Parameter(b[1:]) for b in base]              # misaligned by 4 bytes
    views_b = [nn.Parameter(b[1:].clone()) for b in base]      # aligned copies
    ref = torch.optim.Adam([{"params": [v], "lr": 1e-2 * (i + 1)} for i, v in enumerate(views_b)], eps=1e-15)
    ours = FusedAdam([{"params": [v], "lr": 1e-2 * (i + 1)} for i, v in enumerate(views_a)], eps=1e-15)
    for it in range(3):
        for a, b in zip(views_a, views_b):
            gr = torch.randn(a.shape, generator=g).to(DEV)
            a.grad, b.grad = gr.clone(), gr.clone()
        ref.step()
        ours.step()
    for i, (a, b) in enumerate(zip(views_a, views_b)):
        # params travel ~lr per step here: allow an ulp of that movement
        torch.testing.assert_close(a.data, b.data, rtol=1e-5, atol=1e-6 * (i + 1))


def _keep(P, kind, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    if kind == "all":
        return torch.ones(P, dtype=torch.bool, device=DEV)
    if kind == "none":
        return torch.zeros(P, dtype=torch.bool, device=DEV)
    return (torch.rand(P, generator=g) < 0.7).to(DEV)


@pytest.mark.parametrize("P", [0, 1, 17, 4095, 4096, 4097, 100_003])
@pytest.mark.parametrize("kind", ["random", "all", "none"])
def test_compact_rows_matches_boolean_index(P, kind):
    from wgsr.densify import compact_rows
    keep = _keep(P, kind, seed=P + 7)
    g = torch.Generator(device="cpu").manual_seed(P)
    tensors = [torch.randn(P, 3, generator=g).to(DEV), torch.randn(P, 15, 3, generator=g).to(DEV),
               torch.randn(P, 1, generator=g).to(DEV), torch.randint(0, 1 << 30, (P,), generator=g,
                                                                     dtype=torch.int32).to(DEV),
               torch.randint(-(1 << 40), 1 << 40, (P, 2), generator=g, dtype=torch.int64).to(DEV)]
    outs = compact_rows(keep, tensors)
    for t, o in zip(tensors, outs):
        exp = t[keep]
        assert o.shape == exp.shape and o.dtype == exp.dtype
        assert torch.equal(o, exp)


def _ref_prune(optimizer, mask):
    """gaussian_model.py:526-546, verbatim behaviour."""
    out = {}
    for group in optimizer.param_groups:
        st = optimizer.state.get(group["params"][0], None)
        if st is not None:
            st["exp_avg"] = st["exp_avg"][mask]
            st["exp_avg_sq"] = st["exp_avg_sq"][mask]
            del optimizer.state[group["params"][0]]
            group["params"][0] = nn.Parameter(group["params"][0][mask].requires_grad_(True))
            optimizer.state[group["params"][0]] = st
        else:
            group["params"][0] = nn.Parameter(group["params"][0][mask].requires_grad_(True))
        out[group["name"]] = group["params"][0]
    return out


def test_prune_then_densify_then_step_matches_reference():
    from wgsr.densify import cat_tensors_to_optimizer, prune_optimizer
    from wgsr.optim import FusedAdam
    P = 20_011
    t = _make_params(P, seed=11)
    ref, ours = _optimizer(torch.optim.Adam, t), _optimizer(FusedAdam, t)
    for it in range(3):
        _step_both(ref, ours, seed=200 + it)
    keep = _keep(P, "random", seed=5)
    stats = torch.rand(P, 1, device=DEV)
    r = _ref_prune(ref, keep)
    o, (stats_o,) = prune_optimizer(ours, keep, extra=[stats])
    assert torch.equal(stats_o, stats[keep])
    assert set(r) == set(o)
    for k in r:
        assert o[k].shape == r[k].shape
    _assert_same_state(ref, ours)
    # densification_postfix appends new Gaussians with zero moments
    new = _make_params(777, seed=12)
    cat_tensors_to_optimizer(ours, new)
    for group in ref.param_groups:  # gaussian_model.py:566-600
        ext = new[group["name"]]
        st = ref.state.get(group["params"][0], None)
        st["exp_avg"] = torch.cat((st["exp_avg"], torch.zeros_like(ext)), dim=0)
        st["exp_avg_sq"] = torch.cat((st["exp_avg_sq"], torch.zeros_like(ext)), dim=0)
        del ref.state[group["params"][0]]
        group["params"][0] = nn.Parameter(torch.cat((group["params"][0], ext), dim=0).requires_grad_(True))
        ref.state[group["params"][0]] = st
    _assert_same_state(ref, ours)
    for it in range(2):
        _step_both(ref, ours, seed=300 + it)
    torch.cuda.synchronize()
    _assert_same_state(ref, ours)
