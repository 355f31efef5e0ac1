"""GPU parity of the uncertainty MLP (wgsr.mlp.UncertaintyMLP; SURVEY.md 8(f)
row f2) against a torch fp32 restatement of MLPNetwork (src/utils/
dyn_uncertainty/uncertainty_model.py:5-64) with the same weights: with
dropout off, and with dropout on using the kernel's masks (restated in
wgsr.mlp.dropout_mask).  Tolerances: outputs rel 1e-5, parameter gradients
rel-L1 1e-5 (fp32 reduction order differs from hipBLASLt's)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().sum() / b.abs().sum().clamp_min(1e-30))


def _torch_mlp(net, x, masks=None, p=0.0):
    """MLPNetwork.forward with explicit dropout masks (torch's dropout:
    x * mask / (1 - p))."""
    H, W, C = x.shape[-3:]
    y = x.reshape(-1, C)
    for i, layer in enumerate(net.layers):
        y = F.relu(F.linear(y, layer.weight, layer.bias))
        if masks is not None:
            y = y * masks[i] * (1.0 / (1.0 - p))
    y = F.softplus(F.linear(y, net.output_layer.weight, net.output_layer.bias))
    return y.view(x.shape[:-1])


@pytest.mark.parametrize("shape,p", [((27, 36, 384), 0.0), ((77, 137, 384), 0.0), ((2, 9, 13, 128), 0.0),
                                     ((27, 36, 384), 0.2), ((5, 7, 64), 0.5)])
def test_forward_backward_matches_torch(shape, p):
    from wgsr.mlp import UncertaintyMLP, dropout_mask
    torch.manual_seed(0)
    C = shape[-1]
    net = UncertaintyMLP(input_dim=C, dropout_p=p).to(DEV)
    x = torch.randn(*shape, device=DEV)
    u = net(x)
    g = torch.randn_like(u)
    (u * g).sum().backward()
    got = [prm.grad.clone() for prm in net.parameters()]
    for prm in net.parameters():
        prm.grad = None
    N = x.numel() // C
    masks = None
    if p > 0:
        masks = [torch.from_numpy(dropout_mask(net.last_seed, i, N, p)).to(DEV).float() for i in range(2)]
    want_u = _torch_mlp(net, x, masks, p)
    (want_u * g).sum().backward()
    assert u.shape == want_u.shape
    assert _rel(u, want_u) <= 1e-5
    for a, b in zip(got, [prm.grad for prm in net.parameters()]):
        assert _rel(a, b) <= 1e-5


def test_dropout_rate_and_fresh_masks():
    from wgsr.mlp import UncertaintyMLP
    torch.manual_seed(1)
    net = UncertaintyMLP(input_dim=64).to(DEV)
    x = torch.randn(100, 100, 64, device=DEV)
    u1, s1 = net(x), net.last_seed
    u2, s2 = net(x), net.last_seed
    assert s1 != s2 and not torch.equal(u1, u2)   # new masks per call, like F.dropout
    torch.manual_seed(1)
    net2 = UncertaintyMLP(input_dim=64).to(DEV)
    assert torch.equal(net2(x), u1)               # torch.manual_seed makes it repeatable


def test_state_dict_matches_reference_layout():
    from wgsr.mlp import UncertaintyMLP
    net = UncertaintyMLP(input_dim=384)
    assert sorted(net.state_dict()) == sorted(["layers.0.weight", "layers.0.bias", "layers.1.weight",
                                               "layers.1.bias", "output_layer.weight", "output_layer.bias"])
    assert net.layers[0].weight.shape == (64, 384) and net.output_layer.weight.shape == (1, 64)


def test_single_row_and_batched_shapes():
    from wgsr.mlp import UncertaintyMLP
    torch.manual_seed(2)
    net = UncertaintyMLP(input_dim=64, dropout_p=0.0).to(DEV)
    for shape in ((1, 1, 64), (1, 303, 64), (3, 2, 5, 64)):
        x = torch.randn(*shape, device=DEV)
        u = net(x)
        assert u.shape == x.shape[:-1]
        torch.testing.assert_close(u, _torch_mlp(net, x), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("N,C,p", [(1275, 384, 0.2), (972, 384, 0.0), (300, 128, 0.2), (17, 64, 0.5)])
def test_matrix_core_forward_is_bitwise_the_valu_forward(N, C, p):
    """k_mlp_fwd_small (layers 1-2 on v_mfma_f32_16x16x4_f32) against the
    VALU kernel k_mlp_fwd (taken when X is not 16-byte aligned): every output
    -- both dropout-masked hidden layers, the pre-activation and the
    softplus -- bit for bit (the matrix-core step is a k-ordered fmaf chain)."""
    from wgsr import _lib
    L = _lib.load()
    torch.manual_seed(7)
    f = dict(device=DEV, dtype=torch.float32)
    W1, b1 = torch.randn(64, C, **f) * 0.1, torch.randn(64, **f) * 0.1
    W2, b2 = torch.randn(64, 64, **f) * 0.1, torch.randn(64, **f) * 0.1
    W3, b3 = torch.randn(1, 64, **f) * 0.1, torch.randn(1, **f) * 0.1
    x = torch.randn(N, C, **f)
    xm = torch.empty(N * C + 1, **f)[1:]          # the same rows at a 4-byte offset
    xm.copy_(x.reshape(-1))
    outs = []
    for X in (x, xm):
        o = [torch.full((N, 64), float("nan"), **f), torch.full((N, 64), float("nan"), **f),
             torch.full((N,), float("nan"), **f), torch.full((N,), float("nan"), **f)]
        p_ = _lib.ptr
        _lib.check(L.wgsr_mlp_forward(N, C, p_(X), p_(W1), p_(b1), p_(W2), p_(b2), p_(W3), p_(b3), float(p), 12345,
                                      p_(o[0]), p_(o[1]), p_(o[2]), p_(o[3]), _lib.stream_handle(DEV)))
        outs.append(o)
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("N,C,p", [(1275, 384, 0.2), (130, 128, 0.0), (17, 64, 0.5)])
def test_matrix_core_backward_is_bitwise_the_valu_backward(N, C, p):
    """k_mlp_bwd2 (its three 64 x 64 x 64 products on v_mfma_f32_16x16x4_f32)
    against the VALU kernel k_mlp_bwd (taken when X is not 16-byte aligned):
    the summed parameter gradient bit for bit."""
    from wgsr import _lib
    L = _lib.load()
    torch.manual_seed(8)
    f = dict(device=DEV, dtype=torch.float32)
    W1, b1 = torch.randn(64, C, **f) * 0.1, torch.randn(64, **f) * 0.1
    W2, b2 = torch.randn(64, 64, **f) * 0.1, torch.randn(64, **f) * 0.1
    W3, b3 = torch.randn(1, 64, **f) * 0.1, torch.randn(1, **f) * 0.1
    x = torch.randn(N, C, **f)
    xm = torch.empty(N * C + 1, **f)[1:]
    xm.copy_(x.reshape(-1))
    du = torch.randn(N, **f)
    p_ = _lib.ptr
    st = _lib.stream_handle(DEV)
    h1, h2, o, u = (torch.empty(N, 64, **f), torch.empty(N, 64, **f), torch.empty(N, **f), torch.empty(N, **f))
    _lib.check(L.wgsr_mlp_forward(N, C, p_(x), p_(W1), p_(b1), p_(W2), p_(b2), p_(W3), p_(b3), float(p), 99,
                                  p_(h1), p_(h2), p_(o), p_(u), st))
    nscr = int(L.wgsr_mlp_scratch_bytes(N, C)) // 4
    G = []
    for X in (x, xm):
        scr = torch.empty(max(nscr, 1), **f)
        g = torch.full((int(L.wgsr_mlp_grad_floats(C)),), float("nan"), **f)
        _lib.check(L.wgsr_mlp_backward(N, C, p_(X), p_(W2), p_(W3), float(p), p_(h1), p_(h2), p_(o), p_(du), p_(scr),
                                       p_(g), st))
        G.append(g)
    assert torch.isfinite(G[0]).all() and torch.equal(G[0], G[1])
