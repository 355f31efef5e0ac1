"""The uncertainty MLP on the gfx950 path.

``UncertaintyMLP`` is a drop-in for the reference's ``MLPNetwork`` with its
defaults (src/utils/dyn_uncertainty/uncertainty_model.py:5-68: C -> 64 -> 64
-> 1, ReLU, ``F.dropout(p=0.2)`` after each hidden layer -- applied in train
AND eval mode, as the reference does -- softplus output): same parameter
names (``layers.0``, ``layers.1``, ``output_layer``), so ``state_dict``s load
both ways, same initialisation, same input/output shapes ([H, W, C] ->
[H, W], [B, H, W, C] -> [B, H, W]).  The forward is one HIP launch and the
backward two (per-workgroup partial weight gradients, then a fixed-order
sum) instead of ~10 GEMM / elementwise launches each way, and torch.optim
(or wgsr.optim.FusedAdam) steps its parameters as usual.

Dropout masks are a counter hash of (seed, layer, row, column); the seed is
drawn from torch's default CPU generator per forward, so ``torch.manual_seed``
makes runs repeatable (the masks differ from torch's own Philox draws:
dropout is random in the reference too).  ``dropout_mask`` restates the hash
for tests.  No fallback: without libwgsr.so, or on CPU tensors, this raises.
"""
from __future__ import annotations

import numpy as np
import torch
from torch import nn

from . import _lib

HIDDEN = 64


def _mix32(x):
    x = x.astype(np.uint32)
    x ^= x >> np.uint32(16)
    x *= np.uint32(0x7feb352d)
    x ^= x >> np.uint32(15)
    x *= np.uint32(0x846ca68b)
    x ^= x >> np.uint32(16)
    return x


def dropout_mask(seed: int, layer: int, rows: int, p: float) -> np.ndarray:
    """[rows, 64] bool keep-mask of dropout layer ``layer`` (csrc/mlp.hip keep_elem)."""
    with np.errstate(over="ignore"):
        r = np.arange(rows, dtype=np.uint32)[:, None]
        c = np.arange(HIDDEN, dtype=np.uint32)[None, :]
        inner = _mix32(r * np.uint32(64) + c)
        mid = _mix32(np.uint32((layer * 0x9E3779B9) & 0xFFFFFFFF) ^ inner)
        h = _mix32(np.uint32(seed & 0xFFFFFFFF) ^ mid)
    u = (h >> np.uint32(8)).astype(np.float32) * np.float32(1.0 / 16777216.0)
    return u >= np.float32(p)


class _MLPFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, W1, b1, W2, b2, W3, b3, p, seed):
        N, C = x.shape
        dev = x.device
        L = _lib.load()
        xs = x.detach().contiguous()
        ws = [t.detach().contiguous() for t in (W1, b1, W2, b2, W3, b3)]
        h1d = torch.empty(N, HIDDEN, device=dev)
        h2d = torch.empty(N, HIDDEN, device=dev)
        o = torch.empty(N, device=dev)
        u = torch.empty(N, device=dev)
        pt = _lib.ptr
        with torch.cuda.device(dev):
            _lib.check(L.wgsr_mlp_forward(N, C, pt(xs), *[pt(t) for t in ws], float(p), int(seed) & 0xFFFFFFFF,
                                          pt(h1d), pt(h2d), pt(o), pt(u), _lib.stream_handle(dev)))
        ctx.save_for_backward(xs, ws[2], ws[4], h1d, h2d, o)
        ctx.p = float(p)
        return u

    @staticmethod
    def backward(ctx, du):
        xs, W2, W3, h1d, h2d, o = ctx.saved_tensors
        N, C = xs.shape
        dev = xs.device
        L = _lib.load()
        du = du.detach().to(torch.float32).contiguous()
        total = int(L.wgsr_mlp_grad_floats(C))
        grad = torch.empty(total, device=dev)
        scratch = torch.empty(max(1, int(L.wgsr_mlp_scratch_bytes(N, C)) // 4), device=dev)
        pt = _lib.ptr
        with torch.cuda.device(dev):
            _lib.check(L.wgsr_mlp_backward(N, C, pt(xs), pt(W2), pt(W3), ctx.p, pt(h1d), pt(h2d), pt(o), pt(du),
                                           pt(scratch), pt(grad), _lib.stream_handle(dev)))
        o0 = HIDDEN * C
        gW1 = grad[:o0].view(HIDDEN, C)
        gb1 = grad[o0:o0 + HIDDEN]
        o1 = o0 + HIDDEN
        gW2 = grad[o1:o1 + HIDDEN * HIDDEN].view(HIDDEN, HIDDEN)
        o2 = o1 + HIDDEN * HIDDEN
        gb2 = grad[o2:o2 + HIDDEN]
        gW3 = grad[o2 + HIDDEN:o2 + 2 * HIDDEN].view(1, HIDDEN)
        gb3 = grad[o2 + 2 * HIDDEN:o2 + 2 * HIDDEN + 1]
        if ctx.needs_input_grad[0]:
            raise NotImplementedError("UncertaintyMLP: no gradient w.r.t. the input features")
        return None, gW1, gb1, gW2, gb2, gW3, gb3, None, None


def forward_raw(net, x, seed_dev):
    """The forward of ``net`` on x [N, C] without autograd, the dropout seed
    read from device memory (``seed_dev``: int32 [1] holding the uint32 bits):
    -> (u [N], saved) for ``backward_raw``.  What a graph-replayed mapping
    iteration runs (wgsr.online); the launches and arithmetic are
    ``_MLPFn``'s."""
    N, C = x.shape
    dev = x.device
    L = _lib.load()
    l1, l2, lo = net.layers[0], net.layers[1], net.output_layer
    ws = [t.detach() for t in (l1.weight, l1.bias, l2.weight, l2.bias, lo.weight, lo.bias)]
    h1d = torch.empty(N, HIDDEN, device=dev)
    h2d = torch.empty(N, HIDDEN, device=dev)
    o = torch.empty(N, device=dev)
    u = torch.empty(N, device=dev)
    pt = _lib.ptr
    with torch.cuda.device(dev):
        _lib.check(L.wgsr_mlp_forward_dev_seed(N, C, pt(x), *[pt(t) for t in ws], float(net.dropout_p), pt(seed_dev),
                                               pt(h1d), pt(h2d), pt(o), pt(u), _lib.stream_handle(dev)))
    return u, (x, ws[2], ws[4], h1d, h2d, o, float(net.dropout_p))


def backward_raw(saved, du, scale: float = 1.0, accumulate_into=None):
    """-> the flat parameter gradient (wgsr_mlp_grad_floats(C) floats, the
    parameters' order) of a ``forward_raw`` for dL/du = scale * du [N]; with
    ``accumulate_into`` (an earlier result) the gradient is added to it in
    place (autograd's accumulation of a second backward) and it is returned."""
    x, W2, W3, h1d, h2d, o, p = saved
    N, C = x.shape
    dev = x.device
    L = _lib.load()
    grad = accumulate_into if accumulate_into is not None else torch.empty(int(L.wgsr_mlp_grad_floats(C)), device=dev)
    scratch = torch.empty(max(1, int(L.wgsr_mlp_scratch_bytes(N, C)) // 4), device=dev)
    pt = _lib.ptr
    with torch.cuda.device(dev):
        _lib.check(L.wgsr_mlp_backward_acc(N, C, pt(x), pt(W2), pt(W3), p, pt(h1d), pt(h2d), pt(o), pt(du),
                                           float(scale), int(accumulate_into is not None), pt(scratch), pt(grad),
                                           _lib.stream_handle(dev)))
    return grad


def forward_raw2(net, x1, x2, seed1_dev, seed2_dev):
    """``forward_raw`` of x1 [N1, C] (dropout seed ``seed1_dev``) and of x2
    [N2, C] (``seed2_dev``) in one launch (wgsr_mlp_forward_seg2): -> (u
    [N1 + N2], saved) for ``backward_raw2``; each segment's dropout draw and
    output are those of its own ``forward_raw``."""
    N1, C = x1.shape
    N2 = x2.shape[0]
    dev = x1.device
    L = _lib.load()
    l1, l2, lo = net.layers[0], net.layers[1], net.output_layer
    ws = [t.detach() for t in (l1.weight, l1.bias, l2.weight, l2.bias, lo.weight, lo.bias)]
    N = N1 + N2
    h1d = torch.empty(N, HIDDEN, device=dev)
    h2d = torch.empty(N, HIDDEN, device=dev)
    o = torch.empty(N, device=dev)
    u = torch.empty(N, device=dev)
    pt = _lib.ptr
    with torch.cuda.device(dev):
        _lib.check(L.wgsr_mlp_forward_seg2(N1, N2, C, pt(x1), pt(x2), *[pt(t) for t in ws], float(net.dropout_p),
                                           pt(seed1_dev), pt(seed2_dev), pt(h1d), pt(h2d), pt(o), pt(u),
                                           _lib.stream_handle(dev)))
    return u, (x1, x2, ws[2], ws[4], h1d, h2d, o, float(net.dropout_p))


def backward_raw2(saved, du1, du2, scale1: float = 1.0, scale2: float = 1.0, accumulate_into=None):
    """-> the flat parameter gradient of a ``forward_raw2`` for upstream
    gradients scale1 x du1 [N1] and scale2 x du2 [N2] (one backward launch
    over both segments; ``accumulate_into`` as in ``backward_raw``)."""
    x1, x2, W2, W3, h1d, h2d, o, p = saved
    N1, C = x1.shape
    N2 = x2.shape[0]
    dev = x1.device
    L = _lib.load()
    grad = accumulate_into if accumulate_into is not None else torch.empty(int(L.wgsr_mlp_grad_floats(C)), device=dev)
    scratch = torch.empty(max(1, int(L.wgsr_mlp_scratch_bytes(N1 + N2, C)) // 4), device=dev)
    pt = _lib.ptr
    with torch.cuda.device(dev):
        _lib.check(L.wgsr_mlp_backward_seg2(N1, N2, C, pt(x1), pt(x2), pt(W2), pt(W3), p, pt(h1d), pt(h2d), pt(o),
                                            pt(du1), pt(du2), float(scale1), float(scale2),
                                            int(accumulate_into is not None), pt(scratch), pt(grad),
                                            _lib.stream_handle(dev)))
    return grad


class UncertaintyMLP(nn.Module):
    """MLPNetwork(input_dim=C) with the reference defaults, on libwgsr."""

    def __init__(self, input_dim: int = 384, hidden_dim: int = 64, output_dim: int = 1, net_depth: int = 2,
                 weight_init: str = "he_uniform", dropout_p: float = 0.2):
        super().__init__()
        if hidden_dim != HIDDEN or output_dim != 1 or net_depth != 2:
            raise NotImplementedError("UncertaintyMLP: the reference defaults only (hidden 64, depth 2, output 1)")
        if input_dim % 64:
            raise NotImplementedError("UncertaintyMLP: input_dim must be a multiple of 64")
        self.output_layer_input_dim = hidden_dim
        self.layers = nn.ModuleList()
        for i in range(net_depth):
            layer = nn.Linear(input_dim if i == 0 else hidden_dim, hidden_dim)
            if weight_init == "he_uniform":
                nn.init.kaiming_uniform_(layer.weight, nonlinearity="relu")
            elif weight_init == "xavier_uniform":
                nn.init.xavier_uniform_(layer.weight)
            else:
                raise NotImplementedError(f"Unknown Weight initialization method {weight_init}")
            self.layers.append(layer)
        self.output_layer = nn.Linear(hidden_dim, output_dim)
        nn.init.kaiming_uniform_(self.output_layer.weight, nonlinearity="relu")
        self.dropout_p = float(dropout_p)
        self.last_seed = None
        self.seed_source = None  # optional callable -> the next forward's dropout seed (tests feed fixtures)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        H, W, C = x.shape[-3:]
        batched = x.dim() == 4
        flat = x.reshape(-1, C)
        if flat.dtype != torch.float32 or not flat.is_cuda:
            raise RuntimeError("UncertaintyMLP: fp32 device features only (the HIP path has no CPU fallback)")
        if self.seed_source is not None:
            seed = int(self.seed_source())
        else:
            seed = int(torch.randint(0, 2 ** 31 - 1, (1,)).item())  # host generator: no device sync
        self.last_seed = seed
        l1, l2, lo = self.layers[0], self.layers[1], self.output_layer
        u = _MLPFn.apply(flat, l1.weight, l1.bias, l2.weight, l2.bias, lo.weight, lo.bias, self.dropout_p, seed)
        return u.view(x.shape[0], H, W) if batched else u.view(H, W)


def generate_uncertainty_mlp(n_features: int) -> UncertaintyMLP:
    """uncertainty_model.generate_uncertainty_mlp (:66-68)."""
    return UncertaintyMLP(input_dim=n_features).cuda()
