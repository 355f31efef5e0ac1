"""The graph-replayed mapping iteration (wgsr.online_graph) and the pieces it
is built from, against their eager counterparts:

* wgsr_rasterize_forward_cap (capacity mode, no host wait) renders exactly
  what wgsr_rasterize_forward renders, reports upstream's num_rendered in
  counts[0], and its backward (num_rendered = cap) matches; an overflow
  (cap < N_rect) is flagged and leaves all-zero gradients;
* wgsr_adam_step_dev (device scalars, skip word, L2 weight decay) equals
  wgsr_adam_step / torch.optim.Adam;
* wgsr_mlp_forward_dev_seed equals wgsr_mlp_forward with the same seed, and
  wgsr_random_keys equals its numpy restatement;
* OnlineMapper.map_opt_online / final_refine with graphs: the same map, MLP
  and exposures as the eager loop from the same seeds, iterations replayed,
  and a forced capacity overflow recovers (recapture, event recorded).
"""
import numpy as np
import pytest
import torch

from test_gpu_online import _keyframes

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _scene(P=20000, W=160, H=120, seed=0):
    from wgsr.camera import synthetic_camera
    g = torch.Generator().manual_seed(seed)
    xyz = (torch.rand(P, 3, generator=g) - 0.5) * torch.tensor([4.0, 3.0, 2.0]) + torch.tensor([0.0, 0.0, 5.0])
    scales = torch.full((P, 3), 0.03) * (0.5 + torch.rand(P, 3, generator=g))
    rots = torch.nn.functional.normalize(torch.randn(P, 4, generator=g), dim=1)
    opac = 0.2 + 0.7 * torch.rand(P, 1, generator=g)
    shs = torch.randn(P, 1, 3, generator=g) * 0.5
    cam = synthetic_camera(W, H).raster_fields()
    cam = {k: (v.to(DEV) if torch.is_tensor(v) else v) for k, v in cam.items()}
    return [t.to(DEV).contiguous() for t in (xyz, opac, scales, rots, shs)], cam, W, H


def _backward(args, cam, fwd, W, H, dcol, ddep):
    from diff_gaussian_rasterization import _C
    xyz, opac, scales, rots, shs = args
    e = torch.empty(0, device=DEV)
    return _C.rasterize_gaussians_backward(torch.zeros(3, device=DEV), xyz, fwd[2], e, scales, rots, 1.0, e,
                                           cam["viewmatrix"], cam["projmatrix"], cam["projmatrix_raw"],
                                           cam["tanfovx"], cam["tanfovy"], dcol, ddep, shs, 0, cam["campos"],
                                           fwd[3], fwd[0], fwd[4], fwd[5], False)


def test_capacity_forward_matches_and_overflow_zeroes_gradients():
    from diff_gaussian_rasterization import _C
    from wgsr.mapping import rasterize_forward_cap
    args, cam, W, H = _scene()
    xyz, opac, scales, rots, shs = args
    bg = torch.zeros(3, device=DEV)
    e = torch.empty(0, device=DEV)
    ref = _C.rasterize_gaussians(bg, xyz, e, opac, scales, rots, 1.0, e, cam["viewmatrix"], cam["projmatrix"],
                                 cam["projmatrix_raw"], cam["tanfovx"], cam["tanfovy"], H, W, shs, 0, cam["campos"],
                                 False, False)
    N = ref[0]
    assert N > 1000
    counts = torch.zeros(5, dtype=torch.int32, device=DEV)
    out = rasterize_forward_cap(bg, xyz, opac, scales, rots, shs, 0, cam, H, W, N + 12345, counts)
    c = counts.cpu().tolist()
    assert c[0] == N and c[3] == 0 and 0 < c[2] <= c[1] <= N and c[4] == c[2]
    for i in (1, 2, 6, 7, 8):
        assert torch.equal(out[i], ref[i]), i
    g = torch.Generator(device=DEV).manual_seed(1)
    dcol = torch.randn(3, H, W, device=DEV, generator=g)
    ddep = torch.randn(1, H, W, device=DEV, generator=g)
    gr = _backward(args, cam, ref, W, H, dcol, ddep)
    gc = _backward(args, cam, out, W, H, dcol, ddep)
    for a, b in zip(gr, gc):
        assert torch.equal(a, b)
    # overflow: flagged, no host error, every gradient zero
    counts.zero_()
    small = rasterize_forward_cap(bg, xyz, opac, scales, rots, shs, 0, cam, H, W, N // 3, counts)
    c = counts.cpu().tolist()
    assert c[0] == N and c[3] == 1 and c[4] == min(c[2], N // 3)
    # the truncated forward's tile lists stay inside the capacity-sized region
    from wgsr.mapping import check_tile_lists
    bad = torch.zeros(3, dtype=torch.int32, device=DEV)
    for f in (ref, out, small):
        check_tile_lists(f, xyz, cam, H, W, 0, shs, bad)
    assert bad.tolist() == [0, 0, 0]
    # (and it sees a broken one: tile 0's range -- the image buffer's first
    # word pair -- pointed past the region)
    img = out[5].clone()
    img[:8].view(torch.int32).copy_(torch.tensor([0, 1 << 30], dtype=torch.int32))
    check_tile_lists(out[:5] + (img,) + out[6:], xyz, cam, H, W, 0, shs, bad)
    assert bad.tolist()[0] == 1
    go = _backward(args, cam, small, W, H, dcol, ddep)
    for t in go:
        assert not t.any()
    # the activation backward's densification statistics skip on the same word
    # (an overflowed replay must not count denom / max_radii2D)
    from wgsr import _lib
    L = _lib.load()
    P = xyz.shape[0]
    p = _lib.ptr
    raw_o, raw_s, raw_r = torch.randn(P, 1, device=DEV), torch.randn(P, 3, device=DEV), torch.randn(P, 4, device=DEV)
    g_o, g_s, g_r = torch.randn(P, 1, device=DEV), torch.randn(P, 3, device=DEV), torch.randn(P, 4, device=DEV)
    d_o, d_s, d_r = torch.empty_like(g_o), torch.empty_like(g_s), torch.empty_like(g_r)
    for skip_set, radii, m2d in ((True, small[2], go[0]), (False, ref[2], gr[0])):
        mr, acc, den = torch.full((P,), 2.0, device=DEV), torch.full((P, 1), 0.5, device=DEV), torch.ones(P, 1,
                                                                                                         device=DEV)
        word = counts[3:4] if skip_set else torch.zeros(1, dtype=torch.int32, device=DEV)
        _lib.check(L.wgsr_gaussian_activate_backward_stats(
            P, p(raw_o), p(raw_s), p(raw_r), p(g_o), p(g_s), p(g_r), 0.0, p(d_o), p(d_s), p(d_r), p(radii), p(m2d),
            p(mr), p(acc), p(den), p(word), _lib.stream_handle(DEV)))
        torch.cuda.synchronize()
        vis = radii > 0
        assert vis.any()
        if skip_set:
            assert (mr == 2.0).all() and (acc == 0.5).all() and (den == 1.0).all()
        else:
            assert (den[vis] == 2.0).all() and (den[~vis] == 1.0).all()
            assert torch.equal(mr[vis], torch.maximum(radii[vis].float(), torch.tensor(2.0, device=DEV)))


def test_adam_step_dev_matches_host_scalars_and_torch_weight_decay():
    from wgsr import _lib
    L = _lib.load()
    g = torch.Generator(device=DEV).manual_seed(3)
    n = 1037
    mk = lambda: torch.randn(n, device=DEV, generator=g)  # noqa: E731
    p, gr, m, v = mk(), mk(), mk().abs() * 0.1, mk().abs() * 0.01
    st = _lib.stream_handle(DEV)
    outs = []
    for dev_mode in (False, True):
        pp, mm, vv = p.clone(), m.clone(), v.clone()
        t = _lib.AdamTensor(pp.data_ptr(), gr.data_ptr(), mm.data_ptr(), vv.data_ptr(), n, 1e-3 / 0.1, 0.03)
        arr = (_lib.AdamTensor * 1)(t)
        if dev_mode:
            sc = torch.tensor([1e-3 / 0.1, 0.03, 0.0], device=DEV)
            skip = torch.zeros(1, dtype=torch.int32, device=DEV)
            _lib.check(L.wgsr_adam_step_dev(arr, 1, 0.9, 0.999, 1e-15, 0.0, sc.data_ptr(), skip.data_ptr(), st))
        else:
            _lib.check(L.wgsr_adam_step(arr, 1, 0.9, 0.999, 1e-15, st))
        outs.append((pp, mm, vv))
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    # skip word set: nothing moves
    pp, mm, vv = p.clone(), m.clone(), v.clone()
    t = _lib.AdamTensor(pp.data_ptr(), gr.data_ptr(), mm.data_ptr(), vv.data_ptr(), n, 1.0, 1.0)
    sc = torch.tensor([1.0, 1.0, 0.0], device=DEV)
    skip = torch.ones(1, dtype=torch.int32, device=DEV)
    _lib.check(L.wgsr_adam_step_dev((_lib.AdamTensor * 1)(t), 1, 0.9, 0.999, 1e-8, 0.0, sc.data_ptr(),
                                    skip.data_ptr(), st))
    assert torch.equal(pp, p) and torch.equal(mm, m) and torch.equal(vv, v)
    # weight decay: torch.optim.Adam(weight_decay=wd), three steps
    wd, lr = 1e-2, 4e-3
    ref = p.clone().requires_grad_(True)
    opt = torch.optim.Adam([ref], lr=lr, weight_decay=wd)
    pp = p.clone()
    mm, vv = torch.zeros_like(p), torch.zeros_like(p)
    for k in range(1, 4):
        gk = mk()
        ref.grad = gk.clone()
        opt.step()
        t = _lib.AdamTensor(pp.data_ptr(), gk.data_ptr(), mm.data_ptr(), vv.data_ptr(), n, 0.0, 1.0)
        sc = torch.tensor([lr / (1 - 0.9 ** k), (1 - 0.999 ** k) ** 0.5, 0.0], device=DEV)
        _lib.check(L.wgsr_adam_step_dev((_lib.AdamTensor * 1)(t), 1, 0.9, 0.999, 1e-8, wd, sc.data_ptr(), None, st))
    torch.testing.assert_close(pp, ref.detach(), rtol=1e-5, atol=1e-6)


def test_mlp_device_seed_and_random_keys():
    from wgsr import _lib
    from wgsr.mlp import UncertaintyMLP, _mix32, forward_raw
    torch.manual_seed(0)
    net = UncertaintyMLP(128).to(DEV)
    x = torch.randn(300, 128, device=DEV)
    seed = 123456789
    net.seed_source = lambda: seed
    u_ref = net(x.view(1, 300, 128))[0]
    u, _ = forward_raw(net, x, torch.tensor([seed], dtype=torch.int32, device=DEV))
    assert torch.equal(u, u_ref)
    L = _lib.load()
    n = 5000
    keys = torch.empty(n, dtype=torch.int32, device=DEV)
    sd = torch.tensor([seed], dtype=torch.int32, device=DEV)
    _lib.check(L.wgsr_random_keys(n, 0, sd.data_ptr(), keys.data_ptr(), _lib.stream_handle(DEV)))
    with np.errstate(over="ignore"):
        i = np.arange(n, dtype=np.uint32)
        want = (_mix32(np.uint32(seed) ^ _mix32(i * np.uint32(0x9E3779B9) + np.uint32(0x632BE5AB))) >> 1)
    assert np.array_equal(keys.cpu().numpy(), want.astype(np.int32))


CFG = {"init_itr_num": 30, "init_gaussian_update": 100, "init_gaussian_reset": 10_000, "mapping_itr_num": 60,
       "gaussian_update_every": 100_000, "gaussian_update_offset": 99_999, "gaussian_reset": 100_001,
       "window_size": 4}


def _run(graphs: bool, cap=None, refine=0):
    from wgsr.online import OnlineMapper
    kfs = _keyframes(4)
    m = OnlineMapper(sh_degree=0, device=DEV, config=CFG, seed=3)
    if not graphs:
        m.graphs = None
    m.initialize(kfs[:2])
    # every forward's tile lists checked on the device (inside the captured
    # graphs too): ranges inside the capacity-sized list region, ids < P
    m.ms.list_check = torch.zeros(3, dtype=torch.int32, device=DEV)
    if graphs and cap is not None:  # capacities far below the pair counts: every map state overflows
        m.graphs.cap, m.graphs.min_cap, m.graphs.cap_scale, m.graphs.cap_margin = cap, cap, 0.25, 0
    for kf in kfs[2:]:
        m.insert_keyframe(kf, iters=60)
    if refine:
        m.iterations_after_densify_or_reset = 1000
        m.final_refine(refine)
    torch.cuda.synchronize()
    return m


def _state(m):
    out = {n: m.ms.store.param(n).clone() for n in m.ms.GROUPS}
    out.update({f"mlp{i}": p.detach().clone() for i, p in enumerate(m.net.parameters())})
    out["exposure"] = torch.stack([torch.cat([k.exposure_a, k.exposure_b]) for k in m.keyframes.values()])
    return out


def test_graph_replayed_loop_matches_eager():
    a = _state(_run(False, refine=40))
    mg = _run(True, refine=40)
    assert mg.ms.list_check.tolist() == [0, 0, 0]
    b = _state(mg)
    st = mg.graphs.stats
    assert st["replays"] > 100 and st["captures"] >= 2 and st["overflows"] == 0, st
    assert mg.graphs.disabled is None
    for k in a:
        assert a[k].shape == b[k].shape, k
        rel = float((a[k] - b[k]).norm() / a[k].norm().clamp_min(1e-12))
        assert rel <= 2e-3, (k, rel)


def test_graph_capacity_overflow_recovers():
    m = _run(True, cap=512)
    st = m.graphs.stats
    assert st["overflows"] >= 1 and st["skipped_iterations"] >= 1, st
    # the overflowed (truncated) forwards left consistent tile lists
    assert m.ms.list_check.tolist() == [0, 0, 0]
    assert any(k == "capacity_overflow" for _, k, _ in m.events)
    assert int(m.graphs.sticky_np[0]) == 0 or st["overflows"] >= 2
    for n in m.ms.GROUPS:
        assert torch.isfinite(m.ms.store.param(n)).all()


def test_random_perm_gather_exposure_step_and_mlp_accumulate():
    from wgsr import _lib
    from wgsr.mlp import UncertaintyMLP, _mix32, backward_raw, forward_raw
    L = _lib.load()
    st = _lib.stream_handle(DEV)
    p = _lib.ptr
    # wgsr_random_perm == numpy's stable argsort of the restated keys
    seed, n = 987654321, 4860
    keys = torch.empty(n, dtype=torch.int32, device=DEV)
    perm = torch.empty(n, dtype=torch.int32, device=DEV)
    _lib.check(L.wgsr_random_perm(n, seed, None, p(keys), p(perm), st))
    with np.errstate(over="ignore"):
        i = np.arange(n, dtype=np.uint32)
        want = (_mix32(np.uint32(seed) ^ _mix32(i * np.uint32(0x9E3779B9) + np.uint32(0x632BE5AB))) >> 1)
    assert np.array_equal(perm.cpu().numpy(), np.argsort(want.astype(np.int64), kind="stable"))
    assert int(L.wgsr_random_perm_max()) >= 4096
    # wgsr_gather_rows: rows by a device index, vector and scalar jobs, a strided source
    g = torch.Generator(device=DEV).manual_seed(0)
    bank = torch.randn(10, 3, 8, 12, device=DEV, generator=g)
    ex = torch.randn(10, 3, 2, device=DEV, generator=g)
    ex[:, 2].abs_()  # exp_avg_sq >= 0 (a negative one makes both steps NaN, and NaN != NaN)
    idx = torch.tensor([7, 2, 4, 9], dtype=torch.int64, device=DEV)
    d1 = torch.empty(1, 3, 8, 12, device=DEV)
    d3 = torch.empty(3, 3, 8, 12, device=DEV)
    de = torch.empty(2, device=DEV)
    jobs = (_lib.GatherJob * 3)(_lib.GatherJob(p(bank), p(d1), 288, 288, 0, 1),
                                _lib.GatherJob(p(bank), p(d3), 288, 288, 1, 3),
                                _lib.GatherJob(p(ex), p(de), 2, 6, 0, 1))
    _lib.check(L.wgsr_gather_rows(jobs, 3, p(idx), st))
    assert torch.equal(d1[0], bank[7]) and torch.equal(d3, bank[[2, 4, 9]]) and torch.equal(de, ex[7, 0])
    # wgsr_exposure_step == wgsr_adam_step on the same bank row; skip words; overflow bookkeeping
    grad = torch.randn(2, device=DEV, generator=g)
    sc = torch.tensor([0.01 / 0.1, 0.0316], device=DEV)
    ref = ex.clone()
    r = ref[7]
    t = _lib.AdamTensor(r[0].data_ptr(), grad.data_ptr(), r[1].data_ptr(), r[2].data_ptr(), 2, 0.01 / 0.1, 0.0316)
    _lib.check(L.wgsr_adam_step((_lib.AdamTensor * 1)(t), 1, 0.9, 0.999, 1e-8, st))
    zero = torch.zeros(1, dtype=torch.int32, device=DEV)
    one = torch.ones(1, dtype=torch.int32, device=DEV)
    counts = torch.tensor([1234, 0, 0, 0, 0], dtype=torch.int32, device=DEV)
    sticky = torch.tensor([0, 99], dtype=torch.int64, device=DEV)
    got = ex.clone()
    _lib.check(L.wgsr_exposure_step(p(got), p(idx), p(grad), 1, p(sc), p(zero), p(zero), 0.9, 0.999, 1e-8, p(sticky),
                                    p(counts), None, st))
    # (the same arithmetic as the Adam kernel; the compiler may contract its
    # multiply-adds differently in the two kernels: a few ulp)
    assert torch.allclose(got, ref, rtol=1e-6, atol=1e-7) and sticky.tolist() == [0, 1234]
    assert torch.equal(got[:7], ex[:7]) and torch.equal(got[8:], ex[8:])  # only the indexed row moves
    before = got.clone()
    counts[3] = 1
    slot_skips = torch.zeros(ex.shape[0], dtype=torch.int64, device=DEV)
    _lib.check(L.wgsr_exposure_step(p(got), p(idx), p(grad), 1, p(sc), p(one), p(zero), 0.9, 0.999, 1e-8, p(sticky),
                                    p(counts), p(slot_skips), st))
    # (a step the host did not count -- skip_b set -- is not a held-back one)
    _lib.check(L.wgsr_exposure_step(p(got), p(idx), p(grad), 1, p(sc), p(one), p(one), 0.9, 0.999, 1e-8, None, None,
                                    p(slot_skips), st))
    _lib.check(L.wgsr_exposure_step(p(got), p(idx), p(grad), 1, p(sc), p(zero), p(one), 0.9, 0.999, 1e-8, None, None,
                                    None, st))
    assert torch.equal(got, before) and sticky.tolist() == [1, 1234]
    want_sk = torch.zeros_like(slot_skips)
    want_sk[int(idx[0])] = 1
    assert torch.equal(slot_skips, want_sk)
    # the gradient as per-block partial rows, summed inside the step
    parts = torch.randn(768, 2, device=DEV, generator=g)
    got = ex.clone()
    _lib.check(L.wgsr_exposure_step(p(got), p(idx), p(parts), 768, p(sc), p(zero), p(zero), 0.9, 0.999, 1e-8, None,
                                    None, None, st))
    ref2 = ex.clone()
    gsum = parts.double().sum(0).float().contiguous()
    _lib.check(L.wgsr_exposure_step(p(ref2), p(idx), p(gsum), 1, p(sc), p(zero), p(zero), 0.9, 0.999, 1e-8, None,
                                    None, None, st))
    assert torch.allclose(got, ref2, rtol=1e-5, atol=1e-6)
    # MLP backward: scaled upstream gradient accumulated into an earlier one
    torch.manual_seed(1)
    net = UncertaintyMLP(384).to(DEV)
    x = torch.randn(303, 384, device=DEV)
    s = torch.tensor([42], dtype=torch.int32, device=DEV)
    _, sv = forward_raw(net, x, s)
    du1, du2 = torch.randn(303, device=DEV), torch.randn(303, device=DEV)
    G1 = backward_raw(sv, du1)
    want = G1 + backward_raw(sv, du2 * 0.5)
    got = backward_raw(sv, du2, scale=0.5, accumulate_into=G1.clone())
    assert torch.allclose(got, want, rtol=1e-6, atol=1e-6 * float(want.abs().max()))


@pytest.mark.gpu
def test_random_perm_prefix_and_mlp_two_segments():
    from wgsr import _lib
    from wgsr.mlp import UncertaintyMLP, _mix32, backward_raw, backward_raw2, forward_raw, forward_raw2
    L = _lib.load()
    st = _lib.stream_handle(DEV)
    p = _lib.ptr
    assert int(L.wgsr_random_perm_prefix_max_n()) >= 8192 and int(L.wgsr_random_perm_prefix_max_k()) >= 1024
    # the first k entries of the stable ascending key order, host and device seeds
    for seed, n, k in ((987654321, 4860, 303), (5, 1, 1), (77, 1000, 1000), (123, 8192, 1024), (9, 3000, 1)):
        perm = torch.full((k,), -1, dtype=torch.int32, device=DEV)
        _lib.check(L.wgsr_random_perm_prefix(n, k, seed, None, p(perm), st))
        with np.errstate(over="ignore"):
            i = np.arange(n, dtype=np.uint32)
            want = (_mix32(np.uint32(seed) ^ _mix32(i * np.uint32(0x9E3779B9) + np.uint32(0x632BE5AB))) >> 1)
        ref = np.argsort(want.astype(np.int64), kind="stable")[:k]
        assert np.array_equal(perm.cpu().numpy(), ref), (n, k)
        sd = torch.tensor([seed], dtype=torch.int64, device=DEV).to(torch.int32)
        perm2 = torch.full((k,), -1, dtype=torch.int32, device=DEV)
        _lib.check(L.wgsr_random_perm_prefix(n, k, 0, p(sd), p(perm2), st))
        assert torch.equal(perm, perm2)
    with pytest.raises(RuntimeError):
        _lib.check(L.wgsr_random_perm_prefix(100, 101, 1, None, p(perm), st))
    # two MLP segments in one launch == one launch per segment (outputs bitwise;
    # the summed gradient up to the order of the sums)
    torch.manual_seed(3)
    net = UncertaintyMLP(384).to(DEV)
    x1, x2 = torch.randn(972, 384, device=DEV), torch.randn(303, 384, device=DEV)
    s1 = torch.tensor([11], dtype=torch.int32, device=DEV)
    s2 = torch.tensor([-7], dtype=torch.int32, device=DEV)
    ua, sv = forward_raw2(net, x1, x2, s1, s2)
    u1, sv1 = forward_raw(net, x1, s1)
    u2, sv2 = forward_raw(net, x2, s2)
    assert torch.equal(ua, torch.cat([u1, u2]))
    assert torch.equal(sv[4], torch.cat([sv1[3], sv2[3]])) and torch.equal(sv[5], torch.cat([sv1[4], sv2[4]]))
    du1, du2 = torch.randn(972, device=DEV), torch.randn(303, device=DEV)
    G = backward_raw2(sv, du1, du2, 1.0, 0.5)
    want = backward_raw(sv1, du1) + backward_raw(sv2, du2 * 0.5)
    assert torch.allclose(G, want, rtol=1e-5, atol=1e-5 * float(want.abs().max()))
    Gacc = backward_raw2(sv, du1, du2, 1.0, 0.5, accumulate_into=want.clone())
    assert torch.allclose(Gacc, 2 * want, rtol=1e-5, atol=2e-5 * float(want.abs().max()))


@pytest.mark.gpu
def test_adam_two_optimisers_one_launch():
    """wgsr_adam_step_dev2 == wgsr_adam_step_dev per group (the Gaussians'
    eps / no decay, the MLP's eps / L2 decay), bit for bit."""
    from wgsr import _lib
    L = _lib.load()
    st = _lib.stream_handle(DEV)
    p = _lib.ptr
    g = torch.Generator(device=DEV).manual_seed(5)
    sizes = [(3000, 0), (4801, 3), (17, 0), (256, 0), (6, 0)]
    def make():
        out = []
        for n, _ in sizes:
            prm, grd = torch.randn(n, device=DEV, generator=g), torch.randn(n, device=DEV, generator=g)
            m, v = torch.randn(n, device=DEV, generator=g), torch.rand(n, device=DEV, generator=g)
            out.append([prm, grd, m, v])
        return out
    A, B = make(), make()
    sc1 = torch.rand(3 * 3, device=DEV, generator=g) + 0.5
    sc2 = torch.rand(2 * 3, device=DEV, generator=g) + 0.5
    skip = torch.zeros(1, dtype=torch.int32, device=DEV)
    def tens(T, lo, hi):
        return [_lib.AdamTensor(p(T[i][0]), p(T[i][1]), p(T[i][2]), p(T[i][3]), T[i][0].numel(), 0.0, 1.0)
                for i in range(lo, hi)]
    ref = [[t.clone() for t in row] for row in A]
    t1, t2 = tens(ref, 0, 3), tens(ref, 3, 5)
    _lib.check(L.wgsr_adam_step_dev((_lib.AdamTensor * 3)(*t1), 3, 0.9, 0.999, 1e-15, 0.0, p(sc1), p(skip), st))
    _lib.check(L.wgsr_adam_step_dev((_lib.AdamTensor * 2)(*t2), 2, 0.9, 0.999, 1e-8, 1e-5, p(sc2), p(skip), st))
    got = [[t.clone() for t in row] for row in A]
    ta = tens(got, 0, 5)
    _lib.check(L.wgsr_adam_step_dev2((_lib.AdamTensor * 5)(*ta), 3, 5, 0.9, 0.999, 1e-15, 0.0, p(sc1), 1e-8, 1e-5,
                                     p(sc2), p(skip), st))
    for r, q in zip(ref, got):
        for a, b in zip(r, q):
            assert torch.equal(a, b)
