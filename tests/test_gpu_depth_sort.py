"""The depth orderings of the forward against each other:

* the Gaussian-level depth sort over the visible key range (csrc/sort.hip
  launch_depth_sort, DepthKeyPlan in csrc/wgsr_common.h; WGSR_DEPTH_SORT=
  global) against the four 8-bit passes over the whole 32-bit keys
  (WGSR_DEPTH_SORT=full): identical depth order and outputs;
* the default, per-bin depth sort after the bin sort (csrc/raster_fwd.hip
  k_bin_depth_sort: pairs duplicated in index order, every sort bin ordered by
  depth key, ties by index), which has no Gaussian-level order: every raster
  output bit-identical to the global schedules, incl. bins larger than one
  LDS tile (the chunked pass through global scratch; its keys gathered from
  the Gaussians' depth keys through each bin's ids).

Both are stable sorts of the same keys, so the depth order (rank -> Gaussian,
read from the geometry buffer at wgsr_depth_order_offset()) and every raster
output must be bit-identical.  The scenes cover each branch of the plan:
depth ranges giving 24 key bits (three 8-bit passes), 26 and 28 bits (9- and
10-bit digit passes), 29+ bits (far Gaussians: the host-queued fix-up pass and
the re-run scan), equal depths (ties keep index order), Gaussians behind the
camera (culled: last), nothing visible, a single Gaussian, and the three
workgroup-tile tiers (<= 256k, <= 2M, more keys).
"""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
W, H = 512, 384


def _scene(P, zlo, zhi, seed=0, far=0, behind=0, ties=0, log_z=False):
    g = torch.Generator().manual_seed(seed)
    tanx = 1.0 / (2.0 * 0.9)
    tany = H / (2.0 * 0.9 * W)
    r = torch.rand(P, generator=g)
    z = torch.exp(math.log(zlo) + (math.log(zhi) - math.log(zlo)) * r) if log_z else zlo + (zhi - zlo) * r
    u = torch.rand(P, generator=g) * 2 - 1
    v = torch.rand(P, generator=g) * 2 - 1
    if far:
        z[:far] = 1e12 * (1.0 + torch.rand(far, generator=g))
    if behind:
        z[far:far + behind] = -1.0 - torch.rand(behind, generator=g)
    means = torch.stack([u * z * tanx * 0.9, v * z * tany * 0.9, z], dim=1)
    if ties:  # identical means (e.g. clones after densification): equal depth keys
        means[P - ties:] = means[far + behind:far + behind + ties]
    scales = torch.exp(math.log(0.004) + (math.log(0.03) - math.log(0.004)) * torch.rand(P, 3, generator=g))
    q = torch.randn(P, 4, generator=g)
    q = q / q.norm(dim=1, keepdim=True)
    opac = 0.05 + 0.9 * torch.rand(P, 1, generator=g)
    shs = torch.randn(P, 1, 3, generator=g) * 0.5
    return means, scales, q, opac, shs


def _forward(scene, w=W, h=H):
    from diff_gaussian_rasterization import _C
    from wgsr import _lib
    from wgsr.camera import synthetic_camera
    f = synthetic_camera(w, h, 0).raster_fields()
    d = lambda x: x.to(DEV).contiguous()  # noqa: E731
    means, scales, q, opac, shs = (d(x) for x in scene)
    e = torch.empty(0, device=DEV)
    out = _C.rasterize_gaussians(d(torch.zeros(3)), means, e, opac, scales, q, 1.0, e, d(f["viewmatrix"]),
                                 d(f["projmatrix"]), d(f["projmatrix_raw"]), f["tanfovx"], f["tanfovy"], h, w,
                                 shs, 0, d(f["campos"]), False, False)
    torch.cuda.synchronize()
    off = int(_lib.load().wgsr_depth_order_offset())
    geom = out[3]
    P = means.shape[0]
    order = geom[off:off + 4 * P].cpu().numpy().view(np.uint32).copy() if off >= 0 else None
    res = dict(num_rendered=out[0], color=out[1].cpu().numpy(), radii=out[2].cpu().numpy(),
               depth=out[6].cpu().numpy(), opacity=out[7].cpu().numpy(), n_touched=out[8].cpu().numpy())
    return order, res


def _same_outputs(ra, rb, tag):
    for k, v in ra.items():
        if k == "num_rendered":
            assert rb[k] == v, tag
        else:
            np.testing.assert_array_equal(rb[k], v, err_msg=f"{tag}: {k}")


def _compare(scene, monkeypatch, w=W, h=H):
    outs = {}
    # (bins: the per-bin sort whatever the bins' load -- no fallback)
    monkeypatch.setenv("WGSR_BIN_DEPTH_MAX_AVG", str(1 << 40))
    for mode in ("full", "global", "bins"):
        monkeypatch.setenv("WGSR_DEPTH_SORT", mode)
        outs[mode] = _forward(scene, w, h)
    (o_full, r_full), (o_rng, r_rng), (o_bins, r_bins) = outs["full"], outs["global"], outs["bins"]
    P = scene[0].shape[0]
    assert np.array_equal(np.sort(o_rng), np.arange(P, dtype=np.uint32))  # a permutation
    np.testing.assert_array_equal(o_rng, o_full)
    assert o_bins is None  # (per-bin ordering: no Gaussian-level depth order)
    _same_outputs(r_full, r_rng, "global vs full")
    _same_outputs(r_full, r_bins, "bins vs full")
    return o_rng, r_full


@pytest.mark.parametrize("P,zlo,zhi,log_z", [
    (100_000, 2.0, 8.0, False),      # 24 key bits: three 8-bit passes
    (60_000, 0.25, 60.0, True),      # 26 bits: 8 + 9 + 9
    (60_000, 0.21, 3.0e4, True),     # 28 bits: 8 + 10 + 10
    (300_000, 0.5, 5.0, False),      # 2048-key tiles
])
def test_depth_sort_matches_full_key_sort(P, zlo, zhi, log_z, monkeypatch):
    _compare(_scene(P, zlo, zhi, log_z=log_z, behind=P // 50, ties=P // 20), monkeypatch)


def test_far_gaussians_take_the_fixup_pass(monkeypatch):
    """Visible Gaussians at 1e12 m next to ones at 0.3 m: the key range needs
    29+ bits, so the host queues one more pass after reading the range."""
    scene = _scene(20_000, 0.3, 10.0, far=40, behind=100, ties=500, log_z=True)
    order, res = _compare(scene, monkeypatch)
    radii = res["radii"]
    far_visible = np.nonzero(radii[:40] > 0)[0]
    assert far_visible.size > 0  # the far ones are on screen, so the range really is that wide
    ranks = np.empty_like(order)
    ranks[order] = np.arange(order.size, dtype=np.uint32)
    visible = np.nonzero(radii > 0)[0]
    # the far ones come right before the culled ones
    assert set(order[visible.size - far_visible.size:visible.size].tolist()) == set(far_visible.tolist())


def test_nothing_visible_and_tiny_inputs(monkeypatch):
    s = _scene(5_000, 1.0, 4.0, behind=5_000)
    order, res = _compare(s, monkeypatch)
    np.testing.assert_array_equal(order, np.arange(5_000, dtype=np.uint32))  # all culled: index order
    assert res["num_rendered"] == 0
    _compare(_scene(1, 1.0, 4.0), monkeypatch)
    _compare(_scene(7, 1.0, 1.0 + 1e-6), monkeypatch)  # all depths within a few ulps: R <= 8


def test_large_tile_tier(monkeypatch):
    """More than 2M keys: 4096-key workgroup tiles."""
    _compare(_scene(2_200_000, 1.0, 12.0, behind=10_000, ties=50_000), monkeypatch)


def test_depth_order_is_by_depth_then_index(monkeypatch):
    """Independently of the full-key sort: the visible Gaussians come first,
    by non-decreasing view depth (the splat's depth word), equal depths in
    index order."""
    monkeypatch.setenv("WGSR_DEPTH_SORT", "global")
    scene = _scene(50_000, 0.4, 20.0, behind=500, ties=3_000, log_z=True)
    order, res = _forward(scene)
    z = scene[0][:, 2].numpy().astype(np.float32)
    vis = res["radii"] > 0
    nv = int(vis.sum())
    assert vis[order[:nv]].all() and not vis[order[nv:]].any()
    zs = z[order[:nv]]  # view depth = z for the identity camera (view 0)
    assert np.all(np.diff(zs) >= 0)
    same = np.diff(zs) == 0
    assert np.all(np.diff(order[:nv].astype(np.int64))[same] > 0)
    np.testing.assert_array_equal(order[nv:], np.sort(order[nv:]))


def _clustered(P, cx, cy, spread, seed=3):
    """P small Gaussians whose centres fall inside a few pixels around
    (cx, cy) of the W x H view: one sort bin holds (nearly) all of them."""
    means, scales, q, opac, shs = _scene(P, 1.0, 6.0, seed=seed, ties=P // 10, log_z=True)
    z = means[:, 2]
    tanx = 1.0 / (2.0 * 0.9)
    tany = H / (2.0 * 0.9 * W)
    g = torch.Generator().manual_seed(seed + 1)
    u = (cx + spread * (torch.rand(P, generator=g) - 0.5)) / W * 2 - 1
    v = (cy + spread * (torch.rand(P, generator=g) - 0.5)) / H * 2 - 1
    means = torch.stack([u * z * tanx, v * z * tany, z], dim=1)
    means[P - P // 10:] = means[:P // 10]  # exact ties
    return means, scales * 0.05, q, opac, shs


@pytest.mark.parametrize("P", [9_000, 40_000])
def test_bin_beyond_one_lds_tile(P, monkeypatch):
    """A bin with more entries than k_bin_depth_sort sorts in LDS (8192):
    the chunked passes through global scratch give the same images."""
    _compare(_clustered(P, 200.0, 150.0, 6.0), monkeypatch)


def test_bin_sort_1080p_bins(monkeypatch):
    """4 x 4-tile bins (frames beyond 2048 tiles), with one crowded bin."""
    a = _scene(150_000, 0.5, 9.0, behind=1_000, ties=5_000, log_z=True)
    b = _clustered(20_000, 300.0, 200.0, 10.0, seed=9)
    scene = tuple(torch.cat([x, y]) for x, y in zip(a, b))
    _compare(scene, monkeypatch, 1920, 1080)


def test_bins_too_full_fall_back_to_the_gaussian_sort(monkeypatch):
    """Above WGSR_BIN_DEPTH_MAX_AVG entries per bin the host, at its one wait,
    queues the Gaussian-level depth sort and redoes the scan in depth order:
    the same outputs as the global schedule (and a depth order again)."""
    scene = _scene(60_000, 0.3, 12.0, behind=600, ties=2_000, log_z=True)
    monkeypatch.setenv("WGSR_DEPTH_SORT", "global")
    o_glob, r_glob = _forward(scene)
    monkeypatch.setenv("WGSR_DEPTH_SORT", "bins")
    monkeypatch.setenv("WGSR_BIN_DEPTH_MAX_AVG", "0")
    o_fb, r_fb = _forward(scene)
    assert o_fb is not None
    np.testing.assert_array_equal(o_fb, o_glob)
    _same_outputs(r_glob, r_fb, "fallback vs global")


def _forward_backward(scene, deg, w, h):
    from diff_gaussian_rasterization import _C
    from wgsr.camera import synthetic_camera
    f = synthetic_camera(w, h, 0).raster_fields()
    d = lambda x: x.to(DEV).contiguous()  # noqa: E731
    means, scales, q, opac, shs = (d(x) for x in scene)
    e = torch.empty(0, device=DEV)
    bg = d(torch.zeros(3))
    cam = [d(f["viewmatrix"]), d(f["projmatrix"]), d(f["projmatrix_raw"])]
    nr, color, radii, geom, binning, img, depth, opac_o, nt = _C.rasterize_gaussians(
        bg, means, e, opac, scales, q, 1.0, e, *cam, f["tanfovx"], f["tanfovy"], h, w, shs, deg,
        d(f["campos"]), False, False)
    g = torch.Generator().manual_seed(5)
    gc = d(torch.randn(3, h, w, generator=g))
    gd = d(torch.randn(1, h, w, generator=g))
    grads = _C.rasterize_gaussians_backward(bg, means, radii, e, scales, q, 1.0, e, *cam, f["tanfovx"], f["tanfovy"],
                                            gc, gd, shs, deg, d(f["campos"]), geom, nr, binning, img, False)
    torch.cuda.synchronize()
    return nr, [x.cpu().numpy() for x in grads]


@pytest.mark.parametrize("w,h", [(512, 384), (1920, 1080)])
def test_backward_identical_across_depth_schedules(w, h, monkeypatch):
    """The per-Gaussian backward finds a Gaussian's record slots two ways: from
    two index-ordered slot_start words (the per-bin schedule flags that its
    slots follow the index order, ImageLayout::meta[2]) or by gathering
    slot_start and the list length of each live row (the depth-ordered
    schedules).  Same tile lists, same slots within each Gaussian, same sums:
    every gradient is bit-identical."""
    means, scales, q, opac, shs = _scene(80_000, 0.4, 9.0, behind=800, ties=4_000, log_z=True)
    g = torch.Generator().manual_seed(7)
    shs = torch.cat([shs, 0.1 * torch.randn(shs.shape[0], 15, 3, generator=g)], dim=1)  # SH3
    scene = (means, scales, q, opac, shs)
    monkeypatch.setenv("WGSR_BIN_DEPTH_MAX_AVG", str(1 << 40))
    out = {}
    for mode in ("global", "bins"):
        monkeypatch.setenv("WGSR_DEPTH_SORT", mode)
        out[mode] = _forward_backward(scene, 3, w, h)
    (n_g, g_g), (n_b, g_b) = out["global"], out["bins"]
    assert n_g == n_b and n_g > 0
    names = ("means2D", "colors", "opacity", "means3D", "cov3D", "sh", "scales", "rotations", "tau")
    assert any(np.abs(x).max() > 0 for x in g_b)
    for name, a, b in zip(names, g_g, g_b):
        np.testing.assert_array_equal(b, a, err_msg=name)
