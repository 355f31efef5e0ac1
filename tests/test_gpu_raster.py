"""GPU parity tests: the gfx950 path (libwgsr.so through the drop-in
``diff_gaussian_rasterization`` / ``simple_knn`` API) against the oracle.

Tolerances (written here, SURVEY.md 8(c), north_star "<= 1e-4 rel L1"):
  images (colour, depth, opacity)      rel-L1 <= 1e-4
  radii, num_rendered                  exact (the preprocess arithmetic is
                                       bit-identical to the CPU restatement)
  n_touched                            exact on the golden scenes; against
                                       the fp32 CPU restatement exact for
                                       every Gaussian none of whose blend
                                       decisions sits within rounding slack
                                       of a threshold (T vs 0.5, alpha vs
                                       1/255, power vs 0: exp() rounds
                                       differently in every math library, the
                                       upstream CUDA expf included), and
                                       within [firm, firm + soft] for the
                                       rest (oracle/cpu_raster.cpp)
  per-tensor gradients                 rel-L1 <= 1e-4
  pose gradient (summed over P)        rel-L1 <= 1e-3
  distCUDA2                            bit-exact vs the CPU restatement
"""
import math
import os

import numpy as np
import pytest
import torch

from _util import GRAD_KEYS, load_scene, rel_l1, scene_names
from oracle import cpu_oracle

pytestmark = pytest.mark.gpu

IMG_TOL = 1e-4
GRAD_TOL = 1e-4
TAU_TOL = 1e-3
DEV = "cuda"


def _c():
    from diff_gaussian_rasterization import _C
    return _C


def run_c(inputs, settings, grads, debug=False, between=None):
    """Forward + backward through the exact upstream ``_C`` ABI
    (``between()`` runs after the forward, before the backward)."""
    C = _c()
    d = lambda x: None if x is None else x.to(DEV)  # noqa: E731
    e = torch.empty(0, device=DEV)
    st = settings
    shs = d(inputs.get("shs"))
    colors = d(inputs.get("colors_precomp"))
    scales, rots, cov = d(inputs.get("scales")), d(inputs.get("rotations")), d(inputs.get("cov3D_precomp"))
    means = d(inputs["means3D"])
    args = (d(st["bg"]), means, colors if colors is not None else e, d(inputs["opacities"]),
            scales if scales is not None else e, rots if rots is not None else e,
            st["scale_modifier"], cov if cov is not None else e, d(st["viewmatrix"]),
            d(st["projmatrix"]), d(st["projmatrix_raw"]), st["tanfovx"], st["tanfovy"], st["H"],
            st["W"], shs if shs is not None else e, st["sh_degree"], d(st["campos"]), False, debug)
    (nr, color, radii, geom, binning, img, depth, opac, ntouch) = C.rasterize_gaussians(*args)
    if between is not None:
        between()
    bargs = (d(st["bg"]), means, radii, colors if colors is not None else e,
             scales if scales is not None else e, rots if rots is not None else e,
             st["scale_modifier"], cov if cov is not None else e, d(st["viewmatrix"]),
             d(st["projmatrix"]), d(st["projmatrix_raw"]), st["tanfovx"], st["tanfovy"],
             d(grads[0]), d(grads[1]), shs if shs is not None else e, st["sh_degree"],
             d(st["campos"]), geom, nr, binning, img, debug)
    g = C.rasterize_gaussians_backward(*bargs)
    torch.cuda.synchronize()
    names = ("dL_dmeans2D", "dL_dcolors", "dL_dopacity", "dL_dmeans3D", "dL_dcov3D", "dL_dsh",
             "dL_dscales", "dL_drotations", "dL_dtau")
    out = dict(num_rendered=nr, color=color.cpu().numpy(), radii=radii.cpu().numpy(),
               depth=depth.cpu().numpy(), opacity=opac.cpu().numpy(),
               n_touched=ntouch.cpu().numpy())
    out.update({k: v.cpu().numpy() for k, v in zip(names, g)})
    return out


PIX_TOL = 1e-4       # per-pixel abs error (relative to the image's max magnitude) ...
PIX_BAD_FRAC = 1e-5  # ... exceeded by at most this fraction of pixels (threshold flips)
PIX_FLIP_TOL = 1e-2  # and never by more than a couple of 1/255 threshold flips


def check_against(out, expect, grad_keys=GRAD_KEYS, exact_touched=False):
    assert out["num_rendered"] == expect["num_rendered"]
    np.testing.assert_array_equal(out["radii"], expect["radii"])
    if exact_touched or "n_touched_soft" not in expect:
        np.testing.assert_array_equal(out["n_touched"], expect["n_touched"])
    else:
        got, firm, soft = out["n_touched"], expect["n_touched_firm"], expect["n_touched_soft"]
        clear = soft == 0
        np.testing.assert_array_equal(got[clear], expect["n_touched"][clear])
        assert np.all((got >= firm) & (got <= firm + soft)), int(np.count_nonzero((got < firm) | (got > firm + soft)))
    for k in ("color", "depth", "opacity"):
        r = rel_l1(out[k], expect[k])
        assert r <= IMG_TOL, (k, r)
        # per pixel too: a (Gaussian, tile) pair wrongly left out of a tile list
        # (the exact lists cull pairs that cannot reach alpha >= 1/255) would
        # show as a patch of pixels far above fp32 noise.  Single pixels may
        # differ by one alpha = 1/255 threshold flip (__expf vs expf rounding):
        # <= alpha_min * T * c, a few 1e-3.
        scale = max(1.0, float(np.max(np.abs(expect[k]))))
        diff = np.abs(out[k] - expect[k])
        assert float(np.max(diff)) <= PIX_FLIP_TOL * scale, (k, "max abs", float(np.max(diff)))
        nbad = int(np.count_nonzero(diff > PIX_TOL * scale))
        assert nbad <= max(2, PIX_BAD_FRAC * diff.size), (k, "pixels off", nbad)
    for k in grad_keys:
        if k in expect and expect[k] is not None:
            got = out[k]
            if k == "dL_dsh":
                got = got[:, : expect[k].shape[1]]
            r = rel_l1(got, expect[k])
            assert r <= GRAD_TOL, (k, r)
    t = expect["dL_dtau"]
    got = out["dL_dtau"].sum(0) if out["dL_dtau"].ndim == 2 else out["dL_dtau"]
    exp = t.sum(0) if t.ndim == 2 else t
    assert rel_l1(got, exp) <= TAU_TOL, ("tau", got, exp)


@pytest.mark.parametrize("name", scene_names())
def test_c_abi_matches_oracle_golden(name):
    inputs, settings, expect, grads = load_scene(name)
    out = run_c(inputs, settings, grads)
    check_against(out, expect, exact_touched=True)


def test_debug_mode_same_result():
    inputs, settings, expect, grads = load_scene("sh3_pose_p800_128x96")
    a = run_c(inputs, settings, grads, debug=False)
    b = run_c(inputs, settings, grads, debug=True)
    for k in a:
        np.testing.assert_array_equal(np.asarray(a[k]), np.asarray(b[k]))


def _synthetic(P, W, H, deg, view=0, seed=0):
    from wgsr.camera import synthetic_camera
    from wgsr.scene import make_scene, make_upstream_grads
    sc = make_scene(P, W, H, deg, seed=seed)
    gc, gd = make_upstream_grads(W, H, seed=seed + 1)
    f = synthetic_camera(W, H, view).raster_fields()
    settings = dict(H=H, W=W, tanfovx=f["tanfovx"], tanfovy=f["tanfovy"],
                    bg=torch.tensor([0.0, 0.0, 0.0]), scale_modifier=1.0,
                    viewmatrix=f["viewmatrix"], projmatrix=f["projmatrix"],
                    projmatrix_raw=f["projmatrix_raw"], sh_degree=deg, campos=f["campos"])
    inputs = dict(means3D=sc.means3D, opacities=sc.opacities, shs=sc.shs, scales=sc.scales,
                  rotations=sc.rotations)
    return inputs, settings, (gc, gd)


def _cpu_expect(inputs, settings, grads):
    cr = cpu_oracle.CpuRaster(**inputs, **settings)
    g = cr.backward(*grads)
    exp = dict(num_rendered=cr.num_rendered, color=cr.color, depth=cr.depth, opacity=cr.opacity,
               radii=cr.radii, n_touched=cr.n_touched, n_touched_firm=cr.n_touched_firm,
               n_touched_soft=cr.n_touched_soft)
    exp.update(g)
    return exp


@pytest.mark.parametrize("P,W,H,deg,view", [(20_000, 640, 480, 3, 2), (50_000, 512, 384, 0, 0)])
def test_matches_cpu_restatement_random(P, W, H, deg, view):
    inputs, settings, grads = _synthetic(P, W, H, deg, view)
    out = run_c(inputs, settings, grads)
    check_against(out, _cpu_expect(inputs, settings, grads))


@pytest.mark.parametrize("kernel", ["quad", "split"])
@pytest.mark.parametrize("P,W,H,deg,view", [(20_000, 640, 480, 3, 2), (3_000, 200, 136, 1, 1)])
def test_both_backward_render_kernels(P, W, H, deg, view, kernel, monkeypatch):
    """k_render_bwd_quad (one wave per tile) and k_render_bwd_seg (four
    decoupled waves per tile, chosen below 3072 tiles) both match the CPU
    restatement; WGSR_BWD_SPLIT_BELOW forces either."""
    monkeypatch.setenv("WGSR_BWD_SPLIT_BELOW", "0" if kernel == "quad" else "1000000")
    inputs, settings, grads = _synthetic(P, W, H, deg, view)
    out = run_c(inputs, settings, grads)
    check_against(out, _cpu_expect(inputs, settings, grads))


@pytest.mark.parametrize("kernel", ["quad", "split"])
def test_backward_render_kernels_nonzero_background(kernel, monkeypatch):
    """Both render-backward kernels with a coloured background (the quad
    kernel specialises a black one, whose dL/dalpha term vanishes) against
    the CPU restatement."""
    monkeypatch.setenv("WGSR_BWD_SPLIT_BELOW", "0" if kernel == "quad" else "1000000")
    inputs, settings, grads = _synthetic(20_000, 640, 480, 3, 2)
    settings = dict(settings, bg=torch.tensor([0.3, 0.55, 0.8]))
    out = run_c(inputs, settings, grads)
    check_against(out, _cpu_expect(inputs, settings, grads))


@pytest.mark.parametrize("P,W,H,deg,view", [(20_000, 640, 480, 3, 2), (8_000, 320, 240, 1, 1), (5_000, 200, 136, 0, 0)])
def test_per_gaussian_backward_matches_cpu(P, W, H, deg, view):
    """k_gauss_bwd_compact (the Gaussians that received gradient compacted
    per workgroup, their record sums and backward in one launch, every other
    row the render backward's zero fill) against the CPU restatement, and
    its zero rows exactly those of the Gaussians no pixel sends gradient to.
    Golden scenes cover the precomputed colour / covariance paths."""
    inputs, settings, grads = _synthetic(P, W, H, deg, view)
    out = run_c(inputs, settings, grads)
    exp = _cpu_expect(inputs, settings, grads)
    check_against(out, exp)
    zero_out = ~np.any(out["dL_dmeans2D"] != 0, axis=1)
    zero_exp = ~np.any(exp["dL_dmeans2D"] != 0, axis=1)
    # (a Gaussian whose every record sums to exactly 0 in one order may not in another: tolerate a few)
    assert (zero_out != zero_exp).mean() <= 1e-3
    for k in ("dL_dmeans3D", "dL_dscales", "dL_drotations", "dL_dopacity"):
        assert not np.any(out[k][zero_out & zero_exp]), k


@pytest.mark.parametrize("P,W,H,deg,view,bg", [(20_000, 640, 480, 3, 2, 0.0), (30_000, 512, 384, 0, 1, 0.4),
                                               (6_000, 200, 136, 1, 0, 0.0), (50_000, 1000, 120, 0, 0, 0.2)])
def test_forward_decoupled_waves_bit_identical(P, W, H, deg, view, bg, monkeypatch):
    """The forward with decoupled quadrant waves (k_render_fwd_dec,
    WGSR_FWD_DEC=1, the default) against the batch-synchronous k_render_fwd1:
    image, depth, opacity, n_touched, radii and every gradient bit-identical."""
    inputs, settings, grads = _synthetic(P, W, H, deg, view)
    settings = dict(settings, bg=torch.tensor([bg, bg * 0.5, bg * 0.25]))
    outs = {}
    for dec in ("0", "1"):
        monkeypatch.setenv("WGSR_FWD_DEC", dec)
        outs[dec] = run_c(inputs, settings, grads)
    for k, v in outs["0"].items():
        if k == "num_rendered":
            assert outs["1"][k] == v
        else:
            np.testing.assert_array_equal(outs["1"][k], v, err_msg=k)


@pytest.mark.parametrize("P,W,H,deg,view,bg", [(20_000, 640, 480, 3, 2, 0.0), (30_000, 512, 384, 0, 1, 0.4),
                                               (6_000, 200, 136, 1, 0, 0.0)])
def test_backward_render_kernels_agree(P, W, H, deg, view, bg, monkeypatch):
    """The few-tile backward (k_render_bwd_seg: four decoupled quadrant waves
    per tile) against the one-wave k_render_bwd_quad on the same forward: the
    same per-pixel arithmetic, only the order of the cross-quadrant record
    sum differs -- gradients within fp32 summation noise, identical zero
    rows."""
    inputs, settings, grads = _synthetic(P, W, H, deg, view)
    settings = dict(settings, bg=torch.tensor([bg, bg * 0.5, bg * 0.25]))
    outs = {}
    for below in ("0", "1000000"):
        monkeypatch.setenv("WGSR_BWD_SPLIT_BELOW", below)
        outs[below] = run_c(inputs, settings, grads)
    a, b = outs["1000000"], outs["0"]
    for k in GRAD_KEYS + ("dL_dtau", "dL_dcov3D"):
        np.testing.assert_array_equal(a[k] == 0, b[k] == 0, err_msg=f"{k} zero rows")
        np.testing.assert_allclose(a[k], b[k], rtol=2e-5, atol=2e-5 * float(np.abs(b[k]).max() + 1e-30), err_msg=k)


@pytest.mark.parametrize("P", [300_000, 600_000])
def test_compact_backward_large_workgroups(P):
    """k_gauss_bwd_compact with 512 / 1024 Gaussians per workgroup (chosen
    from P so that the grid is one resident round): full-size properties (no
    CPU restatement at this size) -- every Gaussian culled by the forward
    (radius 0) has all-zero gradient rows, every row is finite, and the
    rows with gradient are the ones with a non-zero screen-space mean
    gradient."""
    inputs, settings, grads = _synthetic(P, 640, 480, 1, 1)
    out = run_c(inputs, settings, grads)
    culled = out["radii"] == 0
    assert culled.any() and (~culled).any()
    live = np.any(out["dL_dmeans2D"] != 0, axis=1)
    assert 0.01 < live.mean() < 0.9
    for k in GRAD_KEYS + ("dL_dtau", "dL_dcov3D"):
        v = out[k].reshape(P, -1)
        assert np.isfinite(v).all(), k
        assert not np.any(v[culled]), k
        if k != "dL_dsh":
            assert not np.any(v[~live]), k


@pytest.mark.parametrize("P,W,H,deg,view", [(20_000, 640, 480, 3, 2), (6_000, 200, 136, 1, 1),
                                            (30_000, 1000, 120, 0, 0)])
def test_render_bins_give_identical_results(P, W, H, deg, view, monkeypatch):
    """The sorted lists are built per bin of 2^s x 2^s tiles (WGSR_BIN_SHIFT,
    default 2) and every wave culls the entries that cannot reach it: each
    pixel blends the same entries in the same order for every s, so images,
    n_touched and gradients are bit-identical to the per-tile exact lists
    (s = 0), and match the CPU restatement.  Image sizes that are not
    multiples of a bin (partial bins on the right / bottom edges) included."""
    inputs, settings, grads = _synthetic(P, W, H, deg, view)
    outs = {}
    for sh in (0, 1, 2, 3):
        monkeypatch.setenv("WGSR_BIN_SHIFT", str(sh))
        outs[sh] = run_c(inputs, settings, grads)
    check_against(outs[2], _cpu_expect(inputs, settings, grads))
    for sh in (1, 2, 3):
        for k, v in outs[0].items():
            if k == "num_rendered":
                assert outs[sh][k] == v
            else:
                np.testing.assert_array_equal(outs[sh][k], v, err_msg=f"shift {sh} {k}")


@pytest.mark.parametrize("deg,active,P", [(3, 3, 20_001), (3, 1, 9_999), (2, 2, 5_000), (1, 1, 7_777), (0, 0, 30_000)])
def test_preprocess_sh_degrees_match_cpu(deg, active, P):
    """k_preprocess2 at every SH degree, an active degree below the table's
    and ragged P (the last wave part-filled) against the CPU restatement."""
    inputs, settings, grads = _synthetic(P, 640, 480, deg, 1)
    settings = dict(settings, sh_degree=active)
    check_against(run_c(inputs, settings, grads), _cpu_expect(inputs, settings, grads))


@pytest.mark.parametrize("fwd_shift,bwd_shift", [("2", "0"), ("0", "2")])
def test_backward_finds_lists_whatever_bin_shift(fwd_shift, bwd_shift, monkeypatch):
    """The backward locates the forward's tile lists through the image
    buffer's meta word, not by recomputing the bin shift: a WGSR_BIN_SHIFT
    change between the two calls does not change any result."""
    inputs, settings, grads = _synthetic(20_000, 640, 480, 3, 1)
    monkeypatch.setenv("WGSR_BIN_SHIFT", fwd_shift)
    ref = run_c(inputs, settings, grads)
    out = run_c(inputs, settings, grads, between=lambda: monkeypatch.setenv("WGSR_BIN_SHIFT", bwd_shift))
    for k, v in ref.items():
        np.testing.assert_array_equal(np.asarray(out[k]), np.asarray(v), err_msg=k)


def test_radix_sorts_against_numpy(monkeypatch):
    """The three radix-sort forms the library uses, checked as sorts: the
    wide single pass (the 510 sort bins of 1080p, 9 bits), 8-bit passes with
    superblock digit bases (the bin-less tile sort, 13 bits) and the
    Morton-code sort of distCUDA2 -- through the rasteriser at bin shift 2
    vs 0 (bit-identical outputs) and distCUDA2 vs its CPU restatement."""
    from oracle import cpu_oracle
    from simple_knn._C import distCUDA2
    from wgsr.scene import make_points
    inputs, settings, grads = _synthetic(100_000, 1920, 1080, 3, 1)
    monkeypatch.setenv("WGSR_BIN_SHIFT", "0")
    a = run_c(inputs, settings, grads)
    monkeypatch.delenv("WGSR_BIN_SHIFT")
    b = run_c(inputs, settings, grads)
    for k, v in a.items():
        np.testing.assert_array_equal(np.asarray(b[k]), np.asarray(v), err_msg=k)
    pts = make_points(300_000, seed=9)
    np.testing.assert_array_equal(distCUDA2(pts.to(DEV)).cpu().numpy(), cpu_oracle.dist_knn(pts.numpy()))


_COPY_PATH_SCRIPT = r"""
import os, sys
import numpy as np
root, out = sys.argv[1], sys.argv[2]
for p in (os.path.join(root, "wildgs-slam-blackwell_amd", "python"), root, os.path.join(root, "tests")):
    sys.path.insert(0, p)
from test_gpu_raster import _synthetic, run_c
res = run_c(*_synthetic(60_000, 640, 480, 3, view=1))
np.savez(out, **{k: np.asarray(v) for k, v in res.items()})
"""


def test_published_counts_match_the_copy_path(tmp_path):
    """The forward's pair counts reach the host either as the 16-byte record
    the offsets scan publishes into coherent pinned memory (default) or by a
    D->H copy + event (WGSR_PUBLISH_COUNTS=0, read once per process): a second
    process runs the copy path on the same scene, and every output and
    gradient is bit-identical."""
    import subprocess
    import sys
    root = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
    out = run_c(*_synthetic(60_000, 640, 480, 3, view=1))
    path = tmp_path / "copy_path.npz"
    env = dict(os.environ, WGSR_PUBLISH_COUNTS="0")
    r = subprocess.run([sys.executable, "-c", _COPY_PATH_SCRIPT, root, str(path)], env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    ref = np.load(path)
    assert int(ref["num_rendered"]) == out["num_rendered"] > 0
    for k, v in out.items():
        if k != "num_rendered":
            np.testing.assert_array_equal(v, ref[k], err_msg=k)


def test_repeated_backward_of_one_forward_is_identical():
    """The per-Gaussian 'received gradient' flags are set by each backward of
    a forward (zeroed once by the forward): a second backward with other
    upstream gradients sees the same set and matches a fresh forward."""
    C = _c()
    inputs, settings, (gc, gd) = _synthetic(10_000, 320, 240, 3, 1)
    d = lambda x: x.to(DEV)  # noqa: E731
    e = torch.empty(0, device=DEV)
    st = settings
    fargs = (d(st["bg"]), d(inputs["means3D"]), e, d(inputs["opacities"]), d(inputs["scales"]),
             d(inputs["rotations"]), 1.0, e, d(st["viewmatrix"]), d(st["projmatrix"]), d(st["projmatrix_raw"]),
             st["tanfovx"], st["tanfovy"], st["H"], st["W"], d(inputs["shs"]), 3, d(st["campos"]), False, False)

    def bwd(fw, gcol, gdep):
        nr, _, radii, geom, binning, img = fw[:6]
        return C.rasterize_gaussians_backward(
            fargs[0], fargs[1], radii, e, fargs[4], fargs[5], 1.0, e, fargs[8], fargs[9], fargs[10], st["tanfovx"],
            st["tanfovy"], gcol, gdep, fargs[15], 3, fargs[17], geom, nr, binning, img, False)
    fw = C.rasterize_gaussians(*fargs)
    g1 = bwd(fw, d(gc), d(gd))
    g2 = bwd(fw, d(gc) * 0.5, torch.zeros_like(d(gd)))
    g3 = bwd(fw, d(gc), d(gd))
    fresh = bwd(C.rasterize_gaussians(*fargs), d(gc) * 0.5, torch.zeros_like(d(gd)))
    torch.cuda.synchronize()
    for a, b, c in zip(g1, g3, zip(g2, fresh)):
        assert torch.equal(a, b)
        assert torch.equal(c[0], c[1])


def test_forwards_back_to_back_on_two_streams():
    """The forward's pair counters live in two persistent blocks per host
    thread (one accumulates, k_preprocess zeroes the other for the next
    call): forwards of different scenes alternating between two streams,
    without synchronising, give the counts and images of a lone forward."""
    C = _c()
    scenes = []
    for P, seed in ((10_000, 0), (3_000, 1), (20_000, 2)):
        inputs, st, _ = _synthetic(P, 320, 240, 3, 1, seed=seed)
        d = lambda x: x.to(DEV)  # noqa: E731
        e = torch.empty(0, device=DEV)
        scenes.append((d(st["bg"]), d(inputs["means3D"]), e, d(inputs["opacities"]), d(inputs["scales"]),
                       d(inputs["rotations"]), 1.0, e, d(st["viewmatrix"]), d(st["projmatrix"]),
                       d(st["projmatrix_raw"]), st["tanfovx"], st["tanfovy"], st["H"], st["W"], d(inputs["shs"]), 3,
                       d(st["campos"]), False, False))
    alone = []
    for a in scenes:
        out = C.rasterize_gaussians(*a)
        torch.cuda.synchronize()
        alone.append((out[0], out[1].clone(), out[2].clone()))
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    got = []
    for k in range(9):
        with torch.cuda.stream(streams[k % 2]):
            out = C.rasterize_gaussians(*scenes[k % 3])
            got.append((k % 3, out[0], out[1], out[2]))
    torch.cuda.synchronize()
    for i, nr, color, radii in got:
        assert nr == alone[i][0]
        assert torch.equal(color, alone[i][1]) and torch.equal(radii, alone[i][2])


def test_exact_tile_lists_elongated_splats():
    """Stress the exact tile lists (row_span) and the per-wave ellipse culling:
    needle-like rotated splats (per-axis scales over 2.6 decades) and opacities
    from just below 1/255 to 0.999 -- every culled pair must be one that
    reaches no pixel, so images and gradients still match the rect-based CPU
    restatement pixel for pixel."""
    from wgsr.camera import synthetic_camera
    from wgsr.scene import make_scene, make_upstream_grads
    P, W, H, deg = 30_000, 640, 480, 1
    sc = make_scene(P, W, H, deg, seed=11, opacity_range=(0.003, 0.999),
                    log_scale_range=(math.log(0.0005), math.log(0.2)))
    gc, gd = make_upstream_grads(W, H, seed=12)
    f = synthetic_camera(W, H, 3).raster_fields()
    settings = dict(H=H, W=W, tanfovx=f["tanfovx"], tanfovy=f["tanfovy"],
                    bg=torch.tensor([0.1, 0.2, 0.3]), scale_modifier=1.0,
                    viewmatrix=f["viewmatrix"], projmatrix=f["projmatrix"],
                    projmatrix_raw=f["projmatrix_raw"], sh_degree=deg, campos=f["campos"])
    inputs = dict(means3D=sc.means3D, opacities=sc.opacities, shs=sc.shs, scales=sc.scales,
                  rotations=sc.rotations)
    out = run_c(inputs, settings, (gc, gd))
    exp = _cpu_expect(inputs, settings, (gc, gd))
    cov_keys = ("dL_dscales", "dL_drotations")
    check_against(out, exp, grad_keys=[k for k in GRAD_KEYS if k not in cov_keys])
    # needle axes make the covariance gradients ill-conditioned: fp32
    # reassociation noise alone is 1.4e-4 / 2.6e-4 rel-L1 here -- bit for bit
    # the same with the exact tile lists as with plain rectangle lists
    for k in cov_keys:
        assert rel_l1(out[k], exp[k]) <= 1e-3, k


def test_config1_200k_1080p_sh3_pose_matches_cpu():
    """BASELINE.json configs[1]: 200k Gaussians, 1080p, SH3, pose gradient."""
    inputs, settings, grads = _synthetic(200_000, 1920, 1080, 3, view=1)
    out = run_c(inputs, settings, grads)
    check_against(out, _cpu_expect(inputs, settings, grads))


def test_config2_1M_1080p_full_size_properties():
    """BASELINE.json configs[2] size: exact integers and images vs the CPU
    restatement, determinism (no float atomics -> bitwise identical runs)."""
    inputs, settings, grads = _synthetic(1_000_000, 1920, 1080, 3, view=0)
    a = run_c(inputs, settings, grads)
    b = run_c(inputs, settings, grads)
    for k in a:
        np.testing.assert_array_equal(np.asarray(a[k]), np.asarray(b[k]), err_msg=k)
    exp = _cpu_expect(inputs, settings, grads)
    check_against(a, exp)
    for k in ("dL_dmeans3D", "dL_dsh", "dL_dopacity", "dL_dscales", "dL_drotations"):
        assert np.all(np.isfinite(a[k])), k


def test_autograd_render_contract():
    """Reference render() contract: means2D grad (NDC), theta/rho grads."""
    from wgsr.camera import synthetic_camera
    from wgsr.render import DeviceCamera, render
    inputs, settings, expect, grads = load_scene("sh3_pose_p800_128x96")
    W, H = settings["W"], settings["H"]
    cam = DeviceCamera.from_pinhole(synthetic_camera(W, H, 3), DEV)
    leaf = lambda x: x.to(DEV).clone().requires_grad_(True)  # noqa: E731
    m, o, s, r, sh = (leaf(inputs[k]) for k in ("means3D", "opacities", "scales", "rotations", "shs"))
    pkg = render(cam, m, o, s, r, sh, settings["sh_degree"], settings["bg"].to(DEV))
    loss = (pkg["render"] * grads[0].to(DEV)).sum() + (pkg["depth"] * grads[1].to(DEV)).sum()
    loss.backward()
    assert rel_l1(pkg["render"].detach().cpu().numpy(), expect["color"]) <= IMG_TOL
    np.testing.assert_array_equal(pkg["radii"].cpu().numpy(), expect["radii"])
    assert torch.equal(pkg["visibility_filter"].cpu(), torch.from_numpy(expect["radii"] > 0))
    assert rel_l1(m.grad.cpu().numpy(), expect["dL_dmeans3D"]) <= GRAD_TOL
    assert rel_l1(pkg["viewspace_points"].grad.cpu().numpy(), expect["dL_dmeans2D"]) <= GRAD_TOL
    assert rel_l1(sh.grad.cpu().numpy(), expect["dL_dsh"]) <= GRAD_TOL
    tau = torch.cat([cam.cam_trans_delta.grad, cam.cam_rot_delta.grad]).cpu().numpy()
    assert rel_l1(tau, expect["dL_dtau"]) <= TAU_TOL


def test_empty_and_culled():
    C = _c()
    from wgsr.camera import synthetic_camera
    f = synthetic_camera(40, 24, 0).raster_fields()
    e = torch.empty(0, device=DEV)
    bg = torch.tensor([0.25, 0.5, 0.75], device=DEV)
    args = lambda m, o, s, r, sh: (bg, m, e, o, s, r, 1.0, e, f["viewmatrix"].to(DEV),  # noqa: E731
                                   f["projmatrix"].to(DEV), f["projmatrix_raw"].to(DEV),
                                   f["tanfovx"], f["tanfovy"], 24, 40, sh, 0, f["campos"].to(DEV),
                                   False, False)
    z = lambda *s: torch.zeros(*s, device=DEV)  # noqa: E731
    nr, color, radii, *_ = C.rasterize_gaussians(*args(z(0, 3), z(0, 1), z(0, 3), z(0, 4), z(0, 1, 3)))
    assert nr == 0 and float(color.abs().sum()) == 0.0  # upstream: zero image for P == 0
    m = z(5, 3)
    m[:, 2] = -1.0
    q = z(5, 4)
    q[:, 0] = 1
    out = C.rasterize_gaussians(*args(m, z(5, 1) + 0.5, z(5, 3) + 0.01, q, z(5, 1, 3)))
    nr, color, radii, geom, binning, img, depth, opac, nt = out
    assert nr == 0 and int(radii.abs().sum()) == 0
    np.testing.assert_allclose(color.cpu().numpy(), bg.cpu().numpy()[:, None, None] * np.ones((3, 24, 40)))
    assert float(opac.abs().sum()) == 0.0 and float(depth.abs().sum()) == 0.0


def test_wrong_dtype_or_device_raises():
    """float64 / host / int64 arguments raise RuntimeError instead of being
    read as float32 garbage through a raw pointer."""
    C = _c()
    from wgsr.camera import synthetic_camera
    from wgsr.scene import make_scene
    f = synthetic_camera(32, 24, 0).raster_fields()
    sc = make_scene(64, 32, 24, 0, seed=1)
    e = torch.empty(0, device=DEV)
    d = lambda x: x.to(DEV)  # noqa: E731

    def fwd(bg=None, vm=None, sh=None):
        return C.rasterize_gaussians(
            torch.zeros(3, device=DEV) if bg is None else bg, d(sc.means3D), e, d(sc.opacities), d(sc.scales),
            d(sc.rotations), 1.0, e, d(f["viewmatrix"]) if vm is None else vm, d(f["projmatrix"]),
            d(f["projmatrix_raw"]), f["tanfovx"], f["tanfovy"], 24, 32, d(sc.shs) if sh is None else sh, 0,
            d(f["campos"]), False, False)
    with pytest.raises(RuntimeError, match="bg: expected torch.float32"):
        fwd(bg=torch.zeros(3, device=DEV, dtype=torch.float64))
    with pytest.raises(RuntimeError, match="viewmatrix: expected a tensor on"):
        fwd(vm=f["viewmatrix"])
    with pytest.raises(RuntimeError, match="sh: expected torch.float32"):
        fwd(sh=d(sc.shs).double())
    nr, color, radii, geom, binning, img, *_ = fwd()
    g = torch.zeros(3, 24, 32, device=DEV)
    gd = torch.zeros(1, 24, 32, device=DEV)
    args = lambda r, gc: (torch.zeros(3, device=DEV), d(sc.means3D), r, e, d(sc.scales), d(sc.rotations), 1.0,  # noqa
                          e, d(f["viewmatrix"]), d(f["projmatrix"]), d(f["projmatrix_raw"]), f["tanfovx"],
                          f["tanfovy"], gc, gd, d(sc.shs), 0, d(f["campos"]), geom, nr, binning, img, False)
    with pytest.raises(RuntimeError, match="radii: expected torch.int32"):
        C.rasterize_gaussians_backward(*args(radii.long(), g))
    with pytest.raises(RuntimeError, match="dL_dout_color: expected torch.float32"):
        C.rasterize_gaussians_backward(*args(radii, g.double()))
    C.rasterize_gaussians_backward(*args(radii, g))
    torch.cuda.synchronize()


def test_mark_visible():
    from wgsr.camera import synthetic_camera
    from wgsr.scene import make_scene
    C = _c()
    sc = make_scene(4096, 64, 48, 0, seed=3)
    m = sc.means3D.clone()
    m[::3, 2] = torch.linspace(-1, 0.4, m[::3].shape[0])
    f = synthetic_camera(64, 48, 1).raster_fields()
    vis = C.mark_visible(m.to(DEV), f["viewmatrix"].to(DEV), f["projmatrix"].to(DEV)).cpu()
    pv = torch.cat([m, torch.ones(len(m), 1)], 1) @ f["viewmatrix"]
    assert torch.equal(vis, pv[:, 2] > 0.2)


def test_distcuda2_golden_and_bitexact():
    from simple_knn._C import distCUDA2
    import os
    from _util import GOLDEN
    z = np.load(os.path.join(GOLDEN, "knn_cases.npz"))
    for k in z.files:
        if not k.startswith("pts_"):
            continue
        pts = z[k]
        got = distCUDA2(torch.from_numpy(pts).to(DEV)).cpu().numpy()
        np.testing.assert_array_equal(got, cpu_oracle.dist_knn(pts), err_msg=k)
        ref = z["ref_" + k[4:]]
        if pts.shape[0] >= 4:
            np.testing.assert_allclose(got, ref, rtol=1e-6, err_msg=k)
        else:
            np.testing.assert_array_equal(got, ref.astype(np.float32), err_msg=k)


def test_distcuda2_1M_bitexact_vs_cpu():
    from simple_knn._C import distCUDA2
    from wgsr.scene import make_points
    pts = make_points(1_000_000, seed=77)
    got = distCUDA2(pts.to(DEV)).cpu().numpy()
    np.testing.assert_array_equal(got, cpu_oracle.dist_knn(pts.numpy()))


def test_distcuda2_adversarial_bitexact():
    """Layouts that stress the walk's pruning: the
    frustum scene (Morton-curve jumps between sparse and dense regions), two
    far clusters plus sparse outliers, collinear points (flat boxes), heavy
    exact duplicates, and sizes around the 64-point leaf / 4096-point
    super-box edges.  Bit-exact vs the CPU restatement."""
    from simple_knn._C import distCUDA2
    from wgsr.scene import make_scene
    g = np.random.default_rng(5)
    cases = {
        "frustum_200k": make_scene(200_000, 1920, 1080, 0, seed=11).means3D.numpy(),
        "clusters_outliers": np.concatenate([
            g.normal(0.0, 0.05, (30_000, 3)), g.normal(50.0, 0.05, (30_000, 3)),
            g.uniform(-500.0, 500.0, (300, 3))]).astype(np.float32),
        "line": np.stack([np.linspace(-3, 3, 20_000), np.zeros(20_000), 0.5 * np.linspace(-3, 3, 20_000)],
                         1).astype(np.float32),
        "duplicates": np.repeat(g.uniform(-1, 1, (2_000, 3)), 5, axis=0).astype(np.float32),
    }
    for n in (5, 63, 64, 65, 127, 4095, 4097, 64 * 64 * 3 + 1):
        cases[f"uniform_{n}"] = g.uniform(-2, 2, (n, 3)).astype(np.float32)
    for k, pts in cases.items():
        pts = np.ascontiguousarray(pts, dtype=np.float32)
        got = distCUDA2(torch.from_numpy(pts).to(DEV)).cpu().numpy()
        np.testing.assert_array_equal(got, cpu_oracle.dist_knn(pts), err_msg=k)
