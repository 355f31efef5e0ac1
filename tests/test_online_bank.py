"""CPU tests of wgsr.online_graph.KeyframeBank: the slot-indexed keyframe
banks behind the graph-replayed mapping iteration (adoption keeps every
value, the Keyframe's tensors become views, replaced fields are refreshed,
growth keeps earlier slots, a keyframe of another shape turns the image
banks off but keeps the exposure bank)."""
import types

import torch


def _kf(uid, H=12, W=16, h=3, w=4, C=8, tan=(0.5, 0.4)):
    g = torch.Generator().manual_seed(uid)
    r = lambda *s: torch.rand(*s, generator=g)  # noqa: E731
    cam = {"viewmatrix": r(4, 4), "projmatrix": r(4, 4), "projmatrix_raw": r(4, 4), "campos": r(3),
           "tanfovx": tan[0], "tanfovy": tan[1], "image_height": H, "image_width": W}
    return types.SimpleNamespace(uid=uid, image=r(3, H, W), depth=r(1, H, W), features=r(h, w, C), cam=cam,
                                 median_depth=r(()), exposure_a=r(1), exposure_b=r(1))


def _snap(kf):
    return {"image": kf.image.clone(), "depth": kf.depth.clone(), "features": kf.features.clone(),
            "med": kf.median_depth.clone(), "a": kf.exposure_a.clone(), "b": kf.exposure_b.clone(),
            **{k: kf.cam[k].clone() for k in ("viewmatrix", "projmatrix", "projmatrix_raw", "campos")}}


def _same(kf, s):
    return (torch.equal(kf.image, s["image"]) and torch.equal(kf.depth, s["depth"])
            and torch.equal(kf.features, s["features"]) and torch.equal(kf.median_depth, s["med"])
            and torch.equal(kf.exposure_a, s["a"]) and torch.equal(kf.exposure_b, s["b"])
            and all(torch.equal(kf.cam[k], s[k]) for k in ("viewmatrix", "projmatrix", "projmatrix_raw", "campos")))


def test_adopt_refresh_grow():
    from wgsr.online_graph import KeyframeBank
    B = KeyframeBank("cpu")
    kfs = {u: _kf(u) for u in range(3)}
    snaps = {u: _snap(k) for u, k in kfs.items()}
    B.sync(kfs)
    assert B.uniform and B.image is not None and B.cap >= 3
    for u, k in kfs.items():
        assert _same(k, snaps[u])
        s = B.slots[u]
        assert k.image.data_ptr() == B.image[s].data_ptr()
        assert k.exposure_b.data_ptr() == B.ex[s, 0, 1:2].data_ptr()
        assert torch.equal(B.feat[s], snaps[u]["features"])
    # in-place writes through the views land in the bank
    kfs[1].exposure_a += 1.0
    assert torch.equal(B.ex[B.slots[1], 0, 0:1], snaps[1]["a"] + 1.0)
    # replaced fields (a pose update's new camera, a new depth) are refreshed
    v0 = B.version
    new = _kf(99)
    kfs[2].cam = dict(kfs[2].cam, viewmatrix=new.cam["viewmatrix"], campos=new.cam["campos"])
    kfs[2].depth = new.depth
    B.sync(kfs)
    s2 = B.slots[2]
    assert torch.equal(B.cam[s2, 0:16].view(4, 4), new.cam["viewmatrix"])
    assert torch.equal(B.depth[s2], new.depth) and kfs[2].depth.data_ptr() == B.depth[s2].data_ptr()
    assert torch.equal(kfs[2].cam["projmatrix"], snaps[2]["projmatrix"])
    assert B.version == v0  # (no reallocation)
    # growth past the first capacity keeps every earlier slot
    more = {u: _kf(u) for u in range(3, 40)}
    msn = {u: _snap(k) for u, k in more.items()}
    kfs.update(more)
    B.sync(kfs)
    assert B.cap >= 40 and B.version > v0
    for u in range(3, 40):
        assert _same(kfs[u], msn[u])
    assert torch.equal(kfs[2].depth, new.depth) and torch.equal(kfs[0].image, snaps[0]["image"])
    assert len(set(B.slots.values())) == 40


def test_other_shape_turns_image_banks_off():
    from wgsr.online_graph import KeyframeBank
    B = KeyframeBank("cpu")
    kfs = {0: _kf(0), 1: _kf(1)}
    B.sync(kfs)
    v = B.version
    odd = _kf(2, H=10)
    sn = _snap(odd)
    kfs[2] = odd
    B.sync(kfs)
    assert not B.uniform and B.version > v
    assert _same(odd, sn)  # its own tensors kept, exposure in the bank
    assert odd.exposure_a.data_ptr() == B.ex[B.slots[2], 0, 0:1].data_ptr()
