"""Host-side camera formation on CPU: the batched raster fields the mapper
uses for pose updates (wgsr.camera.raster_fields_batched) equal the
per-camera PinholeCamera.raster_fields bit for bit, and
OnlineMapper.update_keyframes leaves every moved keyframe (and its bank row)
with exactly those fields."""
import numpy as np
import pytest
import torch


def _poses(n, seed):
    g = torch.Generator().manual_seed(seed)
    Rs, Ts = [], []
    for _ in range(n):
        a = torch.randn(3, generator=g) * 0.4
        K = torch.tensor([[0.0, -a[2], a[1]], [a[2], 0.0, -a[0]], [-a[1], a[0], 0.0]])
        Rs.append(torch.linalg.matrix_exp(K))
        Ts.append(torch.randn(3, generator=g))
    return torch.stack(Rs), torch.stack(Ts)


@pytest.mark.parametrize("intr", [(500.0, 500.0, 256.0, 192.0, 512, 384), (517.3, 516.5, 318.6, 255.3, 640, 480),
                                  (57.6, 57.6, 32.0, 24.0, 64, 48)])
def test_batched_raster_fields_bit_identical(intr):
    from wgsr.camera import PinholeCamera, raster_fields_batched
    fx, fy, cx, cy, W, H = intr
    R, T = _poses(9, int(fx))
    f = raster_fields_batched(R, T, fx, fy, cx, cy, W, H)
    for i in range(R.shape[0]):
        want = PinholeCamera(R=R[i], T=T[i], fx=fx, fy=fy, cx=cx, cy=cy, W=W, H=H).raster_fields()
        assert torch.equal(f["viewmatrix"][i], want["viewmatrix"])
        assert torch.equal(f["projmatrix"][i], want["projmatrix"])
        assert torch.equal(f["projmatrix_raw"], want["projmatrix_raw"])
        assert torch.equal(f["campos"][i], want["campos"])


def test_update_keyframes_cameras_and_bank_rows():
    from wgsr.camera import PinholeCamera
    from wgsr.online import Keyframe, OnlineMapper
    m = OnlineMapper(sh_degree=0, feature_dim=64, device="cpu")
    R, T = _poses(6, 3)
    for k in range(6):
        m.keyframes[k] = Keyframe(k, R[k], T[k], 50.0, 50.0, 16.0, 12.0, torch.rand(3, 24, 32),
                                  torch.ones(1, 24, 32), torch.zeros(2, 2, 64))
    m.bank.sync(m.keyframes)
    R2, T2 = _poses(6, 4)
    upd = {}
    for k in (1, 2, 4):
        w = torch.eye(4)
        w[:3, :3], w[:3, 3] = R2[k], T2[k]
        upd[k] = (w, None)
    w = torch.eye(4)
    w[:3, :3], w[:3, 3] = R[5], T[5] + 1e-8          # within allclose: skipped
    upd[5] = (w, None)
    assert m.update_keyframes(upd) == 3
    for k in range(6):
        kf = m.keyframes[k]
        Rk, Tk = (R2[k], T2[k]) if k in (1, 2, 4) else (R[k], T[k])
        want = PinholeCamera(R=Rk, T=Tk, fx=50.0, fy=50.0, cx=16.0, cy=12.0, W=32, H=24).raster_fields()
        for name in ("viewmatrix", "projmatrix", "projmatrix_raw", "campos"):
            assert torch.equal(kf.cam[name].cpu(), want[name]), (k, name)
        # the keyframe's fields are views of its bank row
        row = m.bank.cam[m.bank.slots[k]]
        assert kf.cam["viewmatrix"].data_ptr() == row.data_ptr()
        assert np.array_equal(row[0:16].numpy(), want["viewmatrix"].reshape(-1).numpy())
