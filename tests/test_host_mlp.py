"""Host-side checks of wgsr.mlp (no GPU): the dropout-mask restatement."""
import numpy as np


def test_dropout_mask_rate_and_determinism():
    from wgsr.mlp import dropout_mask
    m = dropout_mask(12345, 0, 20000, 0.2)
    assert m.shape == (20000, 64) and m.dtype == bool
    assert abs(m.mean() - 0.8) < 0.005
    assert np.array_equal(m, dropout_mask(12345, 0, 20000, 0.2))
    assert not np.array_equal(m, dropout_mask(12345, 1, 20000, 0.2))
    assert not np.array_equal(m, dropout_mask(12346, 0, 20000, 0.2))
    assert dropout_mask(7, 0, 10, 0.0).all()
