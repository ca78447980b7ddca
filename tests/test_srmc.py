"""ShiftRows + MixColumns merge (shiftrows_mixcolumns.py) on ideal slot
vectors: Y_k = sum_r D_r * R_{(k+r) mod 4} equals the golden model's column shift k of
ShiftRows(x) (oracle/golden_model.py, REF/shift_rows.py:39-56, REF/mixcol_final.py:101-102),
for one state and for slot-packed batches."""
import numpy as np
import pytest

from oracle import golden_model as gm


class _SlotCtx:
    """EngineContext surface on plain complex slot vectors (encode = identity)"""

    def __init__(self, sc):
        class engine:
            slot_count = sc
        self.engine = engine

    def encode(self, v):
        return np.asarray(v, np.complex128)

    def multiply(self, a, b):
        return a * b

    def add(self, a, b):
        return a + b

    def rotate(self, a, steps):
        return np.roll(a, steps)


@pytest.mark.parametrize("states", [1, 5])
def test_merged_shifts_match_golden(states):
    from shiftrows_mixcolumns import ShiftRowsMixColumnsFusedEnc
    sc = 512
    ctx = _SlotCtx(sc)
    fused = ShiftRowsMixColumnsFusedEnc(ctx, mix=None, states=states)
    rng = np.random.default_rng(states)
    x = np.zeros(sc, np.complex128)
    stride = sc // 16
    for p in range(16):
        x[p * stride: p * stride + states] = np.exp(2j * np.pi * rng.random(states))
    Y = fused._shifts(x)
    sr = gm.shift_rows(x, states=states)
    for k in range(4):
        want = gm.col_shift(sr, k)
        got = Y[k]
        idx = np.concatenate([np.arange(p * stride, p * stride + states) for p in range(16)])
        assert np.allclose(got[idx], want[idx], atol=1e-12), k
