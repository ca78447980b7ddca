"""Slot-packed batch layout on the CPU: the ideal-slot golden model with
B states per vector equals B independent runs of the reference's byte-level AES, and the
host-side packing (StateEncoder, ShiftRows masks, AESPipeline key broadcast) is laid out
as state_encoder.py documents.  No GPU."""
import numpy as np
import pytest

from oracle import aes_plain as A
from oracle import golden_model as G


class _SlotCtx:
    """Noiseless stand-in context: a ciphertext is its slot vector (golden-model semantics)."""

    class engine:
        slot_count = 256  # stride 16

    def encrypt(self, slots):
        return np.array(slots, np.complex128)

    def decrypt(self, ct):
        return np.array(ct, np.complex128)

    def encode(self, slots):
        return np.array(slots, np.complex128)

    def multiply(self, a, b):
        return a * b

    def add(self, a, b):
        return a + b

    def rotate(self, a, steps):
        return np.roll(a, steps)


@pytest.mark.parametrize("states", [1, 5, 16])
def test_state_encoder_packing(states):
    from state_encoder import StateEncoder
    ctx = _SlotCtx()
    enc = StateEncoder(ctx, states)
    rng = np.random.default_rng(states)
    st = rng.integers(0, 256, (states, 16), dtype=np.uint8)
    hi, lo = enc.encode(st[0] if states == 1 else st)
    stride = 16
    for b in range(states):
        for i in range(16):
            assert np.isclose(hi[i * stride + b], np.exp(-2j * np.pi * (st[b, i] >> 4) / 16))
            assert np.isclose(lo[i * stride + b], np.exp(-2j * np.pi * (st[b, i] & 15) / 16))
    mask = np.ones(256, bool)
    for i in range(16):
        mask[i * stride:i * stride + states] = False
    assert np.allclose(hi[mask], 1.0) and np.allclose(lo[mask], 1.0)
    back = enc.decode(hi, lo)
    assert np.array_equal(back, st[0] if states == 1 else st)
    # the same vectors as the golden model's packing
    ghi, glo = G.encode_state(st if states > 1 else st[0], 256)
    assert np.allclose(ghi, hi) and np.allclose(glo, lo)


def test_state_encoder_rejects_bad_batches():
    from state_encoder import StateEncoder
    ctx = _SlotCtx()
    with pytest.raises(ValueError):
        StateEncoder(ctx, 17)  # > stride
    with pytest.raises(ValueError):
        StateEncoder(ctx, 4).encode(np.zeros((3, 16), np.uint8))


@pytest.mark.parametrize("states", [1, 7, 16])
def test_shiftrows_packed_masks(states):
    """ShiftRows with packed masks moves every packed state like aes_plain.shift_rows and
    zeroes the non-state slots (REF/shift_rows.py:39-56 semantics per column b)."""
    from inv_shiftrows import InvShiftRows
    from shift_rows import ShiftRows
    from state_encoder import StateEncoder
    ctx = _SlotCtx()
    enc = StateEncoder(ctx, states)
    rng = np.random.default_rng(3)
    st = rng.integers(0, 256, (states, 16), dtype=np.uint8)
    hi, lo = enc.encode(st[0] if states == 1 else st)
    sh = ShiftRows(ctx, states=states)
    out = sh._apply_one(hi), sh._apply_one(lo)
    got = enc.decode(*out).reshape(states, 16)
    for b in range(states):
        assert np.array_equal(got[b], A.shift_rows(st[b]))
    mask = np.ones(256, bool)
    for i in range(16):
        mask[i * 16:i * 16 + states] = False
    assert np.allclose(out[0][mask], 0.0)
    inv = InvShiftRows(ctx, states=states)
    back = enc.decode(inv._apply_one(out[0]), inv._apply_one(out[1])).reshape(states, 16)
    assert np.array_equal(back, st)
    # golden model's packed masks agree
    assert np.allclose(G.shift_rows(hi, states=states), out[0])


def test_golden_packed_encrypt_decrypt(coeff_dir):
    """B = 6 states in one ideal-slot vector pair: the golden model of AESPipeline.encrypt
    gives each state's reference ciphertext, and decrypt inverts it (REF/pipeline.py:123-254)."""
    B = 6
    rng = np.random.default_rng(2025)
    states = rng.integers(0, 256, (B, 16), dtype=np.uint8)
    np.random.seed(7)
    key = np.random.randint(0, 256, 16, dtype=np.uint8)
    rks = A.expand_key(key)
    g = G.Golden(coeff_dir, states=B)
    stages = {}
    ct = g.encrypt(states, rks, stages=stages)
    got = G.decode_state(*ct, B)
    for b in range(B):
        assert bytes(got[b]) == bytes(A.ref_encrypt(states[b], rks))
    # the per-stage bytes of state b match a one-state run
    one = {}
    G.Golden(coeff_dir).encrypt(states[2], rks, sc=16, stages=one)
    for tag, v in one.items():
        assert bytes(stages[tag][2]) == bytes(v), tag
    back = G.decode_state(*g.decrypt(ct, rks), B)
    assert np.array_equal(back, states)


@pytest.mark.parametrize("states", [1, 4])
def test_periodic_layout(states):
    """periodic layout (state_encoder.SlotLayout): the 16B-slot block repeated,
    rotation unit B; ShiftRows / InvShiftRows and MixColumns' column shifts act per state exactly
    as on the reference layout, and the vectors stay 16B-periodic (the sparse bootstrap's premise)"""
    from shift_rows import ShiftRows
    from inv_shiftrows import InvShiftRows
    from state_encoder import StateEncoder
    ctx = _SlotCtx()
    enc = StateEncoder(ctx, states, periodic=True)
    lay = enc.layout
    assert lay.unit == states and lay.period == 16 * states and lay.renorm_states == 16
    assert lay.boot_period == (16 * states if 16 * states < 256 else None)
    rng = np.random.default_rng(10 + states)
    st = rng.integers(0, 256, (states, 16), dtype=np.uint8)
    hi, lo = enc.encode(st[0] if states == 1 else st)
    P = lay.period
    assert np.allclose(hi, np.tile(hi[:P], 256 // P)) and np.allclose(lo, np.tile(lo[:P], 256 // P))
    for b in range(states):
        for i in range(16):
            assert np.isclose(hi[i * states + b], np.exp(-2j * np.pi * (st[b, i] >> 4) / 16))
    assert np.array_equal(enc.decode(hi, lo), st[0] if states == 1 else st)
    sr, isr = ShiftRows(ctx, states, layout=lay), InvShiftRows(ctx, states, layout=lay)
    h2, l2 = sr.apply(hi, lo)
    want = np.stack([A.shift_rows(s) for s in st])
    assert np.array_equal(enc.decode(h2, l2), want[0] if states == 1 else want)
    assert np.allclose(h2, np.tile(h2[:P], 256 // P))
    h3, l3 = isr.apply(h2, l2)
    assert np.array_equal(enc.decode(h3, l3), st[0] if states == 1 else st)
    # MixColumns' column shift by k (mixcol_final._col_shift_rowmajor): rotate by -4 k unit
    for k in (1, 2, 3):
        r = np.roll(hi, -4 * k * lay.unit)
        got = enc.decode(r, np.roll(lo, -4 * k * lay.unit))
        exp = np.stack([np.roll(s.reshape(4, 4), -k, axis=0).reshape(16) for s in st])
        assert np.array_equal(got, exp[0] if states == 1 else exp), k


def test_layout_tags_are_checked():
    """a ciphertext the encoder tagged with one slot layout is refused by an encoder (and so by
    AESPipeline.decrypt / renorm) using the other one; untagged ciphertexts pass"""
    from state_encoder import SlotLayout, check_layout, tag_layout

    class Ct:
        pass

    ref, per = SlotLayout(256, 4), SlotLayout(256, 4, periodic=True)
    a, b = tag_layout(ref, Ct(), Ct())
    check_layout(ref, a, b)
    check_layout(per, Ct())
    with pytest.raises(ValueError, match="reference"):
        check_layout(per, a, b)
    (c,) = tag_layout(per, Ct())
    with pytest.raises(ValueError, match="periodic"):
        check_layout(ref, c)
    tag_layout(ref, np.zeros(3))  # untaggable ciphertexts (the CPU stand-ins) are left alone


def test_multi_pair_encoder_shapes():
    """StateEncoder(pairs=P): (P, 16) / (P, B, 16) bytes -> one stacked pair and
    back; a single pair's bytes broadcast to every pair (round keys)"""
    from state_encoder import StateEncoder

    class StackCtx(_SlotCtx):
        def stack(self, cts):
            return np.stack(cts)

        def unstack(self, st):
            return list(st)

    ctx = StackCtx()
    rng = np.random.default_rng(3)
    for states, shape in ((1, (4, 16)), (5, (4, 5, 16))):
        enc = StateEncoder(ctx, states, pairs=4)
        st = rng.integers(0, 256, shape, dtype=np.uint8)
        hi, lo = enc.encode(st)
        assert hi.shape == (4, 256)
        assert np.array_equal(enc.decode(hi, lo), st)
        key = st[0]
        assert np.array_equal(enc.decode(*enc.encode(key)), np.stack([key] * 4))
    with pytest.raises(ValueError):
        StateEncoder(_SlotCtx(), 1, pairs=2)  # no stacked ciphertexts in this context
