"""Slot-packed batches on the MI355X engine: B AES states
per ciphertext pair, byte i of state b in slot i*stride + b.  Decoded bytes must equal the
reference's byte-level AES for every state (oracle/aes_plain.py); slot tolerances are
stated in the asserts."""
import numpy as np
import pytest

from conftest import gpu_context

pytestmark = pytest.mark.gpu

Z16 = np.exp(-2j * np.pi / 16)


@pytest.fixture(scope="module")
def ctx():
    return gpu_context(log_n=16, signature=1)


@pytest.mark.parametrize("states", [2, 37, 2048])
def test_renorm_states_snaps_every_packed_slot(ctx, states):
    """Device renorm of a packed pair: every state slot comes back as the exact codeword of
    its (noisy, 256x-scaled) input's nearest zeta16 power, every other slot as 1."""
    from state_encoder import StateEncoder
    E = ctx.engine
    S = E.slot_count
    stride = S // 16
    enc = StateEncoder(ctx, states)
    rng = np.random.default_rng(states)
    st = rng.integers(0, 256, (states, 16), dtype=np.uint8)
    nib_hi, nib_lo = st >> 4, st & 15
    # noisy inputs: angle jitter < pi/32, magnitude 256 (XOR4 output scale)
    def noisy(nib):
        v = rng.standard_normal(S) + 1j * rng.standard_normal(S)  # garbage in non-state slots
        grid = v.reshape(16, stride)
        grid[:, :states] = 256.0 * Z16 ** nib.T * np.exp(1j * rng.uniform(-np.pi / 32, np.pi / 32, (16, states)))
        return v
    hi, lo = ctx.encrypt(noisy(nib_hi)), ctx.encrypt(noisy(nib_lo))
    rh, rl = ctx.renorm_pair(hi, lo, states=states)
    assert rh.level == E.fresh_level
    for ct, nib in ((rh, nib_hi), (rl, nib_lo)):
        z = ctx.decrypt(ct)
        want = np.ones(S, np.complex128)
        want.reshape(16, stride)[:, :states] = Z16 ** nib.T
        assert np.abs(z - want).max() < 2e-4  # fresh-encryption noise at delta ~ 2^29.9 (max over 2^15 slots)
    assert np.array_equal(enc.decode(rh, rl), st)


def test_renorm_states_one_matches_pair(ctx):
    """states=1 through the packed encoder is the reference layout (16-slot device path)."""
    from state_encoder import StateEncoder
    enc = StateEncoder(ctx, 1)
    st = np.arange(16, dtype=np.uint8) * 17
    hi, lo = enc.encode(st)
    assert np.array_equal(enc.decode(*enc.renorm(hi, lo)), st)


def test_renorm_states_rejects_oversize(ctx):
    hi = ctx.encrypt(np.ones(ctx.engine.slot_count))
    with pytest.raises(RuntimeError):
        ctx.renorm_pair(hi, hi, states=ctx.engine.slot_count // 16 + 1)


def test_packed_round_modules(ctx, coeff_dir):
    """SubBytes, ShiftRows, MixColumns (final bootstrap on) and AddRoundKey on 256 packed
    states, each against its byte-level reference."""
    from aes_keyschedule import load_all_coeffs
    from oracle import aes_plain as A
    from pipeline import AESPipeline
    B = 256
    pipe = AESPipeline(ctx, load_all_coeffs(coeff_dir), use_hard_renorm_between_steps=True, states=B)
    rng = np.random.default_rng(11)
    st = rng.integers(0, 256, (B, 16), dtype=np.uint8)
    key = rng.integers(0, 256, (B, 16), dtype=np.uint8)
    enc = pipe.encoder
    ct = enc.encode(st)
    sb = pipe.sub_bytes(*ct)
    assert np.array_equal(enc.decode(*sb), A.SBOX[st])
    sr = pipe.shift_rows(*enc.renorm(*sb))
    want = np.stack([A.shift_rows(A.SBOX[s]) for s in st])
    assert np.array_equal(enc.decode(*sr), want)
    mc = pipe.mix_columns(*sr)
    want = np.stack([A.ref_mix_columns(w) for w in want])
    assert np.array_equal(enc.decode(*mc), want)
    ark = pipe.add_round_key(*mc, *enc.encode(key))
    assert np.array_equal(enc.decode(*ark), want ^ key)


@pytest.mark.parametrize("states", [64, 128, 2048])
def test_packed_config2_encrypt_and_roundtrip(ctx, coeff_dir, states):
    """BASELINE configs 3/5 in the packed layout (128 = C5's per-GPU share of 1,024 states on 8
    GPUs, bench.c5_states_per_rank): `states` independent states under one
    shared key (REF/test/test_aes_pipeline_roundtrip.py:114-163 per state), 10-round
    encrypt with renorm + final bootstraps, then decrypt with InvMixColumns; every state's
    ciphertext equals the reference AES and every plaintext comes back bit-exact."""
    from aes_keyschedule import expand_aes128_key, load_all_coeffs
    from oracle import aes_plain as A
    from pipeline import AESPipeline
    pipe = AESPipeline(ctx, load_all_coeffs(coeff_dir), use_hard_renorm_between_steps=True, states=states)
    np.random.seed(7)
    key = np.random.randint(0, 256, 16, dtype=np.uint8)
    rks = expand_aes128_key(key)
    pts = np.random.default_rng(2025).integers(0, 256, (states, 16), dtype=np.uint8)
    ct = pipe.encrypt(pts, rks)
    got = pipe.encoder.decode(*ct)
    want = np.stack([A.ref_encrypt(p, rks) for p in pts])
    assert np.array_equal(got, want), int((got != want).any(axis=1).sum())
    back = pipe.decrypt(*ct, rks)
    assert np.array_equal(pipe.encoder.decode(*back), pts)


def test_pipeline_refuses_a_pair_in_the_other_layout(ctx, coeff_dir):
    """the pipeline's encrypt output carries its slot layout; its decrypt (and its encoder)
    refuse a pair encoded in the reference layout instead of returning wrong bytes"""
    from aes_keyschedule import expand_aes128_key, load_all_coeffs
    from pipeline import AESPipeline
    from state_encoder import StateEncoder
    pipe = AESPipeline(ctx, load_all_coeffs(coeff_dir), use_hard_renorm_between_steps=True, states=64)
    assert pipe.layout.periodic
    rks = expand_aes128_key(np.arange(16, dtype=np.uint8))
    other = StateEncoder(ctx, 64).encode(np.zeros((64, 16), np.uint8))  # reference layout
    with pytest.raises(ValueError, match="slot layout"):
        pipe.decrypt(*other, rks)
    with pytest.raises(ValueError, match="slot layout"):
        pipe.encoder.decode(*other)
