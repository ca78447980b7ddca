"""The packed XOR stage: hi and lo side by side in ONE ciphertext for the steps
whose LUT is the same for both halves -- MixColumns' XOR4s and the AddRoundKey after it.

- StateEncoder.pack / encode_packed / decode_packed and the two packed renorms
  (aesfhe_renorm_single, aesfhe_renorm_unpack) against the byte model;
- one XOR4 on packed states == the XOR pair (REF/xor4_lut.py:10-78 per nibble);
- MixColFinal.mix_packed == REF/mixcol_final.py's MixColumns bytes (final bootstrap on);
- full C2 encrypts through the packed path == aes_plain.ref_encrypt, one state and a 64-state
  batch, and == the pair path's bytes, and decrypt through the packed AddRoundKey / InvMixColumns
  stage returns the plaintext;
- the strict default (utils.RenormFolds): an encrypt + decrypt with every folding renorm entry
  point of the engine disabled -- each renorm the identity on the message, as REF's -- and the
  folded form's bytes (the bench's secondary leg);
- SubBytes' bivariate giant-step form (sub_bytes_lut._outputs_biv) == the S-box on all bytes.
Decoded bytes must be exact.
"""
import numpy as np
import pytest

from conftest import gpu_context

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    return gpu_context(log_n=16, signature=1)


@pytest.fixture(scope="module")
def co(coeff_dir):
    from aes_keyschedule import load_all_coeffs
    return load_all_coeffs(coeff_dir)


@pytest.mark.parametrize("states", [1, 64])
def test_pack_renorm_roundtrip(ctx, states):
    from state_encoder import StateEncoder
    from utils import NEED_XOR
    enc = StateEncoder(ctx, states, periodic=True)
    rng = np.random.default_rng(states)
    st = rng.integers(0, 256, (states, 16) if states > 1 else 16).astype(np.uint8)
    p = enc.pack(*enc.encode(st))
    assert np.array_equal(enc.decode_packed(p), st)
    assert np.array_equal(enc.decode_packed(enc.encode_packed(st)), st)
    q = enc.renorm_packed(p, level=NEED_XOR)
    assert q.level == NEED_XOR and np.array_equal(enc.decode_packed(q), st)
    hi, lo = enc.renorm_unpack(p, level=NEED_XOR)
    assert hi.level == lo.level == NEED_XOR
    assert np.array_equal(enc.decode(hi, lo), st)
    with pytest.raises(RuntimeError, match="packed period"):
        ctx.engine.renorm_unpack(p, 24)


def test_direct32_packed_renorm_equals_fft_codec(ctx):
    """the packed renorms at period 32 decode / re-encode their 32 slots directly (decode32 /
    encode32, aesfhe_renorm_packed); the FFT codec (aesfhe_renorm_single) gives the same fresh
    codewords in every slot, and the unpacked halves are the packed halves"""
    from state_encoder import StateEncoder
    E = ctx.engine
    enc = StateEncoder(ctx, 1, periodic=True)
    rng = np.random.default_rng(32)
    st = rng.integers(0, 256, 16).astype(np.uint8)
    p = E.multiply(enc.pack(*enc.encode(st)), 256.0)  # off-scale, as an XOR4 output
    direct = E.renorm_single(p, None, period=32)
    fft = E.renorm_single(p)
    zd, zf = ctx.decrypt(direct), ctx.decrypt(fft)
    assert np.abs(zd - zf).max() < 4e-4  # two fresh encryptions of the same codewords
    assert np.abs(np.abs(zd) - 1.0).max() < 2e-4
    assert np.array_equal(enc.decode_packed(direct), st)
    hi, lo = E.renorm_unpack(p, 16)
    zh, zl = ctx.decrypt(hi), ctx.decrypt(lo)
    assert np.abs(zh - np.tile(zd[:16], len(zd) // 16)).max() < 4e-4
    assert np.abs(zl - np.tile(zd[16:32], len(zd) // 16)).max() < 4e-4


def test_xor4_on_packed_states(ctx, co):
    from state_encoder import StateEncoder
    from utils import NEED_XOR, RENORM_FLOOR
    from xor4_lut import XOR4LUT
    enc = StateEncoder(ctx, periodic=True)
    xor4 = XOR4LUT(ctx, co["xor4"])
    rng = np.random.default_rng(5)
    a, b = rng.integers(0, 256, 16).astype(np.uint8), rng.integers(0, 256, 16).astype(np.uint8)
    pa = enc.renorm_packed(enc.encode_packed(a), level=NEED_XOR)
    pb = enc.pack(*enc.renorm(*enc.encode(b), level=NEED_XOR + enc.PACK_DEPTH))
    x = xor4.apply(pa, pb, out_level=RENORM_FLOOR)
    assert np.array_equal(enc.decode_packed(x), a ^ b)
    assert np.array_equal(enc.decode(*enc.renorm_unpack(x)), a ^ b)


def test_mix_packed_matches_mixcolumns(ctx, co):
    from mixcol_final import MixColFinal
    from oracle import aes_plain
    from state_encoder import StateEncoder
    from utils import NEED_SR_MIX, SHIFTROWS_DEPTH
    from xor4_lut import XOR4LUT
    enc = StateEncoder(ctx, periodic=True)
    mc = MixColFinal(ctx, XOR4LUT(ctx, co["xor4"]), layout=enc.layout)
    assert mc.packed_ok()
    rng = np.random.default_rng(6)
    st = rng.integers(0, 256, 16).astype(np.uint8)
    x = enc.renorm(*enc.encode(st), level=NEED_SR_MIX + enc.PACK_DEPTH - SHIFTROWS_DEPTH)
    out = mc.mix_packed(*x)
    assert out.level == ctx.engine.fresh_level
    assert np.array_equal(enc.decode_packed(out), aes_plain.ref_mix_columns(st))


@pytest.mark.parametrize("states,seed", [(1, 7), (1, 42), (64, 3)])
def test_encrypt_through_packed_stage(ctx, co, states, seed):
    from aes_keyschedule import expand_aes128_key
    from oracle import aes_plain
    from pipeline import AESPipeline
    pipe = AESPipeline(ctx, co, use_hard_renorm_between_steps=True, states=states)
    assert pipe.packed_xor and pipe.packed_dec
    rng = np.random.default_rng(seed)
    rks = expand_aes128_key(rng.integers(0, 256, 16).astype(np.uint8))
    pt = rng.integers(0, 256, (states, 16) if states > 1 else 16).astype(np.uint8)
    ct = pipe.encrypt(pt, rks)
    got = pipe.encoder.decode(*ct)
    want = aes_plain.ref_encrypt(pt, rks) if states == 1 else np.stack([aes_plain.ref_encrypt(p, rks) for p in pt])
    assert np.array_equal(got, want)
    # decrypt rounds through the packed AddRoundKey + InvMixColumns XOR stage
    assert np.array_equal(pipe.encoder.decode(*pipe.decrypt(*ct, rks)), pt)
    if states == 1:
        ref = AESPipeline(ctx, co, use_hard_renorm_between_steps=True, packed_xor=False)
        assert not ref.packed_xor
        assert np.array_equal(ref.encoder.decode(*ref.encrypt(pt, rks)), want)


def test_subbytes_bivariate_giant_step_form(ctx, co):
    """SubBytes from one level above its depth takes the bivariate giant-step form
    (sub_bytes_lut._outputs_biv: chunk sums and their giant-step products as ONE bivariate LUT):
    the S-box on all 256 byte values (16 states x 16 bytes), like the batched-product form"""
    from oracle import aes_plain
    from state_encoder import StateEncoder
    from sub_bytes_lut import SubBytesLUT
    from utils import NEED_SUBBYTES, RENORM_FLOOR
    enc = StateEncoder(ctx, 16, periodic=True)
    sb = SubBytesLUT(ctx, co["sub_hi"], co["sub_lo"])
    st = np.arange(256, dtype=np.uint8).reshape(16, 16)
    want = np.asarray(aes_plain.SBOX, np.uint8)[st]
    x = enc.renorm(*enc.encode(st), level=NEED_SUBBYTES + 1)
    hi, lo = sb.apply(*x, out_level=RENORM_FLOOR)
    assert hi.level >= RENORM_FLOOR and lo.level >= RENORM_FLOOR
    got = enc.decode(hi, lo)
    y = enc.renorm(*enc.encode(st), level=NEED_SUBBYTES)
    ref = enc.decode(*sb.apply(*y, out_level=RENORM_FLOOR))  # the batched-product form
    assert np.array_equal(got, want)
    assert np.array_equal(ref, want)


class _NoFolds:
    """the context with every renorm entry point that computes on the decrypted message made to
    raise: the gathering unpack, the packing renorm, the slot permutations, conjugate partners"""

    def __init__(self, ctx):
        self._ctx = ctx

    def __getattr__(self, name):
        if name in ("renorm_unpack", "renorm_unpack_perm", "renorm_periodic_perm", "renorm_pack"):
            def refuse(*a, **k):
                raise AssertionError(f"strict renorm path called the folding renorm {name}")
            return refuse
        attr = getattr(self._ctx, name)
        if name in ("renorm_single", "renorm_periodic", "renorm_pair"):
            def plain(*a, conj=None, **k):
                assert conj is None, f"strict renorm path passed a conjugate partner to {name}"
                return attr(*a, **k)
            return plain
        return attr


@pytest.mark.parametrize("seed", [5, 11])
def test_strict_path_renorms_are_the_identity(ctx, co, seed):
    """the headline (strict) encrypt and decrypt never reach a renorm that permutes, packs, unpacks or
    conjugates the decrypted message, and their bytes are FIPS-197's"""
    from aes_keyschedule import expand_aes128_key
    from oracle import aes_plain
    from pipeline import AESPipeline
    from utils import FOLDS, RENORM_TALLY
    assert not FOLDS.any
    nf = _NoFolds(ctx)
    pipe = AESPipeline(nf, co, use_hard_renorm_between_steps=True)
    assert pipe.packed_xor and pipe.packed_dec
    rng = np.random.default_rng(seed)
    rks = expand_aes128_key(rng.integers(0, 256, 16).astype(np.uint8))
    pt = rng.integers(0, 256, 16).astype(np.uint8)
    n0 = RENORM_TALLY["ciphertexts"]
    ct = pipe.encrypt(pt, rks)
    assert np.array_equal(pipe.encoder.decode(*ct), aes_plain.ref_encrypt(pt, rks))
    # every renorm counted: REF runs 48 pairs (96 ciphertexts); the packed XOR stage renorms single ones
    assert 40 <= RENORM_TALLY["ciphertexts"] - n0 <= 120
    assert np.array_equal(pipe.encoder.decode(*pipe.decrypt(*ct, rks)), pt)


def test_folded_form_bytes(ctx, co):
    """the bench's secondary 'folded' leg: the renorm folds on, the same bytes"""
    from aes_keyschedule import expand_aes128_key
    from oracle import aes_plain
    from pipeline import AESPipeline
    from utils import renorm_folds
    rng = np.random.default_rng(3)
    rks = expand_aes128_key(rng.integers(0, 256, 16).astype(np.uint8))
    pt = rng.integers(0, 256, 16).astype(np.uint8)
    with renorm_folds(True) as f:
        assert f.conj and f.sr and f.pack and f.unpack
        pipe = AESPipeline(ctx, co, use_hard_renorm_between_steps=True)
        ct = pipe.encrypt(pt, rks)
        assert np.array_equal(pipe.encoder.decode(*ct), aes_plain.ref_encrypt(pt, rks))
        assert np.array_equal(pipe.encoder.decode(*pipe.decrypt(*ct, rks)), pt)
