"""Level management around the renorm on the MI355X engine: renorm at a
target level, LUT steps on inputs dropped just above the renorm floor, and the deferred-
tensor add paths the level drops exercise.  Decoded nibbles must be exact; slot
tolerances are stated in the asserts."""
import numpy as np
import pytest

from conftest import gpu_context

pytestmark = pytest.mark.gpu

Z16 = np.exp(-2j * np.pi / 16)


@pytest.fixture(scope="module")
def ctx():
    return gpu_context(log_n=16, signature=1)


@pytest.mark.parametrize("states", [1, 64])
@pytest.mark.parametrize("level", [0, 7, 13, 99])
def test_renorm_at_level(ctx, states, level):
    """renorm re-encrypts at min(level, fresh) with exact codewords in every state slot."""
    from state_encoder import StateEncoder
    E = ctx.engine
    enc = StateEncoder(ctx, states)
    rng = np.random.default_rng(level + states)
    st = rng.integers(0, 256, (states, 16), dtype=np.uint8)
    hi, lo = enc.encode(st[0] if states == 1 else st)
    rh, rl = enc.renorm(hi, lo, level=level)
    assert rh.level == rl.level == min(level, E.fresh_level)
    got = enc.decode(rh, rl)
    assert np.array_equal(got.reshape(-1, 16), st)
    stride = E.slot_count // 16
    z = ctx.decrypt(rh).reshape(16, stride)[:, :states]
    # fresh-encryption noise only: ~3e-5 rms per slot at every level, max over up to 1,024
    # state slots (measured up to 1.1e-4)
    assert np.abs(z - Z16 ** (st.T >> 4)).max() < 2e-4


def test_xor4_and_gf_at_the_floor(ctx, coeff_dir):
    """XOR4 / GF multipliers with out_level: inputs dropped to out_level + LUT2_DEPTH, the
    output lands at out_level and decodes exactly like the undropped evaluation."""
    from aes_keyschedule import load_all_coeffs
    from mixcol_final import MixColFinal
    from oracle import aes_plain as A
    from state_encoder import StateEncoder
    from utils import LUT2_DEPTH, RENORM_FLOOR
    from xor4_lut import XOR4LUT
    co = load_all_coeffs(coeff_dir)
    enc = StateEncoder(ctx)
    xor4 = XOR4LUT(ctx, co["xor4"])
    mix = MixColFinal(ctx, xor4)
    rng = np.random.default_rng(5)
    s1, s2 = rng.integers(0, 256, 16, dtype=np.uint8), rng.integers(0, 256, 16, dtype=np.uint8)
    a, b = enc.encode(s1), enc.encode(s2)
    x = (xor4.apply(a[0], b[0], out_level=RENORM_FLOOR), xor4.apply(a[1], b[1], out_level=RENORM_FLOOR))
    assert x[0].level == RENORM_FLOOR
    assert np.array_equal(enc.decode(*x), s1 ^ s2)
    g = mix.gf_mult_3(*a, out_level=RENORM_FLOOR + LUT2_DEPTH)
    assert g[0].level == RENORM_FLOOR + LUT2_DEPTH
    assert np.array_equal(enc.decode(*g), A.GF_MUL[3][s1])
    # undropped reference evaluation gives the same bytes
    assert np.array_equal(enc.decode(xor4.apply(a[0], b[0]), xor4.apply(a[1], b[1])), s1 ^ s2)


def test_subbytes_from_level_15(ctx, coeff_dir):
    from aes_keyschedule import load_all_coeffs
    from oracle import aes_plain as A
    from state_encoder import StateEncoder
    from sub_bytes_lut import SubBytesLUT
    from utils import RENORM_FLOOR
    co = load_all_coeffs(coeff_dir)
    enc = StateEncoder(ctx)
    sb = SubBytesLUT(ctx, co["sub_hi"], co["sub_lo"])
    st = np.arange(16, dtype=np.uint8) * 13 + 7
    out = sb.apply(*enc.encode(st), out_level=RENORM_FLOOR)
    assert out[0].level >= RENORM_FLOOR
    assert np.array_equal(enc.decode(*out), A.SBOX[st])


def test_deferred_add_with_third_polynomial(ctx):
    """a deferred 3-polynomial product plus / minus a canonical ciphertext (the fused tail
    add, launch_addsub_tail) and a zero minus a product (exact zero operand)."""
    E = ctx.engine
    S = E.slot_count
    rng = np.random.default_rng(9)
    za = np.exp(2j * np.pi * rng.random(S))
    zb = np.exp(2j * np.pi * rng.random(S))
    zc = 0.5 * np.exp(2j * np.pi * rng.random(S))
    a, b, c = ctx.encrypt(za), ctx.encrypt(zb), ctx.encrypt(zc)
    p = ctx.multiply(a, b)  # deferred tensor (3 polys, one owed rescale) under lazy evaluation
    for got, want in ((ctx.add(p, c), za * zb + zc), (ctx.add(c, p), zc + za * zb),
                      (ctx.sub(p, c), za * zb - zc), (ctx.sub(c, p), zc - za * zb),
                      (ctx.sub(ctx.sub(c, c), p), -za * zb)):
        assert np.abs(ctx.decrypt(got) - want).max() < 1e-3


def test_level_down_is_exact_scale(ctx):
    E = ctx.engine
    z = np.exp(2j * np.pi * np.random.default_rng(3).random(E.slot_count))
    ct = ctx.encrypt(z)
    for lv in (12, 7, 2, 0):
        d = ctx.level_down(ct, lv)
        assert d.level == lv
        assert np.abs(ctx.decrypt(d) - z).max() < 5e-4  # fresh-encryption noise, max over 2^15 slots
