"""AES round modules on the MI355X engine vs the golden model (oracle/golden_model.py)
and the reference's own plaintext models.  Decoded nibbles must match exactly; the
angular error of the 16 state slots is reported and bounded (decode margin pi/16)."""
import numpy as np
import pytest

from conftest import gpu_context

pytestmark = pytest.mark.gpu

MARGIN = np.pi / 16


def state_angle_error(ctx, ct, nibbles):
    sc = ctx.engine.slot_count
    z = ctx.decrypt(ct)[: 16 * (sc // 16): sc // 16]
    ref = np.exp(-2j * np.pi * nibbles / 16)
    return float(np.abs(np.angle(z / ref)).max())


@pytest.fixture(scope="module")
def coeffs(coeff_dir):
    from aes_keyschedule import load_all_coeffs
    return load_all_coeffs(coeff_dir)


def test_config1_add_round_key_logn15(coeffs):
    """BASELINE config 1: one AddRoundKey (2x XOR4) at N=2^15, seed 0 (REF/main.py:44-69)."""
    from add_round_key import AddRoundKey
    from state_encoder import StateEncoder
    from xor4_lut import XOR4LUT
    ctx = gpu_context(log_n=15)
    enc = StateEncoder(ctx)
    ark = AddRoundKey(XOR4LUT(ctx, coeffs["xor4"]))
    np.random.seed(0)
    state = np.random.randint(0, 256, 16, dtype=np.uint8)
    key = np.random.randint(0, 256, 16, dtype=np.uint8)
    hi, lo = ark(*enc.encode(state), *enc.encode(key))
    assert np.array_equal(enc.decode(hi, lo), state ^ key)
    assert state_angle_error(ctx, hi, (state ^ key) >> 4) < MARGIN / 4
    # XOR4 magnitude quirk: 256 * zeta^(a^b)
    mag = np.abs(ctx.decrypt(hi)[:: ctx.engine.slot_count // 16][:16])
    assert np.allclose(mag, 256.0, rtol=1e-2)


def test_subbytes_and_inverse(coeffs):
    from oracle import aes_plain
    from state_encoder import StateEncoder
    from sub_bytes_lut import SubBytesLUT
    ctx = gpu_context(log_n=16)
    enc = StateEncoder(ctx)
    np.random.seed(7)
    state = np.random.randint(0, 256, 16, dtype=np.uint8)
    sb = SubBytesLUT(ctx, coeffs["sub_hi"], coeffs["sub_lo"])
    hi, lo = sb.apply(*enc.encode(state))
    out = enc.decode(hi, lo)
    assert np.array_equal(out, aes_plain.SBOX[state])
    assert state_angle_error(ctx, hi, out >> 4) < MARGIN / 2
    isb = SubBytesLUT(ctx, coeffs["inv_sub_hi"], coeffs["inv_sub_lo"])
    back = enc.decode(*isb.apply(*enc.encode(out)))
    assert np.array_equal(back, state)


def test_subbytes_nibble_form(coeffs):
    """the nibble-bivariate (Inv)SubBytes (sub_bytes_lut.use_nibble) on 256 slot-packed
    states covering every byte value: the S-box / inverse S-box bytes, the depth LUT2_DEPTH (an input
    5 levels above out_level suffices), and a slot error far inside the decode margin"""
    from oracle import aes_plain
    from state_encoder import StateEncoder
    from sub_bytes_lut import SubBytesLUT
    from utils import LUT2_DEPTH, RENORM_FLOOR
    ctx = gpu_context(log_n=16)
    enc = StateEncoder(ctx, 256)
    state = np.arange(256 * 16, dtype=np.int64).reshape(256, 16) % 256
    state = state.astype(np.uint8)
    for hi_c, lo_c, table in (("sub_hi", "sub_lo", aes_plain.SBOX), ("inv_sub_hi", "inv_sub_lo", aes_plain.INV_SBOX)):
        lut = SubBytesLUT(ctx, coeffs[hi_c], coeffs[lo_c])
        lut.use_nibble = True
        assert lut.nibble_on() and lut.need_depth() == LUT2_DEPTH
        hi, lo = enc.renorm(*enc.encode(state), level=RENORM_FLOOR + LUT2_DEPTH)
        oh, ol = lut.apply(hi, lo, out_level=RENORM_FLOOR)
        assert min(oh.level, ol.level) >= RENORM_FLOOR
        assert np.array_equal(enc.decode(oh, ol), table[state])


def test_shiftrows_roundtrip():
    from oracle import aes_plain
    from inv_shiftrows import InvShiftRows
    from shift_rows import ShiftRows
    from state_encoder import StateEncoder
    ctx = gpu_context(log_n=16)
    enc = StateEncoder(ctx)
    np.random.seed(42)
    state = np.random.randint(0, 256, 16, dtype=np.uint8)
    s = ShiftRows(ctx).apply(*enc.encode(state))
    assert np.array_equal(enc.decode(*s), aes_plain.shift_rows(state))
    back = InvShiftRows(ctx).apply(*s)
    assert np.array_equal(enc.decode(*back), state)


def test_mixcolumns_stagewise_no_bootstrap(coeffs):
    """REF/mixcol_final.py:250-297 stagewise checks (final bootstrap off)."""
    from mixcol_final import MixColFinal
    from oracle import aes_plain, golden_model as gm
    from state_encoder import StateEncoder
    from xor4_lut import XOR4LUT
    ctx = gpu_context(log_n=16)
    enc = StateEncoder(ctx)
    mc = MixColFinal(ctx, XOR4LUT(ctx, coeffs["xor4"]))
    np.random.seed(0)
    state = np.random.randint(0, 256, 16, dtype=np.uint8)
    dbg = {}
    out = mc(*enc.encode(state), do_final_bootstrap=False, debug=dbg)
    M = state.reshape(4, 4).T
    for k in (1, 2, 3):
        assert np.array_equal(enc.decode(*dbg[f"rotc{k}"]), np.roll(M, -k, axis=1).T.reshape(16))
    assert np.array_equal(enc.decode(*dbg["two"]), aes_plain.GF_MUL[2][state])
    assert np.array_equal(enc.decode(*out), aes_plain.ref_mix_columns(state))
