"""SubBytes ⊕ AddRoundKey fused LUT (sub_bytes_ark.py) on the MI355X engine:
the fused step alone, and the C2 pipeline with fuse_sub_ark=True (last encrypt round and every
decrypt round fused across (Inv)ShiftRows) -- bytes exact against oracle/aes_plain.py."""
import numpy as np
import pytest

from conftest import gpu_context

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    return gpu_context(log_n=16, signature=1)


@pytest.mark.parametrize("inverse", [False, True], ids=["sbox", "inv_sbox"])
def test_sub_ark_step(ctx, coeff_dir, inverse):
    from aes_keyschedule import load_all_coeffs
    from oracle import aes_plain as A
    from state_encoder import StateEncoder
    from sub_bytes_ark import SubBytesARK
    from sub_bytes_lut import SubBytesLUT
    co = load_all_coeffs(coeff_dir)
    pre = "inv_sub" if inverse else "sub"
    ark = SubBytesARK(SubBytesLUT(ctx, co[f"{pre}_hi"], co[f"{pre}_lo"]), co["xor4"])
    enc = StateEncoder(ctx)
    rng = np.random.default_rng(31 + inverse)
    S = A.INV_SBOX if inverse else A.SBOX
    for _ in range(2):
        x, k = rng.integers(0, 256, 16).astype(np.uint8), rng.integers(0, 256, 16).astype(np.uint8)
        out = ark(*enc.encode(x), *enc.encode(k))
        assert np.array_equal(enc.decode(*out), S[x] ^ k)
        assert out[0].level >= 1


def test_pipeline_fused_encrypt_decrypt(ctx, coeff_dir):
    from aes_keyschedule import expand_aes128_key, load_all_coeffs
    from oracle import aes_plain as A
    from pipeline import AESPipeline
    pipe = AESPipeline(ctx, load_all_coeffs(coeff_dir), use_hard_renorm_between_steps=True, fuse_sub_ark=True)
    np.random.seed(7)
    key = np.random.randint(0, 256, 16, dtype=np.uint8)
    pt = np.random.randint(0, 256, 16, dtype=np.uint8)
    rks = expand_aes128_key(key)
    dbg = {}
    ct = pipe.encrypt(pt, rks, debug=dbg)
    assert np.array_equal(pipe.encoder.decode(*ct), A.ref_encrypt(pt, rks))
    assert np.array_equal(dbg["enc.final.sub_ark"]["plain"], A.SBOX[dbg["enc.r9.ark.renorm"]["plain"]] ^ A.inv_shift_rows(rks[10]))
    back = pipe.decrypt(*ct, rks, debug=dbg)
    assert np.array_equal(pipe.encoder.decode(*back), pt)
    assert "dec.r5.isb_ark" in dbg and "dec.r5.isb" not in dbg


def test_pipeline_fused_packed_roundtrip(ctx, coeff_dir):
    from aes_keyschedule import expand_aes128_key, load_all_coeffs
    from oracle import aes_plain as A
    from pipeline import AESPipeline
    B = 64
    pipe = AESPipeline(ctx, load_all_coeffs(coeff_dir), use_hard_renorm_between_steps=True, states=B, fuse_sub_ark=True)
    rng = np.random.default_rng(8)
    rks = expand_aes128_key(rng.integers(0, 256, 16).astype(np.uint8))
    pts = rng.integers(0, 256, (B, 16)).astype(np.uint8)
    ct = pipe.encrypt(pts, rks)
    got = pipe.encoder.decode(*ct)
    assert all(np.array_equal(got[j], A.ref_encrypt(pts[j], rks)) for j in range(B))
    assert np.array_equal(pipe.encoder.decode(*pipe.decrypt(*ct, rks)), pts)


def test_shiftrows_mixcolumns_merged(ctx, coeff_dir):
    """ShiftRows merged into MixColumns' rotations (shiftrows_mixcolumns.py): the step alone with
    the final bootstrap, then a C2 encrypt with both fusions, every debug stage checked"""
    from aes_keyschedule import expand_aes128_key, load_all_coeffs
    from mixcol_final import MixColFinal
    from oracle import aes_plain as A
    from pipeline import AESPipeline
    from shiftrows_mixcolumns import ShiftRowsMixColumnsFusedEnc
    from state_encoder import StateEncoder
    from xor4_lut import XOR4LUT
    co = load_all_coeffs(coeff_dir)
    enc = StateEncoder(ctx)
    srmc = ShiftRowsMixColumnsFusedEnc(ctx, MixColFinal(ctx, XOR4LUT(ctx, co["xor4"])))
    rng = np.random.default_rng(41)
    x = rng.integers(0, 256, 16).astype(np.uint8)
    dbg = {}
    out = srmc(*enc.encode(x), debug=dbg)
    assert np.array_equal(enc.decode(*dbg["sr"]), A.shift_rows(x))
    assert np.array_equal(enc.decode(*out), A.ref_mix_columns(A.shift_rows(x)))
    assert out[0].level == ctx.engine.fresh_level
    pipe = AESPipeline(ctx, co, use_hard_renorm_between_steps=True, fuse_sr_mc=True, fuse_sub_ark=True)
    np.random.seed(42)
    key = np.random.randint(0, 256, 16, dtype=np.uint8)
    pt = np.random.randint(0, 256, 16, dtype=np.uint8)
    rks = expand_aes128_key(key)
    ct = pipe.encrypt(pt, rks, debug=dbg)
    assert np.array_equal(pipe.encoder.decode(*ct), A.ref_encrypt(pt, rks))
    s = pt ^ rks[0]
    for r in range(1, 10):
        s = A.SBOX[s]
        assert np.array_equal(dbg[f"enc.r{r}.sr"]["plain"], A.shift_rows(s)), r
        s = A.ref_mix_columns(A.shift_rows(s))
        assert np.array_equal(dbg[f"enc.r{r}.mc"]["plain"], s), r
        s = s ^ rks[r]
    assert np.array_equal(pipe.encoder.decode(*pipe.decrypt(*ct, rks)), pt)
