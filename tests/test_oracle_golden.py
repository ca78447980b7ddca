"""CPU checks of the oracle against everything the reference itself pins:
its LUT coefficient files (tests/golden/ref_coeff.npz, from REF/gen/coeff/*.json), the
plaintext models of its self-tests, and FIPS-197.  No GPU, no reference code."""
import json

import numpy as np
import pytest

from conftest import GOLDEN

from oracle import aes_plain as A
from oracle import golden_model as G

Z16 = np.exp(-2j * np.pi / 16)
CODE = Z16 ** np.arange(16)  # nibble v -> zeta16^v (REF/utils.py:8-19)


def _hex(s):
    return np.frombuffer(bytes.fromhex(s), np.uint8)


# ---------------------------------------------------------------- coefficient files
def test_coeffgen_reproduces_reference_files(ref_coeffs, coeff_dir):
    """Our coeffgen.py regenerates all 22 JSON files the reference ships."""
    assert len(ref_coeffs) == 22
    for stem, ref in ref_coeffs.items():
        path = coeff_dir / f"{stem}.json"
        mine = G.load_2d(path) if ref.ndim == 2 else G.load_1d(path)
        n = max(len(ref), len(mine))
        a = np.zeros(n if ref.ndim == 1 else (16, 16), np.complex128)
        b = a.copy()
        a[tuple(slice(0, s) for s in ref.shape)] = ref
        b[tuple(slice(0, s) for s in mine.shape)] = mine
        assert np.abs(a - b).max() < 1e-12, stem


def test_xor4_lut_exact_on_all_pairs(ref_coeffs):
    """XOR4(a, b) = 256 zeta^(a xor b) on all 256 codeword pairs."""
    C = ref_coeffs["xor4_coeffs"]
    a, b = np.meshgrid(np.arange(16), np.arange(16), indexing="ij")
    out = G.bivariate(C, CODE[a.ravel()], CODE[b.ravel()])
    assert np.abs(out - 256.0 * CODE[(a ^ b).ravel()]).max() < 1e-8
    assert np.count_nonzero(np.abs(C) > 1e-12) == 64
    assert np.all(np.abs(C[::2, :]) < 1e-12) and np.all(np.abs(C[:, ::2]) < 1e-12)


@pytest.mark.parametrize("m", [1, 2, 3, 9, 11, 13, 14])
def test_gf_luts_exact_unit_magnitude(ref_coeffs, m):
    """gf_mult{m}_{hi|lo}(hi, lo) = zeta^(nibble of m * byte) on all 256 bytes."""
    byte = np.arange(256)
    hi, lo = CODE[byte >> 4], CODE[byte & 15]
    prod = A.GF_MUL[m][byte].astype(int)
    for which, nib in (("hi", prod >> 4), ("lo", prod & 15)):
        out = G.bivariate(ref_coeffs[f"gf_mult{m}_{which}_coeffs"], hi, lo)
        assert np.abs(out - CODE[nib]).max() < 1e-8, (m, which)


@pytest.mark.parametrize("inverse", [False, True])
def test_subbytes_luts_exact(ref_coeffs, inverse):
    """Lift + 255-term hi/lo sums give S(byte) (or S^-1) nibbles on all 256 bytes."""
    pre = "inv_" if inverse else ""
    H, L = ref_coeffs[f"{pre}mod256_to_16_hi"], ref_coeffs[f"{pre}mod256_to_16_lo"]
    byte = np.arange(256)
    out_h, out_l = G.subbytes(CODE[byte >> 4], CODE[byte & 15], H, L)
    box = A.INV_SBOX if inverse else A.SBOX
    assert np.abs(out_h - CODE[box[byte] >> 4]).max() < 1e-6
    assert np.abs(out_l - CODE[box[byte] & 15]).max() < 1e-6


# ---------------------------------------------------------------- byte-level AES
def test_fips197_key_expansion():
    """FIPS-197 Appendix A.1."""
    from aes_keyschedule import expand_aes128_key
    rks = expand_aes128_key(_hex("2b7e151628aed2a6abf7158809cf4f3c"))
    assert bytes(rks[1]).hex() == "a0fafe1788542cb123a339392a6c7605"
    assert bytes(rks[10]).hex() == "d014f9a8c9ee2589e13f0cc8b6630ca6"
    assert all(np.array_equal(a, b) for a, b in zip(rks, A.expand_key(_hex("2b7e151628aed2a6abf7158809cf4f3c"))))


def test_fips197_cipher_kat():
    """FIPS-197 Appendix B and C.1 (standard MixColumns; pins S-box and key schedule)."""
    rks = A.expand_key(_hex("2b7e151628aed2a6abf7158809cf4f3c"))
    assert bytes(A.fips_encrypt(_hex("3243f6a8885a308d313198a2e0370734"), rks)).hex() == "3925841d02dc09fbdc118597196a0b32"
    rks = A.expand_key(_hex("000102030405060708090a0b0c0d0e0f"))
    assert bytes(A.fips_encrypt(_hex("00112233445566778899aabbccddeeff"), rks)).hex() == "69c4e0d86a7b0430d8cdb78070b4c55a"


def test_reference_mixcolumns_orientation():
    """REF/mixcol_final.py:169-221 self-test model: out[r,c] = 2a[r,c]^3a[r,c+1]^a[r,c+2]^a[r,c+3]
    with byte i = r + 4c (column-first packing) -- the reference's quirk 4b."""
    rng = np.random.default_rng(3)
    s = rng.integers(0, 256, 16).astype(np.uint8)
    a = s.reshape(4, 4, order="F")
    out = np.zeros((4, 4), np.uint8)
    for r in range(4):
        for c in range(4):
            out[r, c] = (A.GF_MUL[2][a[r, c]] ^ A.GF_MUL[3][a[r, (c + 1) % 4]]
                         ^ a[r, (c + 2) % 4] ^ a[r, (c + 3) % 4])
    assert np.array_equal(A.ref_mix_columns(s), out.ravel(order="F"))
    assert np.array_equal(A.ref_inv_mix_columns(A.ref_mix_columns(s)), s)


def test_shift_rows_models():
    """REF/shift_rows.py:67-72 and REF/inv_shiftrows.py:51-70: row r rotated left by r."""
    s = np.arange(16, dtype=np.uint8)
    m = s.reshape(4, 4, order="F")
    exp = np.stack([np.roll(m[r], -r) for r in range(4)])
    assert np.array_equal(A.shift_rows(s), exp.ravel(order="F"))
    assert np.array_equal(A.inv_shift_rows(A.shift_rows(s)), s)


# ---------------------------------------------------------------- committed stage fixture
@pytest.fixture(scope="module")
def stages():
    return json.loads((GOLDEN / "stages.json").read_text())


def test_stage_fixture_matches_byte_model(stages):
    for case in stages["seeds"]:
        rks = [np.array(k, np.uint8) for k in case["round_keys"]]
        pt = np.array(case["plaintext"], np.uint8)
        assert bytes(A.ref_encrypt(pt, rks)) == bytes(case["ciphertext"])
        assert np.array_equal(A.ref_decrypt(np.array(case["ciphertext"], np.uint8), rks), pt)


@pytest.mark.parametrize("idx", [0, 1, 2])
def test_golden_slot_model_matches_stages(stages, coeff_dir, idx):
    """The ideal-slot model of the reference modules (oracle/golden_model.py, LUT polynomials
    over Zeta16 slots) decodes to the committed per-stage bytes for seeds 0, 7, 42."""
    case = stages["seeds"][idx]
    rks = [np.array(k, np.uint8) for k in case["round_keys"]]
    got = {}
    ct = G.Golden(coeff_dir).encrypt(np.array(case["plaintext"], np.uint8), rks, sc=16, stages=got)
    for tag, exp in case["stages"].items():
        assert bytes(got[tag]) == bytes(exp), (case["seed"], tag)
    back = G.Golden(coeff_dir).decrypt(ct, rks, sc=16)
    assert bytes(G.decode_state(*back)) == bytes(case["plaintext"])


def test_config1_fixture(stages):
    c = stages["config1"]
    assert bytes(np.array(c["state"], np.uint8) ^ np.array(c["key"], np.uint8)) == bytes(c["ark"])
