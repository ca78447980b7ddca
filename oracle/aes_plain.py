"""oracle/aes_plain.py -- TEST INFRASTRUCTURE, NOT PRODUCT CODE.

Byte-level plaintext models of the reference's AES round logic, restated from the
reference's own self-test models:

* S-box / inverse S-box tables          REF/gen/generate_sobx_coeffs.py (SBOX / INV_SBOX tables)
* FIPS-197 key expansion                REF/test/test_aes_pipeline_roundtrip.py:95-110
* ShiftRows / InvShiftRows (col-first)  REF/shift_rows.py:67-72, REF/inv_shiftrows.py:51-70
* MixColFinal orientation               REF/mixcol_final.py:101-102,112-165 -- out[r,c] =
  2a[r,c] ^ 3a[r,c+1] ^ a[r,c+2] ^ a[r,c+3] under column-first packing
* InvMixColumnsFHE orientation          REF/invmixcolumns_fhe.py:128-170

``ref_encrypt`` is the cipher the reference's AESPipeline.encrypt computes
(REF/pipeline.py:123-188); ``ref_decrypt`` is its inverse with InvMixColumns
inserted after AddRoundKey (REF/README.md:87-94; the shipped REF/pipeline.py:230-237
omits it -- SURVEY quirk 4c).  ``fips_encrypt`` is FIPS-197 AES-128 for the KATs.
"""
from __future__ import annotations

import numpy as np


def _gf_mul(a: int, b: int) -> int:
    r = 0
    for _ in range(8):
        if b & 1:
            r ^= a
        hi = a & 0x80
        a = (a << 1) & 0xFF
        if hi:
            a ^= 0x1B
        b >>= 1
    return r


def _build_sbox():
    # multiplicative inverse in GF(2^8) followed by the FIPS-197 affine map
    inv = [0] * 256
    for x in range(1, 256):
        for y in range(1, 256):
            if _gf_mul(x, y) == 1:
                inv[x] = y
                break
    sbox = []
    for x in range(256):
        b = inv[x]
        s = b
        for k in range(1, 5):
            s ^= ((b << k) | (b >> (8 - k))) & 0xFF
        sbox.append(s ^ 0x63)
    inv_sbox = [0] * 256
    for x, s in enumerate(sbox):
        inv_sbox[s] = x
    return np.array(sbox, np.uint8), np.array(inv_sbox, np.uint8)


SBOX, INV_SBOX = _build_sbox()
RCON = np.array([0x01, 0x02, 0x04, 0x08, 0x10, 0x20, 0x40, 0x80, 0x1B, 0x36], np.uint8)
GF_MUL = np.array([[_gf_mul(x, k) for x in range(256)] for k in range(16)], np.uint8)  # GF_MUL[k][x]


def expand_key(master) -> list:
    """FIPS-197 AES-128 key schedule -> 11 round keys (16 bytes, column-first)."""
    w = [list(np.asarray(master, np.uint8)[4 * i: 4 * i + 4]) for i in range(4)]
    for i in range(4, 44):
        t = list(w[i - 1])
        if i % 4 == 0:
            t = t[1:] + t[:1]
            t = [int(SBOX[b]) for b in t]
            t[0] ^= int(RCON[i // 4 - 1])
        w.append([w[i - 4][j] ^ t[j] for j in range(4)])
    return [np.array(sum(w[4 * r: 4 * r + 4], []), np.uint8) for r in range(11)]


def _as_mat(state16):
    """column-first 16-vector -> 4x4 matrix M[r, c] = state[r + 4c]"""
    return np.asarray(state16, np.uint8).reshape(4, 4).T.copy()


def _as_vec(M):
    return np.ascontiguousarray(M.T).reshape(16).astype(np.uint8)


def shift_rows(s):
    M = _as_mat(s)
    return _as_vec(np.stack([np.roll(M[r], -r) for r in range(4)]))


def inv_shift_rows(s):
    M = _as_mat(s)
    return _as_vec(np.stack([np.roll(M[r], r) for r in range(4)]))


def _row_mix(s, coeffs):
    """out[r,c] = XOR_k coeffs[k] * a[r, c+k] (the reference's column-rotate recipe)."""
    M = _as_mat(s)
    out = np.zeros_like(M)
    for k, m in enumerate(coeffs):
        out ^= GF_MUL[m][np.roll(M, -k, axis=1)]
    return _as_vec(out)


def ref_mix_columns(s):
    return _row_mix(s, (2, 3, 1, 1))


def ref_inv_mix_columns(s):
    return _row_mix(s, (14, 11, 13, 9))


def fips_mix_columns(s):
    M = _as_mat(s)
    out = np.zeros_like(M)
    for k, m in enumerate((2, 3, 1, 1)):
        out ^= GF_MUL[m][np.roll(M, -k, axis=0)]
    return _as_vec(out)


def ref_encrypt(pt, rks):
    """REF/pipeline.py:123-188 on bytes."""
    s = np.asarray(pt, np.uint8) ^ rks[0]
    for r in range(1, 10):
        s = ref_mix_columns(shift_rows(SBOX[s])) ^ rks[r]
    return shift_rows(SBOX[s]) ^ rks[10]


def ref_decrypt(ct, rks):
    """Inverse of ref_encrypt: REF/pipeline.py:193-254 with InvMixColumns after ARK."""
    s = np.asarray(ct, np.uint8) ^ rks[10]
    for r in range(9, 0, -1):
        s = ref_inv_mix_columns(INV_SBOX[inv_shift_rows(s)] ^ rks[r])
    return INV_SBOX[inv_shift_rows(s)] ^ rks[0]


def fips_encrypt(pt, rks):
    s = np.asarray(pt, np.uint8) ^ rks[0]
    for r in range(1, 10):
        s = fips_mix_columns(shift_rows(SBOX[s])) ^ rks[r]
    return shift_rows(SBOX[s]) ^ rks[10]
