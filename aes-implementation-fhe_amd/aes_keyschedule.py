"""Round-key expansion and coefficient bundle of the reference harness
(REF/test/test_aes_pipeline_roundtrip.py:20-110).

``expand_aes128_key`` is the FIPS-197 AES-128 key schedule (11 round keys, 16 bytes each,
column-first); ``load_all_coeffs`` returns the dict AESPipeline expects.
"""
from __future__ import annotations

from pathlib import Path
from typing import Any, Dict, List

import numpy as np

from lut import COEFF_DIR, ensure_coeffs, load_coeff1d, load_coeff2d


def _xtime(b: int) -> int:
    return ((b << 1) ^ (0x1B if b & 0x80 else 0)) & 0xFF


def _sbox() -> np.ndarray:
    # log/antilog tables over generator 3, then the FIPS-197 affine transform
    exp, log = [0] * 255, [0] * 256
    x = 1
    for i in range(255):
        exp[i] = x
        log[x] = i
        x ^= _xtime(x)
    out = []
    for v in range(256):
        inv = 0 if v == 0 else exp[(255 - log[v]) % 255]
        s = inv
        for k in range(1, 5):
            s ^= ((inv << k) | (inv >> (8 - k))) & 0xFF
        out.append(s ^ 0x63)
    return np.array(out, dtype=np.uint8)


SBOX = _sbox()
RCON = np.array([0x01, 0x02, 0x04, 0x08, 0x10, 0x20, 0x40, 0x80, 0x1B, 0x36], dtype=np.uint8)


def expand_aes128_key(master: np.ndarray) -> List[np.ndarray]:
    master = np.asarray(master, dtype=np.uint8)
    assert master.shape == (16,)
    words = [master[4 * i:4 * i + 4].copy() for i in range(4)]
    for i in range(4, 44):
        t = words[i - 1].copy()
        if i % 4 == 0:
            t = SBOX[np.roll(t, -1)]
            t[0] ^= RCON[i // 4 - 1]
        words.append(words[i - 4] ^ t)
    return [np.concatenate(words[4 * r:4 * r + 4]).astype(np.uint8) for r in range(11)]


def load_all_coeffs(coeff_dir: Path = COEFF_DIR) -> Dict[str, Any]:
    d = ensure_coeffs(coeff_dir)
    return {
        "xor4": load_coeff2d(d / "xor4_coeffs.json", 16),
        "sub_hi": load_coeff1d(d / "mod256_to_16_hi.json"),
        "sub_lo": load_coeff1d(d / "mod256_to_16_lo.json"),
        "inv_sub_hi": load_coeff1d(d / "inv_mod256_to_16_hi.json"),
        "inv_sub_lo": load_coeff1d(d / "inv_mod256_to_16_lo.json"),
    }
