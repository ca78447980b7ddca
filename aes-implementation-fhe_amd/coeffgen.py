"""Coefficient generator for the Zeta16 LUT polynomials.

Produces the same JSON files the reference ships in REF/gen/coeff/ (format read by
REF/lut.py:10-62) from truth tables, by inverse DFT over the 16th / 256th roots of
unity ζ = e^{-2πi/n}:

* 8->4 LUTs (SubBytes / InvSubBytes / split), REF/gen/generate_sobx_coeffs.py:65-120:
  a_k = (1/256) Σ_j ζ16^{f(j)} ζ256^{-jk}, so Σ_k a_k (ζ256^j)^k = ζ16^{f(j)}.
* GF(2^8) constant multipliers on (hi, lo) nibbles, REF/gen/generate_gf_mult_2var_coeff.py:15-113:
  c[p,q] = (1/256) Σ_{h,l} ζ16^{nib(k·(16h+l))} ζ16^{-(ph+ql)}.
* 4-bit XOR, REF/gen/generate_xor4_coeffs.py:10-54 -- keeps the reference's n^2 factor
  (REF/gen/generate_xor4_coeffs.py:17): Σ c[p,q] x^p y^q = 256·ζ16^{a⊕b}
  (the pipeline's renorm re-anchors the magnitude).
* Zeta16 snap polynomial (REF/gen/make_zeta16_snap_coeffs.py:11-56): ridge
  least-squares fit of z -> nearest ζ16 codeword on the unit circle.

Run ``python coeffgen.py [outdir]``; the engine's modules load ./coeff/ by default.
"""
from __future__ import annotations

import json
import sys
from pathlib import Path

import numpy as np

COEFF_DIR = Path(__file__).resolve().parent / "coeff"


def _gf_mul(a: int, b: int) -> int:
    out = 0
    while b:
        if b & 1:
            out ^= a
        a = ((a << 1) ^ (0x1B if a & 0x80 else 0)) & 0xFF
        b >>= 1
    return out


def _sboxes():
    inv = [0] * 256
    for x in range(1, 256):
        inv[x] = next(y for y in range(1, 256) if _gf_mul(x, y) == 1)
    rotl = lambda b, k: ((b << k) | (b >> (8 - k))) & 0xFF
    s = [inv[x] ^ rotl(inv[x], 1) ^ rotl(inv[x], 2) ^ rotl(inv[x], 3) ^ rotl(inv[x], 4) ^ 0x63 for x in range(256)]
    si = [0] * 256
    for x, y in enumerate(s):
        si[y] = x
    return s, si


def _zeta(n: int) -> complex:
    return np.exp(-2j * np.pi / n)


def lut_8to4(table) -> np.ndarray:
    """256-point inverse DFT of ζ16^{table[j]} (1-D LUT over ζ256 inputs)."""
    samples = _zeta(16) ** np.asarray(table, dtype=np.int64)
    return np.fft.ifft(samples)


def lut_bivariate(f, scale: float = 1.0) -> np.ndarray:
    """c[p,q] with Σ c[p,q] ζ16^{ph+ql} = scale·ζ16^{f(h,l)}."""
    F = np.array([[_zeta(16) ** f(h, l) for l in range(16)] for h in range(16)])
    return np.fft.ifft2(F) * scale


def _entries_1d(a, tol):
    return [[int(k), float(c.real), float(c.imag)] for k, c in enumerate(a) if abs(c) > tol]


def _entries_2d(A, tol):
    return [[int(p), int(q), float(A[p, q].real), float(A[p, q].imag)]
            for p in range(A.shape[0]) for q in range(A.shape[1]) if abs(A[p, q]) > tol]


def snap_poly(deg: int = 15, n_samples: int = 8192, ridge: float = 1e-5) -> np.ndarray:
    theta = np.linspace(0, 2 * np.pi, n_samples, endpoint=False)
    x = np.exp(1j * theta)
    k = np.round((theta % (2 * np.pi)) / (2 * np.pi / 16)).astype(np.int64) % 16
    y = np.exp(1j * 2 * np.pi * k / 16.0)
    V = x[:, None] ** np.arange(deg + 1)[None, :]
    A = V.conj().T @ V + ridge * np.eye(deg + 1)
    return np.linalg.solve(A, V.conj().T @ y)


def generate(out_dir: Path = COEFF_DIR) -> dict:
    out_dir = Path(out_dir)
    out_dir.mkdir(parents=True, exist_ok=True)
    sbox, inv_sbox = _sboxes()
    files = {}

    def put(name, obj, indent=2):
        files[name] = obj
        (out_dir / name).write_text(json.dumps(obj, indent=indent), encoding="utf-8")

    one_d = {
        "split_mod256_to_16_hi.json": [x >> 4 for x in range(256)],
        "split_mod256_to_16_lo.json": [x & 15 for x in range(256)],
        "mod256_to_16_hi.json": [y >> 4 for y in sbox],
        "mod256_to_16_lo.json": [y & 15 for y in sbox],
        "inv_mod256_to_16_hi.json": [y >> 4 for y in inv_sbox],
        "inv_mod256_to_16_lo.json": [y & 15 for y in inv_sbox],
    }
    for name, table in one_d.items():
        put(name, {"entries": _entries_1d(lut_8to4(table), 1e-12)})

    for mult in (1, 2, 3, 9, 11, 13, 14):
        for which, nib in (("hi", lambda y: y >> 4), ("lo", lambda y: y & 15)):
            C = lut_bivariate(lambda h, l: nib(_gf_mul((h << 4) | l, mult)))
            put(f"gf_mult{mult}_{which}_coeffs.json",
                {"entries": _entries_2d(C, 1e-12), "multiplier": mult, "which": which, "domain": "zeta16", "size": 16},
                indent=0)

    put("xor4_coeffs.json", {"entries": _entries_2d(lut_bivariate(lambda a, b: a ^ b, 256.0), 1e-8)})
    put("zeta16_snap_coeffs.json", {"type": "zeta16_snap_1d_poly", "entries": _entries_1d(snap_poly(), -1.0)})
    return files


if __name__ == "__main__":
    generate(Path(sys.argv[1]) if len(sys.argv) > 1 else COEFF_DIR)
