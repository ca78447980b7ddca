"""SubBytes ⊕ AddRoundKey as one fused LUT per output nibble (the fusion the
reference plans in REF/README.md:133-135, "SubBytes xor AddRoundKey as a single bivariate
nibble LUT", and "likewise on decryption with InvSubBytes xor AddRoundKey").

For one output nibble (hi or lo) of S (the S-box or its inverse) and a round-key nibble k:

    F(b, y) = XOR4(ζ16^{S_n(x)}, ζ16^k),   b = ζ256^x (the byte lift of SubBytes), y = ζ16^k

a bivariate LUT over the byte lift b and the key nibble y.  With the XOR4 coefficients C
(REF/xor4_lut.py:63-74) in the conjugate-split form S1 + conj(S2) (xor4_lut.SplitLUT2), the
powers of the first XOR4 input a = ζ16^{S_n(x)} it needs (a^1, a^3, a^5, a^7 for the XOR4
set) are NOT formed by products of a: each a^p = ζ16^{p S_n(x)} is itself a univariate LUT
of b, with coefficients

    L_p = ifft_256( t(x)^p ),   t(x) = Σ_k H[k] ζ256^{k x} = ζ16^{S_n(x)}   (H: the SubBytes
                                                                            hi / lo JSON set)

evaluated on the SAME baby / giant steps of b as SubBytes itself (sub_bytes_lut BSGS form).
So the XOR4 of the unfused path -- its power basis of the SubBytes output (depth 3), the
renorm between SubBytes and AddRoundKey -- disappears: depth SubBytes + 2 (product with the
key basis, coefficient), one renorm instead of two, the same output as
XOR4(SubBytes(x), k) (the reference's 256x XOR4 magnitude included).

Byte-wise maps commute with ShiftRows, so the pipeline also fuses across it:
SR(SB(x)) ⊕ k = SR(SB(x) ⊕ SR⁻¹(k)) (encrypt, last round) and ISB(ISR(x)) ⊕ k =
ISR(ISB(x) ⊕ SR(k)) (decrypt) with the permuted round key encrypted instead
(pipeline.AESPipeline(fuse_sub_ark=True)).
"""
from __future__ import annotations

from typing import Any, Dict, Tuple

import numpy as np

from sub_bytes_lut import SubBytesLUTFastCached
from utils import SUB_ARK_DEPTH, can_fork, pair  # noqa: F401 (SUB_ARK_DEPTH re-exported)
from xor4_lut import SplitLUT2, std_basis


def fused_powers(H: np.ndarray, powers) -> Dict[int, np.ndarray]:
    """{p: L_p}: coefficients over b^0..b^255 of ζ16^{p S_n(x)}, from the SubBytes nibble LUT H
    (t(x) = Σ_k H[k] ζ256^{kx} = ζ16^{S_n(x)} on the 256 codewords, renormalised to |t| = 1)"""
    x = np.arange(256)
    Hd = np.zeros(256, np.complex128)
    Hd[: len(H)] = H
    t = np.exp(-2j * np.pi * np.outer(x, np.arange(256)) / 256) @ Hd
    t = t / np.abs(t)
    out = {}
    for p in powers:
        L = np.fft.ifft(t ** p)  # sum_k L[k] e^{-2 pi i k x / 256} = t(x)^p
        out[p] = np.where(np.abs(L) > 1e-13, L, 0)
    return out


def fused_table(H: np.ndarray, C: np.ndarray) -> Tuple[SplitLUT2, Dict[int, np.ndarray]]:
    """(the split XOR4 form, {p: L_p} for every power p of the first input it uses)"""
    sp = SplitLUT2(C)
    return sp, fused_powers(H, sorted(p for p in sp.need_a if p >= 1))


class SubBytesARK:
    """(S_hi(x) ⊕ k_hi, S_lo(x) ⊕ k_lo) as two fused LUTs; S = the S-box of `sub` (a
    SubBytesLUT built with the forward or inverse coefficient set), ⊕ = the XOR4 set `xor4`."""

    def __init__(self, sub: SubBytesLUTFastCached, xor4_coeffs: np.ndarray):
        self.sub = sub
        self.ctx = sub.ctx
        self.split = SplitLUT2(xor4_coeffs)
        self.pows = {"hi": fused_powers(sub.hi, sorted(p for p in self.split.need_a if p >= 1)),
                     "lo": fused_powers(sub.lo, sorted(p for p in self.split.need_a if p >= 1))}
        self._key_basis: Dict[int, Any] = {}

    def _ensure_splits(self):
        bs = self.sub._ensure_bsgs()
        for n in ("hi", "lo"):
            for p, L in self.pows[n].items():
                if (n, p) not in bs:
                    bs[(n, p)] = self.sub._split(L, 128)

    def key_basis(self, key_ct) -> Dict[int, Any]:
        """the standard basis of a round-key nibble ciphertext the split needs (cached per key
        ciphertext: the encrypted round keys are reused by every call)"""
        kid = id(key_ct)
        hit = self._key_basis.get(kid)
        if hit is not None and hit[0] is key_ct:
            return hit[1]
        B = std_basis(self.ctx, key_ct, self.split.need_b)
        self._key_basis[kid] = (key_ct, B)
        return B

    def apply(self, ct_hi, ct_lo, key_hi, key_lo) -> Tuple[Any, Any]:
        ctx = self.ctx
        if not getattr(ctx, "fused_luts", False) or getattr(ctx, "multiply_many", None) is None:
            raise RuntimeError("SubBytesARK needs the engine's fused LUT op and batched products")
        self._ensure_splits()
        s = self.sub
        baby, g, ct_b = s._bsgs_bases(ct_hi, ct_lo)
        Bh, Bl = self.key_basis(key_hi), self.key_basis(key_lo)

        def nibble(n, B):
            whiches = [(n, p) for p in sorted(self.pows[n])]
            A = dict(zip((p for _, p in whiches), s._outputs_batched(baby, g, ct_b, whiches)))
            return self.split.eval(ctx, ("sbark", n), A, B)

        if can_fork(ctx):
            return pair(ctx, lambda: nibble("hi", Bh), lambda: nibble("lo", Bl),
                        shared=(*baby.values(), *g.values(), *Bh.values(), *Bl.values()))
        return nibble("hi", Bh), nibble("lo", Bl)

    __call__ = apply
