"""XOR4LUT: 4-bit XOR as a bivariate LUT polynomial (REF/xor4_lut.py:10-78).

    XOR(a, b) = Σ_{p,q} C[p,q] A^p B^q,   A^k = a^k (k <= 8), conj(a^(16-k)) (k >= 9)

with C from xor4_coeffs.json (only odd p, q are non-zero; the output carries the
reference's 256x magnitude).  Depth 5: power basis 3, product 1,
coefficient 1.
"""
from typing import Any, Dict

import numpy as np
from utils import fused_lut, pair


def basis16(ctx, ct, *, retry_intt: bool = True) -> Dict[int, Any]:
    """1, x..x^8, conj(x^7)..conj(x^1) with the reference's level fallbacks (REF/xor4_lut.py:27-60)."""
    try:
        pos = ctx.make_power_basis(ct, 8)
    except RuntimeError:
        if retry_intt:
            try:
                ct = ctx.to_intt(ct)
            except RuntimeError:
                pass
            try:
                pos = ctx.make_power_basis(ct, 8)
            except RuntimeError:
                ct = ctx.bootstrap(ct)
                pos = ctx.make_power_basis(ct, 8)
        else:
            ct = ctx.bootstrap(ct)
            pos = ctx.make_power_basis(ct, 8)
    basis = {0: ctx.add_plain(ctx.sub(ct, ct), 1.0)}
    basis.update({k: pos[k - 1] for k in range(1, 9)})
    basis.update({k: ctx.conjugate(pos[15 - k]) for k in range(9, 16)})
    return basis


class XOR4LUT:
    def __init__(self, ctx, coeffs: np.ndarray):
        self.ctx = ctx
        self.sc = ctx.engine.slot_count
        self.coeffs = coeffs
        self.pt = {(p, q): ctx.encode(np.full(self.sc, coeffs[p, q], dtype=np.complex128))
                   for p in range(16) for q in range(16) if abs(coeffs[p, q]) > 1e-12}

    def _build_power_basis_16(self, ct: Any) -> Dict[int, Any]:
        return basis16(self.ctx, ct)

    def apply(self, a_ct, b_ct):
        ctx = self.ctx
        A, B = pair(ctx, lambda: self._build_power_basis_16(a_ct), lambda: self._build_power_basis_16(b_ct))
        out = fused_lut(ctx, "xor4", self.coeffs, A, B)  # one kernel for all 64 terms
        if out is not None:
            return out
        acc = ctx.sub(A[0], A[0])
        for (p, q), pt in self.pt.items():
            acc = ctx.add(acc, ctx.multiply(ctx.multiply(A[p], B[q]), pt))
        return acc

    __call__ = apply
