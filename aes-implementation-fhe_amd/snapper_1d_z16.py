"""Homomorphic Zeta16 snap with a 1-D LUT polynomial over basis16 (REF/snapper_1d_z16.py:17-91).

Not reachable from AESPipeline in the reference; kept as the north_star-named renorm
option (the fitted polynomial barely contracts noise).
"""
from typing import Any, Dict

import numpy as np

from xor4_lut import basis16


class Zeta16Snap1D:
    def __init__(self, ctx, coeff_1d: np.ndarray, bootstrap_before: bool = False):
        self.ctx = ctx
        self.sc = ctx.engine.slot_count
        self.coeff = np.asarray(coeff_1d, dtype=np.complex128)
        self.K = len(self.coeff) - 1
        self.bootstrap_before = bootstrap_before
        self.pt: Dict[int, Any] = {k: ctx.encode(np.full(self.sc, c, dtype=np.complex128))
                                   for k, c in enumerate(self.coeff) if abs(c) > 1e-12}

    def _power_basis_16(self, ct):
        return basis16(self.ctx, ct, retry_intt=False)

    def apply(self, ct):
        ctx = self.ctx
        if self.bootstrap_before:
            ct = ctx.bootstrap(ct)
        basis = self._power_basis_16(ct)
        res = ctx.multiply(ct, 0.0)
        for k, pt in self.pt.items():
            res = ctx.add(res, ctx.multiply(basis[k % 16], pt))
        return res


class Zeta16SnapPair:
    def __init__(self, snap1d: Zeta16Snap1D):
        self.snap = snap1d

    def apply_pair(self, ct_hi, ct_lo):
        return self.snap.apply(ct_hi), self.snap.apply(ct_lo)
