"""SubBytes / InvSubBytes via two 8->4 LUT polynomials sharing one power basis
(REF/sub_bytes_lut.py:8-73).

1. lift lo: L(y) = Σ_{k<16} ℓ_k y^k with ℓ = ifft(ζ256^0..15) maps ζ16^l -> ζ256^l;
2. b = hi · L(lo) = ζ256^(16h + l) = ζ256^byte;
3. out_hi / out_lo = Σ_{k=1..255} H[k] / Lo[k] · b^k with b^k = conj(b^(256-k)) for k > 128.

``SubBytesLUT`` is the name AESPipeline imports (REF/pipeline.py:9); the snapshot only
defines ``SubBytesLUTFastCached``, so both names are provided.
"""
from typing import Any, Dict, Tuple

import numpy as np
from utils import fused_lut, pair

_TOL = 1e-12


class SubBytesLUTFastCached:
    def __init__(self, ctx, hi_coeffs: np.ndarray, lo_coeffs: np.ndarray):
        self.ctx = ctx
        self.sc = ctx.engine.slot_count
        self.hi = np.asarray(hi_coeffs, dtype=np.complex128)
        self.lo = np.asarray(lo_coeffs, dtype=np.complex128)
        const = lambda c: ctx.encode(np.full(self.sc, c, dtype=np.complex128))

        self.ks_hi = [k for k, c in enumerate(self.hi) if abs(c) > _TOL]
        self.ks_lo = [k for k, c in enumerate(self.lo) if abs(c) > _TOL]
        union = sorted(set(self.ks_hi) | set(self.ks_lo))
        self.ks_union = [k for k in union if k != 0]
        self.deg256 = min(max(union) if union else 0, 128)
        self.pt_hi: Dict[int, Any] = {k: const(self.hi[k]) for k in self.ks_hi}
        self.pt_lo: Dict[int, Any] = {k: const(self.lo[k]) for k in self.ks_lo}
        self.c0_hi = self.hi[0] if self.hi.size else 0j
        self.c0_lo = self.lo[0] if self.lo.size else 0j

        lift = np.fft.ifft(np.exp(-2j * np.pi * np.arange(16) / 256))
        self.ks_lift = [k for k, c in enumerate(lift) if k != 0 and abs(c) > _TOL]
        self.deg16 = min(max(self.ks_lift) if self.ks_lift else 0, 8)
        self.pt_lift = {k: const(lift[k]) for k in self.ks_lift}
        self.c0_lift = lift[0]
        # the same sums as coefficient vectors for the fused LUT form
        self.vec_lift = np.where(np.abs(lift) > _TOL, lift, 0)
        self.vec_lift[0] = 0
        self.vec_hi, self.vec_lo = np.zeros(256, np.complex128), np.zeros(256, np.complex128)
        for k in self.ks_union:
            self.vec_hi[k] = self.hi[k] if k in self.pt_hi else 0
            self.vec_lo[k] = self.lo[k] if k in self.pt_lo else 0

    @staticmethod
    def _power(basis, k: int, domain: int, ctx):
        return basis[k - 1] if k <= len(basis) else ctx.conjugate(basis[domain - k - 1])

    def apply(self, ct_hi: Any, ct_lo: Any) -> Tuple[Any, Any]:
        ctx = self.ctx
        # 1) ζ16^l -> ζ256^l
        pos16 = ctx.make_power_basis(ct_lo, self.deg16) if self.deg16 > 0 else []
        p16 = {k: self._power(pos16, k, 16, ctx) for k in self.ks_lift}
        lifted = fused_lut(ctx, ("sb-lift", id(self)), self.vec_lift, p16, c0=self.c0_lift)
        if lifted is None:
            lifted = ctx.add_plain(ctx.multiply(ct_lo, 0.0), self.c0_lift)
            for k in self.ks_lift:
                lifted = ctx.add(lifted, ctx.multiply(p16[k], self.pt_lift[k]))
        # 2) ζ256^byte
        ct_b = ctx.multiply(ct_hi, lifted)
        # 3) one shared 128-power basis, two 255-term sums
        pos256 = ctx.make_power_basis(ct_b, self.deg256) if self.deg256 > 0 else []
        # b^k for every used k; the conjugate mirrors (k > 128) once each, split over two streams
        mirror = [k for k in self.ks_union if k > len(pos256)]
        half = len(mirror) // 2
        ma, mb = pair(ctx, lambda: {k: self._power(pos256, k, 256, ctx) for k in mirror[:half]},
                      lambda: {k: self._power(pos256, k, 256, ctx) for k in mirror[half:]})
        bk = {**ma, **mb}
        bk.update({k: pos256[k - 1] for k in self.ks_union if k <= len(pos256)})

        def lut(pts, c0):
            res = fused_lut(ctx, ("sb", id(self), pts is self.pt_hi), self.vec_hi if pts is self.pt_hi else self.vec_lo,
                            bk, c0=c0)
            if res is not None:
                return res
            res = ctx.add_plain(ctx.multiply(ct_b, 0.0), c0)
            for k in self.ks_union:
                if k in pts:
                    res = ctx.add(res, ctx.multiply(bk[k], pts[k]))
            return res

        return pair(ctx, lambda: lut(self.pt_hi, self.c0_hi), lambda: lut(self.pt_lo, self.c0_lo), shared=(ct_b,))

    __call__ = apply


SubBytesLUT = SubBytesLUTFastCached
