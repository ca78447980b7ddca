"""SubBytes / InvSubBytes via two 8->4 LUT polynomials sharing one power basis
(REF/sub_bytes_lut.py:8-73).

1. lift lo: L(y) = Σ_{k<16} ℓ_k y^k with ℓ = ifft(ζ256^0..15) maps ζ16^l -> ζ256^l;
2. b = hi · L(lo) = ζ256^(16h + l) = ζ256^byte;
3. out_hi / out_lo = Σ_{k=1..255} H[k] / Lo[k] · b^k with b^k = conj(b^(256-k)) for k > 128.

``SubBytesLUT`` is the name AESPipeline imports (REF/pipeline.py:9); the snapshot only
defines ``SubBytesLUTFastCached``, so both names are provided.

Evaluation forms (same polynomials, same output level, outputs equal up to CKKS noise):

* direct (the reference's, used when the context has no fused LUT op): the 128-power basis
  of b, 127 conjugated mirrors b^k = conj(b^(256-k)), and a 255-term product loop per output;
* baby-step giant-step over the conjugate split: b is a 256th root of unity,
  so f(b) = sum_{k<=128} c_k b^k + conj(sum_{j<128} conj(c_{256-j}) b^j) = P(b) + conj(Q(b));
  P and Q (degree <= 128) are sum_i S_i(b) G_i with inner sums S_i over the baby steps
  b^1..b^15 (one fused LUT kernel each) and giant steps G_i = b^(16 i).  The lift is split
  the same way over y^1..y^8.  Key switches per SubBytes drop from ~270 to ~37.
"""
import os
from typing import Any, Dict, Tuple

import numpy as np
from utils import FOLDS, LUT2_DEPTH, SUBBYTES_DEPTH, can_fork, conj_many, drop_to, fused_lut, mul_many, pair

_TOL = 1e-12
# AESFHE_SB_NIB=0: the pipeline keeps the reference's 8 -> 4 form (lift to b = ζ256^byte, depth 13)
# instead of the nibble-bivariate form (depth LUT2_DEPTH) in the secret-key renorm mode (A/B runs)
_NIB = os.environ.get("AESFHE_SB_NIB", "1") != "0"


def nibble_matrix(coef256) -> np.ndarray:
    """the 8 -> 4 LUT sum_k a_k b^k (b = ζ256^(16h + l), REF/sub_bytes_lut.py:46-73) as the equivalent
    bivariate sum over the nibble inputs: C[p, q] with sum_{p,q} C[p, q] ζ16^(hp + lq) = the same
    ζ16^(out nibble) for all 256 (h, l) -- the table from the 1-D coefficients (a forward DFT,
    F[16h + l] = sum_k a_k ζ256^((16h + l) k), ζ = e^{-2πi/n} as in coeffgen.py), then its 2-D inverse
    DFT (coeffgen.lut_bivariate's form, the GF multipliers' coefficient layout)"""
    a = np.zeros(256, np.complex128)
    c = np.asarray(coef256, np.complex128)
    a[:min(256, c.size)] = c[:256]
    C = np.fft.ifft2(np.fft.fft(a).reshape(16, 16))
    C[np.abs(C) < 1e-12] = 0
    return C


class _NibbleLUTs:
    """the (hi, lo) output nibbles' bivariate matrices in mixcol_final._CoeffCache's interface, so
    that mixcol_final.gf_mult_pair evaluates SubBytes as it does the GF multipliers"""

    def __init__(self, hi_coeffs, lo_coeffs):
        self.mats = {"hi": nibble_matrix(hi_coeffs), "lo": nibble_matrix(lo_coeffs)}
        self.splits = {}
        self.pts = {}

    def matrix(self, mult, which: str) -> np.ndarray:
        return self.mats[which]

    def split(self, mult, which: str):
        from xor4_lut import SplitLUT2
        if which not in self.splits:
            self.splits[which] = SplitLUT2(self.mats[which])
        return self.splits[which]

    def load_plaintexts(self, ctx, mult, which: str):
        if which not in self.pts:
            sc = ctx.engine.slot_count
            M = self.mats[which]
            self.pts[which] = {(p, q): ctx.encode(np.full(sc, M[p, q], dtype=np.complex128))
                               for p in range(16) for q in range(16) if M[p, q] != 0}
        return self.pts[which]


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

    # nibble-bivariate form (round 5): out_hi / out_lo = sum_{p,q} C[p,q] hi^p lo^q, 16 x 16 each, by the
    # GF multipliers' machinery (two conjugate-split fused LUTs over one pair of bases):
    # depth LUT2_DEPTH = 5 instead of 13.  Off unless the owner enables it (AESPipeline in the
    # secret-key renorm mode: `use_nibble`)
    use_nibble = False

    def nibble_on(self) -> bool:
        from xor4_lut import batched
        return bool(self.use_nibble and _NIB and getattr(self.ctx, "fused_luts", False) and batched(self.ctx))

    def need_depth(self) -> int:
        """levels apply() consumes between its inputs and out_level"""
        return LUT2_DEPTH if self.nibble_on() else SUBBYTES_DEPTH

    def _apply_nibble(self, ct_hi: Any, ct_lo: Any, defer_conj: bool = False) -> Tuple[Any, Any]:
        from mixcol_final import gf_mult_pair
        if not hasattr(self, "_nib"):
            self._nib = _NibbleLUTs(self.hi, self.lo)
        return gf_mult_pair(self.ctx, self._nib, "sbox", ct_hi, ct_lo, defer_conj=defer_conj and FOLDS.conj)

    @staticmethod
    def _power(basis, k: int, domain: int, ctx):
        return basis[k - 1] if k <= len(basis) else ctx.conjugate(basis[domain - k - 1])

    def apply(self, ct_hi: Any, ct_lo: Any, out_level=None, defer_conj: bool = False) -> Tuple[Any, Any]:
        """(S_hi, S_lo)(hi, lo); out_level: the lowest level the caller needs the result at
        (inputs dropped to out_level + SUBBYTES_DEPTH first, utils.drop_to); None = as given.
        Inputs one level higher than that take the bivariate giant-step form (_outputs_biv).
        defer_conj: the nibble form may return utils.ConjSum outputs (for StateEncoder.renorm)."""
        if self.nibble_on():
            if out_level is not None:
                lv = out_level + LUT2_DEPTH
                ct_hi, ct_lo = drop_to(self.ctx, ct_hi, lv), drop_to(self.ctx, ct_lo, lv)
            return self._apply_nibble(ct_hi, ct_lo, defer_conj)
        biv = False
        if out_level is not None:
            lv = out_level + SUBBYTES_DEPTH
            if os.environ.get("AESFHE_SB_BIV", "1") != "0" and min(getattr(c, "level", -1) for c in (ct_hi, ct_lo)) > lv:
                biv, lv = True, lv + 1
            ct_hi, ct_lo = drop_to(self.ctx, ct_hi, lv), drop_to(self.ctx, ct_lo, lv)
        if getattr(self.ctx, "fused_luts", False):
            return self._apply_bsgs(ct_hi, ct_lo, biv)
        return self._apply_direct(ct_hi, ct_lo)

    # ------------------------------------------------------------------ BSGS form
    def _lin(self, key, vec, elems, c0, like):
        """c0 + sum_k vec[k] elems[k]: one fused kernel, or scalar products if unavailable"""
        out = fused_lut(self.ctx, key, vec, elems, c0=c0, owner=self)
        if out is not None:
            return out
        ctx = self.ctx
        res = ctx.add_plain(ctx.multiply(like, 0.0), complex(c0))
        for k, c in enumerate(vec):
            if c != 0 and k in elems:
                res = ctx.add(res, ctx.multiply(elems[k], complex(c)))
        return res

    @staticmethod
    def _split(c: np.ndarray, half: int):
        """f(x) = P(x) + conj(Q(x)) on roots of unity of order 2*half: P[k] = c[k] (k <= half),
        Q[j] = conj(c[2*half - j]) (1 <= j < half)"""
        c = np.where(np.abs(c) > _TOL, c, 0)
        P = np.zeros(half + 1, np.complex128)
        Q = np.zeros(half, np.complex128)
        n = min(len(c), half + 1)
        P[:n] = c[:n]
        for j in range(1, half):
            if 2 * half - j < len(c):
                Q[j] = np.conj(c[2 * half - j])
        return P, Q

    def _poly_bsgs(self, key, coef, baby, giant, like):
        """sum_i S_i G_i, S_i = sum_{j<16} coef[16 i + j] b^j (one fused kernel each)"""
        ctx = self.ctx
        acc = None
        for i in range((len(coef) + 15) // 16):
            chunk = np.zeros(16, np.complex128)
            seg = coef[16 * i: 16 * i + 16]
            chunk[: len(seg)] = seg
            if not np.any(chunk):
                continue
            if i == 0:
                term = self._lin((key, i), np.r_[0, chunk[1:]], baby, chunk[0], like)
            elif not np.any(chunk[1:]):
                term = ctx.multiply(giant[i], complex(chunk[0]))
            else:
                term = ctx.multiply(self._lin((key, i), np.r_[0, chunk[1:]], baby, chunk[0], like), giant[i])
            acc = term if acc is None else ctx.add(acc, term)
        return acc if acc is not None else ctx.multiply(like, 0.0)

    def _ensure_bsgs(self):
        """the conjugate-split coefficient sets: lift, hi, lo (sub_bytes_ark adds its own)"""
        if not hasattr(self, "_bsgs"):
            lift = np.fft.ifft(np.exp(-2j * np.pi * np.arange(16) / 256))
            lp, lq = self._split(lift, 8)
            self._bsgs = dict(lift=(lp, lq), hi=self._split(self.hi, 128), lo=self._split(self.lo, 128))
        return self._bsgs

    def _apply_bsgs(self, ct_hi: Any, ct_lo: Any, biv: bool = False) -> Tuple[Any, Any]:
        ctx = self.ctx
        baby, g, ct_b = self._bsgs_bases(ct_hi, ct_lo)
        if biv:
            out = self._outputs_biv(baby, g, ct_b)
            if out is not None:
                return out
        batch = getattr(ctx, "multiply_many", None) is not None
        if batch:
            if can_fork(ctx):  # each output nibble batches its own products, on its own stream
                shared = (*baby.values(), *g.values())
                return pair(ctx, lambda: self._outputs_batched(baby, g, ct_b, ("hi",))[0],
                            lambda: self._outputs_batched(baby, g, ct_b, ("lo",))[0], shared=shared)
            return self._outputs_batched(baby, g, ct_b)

        # 3) out = P(b) + conj(Q(b)) per output nibble
        def lut(which):
            P, Q = self._bsgs[which]
            return ctx.add(self._poly_bsgs((which, "p"), P, baby, g, ct_b),
                           ctx.conjugate(self._poly_bsgs((which, "q"), Q, baby, g, ct_b)))

        return pair(ctx, lambda: lut("hi"), lambda: lut("lo"), shared=(*baby.values(), *g.values()))

    def _bsgs_bases(self, ct_hi: Any, ct_lo: Any):
        """steps 1-2 of the BSGS form: (baby steps b^1..b^15, giant steps G_1..G_8, b)"""
        ctx = self.ctx
        lp, lq = self._ensure_bsgs()["lift"]
        # 1) zeta16^l -> zeta256^l: L(y) = P(y) + conj(Q(y)) over y^1..y^8
        pos16 = ctx.make_power_basis(ct_lo, 8)
        y = {k: pos16[k - 1] for k in range(1, 9)}
        lifted = ctx.add(self._lin("lift-p", np.r_[0, lp[1:]], y, lp[0], ct_lo),
                         ctx.conjugate(self._lin("lift-q", lq, y, 0j, ct_lo)))
        # 2) b = zeta256^byte; baby steps b^1..b^16, giant steps G_i = b^(16 i), i <= 8
        ct_b = ctx.multiply(ct_hi, lifted)
        pw = ctx.make_power_basis(ct_b, 16)
        baby = {k: pw[k - 1] for k in range(1, 16)}
        g = {1: pw[15]}
        batch = getattr(ctx, "multiply_many", None) is not None
        if batch:  # one mul_many per depth
            for stage in (((2, (1, 1)),), ((3, (1, 2)), (4, (2, 2))), ((5, (1, 4)), (6, (2, 4)), (7, (3, 4)), (8, (4, 4)))):
                for (i, _), r in zip(stage, mul_many(ctx, [(g[u], g[v]) for _, (u, v) in stage])):
                    g[i] = r
        else:
            for i, (u, v) in ((2, (1, 1)), (4, (2, 2)), (3, (1, 2)), (5, (1, 4)), (6, (2, 4)), (7, (3, 4)), (8, (4, 4))):
                g[i] = ctx.multiply(g[u], g[v])  # depth: G_2 +1, G_3 / G_4 +2, G_5..G_8 +3 over b^16
        return baby, g, ct_b

    def _outputs_batched(self, baby, g, ct_b, whiches=("hi", "lo")):
        """the output nibbles `whiches`: every chunk sum S_i (one fused kernel each), ALL their
        products S_i G_i in mul_many batches, the conj(Q) in one conj_many"""
        ctx = self.ctx
        terms, prods = {}, []
        for which in whiches:
            for part, coef in zip(("p", "q"), self._bsgs[which]):
                terms[(which, part)] = []
                for i in range((len(coef) + 15) // 16):
                    chunk = np.zeros(16, np.complex128)
                    seg = coef[16 * i: 16 * i + 16]
                    chunk[: len(seg)] = seg
                    if not np.any(chunk):
                        continue
                    key = ((which, part), i)
                    if i == 0:
                        terms[(which, part)].append(self._lin(key, np.r_[0, chunk[1:]], baby, chunk[0], ct_b))
                    elif not np.any(chunk[1:]):
                        terms[(which, part)].append(ctx.multiply(g[i], complex(chunk[0])))
                    else:
                        prods.append(((which, part), self._lin(key, np.r_[0, chunk[1:]], baby, chunk[0], ct_b), g[i]))
        for (wp, _, _), r in zip(prods, mul_many(ctx, [(s_, g_) for _, s_, g_ in prods])):
            terms[wp].append(r)
        acc = {}
        for wp, ts in terms.items():
            a = ts[0] if ts else ctx.multiply(ct_b, 0.0)
            for t in ts[1:]:
                a = ctx.add(a, t)
            acc[wp] = a
        cq = conj_many(ctx, [acc[(w, "q")] for w in whiches])
        return tuple(ctx.add(acc[(w, "p")], c) for w, c in zip(whiches, cq))

    def _outputs_biv(self, baby, g, ct_b):
        """both output nibbles with every part P, Q (f = P(b) + conj(Q(b))) as three fused sums:
        the chunk-0 sum c_0 + sum_j c_j b^j (univariate over the baby steps), the column
        sum_i c_16i G_i (univariate over the giant steps), and the rest, sum_{i>=1, j>=1}
        c_(16i+j) b^j G_i, as ONE bivariate LUT over (baby, giant) -- the chunk sums S_i and their
        products S_i G_i fused into one kernel and one relinearisation instead
        of 8 LUT kernels, 8 products and their rescales per part.  The coefficients meet the
        products at the giant steps' level: one level more than _outputs_batched (the caller's
        inputs sit one level higher).  None when a fused sum is unavailable (level)."""
        ctx = self.ctx
        acc = {}
        for which in ("hi", "lo"):
            for part, coef in zip(("p", "q"), self._bsgs[which]):
                nch = (len(coef) + 15) // 16
                key = (which, part)
                C = np.zeros((16, nch), np.complex128)
                gcol = np.zeros(nch, np.complex128)
                for i in range(1, nch):
                    seg = coef[16 * i: 16 * i + 16]
                    gcol[i] = seg[0]
                    C[1:len(seg), i] = seg[1:]
                c0 = coef[:16]
                t = [self._lin((key, 0), np.r_[0, c0[1:]], baby, c0[0], ct_b)]
                for sub, vec, args in (("g", gcol, (g,)), ("bg", C, (baby, g))):
                    if np.any(vec):
                        r = fused_lut(ctx, (key, sub), vec, *args, owner=self)
                        if r is None:
                            return None
                        t.append(r)
                a = t[0]
                for x in t[1:]:
                    a = ctx.add(a, x)
                acc[key] = a
        cq = conj_many(ctx, [acc[(w, "q")] for w in ("hi", "lo")])
        return tuple(ctx.add(acc[(w, "p")], c) for w, c in zip(("hi", "lo"), cq))

    # ------------------------------------------------------------------ direct (reference) form
    def _apply_direct(self, ct_hi: Any, ct_lo: Any) -> Tuple[Any, Any]:
        ctx = self.ctx
        # 1) ζ16^l -> ζ256^l
        pos16 = ctx.make_power_basis(ct_lo, self.deg16) if self.deg16 > 0 else []
        p16 = {k: self._power(pos16, k, 16, ctx) for k in self.ks_lift}
        lifted = fused_lut(ctx, "sb-lift", self.vec_lift, p16, c0=self.c0_lift, owner=self)
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
            res = fused_lut(ctx, ("sb", pts is self.pt_hi), self.vec_hi if pts is self.pt_hi else self.vec_lo,
                            bk, c0=c0, owner=self)
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
