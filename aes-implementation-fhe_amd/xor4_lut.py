"""XOR4LUT: 4-bit XOR as a bivariate LUT polynomial (REF/xor4_lut.py:10-78).

    XOR(a, b) = Σ_{p,q} C[p,q] A^p B^q,   A^k = a^k (k <= 8), conj(a^(16-k)) (k >= 9)

with C from xor4_coeffs.json (only odd p, q are non-zero; the output carries the
reference's 256x magnitude).  Depth 5: power basis 3, product 1,
coefficient 1.

With a fused-LUT context the sum is split over the conjugate mirrors: a and
b are 16th roots of unity, so the rows p >= 9 (A^p = conj(A^(16-p))) satisfy
    sum_{p>=9,q} C[p,q] conj(A^(16-p)) B^q = conj( sum C'[p',q'] A^p' B^q' ),
    C'[p',q'] = conj(C[16-p', (16-q') mod 16]),
and the whole LUT is S1 + conj(S2) over the positive powers of a and the standard basis of
b: a needs no conjugations at all, only the powers the coefficients use are formed (x^6 and
x^8 are skipped for XOR4), and each S is one fused kernel.  Output level unchanged.
"""
import os
from typing import Any, Dict

import numpy as np
from utils import LUT2_DEPTH, ConjSum, can_fork, conj_many, drop_to, fused_lut, mul_many, pair


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


# ---------------------------------------------------------------- conjugate-split bivariate LUTs
def _chain(need):
    """products (k, u, v), x^k = x^u x^v, forming x^k for every k in need (<= 8) at depth
    ceil(log2 k) -- the engine's power-basis rule, restricted to what is used"""
    have, order = {1}, []

    def get(k):
        if k in have:
            return
        t = 1 << (k.bit_length() - 1)
        u, v = (k // 2, k // 2) if t == k else (t, k - t)
        get(u)
        get(v)
        order.append((k, u, v))
        have.add(k)

    for k in sorted(need):
        if k >= 1:
            get(k)
    return order


def powers(ctx, ct, need) -> Dict[int, Any]:
    """{k: x^k} for k in need (0 = the constant 1 at x's level)"""
    if batched(ctx):
        return joint_bases(ctx, [(ct, need, "pow")])[0]
    pw = {1: ct}
    for k, u, v in _chain(need):
        pw[k] = ctx.multiply(pw[u], pw[v])
    if 0 in need:
        pw[0] = ctx.add_plain(ctx.multiply(ct, 0.0), 1.0)
    return {k: pw[k] for k in need}


def _depth(k: int) -> int:
    return (k - 1).bit_length()  # ceil(log2 k): the multiplicative depth of x^k


# AESFHE_CONJ_CHAIN=0: the std basis' mirrors as conjugations of the powers (one key switch per
# mirror, at three levels) instead of powers of the conjugated input (A/B runs)
_CONJ_CHAIN = os.environ.get("AESFHE_CONJ_CHAIN", "1") != "0"


def joint_bases(ctx, specs):
    """[(ct, need, kind)] -> [{k: element}], kind "pow" (powers(), x^k) or "std" (std_basis():
    the mirrors conj(x)^(16-q) for q >= 9).  The products of one depth across ALL inputs form
    one mul_many batch.  The mirrors: x is conjugated ONCE (all inputs' in one
    conj_many) and its powers join the same product batches -- one key switch per input at its
    own level instead of one per mirror at three levels (conj(x)^k = conj(x^k): same values,
    same depth); AESFHE_CONJ_CHAIN=0 conjugates the powers instead."""
    if _CONJ_CHAIN and any(kind == "std" and any(q >= 9 for q in need) for _, need, kind in specs):
        std = [i for i, (_, need, kind) in enumerate(specs) if kind == "std" and any(q >= 9 for q in need)]
        bars = conj_many(ctx, [specs[i][0] for i in std])
        ext = [(ct, {q for q in need if q <= 8} if kind == "std" else need, "pow") for ct, need, kind in specs]
        ext += [(bar, {16 - q for q in specs[i][1] if q >= 9}, "pow") for i, bar in zip(std, bars)]
        got = joint_bases(ctx, ext)
        out = got[:len(specs)]
        for j, i in enumerate(std):
            out[i].update({16 - k: v for k, v in got[len(specs) + j].items()})
        return out
    needs = [set(need) if kind == "pow" else {q if q <= 8 else 16 - q for q in need} for _, need, kind in specs]
    pws = [{1: ct} for ct, _, _ in specs]
    chains = [_chain(n) for n in needs]
    top = max((_depth(k) for ch in chains for k, _, _ in ch), default=0)
    for d in range(1, top + 1):
        jobs = [(i, k, u, v) for i, ch in enumerate(chains) for k, u, v in ch if _depth(k) == d]
        for (i, k, _, _), r in zip(jobs, mul_many(ctx, [(pws[i][u], pws[i][v]) for i, _, u, v in jobs])):
            pws[i][k] = r
    for i, (ct, _, _) in enumerate(specs):
        if 0 in needs[i]:
            pws[i][0] = ctx.add_plain(ctx.multiply(ct, 0.0), 1.0)
    out = [{k: pws[i][k] for k in (need if kind == "pow" else [q for q in need if q <= 8])}
           for i, (_, need, kind) in enumerate(specs)]
    cj = [(i, q) for i, (_, need, kind) in enumerate(specs) if kind == "std" for q in sorted(need) if q >= 9]
    for (i, q), c in zip(cj, conj_many(ctx, [pws[i][16 - q] for i, q in cj])):
        out[i][q] = c
    return out


def batched(ctx) -> bool:
    return getattr(ctx, "multiply_many", None) is not None


def std_basis(ctx, ct, need) -> Dict[int, Any]:
    """{q: B[q]} for q in need, B[q] = x^q (q <= 8), conj(x^(16-q)) (q >= 9)"""
    if batched(ctx):
        return joint_bases(ctx, [(ct, need, "std")])[0]
    pos = powers(ctx, ct, {q if q <= 8 else 16 - q for q in need})
    return {q: pos[q] if q <= 8 else ctx.conjugate(pos[16 - q]) for q in need}


class SplitLUT2:
    """sum_{p,q} C[p,q] A[p] B[q] over Zeta16 inputs as S1 + conj(S2) (module docstring)."""

    def __init__(self, C: np.ndarray, tol: float = 1e-12):
        C = np.where(np.abs(C) > tol, np.asarray(C, np.complex128), 0)
        self.c1 = C[:9].copy()
        self.c2 = np.zeros((8, 16), np.complex128)
        for pp in range(1, 8):
            for qq in range(16):
                self.c2[pp, qq] = np.conj(C[16 - pp, (16 - qq) % 16])
        rows = lambda M: {i for i in range(M.shape[0]) if np.any(M[i])}
        cols = lambda M: {j for j in range(16) if np.any(M[:, j])}
        self.need_a = rows(self.c1) | rows(self.c2)
        self.need_b = cols(self.c1) | cols(self.c2)
        self.has2 = bool(np.any(self.c2))

    def bases(self, ctx, a, b, B=None):
        """(A, B): powers of a, std basis of b -- B given: only a's (a basis of b computed before)"""
        if B is not None:
            return powers(ctx, a, self.need_a), B
        if batched(ctx) and not can_fork(ctx):
            A, B = joint_bases(ctx, [(a, self.need_a, "pow"), (b, self.need_b, "std")])
            return A, B
        return pair(ctx, lambda: powers(ctx, a, self.need_a), lambda: std_basis(ctx, b, self.need_b))

    def eval_pair(self, ctx, key, AB0, AB1):
        """(eval(A0, B0), eval(A1, B1)) with the two conjugations batched"""
        return eval_two(ctx, (self, key, *AB0), (self, key, *AB1))

    def eval(self, ctx, key, A, B, defer_conj: bool = False):
        """S1 + conj(S2); defer_conj: as a ConjSum for a renorm that folds the conjugation in"""
        s1 = fused_lut(ctx, (key, 1), self.c1, A, B, owner=self)
        if s1 is None:
            return None
        if not self.has2:
            return s1
        s2 = fused_lut(ctx, (key, 2), self.c2, A, B, owner=self)
        if s2 is None:
            return None
        return ConjSum(s1, s2) if defer_conj else ctx.add(s1, ctx.conjugate(s2))


def eval_two(ctx, j0, j1, defer_conj: bool = False):
    """two split-LUT evaluations j = (split, key, A, B) as S1 + conj(S2) each, the two
    conjugations in one conj_many batch; None if a fused sum is unavailable (level).
    defer_conj: each result a utils.ConjSum (S1, S2) for a renorm that folds the conjugation in"""
    out, s2 = [], []
    for sp, key, A, B in (j0, j1):
        s1 = fused_lut(ctx, (key, 1), sp.c1, A, B, owner=sp)
        t2 = fused_lut(ctx, (key, 2), sp.c2, A, B, owner=sp) if sp.has2 else None
        if s1 is None or (sp.has2 and t2 is None):
            return None
        out.append(s1)
        s2.append(t2)
    idx = [i for i in (0, 1) if s2[i] is not None]
    if defer_conj:
        return tuple(ConjSum(out[i], s2[i]) if s2[i] is not None else out[i] for i in (0, 1))
    for i, c in zip(idx, conj_many(ctx, [s2[i] for i in idx])):
        out[i] = ctx.add(out[i], c)
    return out[0], out[1]


def split_lut2(ctx, split: SplitLUT2, key, a, b, keep_b=None, defer_conj: bool = False):
    """the split evaluation, or None (no fused op / not enough level: use the product loop).
    keep_b: a dict caching b's std basis -- filled on the first call, reused by a later call with
    the same b at the same level (an operand shared by two XOR4s of one step)"""
    if not getattr(ctx, "fused_luts", False):
        return None
    cached = None
    if keep_b is not None and keep_b.get("b") is b and keep_b.get("level") == b.level:
        cached = keep_b["B"]
    try:
        A, B = split.bases(ctx, a, b, cached)
    except RuntimeError as e:
        if "level" in str(e):
            return None
        raise
    if keep_b is not None and cached is None:
        keep_b.update(b=b, level=b.level, B=B)
    return split.eval(ctx, key, A, B, defer_conj)


class XOR4LUT:
    def __init__(self, ctx, coeffs: np.ndarray):
        self.ctx = ctx
        self.sc = ctx.engine.slot_count
        self.coeffs = coeffs
        self.pt = {(p, q): ctx.encode(np.full(self.sc, coeffs[p, q], dtype=np.complex128))
                   for p in range(16) for q in range(16) if abs(coeffs[p, q]) > 1e-12}

    def _build_power_basis_16(self, ct: Any) -> Dict[int, Any]:
        return basis16(self.ctx, ct)

    def apply(self, a_ct, b_ct, out_level=None, keep_b=None, defer_conj: bool = False):
        """XOR4(a, b); out_level: the lowest level the caller needs the result at (the inputs
        are dropped to out_level + LUT2_DEPTH first, utils.drop_to); None = as given.
        keep_b: a dict shared by two XOR4s whose second operand is the same ciphertext -- b's
        basis is built once (MixColumns' r1 enters two XOR4s, mixcol_final.mix_packed).
        defer_conj: the split form may return a utils.ConjSum (S1, S2) for a renorm that takes one."""
        ctx = self.ctx
        if keep_b is not None and "b_in" in keep_b and keep_b["b_in"] is b_ct and keep_b.get("out_level") == out_level:
            b_ct = keep_b["b_dropped"]  # the same drop as before: reuse it (and so its basis)
        elif keep_b is not None:
            keep_b.clear()
            keep_b.update(b_in=b_ct, out_level=out_level)
            b_ct = drop_to(ctx, b_ct, out_level + LUT2_DEPTH) if out_level is not None else b_ct
            keep_b["b_dropped"] = b_ct
        elif out_level is not None:
            b_ct = drop_to(ctx, b_ct, out_level + LUT2_DEPTH)
        if out_level is not None:
            a_ct = drop_to(ctx, a_ct, out_level + LUT2_DEPTH)
        if not hasattr(self, "_split"):
            self._split = SplitLUT2(self.coeffs)
        out = split_lut2(ctx, self._split, "xor4", a_ct, b_ct, keep_b, defer_conj)
        if out is not None:
            return out
        A, B = pair(ctx, lambda: self._build_power_basis_16(a_ct), lambda: self._build_power_basis_16(b_ct))
        out = fused_lut(ctx, "xor4", self.coeffs, A, B, owner=self)  # one kernel for all 64 terms
        if out is not None:
            return out
        acc = ctx.sub(A[0], A[0])
        for (p, q), pt in self.pt.items():
            acc = ctx.add(acc, ctx.multiply(ctx.multiply(A[p], B[q]), pt))
        return acc

    def apply_pair(self, a0, b0, a1, b1, out_level=None):
        """(XOR4(a0, b0), XOR4(a1, b1)) -- the hi / lo halves of an AES step.  On two branch
        streams when the context can fork (each XOR batching its own two inputs' bases: on
        this GPU two concurrent half-size batches beat one full batch);
        otherwise the four inputs' bases share mul_many / conj_many batches and the two
        conjugations of the split sums one more."""
        ctx = self.ctx
        if getattr(ctx, "fused_luts", False) and batched(ctx) and not can_fork(ctx):
            if out_level is not None:
                lv = out_level + LUT2_DEPTH
                a0, b0, a1, b1 = (drop_to(ctx, c, lv) for c in (a0, b0, a1, b1))
            if not hasattr(self, "_split"):
                self._split = SplitLUT2(self.coeffs)
            sp = self._split
            try:
                A0, B0, A1, B1 = joint_bases(ctx, [(a0, sp.need_a, "pow"), (b0, sp.need_b, "std"),
                                                   (a1, sp.need_a, "pow"), (b1, sp.need_b, "std")])
            except RuntimeError as e:
                if "level" not in str(e):
                    raise
            else:
                out = sp.eval_pair(ctx, "xor4", (A0, B0), (A1, B1))
                if out is not None:
                    return out
        return pair(ctx, lambda: self.apply(a0, b0, out_level), lambda: self.apply(a1, b1, out_level))

    __call__ = apply
