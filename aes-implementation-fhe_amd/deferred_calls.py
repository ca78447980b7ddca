"""Deferred call sequences of the drop-in API.

The reference's round modules evaluate every LUT as a loop of single primitive calls
(REF/xor4_lut.py:71-73, REF/mixcol_final.py:80-91, REF/sub_bytes_lut.py:66-71):

    term = multiply(A[p], B[q]); term = multiply(term, pt); res = add(res, term)

and every rotation / conjugation as its own call (REF/shift_rows.py:20-50,
REF/xor4_lut.py:57-59).  Issued one by one, such a loop is three kernel launches per term and
one key switch per rotation.  `mi355x_ckks.Engine(defer_calls=True)` (the default) returns
*deferred* ciphertexts for these calls instead and issues the work only when a result is
needed:

- `TermSum`: c0 + sum_i c_i a_i (x) b_i + sum_j d_j x_j -- products of two ciphertexts and
  ciphertexts times constants (scalars or constant plaintexts), summed.  Resolved as ONE fused
  bivariate LUT kernel for the products (aesfhe_lut_eval over the distinct factors, the
  coefficient matrix cached by content) and ONE univariate LUT for the scaled terms; plain
  `add`s of ciphertexts are summed as they are.  A single product or a single scaled term is
  issued as the very calls the caller made, so its bytes equal the undeferred result.
- `GalPending`: rotate / conjugate of a ciphertext.  The first one needed resolves EVERY
  pending one of the engine (this thread) as one heterogeneous batched key switch
  (aesfhe_galois_multi: bit-exact with the separate calls).

A deferred object is a `Ciphertext`: any engine call that needs its handle -- and `.level`,
`.num_polys` -- resolves it first, so callers see no difference beyond CKKS rounding of the
fused sums (decoded AES bytes are checked by tests/test_gpu_deferred_calls.py and the bench's
`deferred_ref_calls` leg).  `AESFHE_DEFER_CALLS=0` or `Engine(defer_calls=False)` turns it off.
"""
from __future__ import annotations

import hashlib
import numbers
import threading
import weakref

import numpy as np

from mi355x_ckks import Ciphertext, Plaintext

_LUT_MAX = 16  # kLutMax (csrc/kernels.h): factors per side of one bivariate LUT


_FALLBACK_LOCK = threading.RLock()  # engines without their own (test stubs)


class Deferred(Ciphertext):
    """a ciphertext whose value is not computed yet; `handle` computes it (once)"""

    __slots__ = ("_eng", "_res")

    def __init__(self, eng):
        self._ctx = eng._ctx
        self._eng = eng
        self._res = None

    @property
    def handle(self):
        if self._res is None:
            # one resolution per object even when two branch threads need it at once:
            # the engine's re-entrant lock (a resolution may resolve the deferred operands it reads)
            with getattr(self._eng, "_defer_lock", None) or _FALLBACK_LOCK:
                if self._res is None:
                    res = self._resolve()
                    self._res = res
                    self._release_operands()
        return self._res.handle

    def resolved(self) -> Ciphertext:
        self.handle  # noqa: B018 -- forces resolution
        return self._res

    def _resolve(self) -> Ciphertext:
        raise NotImplementedError

    def _release_operands(self):
        pass

    def __del__(self):  # the resolved Ciphertext frees its own handle
        pass


def real(x):
    """the resolved Ciphertext behind x (x itself when not deferred)"""
    return x.resolved() if isinstance(x, Deferred) else x


def constant_of(m):
    """the complex constant a multiplier stands for (a number or a constant plaintext), else None"""
    if isinstance(m, bool):
        return None
    if isinstance(m, numbers.Number):
        return complex(m)
    if isinstance(m, Plaintext):
        return getattr(m, "const", None)
    return None


class GalPending(Deferred):
    """X -> X^g of `src` (a rotation or the conjugation), key switch not yet issued"""

    __slots__ = ("src", "g", "raw")

    def __init__(self, eng, src, g: int, raw):
        super().__init__(eng)
        self.src, self.g, self.raw = src, int(g), raw  # raw: () -> the undeferred call (a lone resolution)
        eng._gal_pending().append(weakref.ref(self))

    def _resolve(self):
        return self._eng._flush_gal(self)

    def _release_operands(self):
        self.src = self.raw = None


class TermSum(Deferred):
    """c0 + sum c (a (x) b) [bil] + sum d x [lin]; each term keeps the multipliers the caller
    applied (`chain`) so a lone term is re-issued as exactly those calls"""

    __slots__ = ("c0", "bil", "lin", "_lv")

    def __init__(self, eng, c0=0j, bil=(), lin=()):
        super().__init__(eng)
        self.c0 = complex(c0)
        self.bil = list(bil)  # (a, b, coef, chain)
        self.lin = list(lin)  # (x, coef, chain)

    # ---------------------------------------------------------------- algebra (no launches)
    def scaled(self, m, c: complex):
        return TermSum(self._eng, self.c0 * c, [(a, b, k * c, ch + [m]) for a, b, k, ch in self.bil],
                       [(x, k * c, ch + [m]) for x, k, ch in self.lin])

    def plus(self, other, sign: float = 1.0):
        if isinstance(other, TermSum):
            if sign == 1.0:
                return TermSum(self._eng, self.c0 + other.c0, self.bil + other.bil, self.lin + other.lin)
            neg = other.scaled(-1.0, -1.0)
            return TermSum(self._eng, self.c0 + neg.c0, self.bil + neg.bil, self.lin + neg.lin)
        if sign == 1.0:
            return TermSum(self._eng, self.c0, self.bil, self.lin + [(other, 1.0 + 0j, [])])
        return TermSum(self._eng, self.c0, self.bil, self.lin + [(other, -1.0 + 0j, [-1.0])])

    def _release_operands(self):
        self.bil = self.lin = None

    # ---------------------------------------------------------------- resolution
    def _resolve(self) -> Ciphertext:
        eng = self._eng
        # every pending rotation / conjugation among the operands (and elsewhere) in one batch
        ops = [o for a, b, _, _ in self.bil for o in (a, b)] + [x for x, _, _ in self.lin]
        if any(isinstance(o, GalPending) and o._res is None for o in ops):
            eng._flush_gal(None)
        parts = []
        if self.bil:
            parts.append(self._resolve_bil())
        plain = [x for x, k, ch in self.lin if k == 1 and not ch]
        scaled = [(x, k, ch) for x, k, ch in self.lin if not (k == 1 and not ch)]
        c0 = self.c0
        if scaled:
            r, c0 = self._resolve_lin(scaled, c0)
            parts.append(r)
        parts += [real(x) for x in plain]
        if not parts:
            raise ValueError("deferred sum without terms")
        acc = parts[0]
        for p in parts[1:]:
            acc = eng._raw("add", acc, p)
        if c0 != 0:
            acc = eng._raw("add_scalar", acc, c0)
        return acc

    def _resolve_bil(self) -> Ciphertext:
        eng = self._eng
        terms = [(real(a), real(b), k, ch) for a, b, k, ch in self.bil]
        if len(terms) == 1:
            a, b, _, ch = terms[0]
            r = eng._raw("mul", a, b)
            for m in ch:
                r = eng._raw("mul_by", r, m)
            return r
        fa, fb, C = _bil_matrix(terms)
        if C is not None:
            try:
                return eng._raw_lut(C, fa, fb)
            except RuntimeError as e:
                if "level" not in str(e):
                    raise
        # too many distinct factors or too little level for the fused form: the products in one
        # batched multiply (relinearised + rescaled together), then the constants and the sum
        prods = eng._raw("mul_many", [(a, b) for a, b, _, _ in terms])
        acc = None
        for p, (_, _, k, ch) in zip(prods, terms):
            for m in ch:
                p = eng._raw("mul_by", p, m)
            acc = p if acc is None else eng._raw("add", acc, p)
        return acc

    def _resolve_lin(self, scaled, c0):
        """(the scaled terms' sum, the constant still to add)"""
        eng = self._eng
        live = [t for t in scaled if t[1] != 0]
        if len(live) <= 1:  # a lone term (or only zero products): the caller's own calls
            x, _, ch = live[0] if live else scaled[0]
            r = real(x)
            for m in ch:
                r = eng._raw("mul_by", r, m)
            return r, c0
        xs, ks = [], []
        pos = {}
        for x, k, _ in live:
            x = real(x)
            i = pos.setdefault(id(x), len(xs))
            if i == len(xs):
                xs.append(x)
                ks.append(0j)
            ks[i] += k
        if any(k != 0 for k in ks):
            try:
                return eng._raw_lut(np.array(ks, np.complex128), xs, None, c0), 0j
            except RuntimeError as e:
                if "level" not in str(e):
                    raise
        acc = None
        for x, k, ch in live:
            p = real(x)
            for m in ch:
                p = eng._raw("mul_by", p, m)
            acc = p if acc is None else eng._raw("add", acc, p)
        return acc, c0


def _bil_matrix(terms):
    """distinct first / second factors and the coefficient matrix C[p, q] of sum c a_p b_q; the
    factor of each product that repeats less goes to the rows (the kernel forms one tensor per
    row).  (None, None, None) when a side exceeds the kernel's 16 factors."""
    def index(objs):
        pos, out = {}, []
        for o in objs:
            if id(o) not in pos:
                pos[id(o)] = len(out)
                out.append(o)
        return pos, out
    pa, fa = index(a for a, _, _, _ in terms)
    pb, fb = index(b for _, b, _, _ in terms)
    swap = len(fa) > len(fb)
    if swap:
        pa, fa, pb, fb = pb, fb, pa, fa
    if len(fa) > _LUT_MAX or len(fb) > _LUT_MAX:
        return None, None, None
    C = np.zeros((len(fa), max(2, len(fb))), np.complex128)  # n_b >= 2: the bivariate form
    for a, b, k, _ in terms:
        if swap:
            a, b = b, a
        C[pa[id(a)], pb[id(b)]] += k
    return fa, fb, C


def lut_key(C: np.ndarray, c0: complex) -> bytes:
    return hashlib.blake2b(C.tobytes() + repr(C.shape).encode() + np.complex128(c0).tobytes(), digest_size=16).digest()
