"""Homomorphic Zeta16 snaps: the true-FHE replacement of the secret-key renorm
(REF/zeta16_noise_reducter.py:6-169, REF/noise_reduction.py:14-82).

A renorm re-anchors every state slot to the nearest 16th root of unity ζ.  Without the
secret key it is a bootstrap (fresh levels, REF bootstrap_before=True) followed by a
polynomial f with f(ζ) = ζ and f'(ζ) = 0 at every codeword, so an error ε becomes O(ε²).

``Zeta16NoiseReducer`` -- the reference's f(x) = (17x - x^17)/16 (REF :6-57): x^1..x^8 by the
power basis, x^16 = (x^8)^2, x^17 = x^16 x (depth 5) and its -1/16 scalar: depth 6 as written.  (The reference's ``Zeta16Snap``,
:108-169, forms x^17 as x^8 conj(x^7), which equals x on the unit circle -- the identity, no
snap; it is not rebuilt.)

``Zeta16Snap15`` -- the depth-4 snap this engine's parameter set needs.  After a bootstrap
the state sits at the fresh level 17 and SubBytes needs 13 levels, so the snap may use 4.
Over x and conj(x) (conjugation is a free key switch), with e = x/ζ - 1:

    f(x) = (30 x - 15 x^2 conj(x) + conj(x)^15) / 16
    f(ζ(1+e)) = ζ (1 + O(e^2))      (value 1, both first-order terms cancel; 16 f = 30 - 15 + 1)

conj(x)^15 = conj(x^8 x^7) has depth 4, but its coefficient 1/16 would cost a fifth level.
The bootstrap therefore returns u = κ x with κ^15 = 1/16 (gain folded into its level-0
scaling integer, aesfhe_bootstrap_pair_scaled), so in u

    f = a1 u + a3 u^2 conj(u) + conj(u)^15,   a1 = 30 / (16 κ),  a3 = -15 / (16 κ^3)

with the depth-4 term's coefficient exactly 1 and the others on depth <= 2 products.

``BootstrapSnap`` -- the pair renorm the pipeline uses in true-FHE mode: one batched
scaled bootstrap of (hi, lo), then Zeta16Snap15 on each half (two branch streams), and a second
snap (x κ, then the snap: 5 levels) when the step after the renorm is an XOR4 (<= 8 levels
needed) rather than SubBytes (13): an error ε leaves one snap as ~9 ε², two as ~729 ε^4.
SubBytes / InvSubBytes outputs carry ~3e-2 slot errors (their polynomials' derivatives
amplify the CKKS noise ~60x on average), and an XOR4 can amplify its inputs' errors up to
~17x, so one snap between them is not enough at the tails of a batch (measured:
profiles/r2_true_fhe.json).
"""
from __future__ import annotations

import os
from typing import Any, Tuple

from utils import NEED_SR_ARK, NEED_XOR, pair, stacked_many, stacked_pair
from xor4_lut import powers

SNAP15_DEPTH = 4
DOUBLE_SNAP_MAX_LEVEL = NEED_SR_ARK  # renorms whose consumer needs at most this many levels snap twice
KAPPA = 16.0 ** (-1.0 / 15.0)  # bootstrap gain: conj(u)^15 carries coefficient 1
# AESFHE_FHE_SNAPS=1 / 2: at most that many snaps per renorm (default: the pipeline's choice, max_snaps)
_ENV_SNAPS = os.environ.get("AESFHE_FHE_SNAPS")
# AESFHE_FHE_QUAD=0: two pair bootstraps instead of one quad bootstrap for renorm_two (A/B runs)
_QUAD = os.environ.get("AESFHE_FHE_QUAD", "1") != "0"


class Zeta16NoiseReducer:
    """f(x) = (17/16) x - (1/16) x^17 (REF/zeta16_noise_reducter.py:6-57); depth 6 as written."""

    def __init__(self, ctx, bootstrap_before: bool = False, bootstrap_after: bool = False):
        self.ctx = ctx
        self.alpha = 17.0 / 16.0
        self.beta = -1.0 / 16.0
        self.bootstrap_before = bootstrap_before
        self.bootstrap_after = bootstrap_after

    def _ensure_power_basis(self, ct):
        """x^1..x^8, one bootstrap on a level complaint (REF :20-29)"""
        try:
            return ct, self.ctx.make_power_basis(ct, 8)
        except RuntimeError:
            ct = self.ctx.bootstrap(ct)
            return ct, self.ctx.make_power_basis(ct, 8)

    def apply(self, ct):
        ctx = self.ctx
        x = ctx.bootstrap(ct) if self.bootstrap_before else ct
        x, pos = self._ensure_power_basis(x)
        x16 = ctx.multiply(pos[7], pos[7])
        x17 = ctx.multiply(x16, pos[0])
        y = ctx.add(ctx.multiply_plain(pos[0], self.alpha), ctx.multiply_plain(x17, self.beta))
        return ctx.bootstrap(y) if self.bootstrap_after else y

    def apply_pair(self, ct_hi, ct_lo):
        if self.bootstrap_before or self.bootstrap_after:  # the bootstrapping variants keep two calls
            return pair(self.ctx, lambda: self.apply(ct_hi), lambda: self.apply(ct_lo))
        return stacked_pair(self.ctx, self.apply, ct_hi, ct_lo)


class Zeta16Snap15:
    """f = a1 u + a3 u^2 conj(u) + conj(u)^15 on u = κ x (module docstring); depth 4."""

    def __init__(self, ctx, kappa: float = KAPPA):
        self.ctx = ctx
        self.kappa = kappa
        self.a1 = 30.0 / (16.0 * kappa)
        self.a3 = -15.0 / (16.0 * kappa ** 3)
        self.c15 = 1.0 / (16.0 * kappa ** 15)  # 1 for the default κ: an exact (free) coefficient

    def apply_scaled(self, u):
        """the snap of x given u = κ x"""
        ctx = self.ctx
        pw = powers(ctx, u, {2, 7, 8})               # u^2 (1), u^7, u^8 (3): five products
        ub = ctx.conjugate(u)
        u15 = ctx.multiply(pw[8], pw[7])             # depth 4
        t3 = ctx.multiply(pw[2], ub)                 # u^2 conj(u), depth 2
        c15 = ctx.conjugate(u15)
        if abs(self.c15 - 1.0) > 1e-12:
            c15 = ctx.multiply(c15, self.c15)
        return ctx.add(ctx.add(ctx.multiply(u, self.a1), ctx.multiply(t3, self.a3)), c15)

    def apply(self, x):
        """the snap of a ciphertext at unit gain (scales by κ first: one more level)"""
        return self.apply_scaled(self.ctx.multiply(x, self.kappa))


class BootstrapSnap:
    """True-FHE renorm of a (hi, lo) pair: scaled bootstrap, then the depth-4 snap.

    max_snaps: 2 (round 2's rule for the reference's 8 -> 4 SubBytes, whose outputs carry ~3e-2
    errors): a second snap when the consumer needs <= DOUBLE_SNAP_MAX_LEVEL levels; 1 (the
    pipeline's choice with the nibble-bivariate SubBytes, whose outputs stay ~1e-3 off their
    codewords): one snap everywhere, so the fresh level only needs snap + 8 levels."""

    def __init__(self, ctx, snap: Zeta16Snap15 | None = None, period: int | None = None, max_snaps: int = 2):
        if getattr(ctx, "bootstrap_pair_scaled", None) is None:
            raise RuntimeError("true-FHE renorm needs the engine's scaled pair bootstrap (bootstrappable context)")
        self.ctx = ctx
        self.snap = snap or Zeta16Snap15(ctx)
        self.period = period  # the states' slot period (periodic layout): sparse-slot bootstraps
        self.max_snaps = int(_ENV_SNAPS) if _ENV_SNAPS else max_snaps

    def _twice(self, level) -> bool:
        """a second snap: consumer needs <= DOUBLE_SNAP_MAX_LEVEL (None / 0: the output or a bootstrap
        -- an XOR4 follows in true-FHE mode) and the fresh level leaves it room"""
        need = level if level else NEED_XOR
        return (self.max_snaps > 1 and need <= DOUBLE_SNAP_MAX_LEVEL
                and self.ctx.engine.fresh_level - 2 * SNAP15_DEPTH - 1 >= need)

    def _snap_fn(self, level):
        sn = self.snap
        return (lambda u: sn.apply(sn.apply_scaled(u))) if self._twice(level) else sn.apply_scaled

    def apply_pair(self, ct_hi, ct_lo, level=None) -> Tuple[Any, Any]:
        """level: what the next step needs (the pipeline's renorm hint)"""
        ctx = self.ctx
        if self.period is not None:
            uh, ul = ctx.bootstrap_pair_scaled(ctx.to_intt(ct_hi), ctx.to_intt(ct_lo), self.snap.kappa, self.period)
        else:
            uh, ul = ctx.bootstrap_pair_scaled(ctx.to_intt(ct_hi), ctx.to_intt(ct_lo), self.snap.kappa)
        # the same snap on both halves: one stacked evaluation (utils.stacked_pair)
        return stacked_pair(ctx, self._snap_fn(level), uh, ul)

    __call__ = apply_pair

    def quad_ok(self) -> bool:
        ctx = self.ctx
        return bool(_QUAD and self.period is not None and getattr(ctx, "bootstrap_quad_scaled", None) is not None
                    and 4 * self.period <= ctx.engine.slot_count)

    def apply_quad(self, p, q, level=None):
        """two (hi, lo) pairs renormalised at one point of a step: ONE bootstrap at four times the
        period (EngineContext.bootstrap_quad_scaled) and one snap stacked over the four"""
        if not self.quad_ok():
            return self.apply_pair(*p, level), self.apply_pair(*q, level)
        ctx = self.ctx
        u = ctx.bootstrap_quad_scaled([ctx.to_intt(c) for c in (*p, *q)], self.snap.kappa, self.period)
        out = stacked_many(ctx, self._snap_fn(level), u)
        return (out[0], out[1]), (out[2], out[3])
