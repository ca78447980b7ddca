"""InvMixColumnsFHE: GF×14(x) ⊕ GF×11(r1) ⊕ GF×13(r2) ⊕ GF×9(r3)
(REF/invmixcolumns_fhe.py:34-170), same rotation orientation as MixColFinal so the two
are mutually inverse.  Renorm after each XOR pair when use_hard_renorm (default True).
"""
from __future__ import annotations

import os
from typing import Any, Dict, List

from mixcol_final import _CoeffCache, gf_basis16, gf_eval, gf_mult_pair
from shift_rows import row_masks
from state_encoder import StateEncoder
from xor4_lut import XOR4LUT
from utils import FOLDS, LUT2_DEPTH, takes_kw, NEED_BOOTSTRAP, NEED_GF, NEED_XOR, RENORM_FLOOR, bootstrap1, bootstrap2, pair, rot_many, rot_pair

# AESFHE_IMC_GF_LOW=0: the packed InvMixColumns' GF multiplier pairs at their own depth above the XOR4s
# (inputs at NEED_GF + PACK_DEPTH) instead of at the XOR4 level with renormalised outputs (A/B runs)
_IMC_GF_LOW = os.environ.get("AESFHE_IMC_GF_LOW", "1") != "0"


class InvMixColumnsFHE:
    def __init__(self, ctx, xor4: XOR4LUT, use_hard_renorm: bool = True, states: int = 1, layout=None):
        self.ctx = ctx
        self.xor4 = xor4
        self.sc = ctx.engine.slot_count
        # states > 1: slot-packed batch; layout.periodic: the periodic layout (state_encoder.py)
        self.enc = StateEncoder(ctx, states, periodic=bool(layout is not None and layout.periodic))
        self.layout = self.enc.layout
        self.stride = self.layout.unit
        self._coeffs = _CoeffCache()
        self.use_hard_renorm = use_hard_renorm
        self._pt_row: List[Any] = row_masks(ctx, self.sc, states, self.layout)
        # with the renorm after every XOR pair, the LUTs run just above RENORM_FLOOR (utils.py)
        self._xor_level = RENORM_FLOOR if use_hard_renorm else None
        self._gf_level = RENORM_FLOOR + LUT2_DEPTH if use_hard_renorm else None

    def _basis16(self, ct):
        return gf_basis16(self.ctx, ct)

    def _poly2_eval(self, ct_hi, ct_lo, mult: int, which: str):
        return gf_eval(self.ctx, self._coeffs, mult, which, ct_hi, ct_lo)

    def _xor(self, a, b, out_level=None, defer_conj: bool = False):
        """XOR4(a, b); defer_conj: straight into a secret-key renorm (utils.ConjSum, as
        MixColFinal._xor_ct)"""
        if defer_conj and FOLDS.conj and takes_kw(self.xor4.apply, "defer_conj"):
            return self.xor4.apply(a, b, out_level, defer_conj=True)
        return self.xor4.apply(a, b, out_level)

    def _renorm_pair(self, hi, lo, level=None):
        return self.enc.renorm(hi, lo, level) if self.use_hard_renorm else (hi, lo)

    def _rot_rows_in_col(self, ct, k_rows: int):
        """Masked per-row rotation by k*stride (REF :100-109; unused by __call__)."""
        ctx = self.ctx
        out = ctx.multiply(ct, 0.0)
        for mask in self._pt_row:
            out = ctx.add(out, ctx.rotate(ctx.multiply(ct, mask), k_rows * self.stride))
        return out

    def _xor_pair(self, a, b, out_level=None):
        """(XOR4(a_hi, b_hi), XOR4(a_lo, b_lo)), batched when the XOR4 has apply_pair"""
        if hasattr(self.xor4, "apply_pair"):
            return self.xor4.apply_pair(a[0], b[0], a[1], b[1], out_level)
        return pair(self.ctx, lambda: self._xor(a[0], b[0], out_level), lambda: self._xor(a[1], b[1], out_level))

    def _gf(self, mult, hi, lo, out_level=None, defer_conj: bool = False):
        return gf_mult_pair(self.ctx, self._coeffs, mult, hi, lo, out_level, defer_conj)

    def gf_mult_9(self, hi, lo):
        return self._gf(9, hi, lo, self._gf_level)

    def gf_mult_11(self, hi, lo):
        return self._gf(11, hi, lo, self._gf_level)

    def gf_mult_13(self, hi, lo):
        return self._gf(13, hi, lo, self._gf_level)

    def gf_mult_14(self, hi, lo):
        return self._gf(14, hi, lo, self._gf_level)

    def _col_shift_rowmajor(self, ct, k_up: int):
        return self.ctx.rotate(ct, -4 * k_up * self.stride)

    def packed_ok(self) -> bool:
        """the packed XOR stage applies (see MixColFinal.packed_ok)"""
        return (self.use_hard_renorm and self.layout.packable and self.enc.renorm_hook is None
                and getattr(self.ctx, "fused_luts", False) and getattr(self.ctx, "renorm_unpack", None) is not None)

    def packed_input_need(self) -> int:
        """the level imc_packed needs on its input pair: the GF multipliers' input level"""
        return (NEED_XOR if _IMC_GF_LOW else NEED_GF) + self.enc.PACK_DEPTH

    def imc_packed(self, ct_hi, ct_lo, do_final_bootstrap: bool = True):
        """InvMixColumns with its XOR stage on packed states (MixColFinal.mix_packed):
        the four GF multiplier pairs' outputs packed (inputs one level higher than __call__'s),
        three single XOR4s and single renorms, one sparse bootstrap at period 2P.  Returns the
        PACKED output; the caller's renorm unpacks it."""
        ctx, enc = self.ctx, self.enc
        steps = [-4 * k * self.stride for k in (1, 2, 3)]
        rh, rl = rot_pair(ctx, ct_hi, ct_lo, steps)
        fl = RENORM_FLOOR
        gl = fl + LUT2_DEPTH + enc.PACK_DEPTH
        if _IMC_GF_LOW:
            # the GF multiplier pairs at the XOR4 level, each packed output renormalised (as
            # MixColFinal.mix_packed's rot form, round 5): inputs at gl = packed_input_need()
            direct = getattr(enc, "pack_renorm_direct", lambda ct=None: False)(ct_hi)  # the device renorm packs: no pack level
            if direct:
                gf = lambda m, hi, lo: enc.renorm_pack(*self._gf(m, hi, lo, fl, True), level=NEED_XOR)
            else:
                gf = lambda m, hi, lo: enc.renorm_packed(enc.pack(*self._gf(m, hi, lo, fl + enc.PACK_DEPTH, True)), level=NEED_XOR)
        else:
            gf = lambda m, hi, lo: enc.pack(*self._gf(m, hi, lo, gl))
        p14, p11 = pair(ctx, lambda: gf(14, ct_hi, ct_lo), lambda: gf(11, rh[0], rl[0]))
        p13, p9 = pair(ctx, lambda: gf(13, rh[1], rl[1]), lambda: gf(9, rh[2], rl[2]))
        x1, x2 = pair(ctx, lambda: enc.renorm_packed(self._xor(p14, p11, fl, True), level=NEED_XOR),
                      lambda: enc.renorm_packed(self._xor(p13, p9, fl, True), level=NEED_XOR))
        acc = enc.renorm_packed(self._xor(x1, x2, fl, True), level=NEED_BOOTSTRAP if do_final_bootstrap else None)
        if do_final_bootstrap:
            acc = bootstrap1(ctx, acc, 2 * self.layout.period)
        return acc

    def _call_fhe_quad(self, ct_hi, ct_lo, rot, do_final_bootstrap: bool, final_renorm: bool):
        """true-FHE with the quad bootstrap (zeta16_noise_reducer.BootstrapSnap.apply_quad; as
        MixColFinal.mix_rotated): the four GF multiplier pairs' outputs renormalised two pairs per
        bootstrap before any XOR4 (so the input needs the GF multipliers' levels only, not NEED_GF,
        and each XOR4 meets freshly snapped inputs), then (e14 ^ e11) ^ (e13 ^ e9) with the inner XOR
        pairs renormalised together"""
        enc, fl = self.enc, RENORM_FLOOR
        e14, e11 = enc.renorm_two(self._gf(14, ct_hi, ct_lo, fl), self._gf(11, *rot[1], fl), level=NEED_XOR)
        e13, e9 = enc.renorm_two(self._gf(13, *rot[2], fl), self._gf(9, *rot[3], fl), level=NEED_XOR)
        x1, x2 = enc.renorm_two(self._xor_pair(e14, e11, fl), self._xor_pair(e13, e9, fl), level=NEED_XOR)
        a3 = self._xor_pair(x1, x2, fl)
        if not final_renorm:
            return a3
        return self._renorm_pair(*a3, level=NEED_BOOTSTRAP if do_final_bootstrap else None)

    def __call__(self, ct_hi, ct_lo, do_final_bootstrap: bool = True, debug: Dict[str, Any] | None = None,
                 final_renorm: bool = True):
        """final_renorm=False returns the last XOR pair before its renorm (and without the final
        bootstrap): true-FHE decrypt applies the next round's InvShiftRows there first"""
        log = (lambda k, v: debug.__setitem__(k, v)) if debug is not None else (lambda k, v: None)
        steps = [-4 * k * self.stride for k in (1, 2, 3)]  # _col_shift_rowmajor(ct, k), hoisted
        rh, rl = rot_pair(self.ctx, ct_hi, ct_lo, steps)
        rot = {k: (rh[k - 1], rl[k - 1]) for k in (1, 2, 3)}
        for k in (1, 2, 3):
            log(f"rotc{k}", rot[k])
        if debug is None and self.enc.renorm_hook is not None and getattr(self.enc, "renorm_quad_hook", None) is not None:
            return self._call_fhe_quad(ct_hi, ct_lo, rot, do_final_bootstrap, final_renorm)
        # independent GF multiplier pairs two at a time on the branch streams
        e14, e11 = pair(self.ctx, lambda: self.gf_mult_14(ct_hi, ct_lo), lambda: self.gf_mult_11(*rot[1]))
        log("mul14", e14)
        log("mul11", e11)
        e13, e9 = pair(self.ctx, lambda: self.gf_mult_13(*rot[2]), lambda: self.gf_mult_9(*rot[3]))
        log("mul13", e13)
        log("mul9", e9)
        fl = self._xor_level
        last = NEED_BOOTSTRAP if do_final_bootstrap else None
        if debug is not None:
            # the reference's chain ((e14 ^ e11) ^ e13) ^ e9 and its debug keys (REF :123-134)
            a1 = self._xor_pair(e14, e11, fl)
            log("acc1", a1)
            a2 = self._xor_pair(self._renorm_pair(*a1, level=NEED_XOR), e13, fl)
            log("acc2", a2)
            a3 = self._xor_pair(self._renorm_pair(*a2, level=NEED_XOR), e9, fl)
            if not final_renorm:
                return a3
            out = self._renorm_pair(*a3, level=last)
        else:
            # (e14 ^ e11) ^ (e13 ^ e9): the chain regrouped (see MixColFinal), the two inner XOR
            # pairs on the two branch streams
            x1, x2 = pair(self.ctx, lambda: self._renorm_pair(*self._xor_pair(e14, e11, fl), level=NEED_XOR),
                          lambda: self._renorm_pair(*self._xor_pair(e13, e9, fl), level=NEED_XOR))
            if not final_renorm:
                return self._xor_pair(x1, x2, fl)
            out = self._renorm_pair(*self._xor_pair(x1, x2, fl), level=last)
        if do_final_bootstrap and self.enc.renorm_hook is None:
            out = bootstrap2(self.ctx, out[0], out[1], self.layout.boot_period)
        log("out", out)
        return out
