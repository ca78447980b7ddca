"""ShiftRows and MixColumns merged (the "GHS12 merge refinement" the
reference plans in REF/README.md:137-138 and sketches in
REF/temp/shiftrows_mixcolumns_fused.py:44-258, ``ShiftRowsMixColumnsFusedEnc``).

Layout: byte (r, c) sits in slot (r + 4c)·stride (column-first, REF/state_encoder.py:23-27).
Write R_j = rotate(x, -4j·stride): R_j(r, c) = x(r, c + j).  ShiftRows is
SR(x)(r, c) = x(r, c + r), i.e. SR(x) = Σ_r D_r ⊙ R_r with D_r the mask of row r applied AFTER
the rotation (Gentry-Halevi-Smart 2012's form), and MixColumns reads the column shifts
rot_k(SR(x))(r, c) = x(r, c + k + r):

    Y_k = rot_k(SR(x)) = Σ_r D_r ⊙ R_{(k + r) mod 4},   k = 0..3   (Y_0 = SR(x))

so every ciphertext MixColumns needs is a masked sum of the SAME four rotations of x: three
hoisted rotations of one ciphertext (one ModUp, aesfhe_rotate_hoisted) and 16 mask products,
instead of ShiftRows' three rotations of three masked ciphertexts (three ModUps) followed by
MixColumns' three rotations of the ShiftRows output.  MixColumns then runs unchanged on
(Y_0; Y_1, Y_2, Y_3) (mixcol_final.MixColFinal.mix_rotated); same bytes, same levels (the
masks cost the level ShiftRows cost).  With B slot-packed states the masks cover
(r + 4c)·stride + b, b < B, as ShiftRows' (shift_rows.row_masks).
"""
from __future__ import annotations

from typing import Any, Dict, Tuple

from mixcol_final import MixColFinal
from shift_rows import row_masks
from utils import pair, rot_many


class ShiftRowsMixColumnsFusedEnc:
    def __init__(self, ctx, mix: MixColFinal, states: int = 1):
        self.ctx = ctx
        self.mix = mix
        self.sc = ctx.engine.slot_count
        layout = getattr(mix, "layout", None)  # mix may be None in the plain-slot tests
        self.stride = layout.unit if layout is not None else self.sc // 16
        self.masks = row_masks(ctx, self.sc, states, layout)  # D_r

    def _shifts(self, ct) -> Dict[int, Any]:
        """{k: Y_k} for one nibble ciphertext"""
        ctx = self.ctx
        R = [ct] + rot_many(ctx, ct, [-4 * j * self.stride for j in (1, 2, 3)])
        Y = {}
        for k in range(4):
            acc = None
            for r in range(4):
                t = ctx.multiply(R[(k + r) % 4], self.masks[r])
                acc = t if acc is None else ctx.add(acc, t)
            Y[k] = acc
        return Y

    def shifted(self, ct_hi, ct_lo) -> Dict[int, Tuple[Any, Any]]:
        """{k: (Y_k hi, Y_k lo)}: ShiftRows (k = 0) and MixColumns' column shifts of it"""
        yh, yl = pair(self.ctx, lambda: self._shifts(ct_hi), lambda: self._shifts(ct_lo))
        return {k: (yh[k], yl[k]) for k in range(4)}

    def __call__(self, ct_hi, ct_lo, do_final_bootstrap: bool = True, debug: Dict[str, Any] | None = None):
        Y = self.shifted(ct_hi, ct_lo)
        if isinstance(debug, dict):
            debug["sr"] = Y[0]
        return self.mix.mix_rotated(Y[0], {k: Y[k] for k in (1, 2, 3)}, do_final_bootstrap, debug)
