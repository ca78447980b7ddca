"""ShiftRows under column-first packing (REF/shift_rows.py:7-56).

Row r occupies slots (r + 4c)*stride; ShiftRows rotates row r left by r columns, i.e.
the masked row is rotated by -4r*stride slots (np.roll semantics).
With ``states`` = B slot-packed states (state_encoder.py) the row masks cover slots
(r + 4c)*stride + b for b < B (REF/temp/mixcolumns_desilo_port.py:60-65 builds the same
per-block masks); B = 1 is the reference's mask exactly.
"""
from typing import Any, List

import numpy as np
from utils import _MULTI, pair


def shift_rows_bytes(state: np.ndarray, direction: int = -1) -> np.ndarray:
    """the byte permutation ShiftRows (direction -1) / InvShiftRows (+1) applies to a (16,) or
    (B, 16) column-first state: row r (bytes r + 4c) rotated by direction * r columns; used
    to permute plaintext round keys for the SubBytes-AddRoundKey fusion (sub_bytes_ark.py)"""
    s = np.asarray(state, np.uint8)
    M = s.reshape(*s.shape[:-1], 4, 4)  # [..., c, r]
    out = np.empty_like(M)
    for r in range(4):
        out[..., :, r] = np.roll(M[..., :, r], direction * r, axis=-1)
    return out.reshape(s.shape)


def row_masks(ctx, sc: int, states: int = 1, layout=None) -> List[Any]:
    """the four row masks (REF/shift_rows.py:20-33) in `layout` (default: the reference's)"""
    from state_encoder import SlotLayout
    lay = layout or SlotLayout(sc, states)
    return [ctx.encode(lay.row_mask(r)) for r in range(4)]


class ShiftRows:
    direction = -1

    def __init__(self, ctx, states: int = 1, layout=None):
        from state_encoder import SlotLayout
        self.ctx = ctx
        self.sc = ctx.engine.slot_count
        self.layout = layout or SlotLayout(self.sc, states)
        self.stride = self.layout.unit
        self.states = states
        self._pt_masks = row_masks(ctx, self.sc, states, self.layout)
        self._rot_steps = [self.direction * 4 * r * self.stride for r in range(4)]

    def slot_perm(self):
        """the permutation as output slot i <- input slot perm[i] when the layout holds one state per
        16-slot block (periodic, unit 1: byte i in slot i), else None -- for a renorm that folds it
        (StateEncoder.renorm(perm=)); row r's slots rotate by direction * 4 r (np.roll convention)"""
        if not (self.layout.periodic and self.stride == 1 and self.layout.period == 16):
            return None
        return [(i - self.direction * 4 * (i % 4)) % 16 for i in range(16)]

    def _apply_one(self, ct: Any) -> Any:
        ctx = self.ctx
        out = ctx.multiply(ct, 0.0)
        for mask, step in zip(self._pt_masks, self._rot_steps):
            part = ctx.multiply(ct, mask)
            out = ctx.add(out, ctx.rotate(part, step) if step else part)
        return out

    def apply(self, ct_hi: Any, ct_lo: Any):
        """both halves; with a batching context the 8 masked rows (lazy plaintext products) go
        through ONE rotate_multi -- their rescales stacked, the 6 rotations one batched key switch
         -- instead of 6 separate rotations on two streams; same results"""
        ctx = self.ctx
        if getattr(ctx, "rotate_multi", None) is None or not _MULTI:
            return pair(ctx, lambda: self._apply_one(ct_hi), lambda: self._apply_one(ct_lo))
        parts = [ctx.multiply(ct, mask) for ct in (ct_hi, ct_lo) for mask in self._pt_masks]
        rots = ctx.rotate_multi([(p, s) for p, s in zip(parts, self._rot_steps * 2)])
        out = []
        for h in (0, 4):
            acc = rots[h]
            for r in rots[h + 1:h + 4]:
                acc = ctx.add(acc, r)
            out.append(acc)
        return out[0], out[1]
