"""ShiftRows / InvShiftRows as byte permutations (shift_rows.ShiftRows.slot_perm, folded into the
periodic renorm by pipeline._sr_perm / aesfhe_renorm_periodic_perm): output byte i <- input byte
perm[i] must be the FIPS-197 ShiftRows of oracle/aes_plain.py for the one-state periodic layout,
and None for layouts where a byte is not one slot."""
import numpy as np

from oracle import aes_plain


def _sr(cls, periodic, states=1):
    from inv_shiftrows import InvShiftRows
    from shift_rows import ShiftRows
    from state_encoder import SlotLayout
    k = {"sr": ShiftRows, "isr": InvShiftRows}[cls]
    o = object.__new__(k)
    o.layout = SlotLayout(1 << 15, states, periodic)
    o.stride = o.layout.unit
    return o


def test_shift_rows_permutation_is_fips197():
    perm = _sr("sr", True).slot_perm()
    x = np.arange(16)
    assert np.array_equal(x[perm], aes_plain.shift_rows(x))
    iperm = _sr("isr", True).slot_perm()
    assert np.array_equal(x[iperm], aes_plain.inv_shift_rows(x))


def test_no_permutation_outside_the_one_state_periodic_layout():
    assert _sr("sr", False).slot_perm() is None
    assert _sr("sr", True, states=4).slot_perm() is None
