"""InvShiftRows: ShiftRows with the rotation sign flipped (REF/inv_shiftrows.py:11-47)."""
from shift_rows import ShiftRows


class InvShiftRows(ShiftRows):
    direction = +1

    @property
    def _rot_step(self):  # reference attribute name (REF/inv_shiftrows.py:36)
        return self._rot_steps
