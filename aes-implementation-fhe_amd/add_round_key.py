"""AddRoundKey = nibble-wise XOR4 of state and round key (REF/add_round_key.py:138-144).

The legacy ``AESFHE`` class (REF/add_round_key.py:44-135) duplicates StateEncoder and
XOR4LUT and is not reachable from AESPipeline; it is not rebuilt.
"""
import json
from pathlib import Path
from typing import Any, Tuple

import numpy as np

from lut import COEFF_DIR, ensure_coeffs
from xor4_lut import XOR4LUT
from utils import pair


def load_xor4_coeffs(path: Path) -> np.ndarray:
    mat = np.zeros((16, 16), dtype=np.complex128)
    for i, j, re, im in json.loads(Path(path).read_text(encoding="utf-8"))["entries"]:
        mat[i, j] = complex(re, im)
    return mat


def default_xor4_coeffs() -> np.ndarray:
    return load_xor4_coeffs(ensure_coeffs(COEFF_DIR) / "xor4_coeffs.json")


class AddRoundKey:
    def __init__(self, xor4: XOR4LUT):
        self.xor4 = xor4

    def __call__(self, ct_hi, ct_lo, key_hi, key_lo, out_level=None) -> Tuple[Any, Any]:
        if hasattr(self.xor4, "apply_pair"):
            return self.xor4.apply_pair(ct_hi, key_hi, ct_lo, key_lo, out_level)
        return pair(self.xor4.ctx, lambda: self.xor4.apply(ct_hi, key_hi, out_level),
                    lambda: self.xor4.apply(ct_lo, key_lo, out_level))
