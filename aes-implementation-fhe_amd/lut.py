"""Coefficient loaders (REF/lut.py:10-62) and the generic 1-D LUT evaluator (REF/lut.py:65-90).

File format: {"entries": [[k, re, im], ...]} (1-D) or [[p, q, re, im], ...] (2-D).
"""
import json
from pathlib import Path
from typing import Any, Dict

import numpy as np

COEFF_DIR = Path(__file__).resolve().parent / "coeff"


def ensure_coeffs(coeff_dir: Path = COEFF_DIR) -> Path:
    """Generate the JSON coefficient files with coeffgen.py if they are missing."""
    coeff_dir = Path(coeff_dir)
    if not (coeff_dir / "xor4_coeffs.json").exists():
        import coeffgen
        coeffgen.generate(coeff_dir)
    return coeff_dir


def _entries(path: Path):
    return json.loads(Path(path).read_text(encoding="utf-8")).get("entries", [])


def load_coeff1d(path: Path) -> np.ndarray:
    ent = _entries(path)
    out = np.zeros(max((int(e[0]) for e in ent), default=0) + 1, dtype=np.complex128)
    for k, re, im in ent:
        out[int(k)] = complex(re, im)
    return out


def load_coeff2d(path: Path, size: int) -> np.ndarray:
    out = np.zeros((size, size), dtype=np.complex128)
    for p, q, re, im in _entries(path):
        out[int(p), int(q)] = complex(re, im)
    return out


class LUTEvaluator:
    """Σ_k coeffs[k]·x^k over the basis x^1..x^{d/2} plus conjugate mirrors (REF/lut.py:65-90)."""

    def __init__(self, ctx, coeffs: Dict[int, Any], domain_size: int):
        self.ctx = ctx
        self.coeffs = coeffs
        self.domain = domain_size

    def apply(self, ct):
        ctx, half = self.ctx, self.domain // 2
        pos = ctx.make_power_basis(ct, half)
        basis = {0: ctx.add_plain(ct, 1.0)}
        for k in range(1, self.domain):
            basis[k] = pos[k - 1] if k <= half else ctx.conjugate(pos[self.domain - k - 1])
        res = ctx.multiply(ct, 0.0)
        for k, pt in self.coeffs.items():
            res = ctx.add(res, pt if k == 0 else ctx.multiply(basis[k], pt))
        return res
