"""Regenerate tests/golden/ref_coeff.npz from the reference's shipped coefficient data
(REF/gen/coeff/*.json, the LUT polynomials read by REF/lut.py:10-62).

The fixture is data only: for every file, an int array of the index columns and a
complex array of the coefficients, in file order.  Run in the build container (the
GPU box has no /root/reference):  python tests/golden/make_ref_coeff_fixture.py
"""
import json
from pathlib import Path

import numpy as np

REF = Path("/root/reference/gen/coeff")
OUT = Path(__file__).resolve().parent / "ref_coeff.npz"

arrays = {}
for f in sorted(REF.glob("*.json")):
    ent = json.loads(f.read_text())["entries"]
    stem = f.stem
    arrays[stem + "__idx"] = np.array([e[:-2] for e in ent], dtype=np.int64)
    arrays[stem + "__val"] = np.array([complex(e[-2], e[-1]) for e in ent], dtype=np.complex128)
np.savez_compressed(OUT, **arrays)
print(f"wrote {OUT} ({len(arrays) // 2} files)")
