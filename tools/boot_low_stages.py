"""Stage-by-stage comparison of the low-level sparse bootstrap with the standard one
on the same input: each stage of the debug path (aesfhe_debug_boot_stage_sparse) decrypted, its
level and its slot values against the standard form's.  Run twice by the caller: with
AESFHE_DEBUG_BOOT_FLOOR unset (standard) and =7 (low); prints one JSON line per stage."""
import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "aes-implementation-fhe_amd")]

from engine_context import EngineContext  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    out = Path(sys.argv[2]) if len(sys.argv) > 2 else None
    E = EngineContext(signature=1, max_level=17, seed=0x5EED, enc_nonce=3).engine
    rng = np.random.default_rng(1)
    z = np.tile(np.exp(2j * np.pi * rng.integers(0, 16, n) / 16), E.slot_count // n)
    ct = E.encrypt(z)
    res = {}
    for st in (12, 4, 5, 9, 10, 11):
        c = E.debug_boot_stage_sparse(ct, st, n)
        v = E.decrypt(c)
        res[st] = {"level": c.level, "max_abs": float(np.abs(v).max()), "vals": v[:2 * n].tolist()}
        print(json.dumps({"stage": st, "floor": os.environ.get("AESFHE_DEBUG_BOOT_FLOOR"), "level": c.level,
                          "max_abs": float(np.abs(v).max()), "err_vs_input": float(np.abs(v - z).max())}), flush=True)
    if out:
        out.write_text(json.dumps({k: {"level": v["level"], "re": [x.real for x in v["vals"]], "im": [x.imag for x in v["vals"]]}
                                   for k, v in res.items()}))


if __name__ == "__main__":
    main()
