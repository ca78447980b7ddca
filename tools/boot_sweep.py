"""Pair-bootstrap time and accuracy of one bootstrap configuration (set through the
environment: AESFHE_BOOT_CTS = CoeffToSlot groups, AESFHE_BOOT_BMAX = baby-step cap),
N = 2^16 bootstrappable set at fresh level 17."""
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "aes-implementation-fhe_amd")]

from engine_context import EngineContext  # noqa: E402


def main(n=10):
    ctx = EngineContext(signature=1, max_level=17, seed=0x5EED)
    E = ctx.engine
    rng = np.random.default_rng(0)
    za = np.exp(2j * np.pi * rng.random(E.slot_count))
    zb = np.exp(2j * np.pi * rng.random(E.slot_count)) * rng.random(E.slot_count)
    a, b = ctx.encrypt(za), ctx.encrypt(zb)
    pa, pb = E.bootstrap_pair(a, b)
    E.sync()
    err = max(np.abs(ctx.decrypt(pa) - za).max(), np.abs(ctx.decrypt(pb) - zb).max())
    t = time.perf_counter()
    for _ in range(n):
        E.bootstrap_pair(a, b)
    E.sync()
    ms = (time.perf_counter() - t) / n * 1e3
    print(json.dumps({"cts_groups": os.environ.get("AESFHE_BOOT_CTS", "3"), "baby_max": os.environ.get("AESFHE_BOOT_BMAX", "16"),
                      "log_pq": round(E.log_pq, 1), "top_limbs": E.nl(E.L), "pair_ms": round(ms, 2), "max_err": float(err),
                      "out_level": pa.level}), flush=True)


if __name__ == "__main__":
    main()
