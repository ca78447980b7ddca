"""Single sparse-slot bootstrap at the pipeline's packed period (n = 32: one state, hi | lo)
under the EvalMod configuration in the environment (AESFHE_BOOT_K / _R / _DEG, read once per
process): time and slot error on 32-periodic inputs of modulus <= 1 and on Zeta16 codewords.
One JSON line; run once per configuration (tools/evalmod sweep in DESIGN.md §4)."""
import hashlib
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "aes-implementation-fhe_amd")]

from engine_context import EngineContext  # noqa: E402


def main(n=32, reps=10):
    ctx = EngineContext(signature=1, max_level=17, seed=0x5EED)
    E = ctx.engine
    S = E.slot_count
    rng = np.random.default_rng(5)
    za = np.tile(np.exp(2j * np.pi * rng.random(n)) * rng.random(n), S // n)
    zz = np.tile(np.exp(2j * np.pi * rng.integers(0, 16, n) / 16), S // n)
    a, z = ctx.encrypt(za), ctx.encrypt(zz)
    out = E.bootstrap_sparse(a, n)
    oz = E.bootstrap_sparse(z, n)
    E.sync()
    t = time.perf_counter()
    for _ in range(reps):
        E.bootstrap_sparse(a, n)
    E.sync()
    ms = (time.perf_counter() - t) / reps * 1e3
    print(json.dumps({"K_r_deg": [os.environ.get(k, "default") for k in ("AESFHE_BOOT_K", "AESFHE_BOOT_R", "AESFHE_BOOT_DEG")],
                      "evalmod_batch": os.environ.get("AESFHE_EVALMOD_BATCH", "1"),
                      "digest": hashlib.md5(E.export(out).tobytes() + E.export(oz).tobytes()).hexdigest(),
                      "n": n, "level": out.level, "ms": ms,
                      "max_err": float(np.abs(ctx.decrypt(out) - za).max()),
                      "max_err_zeta16": float(np.abs(ctx.decrypt(oz) - zz).max())}), flush=True)


if __name__ == "__main__":
    main()
