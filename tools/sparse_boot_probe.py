"""Sparse-slot bootstrap (aesfhe_bootstrap[_pair]_sparse): slot error on
n-periodic inputs and pair time against the full-slot pair bootstrap, N = 2^16 bootstrappable
set at fresh level 17."""
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "aes-implementation-fhe_amd")]

from engine_context import EngineContext  # noqa: E402


def timed(E, fn, n=8):
    fn()
    E.sync()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    E.sync()
    return (time.perf_counter() - t) / n * 1e3


def main():
    ctx = EngineContext(signature=1, max_level=17, seed=0x5EED)
    E = ctx.engine
    S = E.slot_count
    rng = np.random.default_rng(3)
    out = {}
    full_a = ctx.encrypt(np.exp(2j * np.pi * rng.random(S)))
    full_b = ctx.encrypt(np.exp(2j * np.pi * rng.random(S)))
    out["full_pair_ms"] = timed(E, lambda: E.bootstrap_pair(full_a, full_b))
    for n in [int(x) for x in (sys.argv[1:] or ["16", "256", "4096", "16384"])]:
        za = np.tile(np.exp(2j * np.pi * rng.random(n)) * rng.random(n), S // n)
        zb = np.tile(np.exp(2j * np.pi * rng.random(n)), S // n)
        a, b = ctx.encrypt(za), ctx.encrypt(zb)
        pa, pb = E.bootstrap_pair_sparse(a, b, n)
        sa = E.bootstrap_sparse(a, n)
        da, db = ctx.decrypt(pa), ctx.decrypt(pb)
        rec = {"level": pa.level, "max_err": float(max(np.abs(da - za).max(), np.abs(db - zb).max())),
               "rms_err": float(np.sqrt(np.mean(np.abs(da - za) ** 2))),
               "pair_equals_single": bool(np.array_equal(E.export(pa), E.export(sa))),
               "pair_ms": timed(E, lambda: E.bootstrap_pair_sparse(a, b, n))}
        out[f"n={n}"] = rec
        print(json.dumps({f"n={n}": rec}), flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
