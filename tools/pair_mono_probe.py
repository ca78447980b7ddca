"""Pair bootstrap of two n-periodic messages: time and max slot error, for the 2n-periodic
monomial packing (default) and, with AESFHE_PAIR_MONO=0, the stacked pair / pair4 path.
usage: pair_mono_probe.py [periods...]"""
import json
import os
import sys
import time

sys.path[:0] = ["/root/repo", "/root/repo/aes-implementation-fhe_amd"]
import numpy as np  # noqa: E402
from engine_context import EngineContext  # noqa: E402

ctx = EngineContext(signature=1, max_level=17, seed=3)
E = ctx.engine
S = E.slot_count
res = {"mono": os.environ.get("AESFHE_PAIR_MONO", "1")}
for p in [int(x) for x in (sys.argv[1:] or ["16", "1024", "16384"])]:
    rng = np.random.default_rng(p)
    za = np.tile(np.exp(2j * np.pi * rng.random(p)) * rng.random(p), S // p)
    zb = np.tile(np.exp(2j * np.pi * rng.random(p)), S // p)
    a, b = ctx.encrypt(za), ctx.encrypt(zb)
    pa, pb = E.bootstrap_pair_sparse(a, b, p)
    E.sync()
    t0 = time.perf_counter()
    for _ in range(6):
        E.bootstrap_pair_sparse(a, b, p)
    E.sync()
    ms = (time.perf_counter() - t0) / 6 * 1e3
    ea, eb = np.abs(ctx.decrypt(pa) - za), np.abs(ctx.decrypt(pb) - zb)
    res[f"n={p}"] = {"pair_ms": round(ms, 3), "level": pa.level, "max_err_a": float(ea.max()), "max_err_b": float(eb.max()),
                     "rms_err": float(np.sqrt(np.mean(np.concatenate([ea, eb]) ** 2)))}
    print(json.dumps({f"n={p}": res[f"n={p}"]}), flush=True)
print(json.dumps(res), flush=True)
