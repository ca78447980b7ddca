"""Sparse-slot bootstrap timings: single (period 16, 32, 64) vs the pair-packed pair (period 16).
A pair of 16-periodic messages packed into ONE 32-periodic one (hi + X^(N/64) lo) costs one
single bootstrap at period 32 plus the split (one rotation)."""
import json
import sys
import time

sys.path[:0] = ["/root/repo", "/root/repo/aes-implementation-fhe_amd"]
import numpy as np  # noqa: E402
from engine_context import EngineContext  # noqa: E402

ctx = EngineContext(signature=1, max_level=17, seed=1)
E = ctx.engine
S = E.slot_count
z = np.tile(np.exp(2j * np.pi * np.random.default_rng(0).random(16)), S // 16)
a, b = ctx.encrypt(z), ctx.encrypt(z)


def t(fn, n=8):
    fn()
    E.sync()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    E.sync()
    return round((time.perf_counter() - t0) / n * 1e3, 3)


res = {f"single_sparse{p}_ms": t(lambda: E.bootstrap_sparse(a, p)) for p in (16, 32, 64)}
res["pair_sparse16_ms"] = t(lambda: E.bootstrap_pair_sparse(a, b, 16))
res["rotate_fresh_ms"] = t(lambda: E.rotate(a, delta=3))
print(json.dumps(res), flush=True)
