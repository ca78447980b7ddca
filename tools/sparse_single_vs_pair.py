import sys, time
sys.path[:0] = ["/root/repo", "/root/repo/aes-implementation-fhe_amd"]
import numpy as np
from engine_context import EngineContext
ctx = EngineContext(signature=1, max_level=17, seed=1)
E = ctx.engine
S = E.slot_count
z = np.tile(np.exp(2j*np.pi*np.random.default_rng(0).random(16)), S // 16)
a, b = ctx.encrypt(z), ctx.encrypt(z)
def t(fn, n=8):
    fn(); E.sync(); t0 = time.perf_counter()
    for _ in range(n): fn()
    E.sync(); return (time.perf_counter() - t0) / n * 1e3
print("single sparse16", t(lambda: E.bootstrap_sparse(a, 16)))
print("pair sparse16", t(lambda: E.bootstrap_pair_sparse(a, b, 16)))
import os
