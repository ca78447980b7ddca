import sys, time
sys.path[:0] = ["/root/repo", "/root/repo/aes-implementation-fhe_amd"]
import numpy as np
from engine_context import EngineContext
ctx = EngineContext(signature=1, max_level=17, seed=1)
E = ctx.engine
from state_encoder import StateEncoder
enc = StateEncoder(ctx)
hi, lo = enc.encode(np.arange(16, dtype=np.uint8))
for states in (1, 2, 2048):
    E.renorm_pair(hi, lo, states, level=13); E.sync()
    t = time.perf_counter()
    for _ in range(50):
        E.renorm_pair(hi, lo, states, level=13)
    E.sync()
    print("renorm states", states, (time.perf_counter() - t) / 50 * 1e3, "ms", flush=True)
