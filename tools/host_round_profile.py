"""cProfile of the host side of encrypt rounds (C2 bench workload): where the Python driver and
the ctypes engine calls spend their time, to tell a host-bound round from a GPU-bound one
(tools/round_timeline.py reports host enqueue time ~ wall time when the host is the limit)."""
import cProfile
import io
import json
import pstats
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "aes-implementation-fhe_amd"), str(ROOT / "tools")]

import round_timeline  # noqa: E402


def main():
    import numpy as np
    from aes_keyschedule import expand_aes128_key, load_all_coeffs
    from engine_context import EngineContext
    from pipeline import AESPipeline
    ctx = EngineContext(signature=1, max_level=17, seed=0x5EED)
    E = ctx.engine
    pipe = AESPipeline(ctx, load_all_coeffs(), use_hard_renorm_between_steps=True)
    np.random.seed(7)
    rk = pipe._prepare_round_keys(expand_aes128_key(np.random.randint(0, 256, 16, dtype=np.uint8)))
    c = pipe._ark_renorm(pipe.encoder.encode(np.random.randint(0, 256, 16, dtype=np.uint8)), rk[0], level=pipe.need_sub)
    c = pipe.encrypt_round(c, rk[1], r=1)
    E.sync()
    pr = cProfile.Profile()
    t = time.perf_counter()
    pr.enable()
    for r in range(6):
        c = pipe.encrypt_round(c, rk[2 + r], r=2 + r)
    pr.disable()
    host = (time.perf_counter() - t) / 6 * 1e3
    E.sync()
    wall = (time.perf_counter() - t) / 6 * 1e3
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
    print(json.dumps({"host_ms_per_round_profiled": host, "wall_ms_per_round_profiled": wall}))
    print(s.getvalue())


if __name__ == "__main__":
    main()
