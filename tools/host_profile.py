"""Host-side cost of one C2 encrypt (bench.py's workload): time until pipeline.encrypt
returns (everything enqueued, no sync) vs time until the GPU is done, for the two-stream
and the serial pipeline, plus a cProfile of the serial encrypt (top functions by own time).
If the enqueue time is close to the total, the host, not the GPU, sets the pace."""
import cProfile
import io
import json
import pstats
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "aes-implementation-fhe_amd")]

from aes_keyschedule import expand_aes128_key, load_all_coeffs  # noqa: E402
from engine_context import EngineContext  # noqa: E402
from mixcol_final import MixColFinal  # noqa: E402
from pipeline import AESPipeline  # noqa: E402
from xor4_lut import XOR4LUT  # noqa: E402
from mi355x_ckks import EXPORTED as SYMS  # noqa: E402


def run(concurrent, reps=3, prof=False):
    coeffs = load_all_coeffs()
    ctx = EngineContext(signature=1, max_level=17, thread_count=1, seed=0x5EED, lazy=True, concurrent=concurrent)
    mix = MixColFinal(ctx, XOR4LUT(ctx, coeffs["xor4"]))
    pipe = AESPipeline(ctx, coeffs, mixcolumns=mix, use_hard_renorm_between_steps=True)
    rks = expand_aes128_key(np.arange(16, dtype=np.uint8))
    st = np.arange(16, dtype=np.uint8)
    E = ctx.engine
    pipe.encrypt(st, rks)
    E.sync()
    enq, tot = [], []
    for _ in range(reps):
        t0 = time.perf_counter()
        out = pipe.encrypt(st, rks)
        t1 = time.perf_counter()
        E.sync()
        t2 = time.perf_counter()
        enq.append(t1 - t0)
        tot.append(t2 - t0)
        del out
    res = {"enqueue_ms": 1e3 * float(np.median(enq)), "total_ms": 1e3 * float(np.median(tot))}
    if prof:
        # host time inside each C-ABI entry point (ctypes releases the GIL; serial pipeline)
        lib = ctx.engine._ctx.lib
        acc, cnt = {}, {}
        for name in [n for n in dir(lib) if n.startswith("aesfhe_")] + sorted(SYMS):
            if not name.startswith("aesfhe_"):
                continue
            try:
                f = getattr(lib, name)
            except AttributeError:
                continue

            def wrap(f=f, name=name):
                def w(*a):
                    t = time.perf_counter()
                    r = f(*a)
                    acc[name] = acc.get(name, 0.0) + time.perf_counter() - t
                    cnt[name] = cnt.get(name, 0) + 1
                    return r
                return w
            setattr(lib, name, wrap())
        out = pipe.encrypt(st, rks)
        E.sync()
        res["api_ms"] = {k: [round(1e3 * v, 2), cnt[k], round(1e6 * v / cnt[k], 1)] for k, v in sorted(acc.items(), key=lambda kv: -kv[1])}
        pr = cProfile.Profile()
        pr.enable()
        out = pipe.encrypt(st, rks)
        pr.disable()
        E.sync()
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
        res["cprofile_top"] = s.getvalue().splitlines()[:45]
    return res


def main():
    out = {"concurrent": run(True), "serial": run(False, prof=True)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
