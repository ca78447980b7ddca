"""Cumulative wall time of bootstrapping up to each stage (engine.bootstrap stop_after),
N = 2^16 bootstrappable parameters; stage costs are the differences."""
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "aes-implementation-fhe_amd")]

from engine_context import EngineContext  # noqa: E402

STAGES = ["q0-only", "SSE", "ModRaise", "to-dense", "CoeffToSlot", "real", "imag", "EvalMod(re)", "EvalMod(im)",
          "recombine", "SlotToCoeff"]


def main():
    ctx = EngineContext(signature=1, max_level=17)
    E = ctx.engine
    rng = np.random.default_rng(0)
    ct = ctx.encrypt(np.exp(2j * np.pi * rng.random(E.slot_count)))
    ct = E.intt(ct)
    E.bootstrap(ct)
    E.sync()
    res = {}
    prev = 0.0
    for s in range(1, 12):
        ts = []
        for _ in range(3):
            E.sync()
            t = time.perf_counter()
            o = E.debug_boot_stage(ct, s) if s < 11 else E.bootstrap(ct)
            E.sync()
            ts.append(time.perf_counter() - t)
            del o
        m = float(np.median(ts)) * 1e3
        res[STAGES[s - 1]] = {"cum_ms": m, "stage_ms": m - prev}
        prev = m
    E.reset_counters()
    E.bootstrap(ct)
    res["counters_one_bootstrap"] = E.counters()
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
