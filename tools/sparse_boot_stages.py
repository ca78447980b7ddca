"""Cumulative wall time of the packed sparse-slot bootstrap up to each stage (period from
argv[1], default 32 -- the pair's 2n-periodic packing), stage costs as differences.
Runs with AESFHE_DEBUG_PERIOD=<period> so aesfhe_debug_boot_stage takes the sparse path."""
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "aes-implementation-fhe_amd")]
P = int(sys.argv[1]) if len(sys.argv) > 1 else 32
TRACE = "--trace" in sys.argv  # warm run, 100 ms pause, 5 bootstraps (tools/round_timeline.py analyse)
os.environ["AESFHE_DEBUG_PERIOD"] = str(P)

import numpy as np  # noqa: E402
from engine_context import EngineContext  # noqa: E402

STAGES = {1: "q0-only", 2: "SSE", 3: "ModRaise", 4: "to-dense+trace", 5: "CoeffToSlot", 9: "w+conj(w)", 10: "EvalMod",
          11: "SlotToCoeff+level_down"}


def main():
    ctx = EngineContext(signature=1, max_level=17)
    E = ctx.engine
    S = E.slot_count
    rng = np.random.default_rng(0)
    ct = ctx.encrypt(np.tile(np.exp(2j * np.pi * rng.random(P)), S // P))
    E.bootstrap_sparse(ct, P)
    E.sync()
    if TRACE:
        time.sleep(0.1)
        for _ in range(5):
            E.bootstrap_sparse(ct, P)
        E.sync()
        return
    res = {"period": P}
    prev = 0.0
    for s, name in STAGES.items():
        ts = []
        for _ in range(5):
            E.sync()
            t = time.perf_counter()
            o = E.debug_boot_stage(ct, s) if s < 11 else E.bootstrap_sparse(ct, P)
            E.sync()
            ts.append(time.perf_counter() - t)
            del o
        m = float(np.median(ts)) * 1e3
        res[name] = {"cum_ms": round(m, 3), "stage_ms": round(m - prev, 3)}
        prev = m
    E.reset_counters()
    E.bootstrap_sparse(ct, P)
    res["counters_one_bootstrap"] = E.counters()
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
