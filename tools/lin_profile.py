"""One CoeffToSlot butterfly group (bootstrap linear transform, BSGS) repeated, for
rocprofv3 --kernel-trace --stats: per-kernel cost of the bootstrap's dominant stage."""
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "aes-implementation-fhe_amd")]

from engine_context import EngineContext  # noqa: E402


def main():
    which = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    ctx = EngineContext(signature=1, max_level=17)
    E = ctx.engine
    rng = np.random.default_rng(0)
    ct = ctx.encrypt(np.exp(2j * np.pi * rng.random(E.slot_count)))
    top = E.import_ct(np.zeros((2, E.nl(E.L), E.n), np.uint32), E.L) if which < 3 else ct
    o = E.debug_lin_group(top, which)
    E.sync()
    t = time.perf_counter()
    for _ in range(reps):
        o = E.debug_lin_group(top, which)
    E.sync()
    print("group", which, "level", top.level, "->", o.level, "ms per group %.3f" % ((time.perf_counter() - t) * 1e3 / reps),
          E.counters())


if __name__ == "__main__":
    main()
