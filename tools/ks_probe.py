"""Short key-switch workload for rocprofv3 PMC passes: the bench's parameter set
(bootstrappable N=2^16), relinearised products and rotations from the fresh level down.
Prints the engine's per-kernel stats (launches, ms, algorithmic bytes) as JSON; with
AESFHE_PROFILE_FROM_START=<ids> they cover the whole process, like a --pmc pass."""
import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "aes-implementation-fhe_amd")]

from engine_context import EngineContext  # noqa: E402


KIDS = ["key_inner", "base_convert", "ntt_cols_fwd", "ntt_rows_fwd", "moddown"]


def main():
    # whole-process accounting (keys included) when rocprofv3 counts the whole process too
    whole = bool(os.environ.get("AESFHE_PROFILE_FROM_START"))
    ctx = EngineContext(signature=1, max_level=17)
    E = ctx.engine
    rng = np.random.default_rng(0)
    ct = ctx.encrypt(np.exp(2j * np.pi * rng.random(E.slot_count)))
    E.sync()
    if not whole:
        E.profile(KIDS)
        E.kernel_stats(reset=True)
    x = ct
    while x.level > 1:
        y = ctx.rotate(x, 4096)
        x = ctx.multiply(y, x)
        x = ctx.conjugate(x)
    E.sync()
    print(json.dumps(E.kernel_stats(reset=True)))


if __name__ == "__main__":
    main()
