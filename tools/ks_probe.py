"""Short key-switch workload for rocprofv3 PMC passes: the bench's parameter set
(bootstrappable N=2^16), relinearised products and rotations from the fresh level down.
Prints the engine's per-kernel stats (launches, ms, algorithmic bytes) as JSON."""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "aes-implementation-fhe_amd")]

from engine_context import EngineContext  # noqa: E402


def main():
    ctx = EngineContext(signature=1, max_level=17)
    E = ctx.engine
    rng = np.random.default_rng(0)
    ct = ctx.encrypt(np.exp(2j * np.pi * rng.random(E.slot_count)))
    E.sync()
    E.profile(["key_inner", "base_convert", "ntt_cols_fwd", "ntt_rows_fwd", "moddown"])
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
