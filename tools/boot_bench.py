"""Repeated bootstraps of one full-slot ciphertext (N = 2^16 bootstrappable set), for
`rocprofv3 --kernel-trace --stats` breakdowns of the bootstrap's kernel mix."""
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "aes-implementation-fhe_amd")]

from engine_context import EngineContext  # noqa: E402


def main(n=int(sys.argv[1]) if len(sys.argv) > 1 else 10):
    ctx = EngineContext(signature=1, max_level=17)
    E = ctx.engine
    rng = np.random.default_rng(0)
    z = np.exp(2j * np.pi * rng.random(E.slot_count))
    ct = E.intt(ctx.encrypt(z))
    E.bootstrap(ct)
    E.sync()
    t = time.perf_counter()
    for _ in range(n):
        out = E.bootstrap(ct)
    E.sync()
    dt = (time.perf_counter() - t) / n
    err = np.abs(ctx.decrypt(out) - z).max()
    print(f"bootstrap {dt * 1e3:.2f} ms  max err {err:.2e}", flush=True)


if __name__ == "__main__":
    main()
