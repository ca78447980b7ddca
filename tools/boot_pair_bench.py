"""Bootstrap pair throughput: two single bootstraps on two streams (the hi / lo branches)
vs one batched bootstrap_pair on one stream, N = 2^16 bootstrappable set."""
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "aes-implementation-fhe_amd")]

from engine_context import EngineContext  # noqa: E402
from utils import pair  # noqa: E402


def main(n=10):
    ctx = EngineContext(signature=1, max_level=17)
    E = ctx.engine
    rng = np.random.default_rng(0)
    a = ctx.encrypt(np.exp(2j * np.pi * rng.random(E.slot_count)))
    b = ctx.encrypt(np.exp(2j * np.pi * rng.random(E.slot_count)))
    for name, fn in (("two streams", lambda: pair(ctx, lambda: E.bootstrap(a), lambda: E.bootstrap(b))),
                     ("bootstrap_pair", lambda: E.bootstrap_pair(a, b))):
        fn()
        E.sync()
        t = time.perf_counter()
        for _ in range(n):
            fn()
        E.sync()
        print(f"{name}: {(time.perf_counter() - t) / n * 1e3:.2f} ms per pair", flush=True)


if __name__ == "__main__":
    main()
