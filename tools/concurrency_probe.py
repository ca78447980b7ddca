"""How much throughput do independent bootstraps gain from running concurrently?  k separate
contexts (own streams, own keys), one host thread each, n bootstraps per thread; prints
bootstraps/s for k = 1, 2, 4."""
import sys
import threading
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "aes-implementation-fhe_amd")]

from engine_context import EngineContext  # noqa: E402


def main(n=8):
    ctxs = [EngineContext(signature=1, max_level=17, seed=11 + i) for i in range(4)]
    cts = []
    for c in ctxs:
        E = c.engine
        z = np.exp(2j * np.pi * np.random.default_rng(0).random(E.slot_count))
        ct = E.intt(c.encrypt(z))
        E.bootstrap(ct)
        E.sync()
        cts.append(ct)
    for k in (1, 2, 4):
        def work(i):
            E = ctxs[i].engine
            for _ in range(n):
                E.bootstrap(cts[i])
            E.sync()
        th = [threading.Thread(target=work, args=(i,)) for i in range(k)]
        t = time.perf_counter()
        for x in th:
            x.start()
        for x in th:
            x.join()
        dt = time.perf_counter() - t
        print(f"k={k}: {k * n / dt:.1f} bootstraps/s ({dt / n * 1e3:.1f} ms per round of {k})", flush=True)


if __name__ == "__main__":
    main()
