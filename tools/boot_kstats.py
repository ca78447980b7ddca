"""Per-kernel-id time and algorithmic bytes of one bootstrap (engine profiler, every launch
timed): where the bootstrap's time goes and how close each kernel class runs to HBM peak.
usage: python tools/boot_kstats.py [--pair | --sparse P]"""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "aes-implementation-fhe_amd")]

from engine_context import EngineContext  # noqa: E402
from mi355x_ckks import KERNEL_IDS  # noqa: E402


def main(n=5):
    ctx = EngineContext(signature=1, max_level=17)
    E = ctx.engine
    z = np.exp(2j * np.pi * np.random.default_rng(0).random(E.slot_count))
    ct = E.intt(ctx.encrypt(z))
    pair = "--pair" in sys.argv  # the batched hi / lo bootstrap
    # --sparse P: the sparse-slot bootstrap at period P (C2's MixColumns final bootstrap: one
    # packed ciphertext, P = 2 x 16 = 32); the input is made P-periodic
    sp = int(sys.argv[sys.argv.index("--sparse") + 1]) if "--sparse" in sys.argv else 0
    if sp:
        z = np.tile(z[:sp], E.slot_count // sp)
        ct = E.intt(ctx.encrypt(z))
        boot = lambda: E.bootstrap_sparse(ct, sp)  # noqa: E731
    else:
        boot = (lambda: E.bootstrap_pair(ct, ct)) if pair else (lambda: E.bootstrap(ct))
    boot()
    E.sync()
    E.profile(list(KERNEL_IDS), every=1)
    E.kernel_stats(reset=True)
    for _ in range(n):
        boot()
    E.sync()
    st = E.kernel_stats(reset=True)
    E.profile(())
    out = {}
    for k, v in sorted(st.items(), key=lambda kv: -kv[1]["ms"]):
        if not v["launches"]:
            continue
        out[k] = {"launches": v["launches"] / n, "ms": v["ms"] / n, "GB": v["bytes"] / n / 1e9,
                  "GBps": v["bytes"] / (v["ms"] * 1e-3) / 1e9 if v["ms"] else 0.0,
                  "avg_us": v["ms"] / v["launches"] * 1e3}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
