"""Throughput of multi-pair batches against the stack size: AESPipeline(pairs=P)
full encrypts, one state per pair (BASELINE config 3's shape) for P in argv (default 1 4 16 64),
and stacked slot-packed pairs of 2048 states (k = 1, 2, 4; --packed).  --ref: the one-state pairs in the reference's slot layout.
Prints one JSON line per shape (blocks/s, ms per encrypt, launches per encrypt, outputs checked against the plaintext AES)."""
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "aes-implementation-fhe_amd")]

from aes_keyschedule import expand_aes128_key, load_all_coeffs  # noqa: E402
from engine_context import EngineContext  # noqa: E402
from mi355x_ckks import launch_count  # noqa: E402
from oracle import aes_plain  # noqa: E402
from pipeline import AESPipeline  # noqa: E402


def probe(ctx, coeffs, rks, pairs, states, reps=2, periodic=None):
    pipe = AESPipeline(ctx, coeffs, use_hard_renorm_between_steps=True, states=states, pairs=pairs, periodic=periodic)
    rng = np.random.default_rng(pairs * 7 + states)
    shape = (pairs, 16) if states == 1 else (pairs, states, 16)
    E = ctx.engine
    pipe.encrypt(rng.integers(0, 256, shape, dtype=np.uint8), rks)
    E.sync()
    ins = [rng.integers(0, 256, shape, dtype=np.uint8) for _ in range(reps)]
    n0, t0 = launch_count(), time.perf_counter()
    outs = [pipe.encrypt(b, rks) for b in ins]
    E.sync()
    dt = (time.perf_counter() - t0) / reps
    launches = (launch_count() - n0) / reps
    ok = all(np.array_equal(pipe.encoder.decode(*o).reshape(-1, 16)[j], aes_plain.ref_encrypt(s, rks))
             for b, o in zip(ins, outs) for j, s in enumerate(b.reshape(-1, 16)))
    return {"pairs": pairs, "states_per_pair": states, "layout": "periodic" if pipe.layout.periodic else "reference",
            "ms_per_encrypt": dt * 1e3, "blocks_per_s": pairs * states / dt, "launches_per_encrypt": launches, "ok": bool(ok)}


def main():
    ps = [int(a) for a in sys.argv[1:] if a.isdigit()] or [1, 4, 16, 64]
    ps = [p for p in ps if p > 0]  # "0": no one-state shapes (e.g. --packed alone)
    ctx = EngineContext(signature=1, max_level=17)
    coeffs = load_all_coeffs()
    rks = expand_aes128_key(np.arange(16, dtype=np.uint8))
    ref = "--ref" in sys.argv  # the reference's slot layout (full-slot bootstraps) instead of the periodic one
    for p in ps:
        print(json.dumps(probe(ctx, coeffs, rks, p, 1, periodic=False if ref else None)), flush=True)
    if "--packed" in sys.argv:
        for k in (1, 2, 4):
            print(json.dumps(probe(ctx, coeffs, rks, k, 2048, reps=1)), flush=True)


if __name__ == "__main__":
    main()
