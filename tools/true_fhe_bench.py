"""True-FHE C2 encrypt (bootstrap + snap at every renorm point) beside the
secret-key-renorm encrypt, one state and a slot-packed batch, N = 2^16; prints JSON."""
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "aes-implementation-fhe_amd")]

from aes_keyschedule import expand_aes128_key, load_all_coeffs  # noqa: E402
from engine_context import EngineContext  # noqa: E402
from oracle import aes_plain  # noqa: E402  (checker, after timing)
from pipeline import AESPipeline  # noqa: E402


def run(ctx, co, rks, B, reps, **kw):
    pipe = AESPipeline(ctx, co, states=B, **kw)
    rng = np.random.default_rng(77 + B)
    pts = [rng.integers(0, 256, (B, 16) if B > 1 else 16).astype(np.uint8) for _ in range(reps + 1)]
    pipe.encrypt(pts[0], rks)
    ctx.engine.sync()
    n0 = ctx.bootstrap_stats()["count"]
    t0 = time.perf_counter()
    outs = [pipe.encrypt(p, rks) for p in pts[1:]]
    ctx.engine.sync()
    dt = (time.perf_counter() - t0) / reps
    nb = (ctx.bootstrap_stats()["count"] - n0) / reps
    ok = True
    for p, o in zip(pts[1:], outs):
        got = pipe.encoder.decode(*o)
        ok &= all(np.array_equal(np.atleast_2d(got)[j], aes_plain.ref_encrypt(np.atleast_2d(p)[j], rks)) for j in range(B))
    return {"states": B, "ms_per_encrypt": dt * 1e3, "rounds_per_s": 10.0 * B / dt, "blocks_per_s": B / dt,
            "bootstraps_per_encrypt": nb, "verified_against_plaintext_model": bool(ok)}


def main():
    ctx = EngineContext(signature=1, max_level=17)
    co = load_all_coeffs()
    np.random.seed(7)
    rks = expand_aes128_key(np.random.randint(0, 256, 16, dtype=np.uint8))
    out = {"secret_key_renorm": run(ctx, co, rks, 1, 2, use_hard_renorm_between_steps=True),
           "true_fhe": run(ctx, co, rks, 1, 2, use_hard_renorm_between_steps=False, true_fhe=True),
           "true_fhe_batch_1024": run(ctx, co, rks, 1024, 1, use_hard_renorm_between_steps=False, true_fhe=True)}
    print(json.dumps(out, indent=1), flush=True)


if __name__ == "__main__":
    main()
