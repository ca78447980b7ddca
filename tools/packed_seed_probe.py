"""Diagnostic: the 2,048-state packed encrypt -> decrypt round trip (tests/test_gpu_packed.py)
for several context seeds (key and encryption randomness), serial or concurrent; prints
pass / fail per seed and how many states differ.  Used to tell a data-dependent failure
(same seed fails every time) from a race (failures move between runs)."""
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "aes-implementation-fhe_amd")]

from aes_keyschedule import expand_aes128_key, load_all_coeffs  # noqa: E402
from engine_context import EngineContext  # noqa: E402
from oracle import aes_plain as A  # noqa: E402
from pipeline import AESPipeline  # noqa: E402


def main():
    states = 2048
    concurrent = "--concurrent" in sys.argv
    seeds = [int(a, 0) for a in sys.argv[1:] if not a.startswith("--")]
    co = load_all_coeffs()
    for seed in seeds:
        t = time.time()
        ctx = EngineContext(signature=1, max_level=17, seed=seed, concurrent=concurrent)
        pipe = AESPipeline(ctx, co, use_hard_renorm_between_steps=True, states=states)
        np.random.seed(7)
        rks = expand_aes128_key(np.random.randint(0, 256, 16, dtype=np.uint8))
        pts = np.random.default_rng(2025).integers(0, 256, (states, 16), dtype=np.uint8)
        ct = pipe.encrypt(pts, rks)
        got = pipe.encoder.decode(*ct)
        want = np.stack([A.ref_encrypt(p, rks) for p in pts])
        bad_enc = int((got != want).any(axis=1).sum())
        back = pipe.encoder.decode(*pipe.decrypt(*ct, rks))
        bad_dec = int((back != pts).any(axis=1).sum())
        print(f"seed {seed:#x} concurrent={concurrent}: enc_bad_states={bad_enc} dec_bad_states={bad_dec} ({time.time() - t:.1f} s)", flush=True)
        del ctx, pipe, ct


if __name__ == "__main__":
    main()
