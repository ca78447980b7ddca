"""One middle encrypt round of the bench workload (C2: bootstrappable N = 2^16, renorm on,
MixColumns' final bootstrap pair) on one stream, for rocprofv3 --pmc passes: the full bench
aborts inside rocprofv3's counter-collection dispatch path (profiles/r2_pmc_bench_failure.log),
this is the same kernels with the same shapes, ~6k dispatches.  With
AESFHE_PROFILE_FROM_START=<ids> the engine's algorithmic bytes of exactly the same launches
(whole process, keys included, as a --pmc pass counts them) go to argv[1] as JSON.
pairs=P (an argument): the round of a stack of P one-state ciphertext pairs (BASELINE C3's shape,
DESIGN.md §3.16) instead of one pair."""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "aes-implementation-fhe_amd")]

from aes_keyschedule import expand_aes128_key, load_all_coeffs  # noqa: E402
from engine_context import EngineContext  # noqa: E402
from pipeline import AESPipeline  # noqa: E402


def main():
    kv = dict(a.split("=", 1) for a in sys.argv[1:] if "=" in a)
    out = [a for a in sys.argv[1:] if "=" not in a]
    pairs = int(kv.get("pairs", 1))
    ctx = EngineContext(signature=1, max_level=17, thread_count=1, seed=0x5EED, concurrent=False)
    E = ctx.engine
    pipe = AESPipeline(ctx, load_all_coeffs(), use_hard_renorm_between_steps=True, pairs=pairs)
    np.random.seed(7)
    rks = expand_aes128_key(np.random.randint(0, 256, 16, dtype=np.uint8))
    st = np.random.randint(0, 256, (16,) if pairs == 1 else (pairs, 16), dtype=np.uint8)
    rk = pipe._prepare_round_keys(rks)
    ct = pipe._ark_renorm(pipe.encoder.encode(st), rk[0], level=pipe.need_sub)
    ct = pipe.encrypt_round(ct, rk[1], r=1)
    E.sync()
    print(json.dumps({"round1_state_decodes": pipe.encoder.decode(*ct).tolist()}), flush=True)
    if out:
        Path(out[0]).write_text(json.dumps(E.kernel_stats(reset=True), indent=1))


if __name__ == "__main__":
    main()
