"""Post-trace stage of a sparse bootstrap (aesfhe_debug_boot_stage_sparse, stop after the trace to the
subring), decrypted: run with AESFHE_S2D_TRACE=1 (the sparse -> dense switch fused into the first trace
step) and =0 (separate), the slot values must agree within the bootstrap tolerance
(tests/test_gpu_flag_identity.py).  Prints one JSON object: the first 64 slots (re, im)."""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "aes-implementation-fhe_amd")]

from engine_context import EngineContext  # noqa: E402


def main():
    ctx = EngineContext(signature=1, max_level=17, seed=0x5EED, enc_nonce=0xC0FFEE)
    E = ctx.engine
    P = 32
    z = np.exp(2j * np.pi * np.random.default_rng(3).random(P))
    ct = E.intt(ctx.encrypt(np.tile(z, E.slot_count // P)))
    out = {}
    for stage, name in ((4, "trace"), (5, "cts")):
        s = ctx.decrypt(E.debug_boot_stage_sparse(ct, stage, P))[:64]
        out[name] = [s.real.tolist(), s.imag.tolist()]
    out["input"] = [np.tile(z, 2).real.tolist(), np.tile(z, 2).imag.tolist()]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
