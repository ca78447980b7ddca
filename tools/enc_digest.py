"""Bit-identity A/B of a C2 encrypt across two builds of libaesfhe.so (the renorms' fresh
encryptions included): python3 tools/enc_digest.py [LIB.so] prints a digest of the ciphertext
residues after 2 AES rounds and after the full encrypt, for a pinned key set and encryption nonce."""
import hashlib
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "aes-implementation-fhe_amd")]

import mi355x_ckks  # noqa: E402


def main():
    if len(sys.argv) > 1:
        mi355x_ckks.load_library(Path(sys.argv[1]))
    from aes_keyschedule import expand_aes128_key, load_all_coeffs
    from engine_context import EngineContext
    from pipeline import AESPipeline
    ctx = EngineContext(signature=1, max_level=17, seed=0x5EED, enc_nonce=0)
    E = ctx.engine
    pipe = AESPipeline(ctx, load_all_coeffs(), use_hard_renorm_between_steps=True)
    rng = np.random.default_rng(7)
    rks = expand_aes128_key(rng.integers(0, 256, 16, dtype=np.uint8))
    st = rng.integers(0, 256, 16, dtype=np.uint8)
    hi, lo = pipe.encrypt(st, rks)
    h = hashlib.blake2b(digest_size=16)
    for c in (hi, lo):
        h.update(E.export(c).tobytes())
    print(json.dumps({"lib": sys.argv[1] if len(sys.argv) > 1 else "in-tree", "digest": h.hexdigest()}), flush=True)


if __name__ == "__main__":
    main()
