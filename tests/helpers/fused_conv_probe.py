"""Digest of every key-switching path's raw output (RNS limbs) for one pinned key set and one
pinned encryption nonce: run once with AESFHE_FUSED_CONV=0 and once with it on, the digests must
be equal (tests/test_gpu_fused_conv.py).  Covers ModUp / ModDown of relinearisation (fused with
the rescale and plain), a rotation, a conjugation, a batched rotation set, a stacked key switch,
and the sparse bootstrap (its dense <-> sparse key switches).  Prints one JSON object."""
import hashlib
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "aes-implementation-fhe_amd")]

from mi355x_ckks import Engine  # noqa: E402


def main():
    E = Engine(log_n=16, max_level=17, seed=0x5EED, enc_nonce=0xC0FFEE, use_bootstrap=True)
    rng = np.random.default_rng(5)
    z = np.exp(2j * np.pi * rng.random(E.slot_count))
    w = np.exp(2j * np.pi * rng.random(E.slot_count))
    a, b = E.encrypt(z), E.encrypt(w)
    out = {}

    def dig(name, ct):
        out[name] = hashlib.sha256(np.ascontiguousarray(E.export(ct)).tobytes()).hexdigest()[:24]

    E.set_lazy(False)
    ab = E.multiply(a, b, "rlk")
    dig("relin+rescale", ab)
    x = ab
    for k in range(4):  # lower levels: fewer digits, a partial last digit
        x = E.multiply(x, x, "rlk")
        dig(f"square{k}", x)
    dig("rotate", E.rotate(a, None, 7))
    dig("rotate_low", E.rotate(x, None, 3))
    dig("conjugate", E.conjugate(b))
    for i, r in enumerate(E.rotate_multi([(a, 1), (a, 5), (b, 2)])):
        dig(f"rotate_multi{i}", r)
    st = E.stack([a, b, a])
    dig("stacked_rotate", E.rotate(st, None, 4))
    dig("relinearize", E.relinearize(E.multiply(a, b)))
    p = 32
    zs = np.tile(z[:p], E.slot_count // p)
    dig("bootstrap_sparse", E.bootstrap_sparse(E.intt(E.encrypt(zs)), p))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
