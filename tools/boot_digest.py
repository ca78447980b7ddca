"""Bit-exactness A/B of the bootstrap across two builds of libaesfhe.so on the GPU box:

    python3 tools/boot_digest.py [LIB.so]

prints a digest of the residues of bootstrap(ct) and bootstrap_pair(ct_a, ct_b) for fixed
seeds (key set, inputs), plus the pair bootstrap's wall time and the k_lin_mac kernel average.
Two builds whose digests agree produce identical bootstraps on these inputs."""
import hashlib
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "aes-implementation-fhe_amd")]

import mi355x_ckks  # noqa: E402


def main():
    if len(sys.argv) > 1:
        mi355x_ckks.load_library(Path(sys.argv[1]))
    from engine_context import EngineContext
    ctx = EngineContext(signature=1, max_level=17, seed=0xB007, enc_nonce=0)  # pinned: digests compare builds
    E = ctx.engine
    rng = np.random.default_rng(5)
    za = np.exp(2j * np.pi * rng.random(E.slot_count))
    zb = np.exp(2j * np.pi * rng.random(E.slot_count)) * rng.random(E.slot_count)
    a, b = ctx.encrypt(za), ctx.encrypt(zb)
    h = hashlib.blake2b(digest_size=16)
    s = ctx.bootstrap(a)
    pa, pb = ctx.bootstrap_pair(a, b)
    for c in (s, pa, pb):
        h.update(E.export(c).tobytes())
    err = float(max(np.abs(ctx.decrypt(pa) - za).max(), np.abs(ctx.decrypt(pb) - zb).max()))
    E.sync()
    E.profile(["lin_mac"], every=1)
    E.kernel_stats(reset=True)
    t0 = time.perf_counter()
    for _ in range(5):
        ctx.bootstrap_pair(a, b)
    E.sync()
    dt = (time.perf_counter() - t0) / 5
    st = E.kernel_stats(reset=True).get("lin_mac", {})
    E.profile(())
    print(json.dumps({"lib": sys.argv[1] if len(sys.argv) > 1 else "default", "digest": h.hexdigest(),
                      "pair_bootstrap_ms": dt * 1e3, "max_slot_err": err,
                      "lin_mac_avg_us": st.get("ms", 0) / max(st.get("launches", 1), 1) * 1e3,
                      "lin_mac_GBps": st.get("bytes", 0) / (st.get("ms", 1e-9) * 1e-3) / 1e9}), flush=True)


if __name__ == "__main__":
    main()
