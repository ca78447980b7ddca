"""Digest of a full-slot bootstrap of a pinned input (pinned key set and encryption nonce).  With
AESFHE_TEST_FAIL_GIANT=k the engine's k-th giant-step accumulation throws: the probe runs one bootstrap
that must fail mid-group first, then the digested one -- which must equal a clean process's
(tests/test_gpu_flag_identity.py; ADVICE r4: the fused form's P rows were engine-wide state a failed
group could leave to the next call).  Prints one JSON object."""
import hashlib
import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "aes-implementation-fhe_amd")]

from mi355x_ckks import Engine  # noqa: E402


def main():
    E = Engine(log_n=16, max_level=17, seed=0x5EED, enc_nonce=0xC0FFEE, use_bootstrap=True)
    z = np.exp(2j * np.pi * np.random.default_rng(9).random(E.slot_count))
    ct = E.intt(E.encrypt(z))
    failed = None
    if os.environ.get("AESFHE_TEST_FAIL_GIANT"):
        try:
            E.bootstrap(ct)
            failed = False
        except RuntimeError as e:
            failed = "test failure" in str(e)
    out = E.bootstrap(ct)
    d = hashlib.sha256(np.ascontiguousarray(E.export(out)).tobytes()).hexdigest()[:24]
    print(json.dumps({"failed_first": failed, "digest": d}))


if __name__ == "__main__":
    main()
