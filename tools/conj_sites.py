"""Which round-module lines issue single conjugations / rotations / products during one C2 encrypt
(the launch census's aesfhe_conjugate entry): counts EngineContext calls by the calling
file:line of the package.  usage: python3 tools/conj_sites.py > out.json (GPU)"""
import collections
import json
import sys
import traceback
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "aes-implementation-fhe_amd")]

from aes_keyschedule import expand_aes128_key, load_all_coeffs  # noqa: E402
from engine_context import EngineContext  # noqa: E402
from pipeline import AESPipeline  # noqa: E402


def main():
    ctx = EngineContext(signature=1, boot_fresh_level=7, dnum=4)  # the bench's C2 set
    pipe = AESPipeline(ctx, load_all_coeffs(), use_hard_renorm_between_steps=True)
    rng = np.random.default_rng(7)
    rks = expand_aes128_key(rng.integers(0, 256, 16, dtype=np.uint8))
    st = rng.integers(0, 256, 16, dtype=np.uint8)
    pipe.encrypt(st, rks)
    E = ctx.engine
    counts = {name: collections.Counter() for name in ("conjugate", "conjugate_many", "rotate", "galois_multi", "mul_many")}
    for name in counts:
        fn = getattr(E, name, None)
        if fn is None:
            continue

        def wrap(*a, _fn=fn, _name=name, **k):
            site = [f"{Path(f.filename).name}:{f.lineno}" for f in traceback.extract_stack()[:-1]
                    if "aes-implementation-fhe_amd" in f.filename and not f.filename.endswith(("mi355x_ckks.py", "deferred_calls.py"))]
            counts[_name][" < ".join(site[-3:][::-1])] += 1
            return _fn(*a, **k)
        setattr(E, name, wrap)
    pipe.encrypt(st, rks)
    E.sync()
    print(json.dumps({k: dict(v.most_common(30)) for k, v in counts.items()}, indent=1))


if __name__ == "__main__":
    main()
