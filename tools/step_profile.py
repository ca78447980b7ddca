"""Synchronised wall time of each AES step of one middle encrypt round (C2 parameters),
plus the MixColumns breakdown (GF LUTs, XOR4s, renorms, final bootstraps)."""
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "aes-implementation-fhe_amd")]

from aes_keyschedule import expand_aes128_key, load_all_coeffs  # noqa: E402
from engine_context import EngineContext  # noqa: E402
from pipeline import AESPipeline  # noqa: E402


def main():
    lazy = "--eager" not in sys.argv
    ctx = EngineContext(signature=1, max_level=17, lazy=lazy)
    E = ctx.engine
    pipe = AESPipeline(ctx, load_all_coeffs(), use_hard_renorm_between_steps=True)
    np.random.seed(7)
    rks = expand_aes128_key(np.random.randint(0, 256, 16, dtype=np.uint8))
    st = np.random.randint(0, 256, 16, dtype=np.uint8)
    rk = pipe._prepare_round_keys(rks)
    ct = pipe._renorm_pair(*pipe.add_round_key(*pipe.encoder.encode(st), *rk[0]))
    pipe.encrypt_round(ct, rk[1])  # warm caches (plaintext encodings, keys, bootstrap plan)
    E.sync()
    res = {}

    def timed(name, fn, *a):
        E.sync()
        t = time.perf_counter()
        out = fn(*a)
        E.sync()
        res[name] = res.get(name, 0.0) + (time.perf_counter() - t) * 1e3
        return out

    mix = pipe.mix
    orig_xor, orig_renorm, orig_boot = mix._xor_ct, mix._renorm_pair, ctx.bootstrap
    mix._xor_ct = lambda a, b: timed("mc.xor4", orig_xor, a, b)
    mix._renorm_pair = lambda h, l: timed("mc.renorm", orig_renorm, h, l)
    ctx.bootstrap = lambda c: timed("bootstrap", orig_boot, c)
    t0 = time.perf_counter()
    c = timed("sub_bytes", pipe.sub_bytes, *ct)
    c = timed("renorm", pipe._renorm_pair, *c)
    c = timed("shift_rows", pipe.shift_rows, *c)
    c = timed("mix_columns(total)", pipe.mix_columns, *c)
    c = timed("add_round_key", pipe.add_round_key, *c, *rk[2])
    c = timed("renorm", pipe._renorm_pair, *c)
    res["round_total"] = (time.perf_counter() - t0) * 1e3
    res["mc.gf_luts+rest"] = res["mix_columns(total)"] - res.get("mc.xor4", 0) - res.get("mc.renorm", 0) - res.get("bootstrap", 0)
    print(json.dumps({"lazy": lazy, "ms": {k: round(v, 2) for k, v in res.items()}}, indent=1))


if __name__ == "__main__":
    main()
