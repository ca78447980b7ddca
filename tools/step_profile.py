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
from utils import pair  # noqa: E402


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
    t0 = time.perf_counter()
    c = timed("sub_bytes", pipe.sub_bytes, *ct)
    c = timed("renorm", pipe._renorm_pair, *c)
    c = timed("shift_rows", pipe.shift_rows, *c)
    # MixColFinal.__call__ step by step (same calls, each pair timed as a whole)
    t_mc = time.perf_counter()
    hi, lo = c
    rh, rl = timed("mc.rotations", lambda: pair(ctx, lambda: [mix._col_shift_rowmajor(hi, k) for k in (1, 2, 3)],
                                                  lambda: [mix._col_shift_rowmajor(lo, k) for k in (1, 2, 3)]))
    two = timed("mc.gf_mult_2", mix.gf_mult_2, hi, lo)
    thr = timed("mc.gf_mult_3", mix.gf_mult_3, rh[0], rl[0])
    xor_pair = lambda a, b: pair(ctx, lambda: mix._xor_ct(a[0], b[0]), lambda: mix._xor_ct(a[1], b[1]))
    acc = timed("mc.xor4_pairs", xor_pair, two, thr)
    acc = timed("mc.renorm", mix._renorm_pair, *acc)
    acc = timed("mc.xor4_pairs", xor_pair, acc, (rh[1], rl[1]))
    acc = timed("mc.renorm", mix._renorm_pair, *acc)
    acc = timed("mc.xor4_pairs", xor_pair, acc, (rh[2], rl[2]))
    acc = timed("mc.renorm", mix._renorm_pair, *acc)
    c = timed("mc.bootstrap_pair", lambda: pair(ctx, lambda: ctx.bootstrap(ctx.to_intt(acc[0])),
                                                lambda: ctx.bootstrap(ctx.to_intt(acc[1]))))
    res["mix_columns(total)"] = (time.perf_counter() - t_mc) * 1e3
    c = timed("add_round_key", pipe.add_round_key, *c, *rk[2])
    c = timed("renorm", pipe._renorm_pair, *c)
    res["round_total"] = (time.perf_counter() - t0) * 1e3
    print(json.dumps({"lazy": lazy, "ms": {k: round(v, 2) for k, v in res.items()}}, indent=1))


if __name__ == "__main__":
    main()
