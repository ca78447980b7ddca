"""Launch census of the C2 bench workload: kernel launches (aesfhe_launch_count) and synchronised
wall time of each AES step of a middle encrypt round, of the sparse bootstrap alone, and of one
full 10-round encrypt (launches per encrypt, the VERDICT r2 target).  Same steps as
tools/step_profile.py.  usage: python tools/launch_census.py [--concurrent]"""
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "aes-implementation-fhe_amd")]

from aes_keyschedule import expand_aes128_key, load_all_coeffs  # noqa: E402
from engine_context import EngineContext  # noqa: E402
from mi355x_ckks import launch_count  # noqa: E402
from pipeline import AESPipeline  # noqa: E402
from utils import NEED_SR_MIX, SHIFTROWS_DEPTH, bootstrap1  # noqa: E402


def main():
    serial = "--concurrent" not in sys.argv
    reps = 3
    ctx = EngineContext(signature=1, max_level=17, concurrent=not serial)
    E = ctx.engine
    pipe = AESPipeline(ctx, load_all_coeffs(), use_hard_renorm_between_steps=True)
    np.random.seed(7)
    rks = expand_aes128_key(np.random.randint(0, 256, 16, dtype=np.uint8))
    st = np.random.randint(0, 256, 16, dtype=np.uint8)
    rk = pipe._prepare_round_keys(rks)
    ct0 = pipe._ark_renorm(pipe.encoder.encode(st), rk[0], level=pipe.need_sub)
    pipe.encrypt_round(ct0, rk[1], r=1)  # warm caches
    pipe._packed_round_key(2)
    pipe.encrypt(st, rks)
    E.sync()
    res = {}

    def timed(name, fn, *a):
        E.sync()
        n0, t = launch_count(), time.perf_counter()
        out = fn(*a)
        E.sync()
        r = res.setdefault(name, {"ms": 0.0, "launches": 0})
        r["ms"] += (time.perf_counter() - t) * 1e3
        r["launches"] += launch_count() - n0
        return out

    packed = pipe.packed_xor
    for _ in range(reps):
        lv = pipe.mix.packed_input_need() + SHIFTROWS_DEPTH if packed else NEED_SR_MIX  # the pipeline's own level

        perm = pipe._sr_perm(ct0, None) if packed else None  # the pipeline folds ShiftRows into this renorm

        def sub_step():
            if perm is not None:
                out = pipe.encoder.renorm_perm(*pipe._sub_apply(ct0, defer_conj=True), perm, level=lv - SHIFTROWS_DEPTH)
            else:
                out = pipe._sub_renorm(ct0, level=lv)
            E.settle(*out)  # the step's deferred products executed inside its own timing
            return out
        c = timed("sub_bytes+renorm" + ("+shift_rows(folded)" if perm is not None else ""), sub_step)
        if perm is None:
            c = timed("shift_rows", pipe.shift_rows, *c)
        mix = pipe.mix.mix_packed if packed else pipe.mix
        acc = timed("mix_columns(no final bootstrap)", lambda: mix(*c, do_final_bootstrap=False))
        timed("final_bootstrap", lambda: bootstrap1(ctx, acc, 2 * pipe.layout.period) if packed else None)
        c2 = timed("mix_columns(total)", lambda: mix(*c))
        if packed:
            timed("add_round_key+renorm", lambda: pipe.encoder.renorm_unpack(pipe._ark_packed(c2, 2), level=pipe.need_sub))
        timed("encrypt(10 rounds)", lambda: pipe.encrypt(st, rks))
    out = {k: {"ms": round(v["ms"] / reps, 3), "launches": v["launches"] / reps} for k, v in res.items()}
    steps = ("sub_bytes+renorm", "sub_bytes+renorm+shift_rows(folded)", "shift_rows", "mix_columns(total)", "add_round_key+renorm")
    out["round(sum of steps)"] = {"ms": round(sum(out[s]["ms"] for s in steps if s in out), 3),
                                  "launches": sum(out[s]["launches"] for s in steps if s in out)}
    print(json.dumps({"serial": serial, "packed_xor": packed, "reps": reps, "steps": out}, indent=1))


if __name__ == "__main__" and "--by-op" not in sys.argv:
    main()


def by_op():
    """launches per Engine method (top-level calls only) over one middle round (--by-op)"""
    import functools
    import mi355x_ckks
    from collections import defaultdict
    stats = defaultdict(lambda: [0, 0])
    depth = [0]

    def wrap(name, f):
        @functools.wraps(f)
        def g(*a, **k):
            if depth[0]:
                return f(*a, **k)
            depth[0] += 1
            n0 = launch_count()
            try:
                return f(*a, **k)
            finally:
                depth[0] -= 1
                s = stats[name]
                s[0] += 1
                s[1] += launch_count() - n0
        return g

    for name in dir(mi355x_ckks.Engine):
        f = getattr(mi355x_ckks.Engine, name)
        if callable(f) and not name.startswith("_") and name not in ("sync", "parallel", "can_fork", "settle", "nl", "galois_rotate"):
            setattr(mi355x_ckks.Engine, name, wrap(name, f))
    ctx = EngineContext(signature=1, max_level=17, concurrent=False)
    pipe = AESPipeline(ctx, load_all_coeffs(), use_hard_renorm_between_steps=True)
    np.random.seed(7)
    rks = expand_aes128_key(np.random.randint(0, 256, 16, dtype=np.uint8))
    st = np.random.randint(0, 256, 16, dtype=np.uint8)
    rk = pipe._prepare_round_keys(rks)
    ct0 = pipe._ark_renorm(pipe.encoder.encode(st), rk[0], level=pipe.need_sub)
    pipe.encrypt_round(ct0, rk[1], r=1)
    pipe._packed_round_key(2)
    ctx.engine.sync()
    stats.clear()
    n0 = launch_count()
    pipe.encrypt_round(ct0, rk[2], r=2)
    ctx.engine.sync()
    total = launch_count() - n0
    rows = sorted(stats.items(), key=lambda kv: -kv[1][1])
    print(json.dumps({"round_launches": total, "by_op": {k: {"calls": v[0], "launches": v[1], "per_call": round(v[1] / max(v[0], 1), 1)}
                                                          for k, v in rows}}, indent=1))


if __name__ == "__main__" and "--by-op" in sys.argv:
    by_op()
    sys.exit(0)
