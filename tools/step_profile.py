"""Synchronised wall time of each AES step of one middle encrypt round (C2 parameters), the
steps as AESPipeline.encrypt_round runs them (level-targeted renorms); the
final bootstrap pair of MixColumns is the difference of MixColumns with and without it.
Arguments: pairs=P (stacked ciphertext pairs), states=S (slot-packed states per
pair), reps=R, fresh=L dnum=d (the context's set, default the bench's 9 / 4), --eager, --concurrent.  One more profiled round gives each step's time per kernel
class (engine profiler, every launch: in-kernel spans / dispatch-stamped events)."""
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
    serial = "--concurrent" not in sys.argv
    kv = dict(a.split("=", 1) for a in sys.argv[1:] if "=" in a)
    pairs, states, reps = int(kv.get("pairs", 1)), int(kv.get("states", 1)), int(kv.get("reps", 3))
    fresh, dnum = int(kv.get("fresh", 7)), int(kv.get("dnum", 4))  # the bench's C2 set (bench.py --fresh-level / --dnum)
    ctx = EngineContext(signature=1, boot_fresh_level=fresh, dnum=dnum, lazy=lazy, concurrent=not serial)
    E = ctx.engine
    pipe = AESPipeline(ctx, load_all_coeffs(), use_hard_renorm_between_steps=True, states=states, pairs=pairs)
    np.random.seed(7)
    rks = expand_aes128_key(np.random.randint(0, 256, 16, dtype=np.uint8))
    shape = (16,) if states == 1 else (states, 16)
    if pairs > 1:
        shape = (pairs,) + shape
    st = np.random.randint(0, 256, shape, dtype=np.uint8)
    rk = pipe._prepare_round_keys(rks)
    ct = pipe._ark_renorm(pipe.encoder.encode(st), rk[0], level=pipe.need_sub)
    pipe.encrypt_round(ct, rk[1], r=1)  # warm caches (plaintext encodings, keys, bootstrap plan)
    if pipe.packed_xor:
        pipe._packed_round_key(2)  # the packed round key the timed AddRoundKey uses
    E.sync()
    res = {}

    def timed(name, fn, *a):
        E.sync()
        t = time.perf_counter()
        out = fn(*a)
        E.sync()
        res[name] = res.get(name, 0.0) + (time.perf_counter() - t) * 1e3
        return out

    for _ in range(reps):
        round_steps(pipe, ct, rk, res, timed)
    res = {k: v / reps for k, v in res.items()}
    res["mc.final_bootstrap_pair(derived)"] = res["mix_columns(total)"] - res["mix_columns(no final bootstrap)"]
    # one more round with every launch profiled: kernel-class ms and launches per step
    from mi355x_ckks import KERNEL_IDS, launch_count
    classes = {}
    E.profile(KERNEL_IDS, every=1)
    E.kernel_stats(reset=True)

    def prof(name, fn, *a):
        E.sync()
        E.kernel_stats(reset=True)
        l0 = launch_count()
        out = fn(*a)
        E.sync()
        ks = E.kernel_stats(reset=True)
        classes[name] = {"launches": launch_count() - l0,
                         "ms": {k: round(v["ms"], 3) for k, v in sorted(ks.items(), key=lambda kv: -kv[1]["ms"])},
                         "launches_by_class": {k: v["launches"] for k, v in ks.items()}}
        return out

    round_steps(pipe, ct, rk, {}, prof)
    E.profile(())
    print(json.dumps({"lazy": lazy, "serial": serial, "packed_xor": pipe.packed_xor, "pairs": pairs, "states": states, "reps": reps,
                      "ms": {k: round(v, 2) for k, v in res.items()}, "kernel_classes_per_step": classes}, indent=1))


def round_steps(pipe, ct, rk, res, timed):
    from utils import NEED_SR_MIX, NEED_SUBBYTES
    t0 = time.perf_counter()
    packed = pipe.packed_xor  # MixColumns' XOR stage + AddRoundKey on packed states
    c = timed("sub_bytes+renorm", lambda: pipe._sub_renorm(ct, level=NEED_SR_MIX + (pipe.encoder.PACK_DEPTH if packed else 0)))
    c = timed("shift_rows", pipe.shift_rows, *c)
    mix = pipe.mix.mix_packed if packed else pipe.mix
    nb0 = res.get("mix_columns(no final bootstrap)", 0.0)
    c_nb = timed("mix_columns(no final bootstrap)", lambda: mix(*c, do_final_bootstrap=False))
    c = timed("mix_columns(total)", lambda: mix(*c))
    res["mix_columns(no final bootstrap)"] = res.get("mix_columns(no final bootstrap)", 0.0)
    if packed:
        c = timed("add_round_key+renorm", lambda: pipe.encoder.renorm_unpack(
            pipe._ark_packed(c, 2), level=pipe.need_sub))
    else:
        c = timed("add_round_key+renorm", lambda: pipe._ark_renorm(c, rk[2], level=pipe.need_sub))
    res["round_total"] = res.get("round_total", 0.0) + (time.perf_counter() - t0) * 1e3 - (res["mix_columns(no final bootstrap)"] - nb0)


if __name__ == "__main__":
    main()
