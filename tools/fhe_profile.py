"""Where a true-FHE C2 encrypt goes (AESPipeline(true_fhe=True), bench.py's true-FHE leg): every
bootstrap, snap, (Inv)SubBytes, GF multiplier, XOR4 and ShiftRows call synchronised and timed on
its own (the outermost timed call only), with the engine's launch count per class.  Sub-step
syncs serialise the branch streams, so the sum is an upper bound of the unsynchronised encrypt,
which is timed separately first.
usage: python3 tools/fhe_profile.py [reps] [fresh_level] [dnum]   (GPU; env flags as the bench)"""
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "aes-implementation-fhe_amd")]

import zeta16_noise_reducer as zn  # noqa: E402
from aes_keyschedule import expand_aes128_key, load_all_coeffs  # noqa: E402
from engine_context import EngineContext  # noqa: E402
from mi355x_ckks import launch_count  # noqa: E402
from oracle import aes_plain  # noqa: E402
from pipeline import AESPipeline  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    fresh = int(sys.argv[2]) if len(sys.argv) > 2 else None
    dnum = int(sys.argv[3]) if len(sys.argv) > 3 else None
    kw = {"boot_fresh_level": fresh} if fresh else {}
    if dnum:
        kw["dnum"] = dnum
    ctx = EngineContext(signature=1, seed=0xF4E, **kw)
    E = ctx.engine
    pipe = AESPipeline(ctx, load_all_coeffs(), use_hard_renorm_between_steps=False, true_fhe=True)
    rng = np.random.default_rng(11)
    rks = expand_aes128_key(rng.integers(0, 256, 16).astype(np.uint8))
    pts = rng.integers(0, 256, (reps + 1, 16)).astype(np.uint8)

    def run(pt):
        ct = pipe.encrypt(pt, rks)
        E.settle(*ct)
        return ct

    run(pts[0])  # warm: plans, keys, plaintext caches
    E.sync()
    t0, n0, b0 = time.perf_counter(), launch_count(), ctx.bootstrap_stats()["count"]
    cts = [run(pt) for pt in pts[1:]]
    E.sync()
    whole = (time.perf_counter() - t0) * 1e3 / reps
    launches = (launch_count() - n0) / reps
    boots = (ctx.bootstrap_stats()["count"] - b0) / reps
    ok = all(np.array_equal(pipe.encoder.decode(*ct), aes_plain.ref_encrypt(pt, rks)) for ct, pt in zip(cts, pts[1:]))
    del cts
    from bench import measure_precision
    prec = measure_precision(pipe, ctx, rks, pts[0], "one state, true-FHE")

    times, depth = {}, [0]

    def timed(name, f):
        def w(*a, **k):
            if depth[0]:
                return f(*a, **k)
            depth[0] += 1
            try:
                E.sync()
                l0, t = launch_count(), time.perf_counter()
                r = f(*a, **k)
                flat, todo = [], [r]
                while todo:
                    v = todo.pop()
                    if isinstance(v, (tuple, list)):
                        todo.extend(v)
                    elif v is not None:
                        flat.append(v)
                E.settle(*flat)
                E.sync()
                s = times.setdefault(name, [0.0, 0, 0])
                s[0] += (time.perf_counter() - t) * 1e3
                s[1] += launch_count() - l0
                s[2] += 1
                return r
            finally:
                depth[0] -= 1
        return w

    ctx.bootstrap_pair_scaled = timed("bootstrap", ctx.bootstrap_pair_scaled)
    zn.stacked_pair = timed("snap", zn.stacked_pair)
    for name, obj, meth in (("subbytes", pipe.sub, "apply"), ("gf_mult", pipe.mix, "gf_mult_2"),
                            ("gf_mult", pipe.mix, "gf_mult_3"), ("xor4", pipe.xor4, "apply"),
                            ("shiftrows", pipe.shift, "apply")):
        setattr(obj, meth, timed(name, getattr(obj, meth)))
    E.sync()
    t0 = time.perf_counter()
    for pt in pts[1:]:
        run(pt)
    E.sync()
    synced = (time.perf_counter() - t0) * 1e3 / reps
    out = {"fresh_level": E.fresh_level, "dnum": E.dnum, "ms_per_encrypt": round(whole, 2),
           "rounds_per_s": round(10e3 / whole, 2), "launches_per_encrypt": launches,
           "bootstraps_per_encrypt": boots, "verified": ok,
           "precision": {k: prec[k] for k in ("max_slot_angle_error_rad", "worst_stage", "margin_factor")}, "ms_per_encrypt_synced": round(synced, 2),
           "steps": {k: {"ms_per_encrypt": round(v[0] / reps, 2), "calls": v[2] / reps,
                         "ms_per_call": round(v[0] / v[2], 3), "launches_per_call": round(v[1] / v[2], 1)}
                     for k, v in sorted(times.items(), key=lambda kv: -kv[1][0])}}
    out["steps"]["other"] = {"ms_per_encrypt": round(synced - sum(v[0] for v in times.values()) / reps, 2)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
