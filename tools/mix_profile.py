"""Sub-step times of MixColumns' packed rot form (mixcol_final.mix_packed, AESFHE_MC_FORM=rot, with
the GF pair at the XOR4 level: AESFHE_MC_GF_LOW) on one C2 state, each step synchronised and its
deferred products settled inside it (launch counts from the engine): where a round's MixColumns
without its bootstrap goes.  usage: python3 tools/mix_profile.py [reps] (GPU)"""
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
from utils import LUT2_DEPTH, NEED_BOOTSTRAP, NEED_XOR, RENORM_FLOOR, SHIFTROWS_DEPTH, rot_pair  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    ctx = EngineContext(signature=1, max_level=17)
    E = ctx.engine
    pipe = AESPipeline(ctx, load_all_coeffs(), use_hard_renorm_between_steps=True)
    mix, enc = pipe.mix, pipe.encoder
    rng = np.random.default_rng(3)
    st = rng.integers(0, 256, 16, dtype=np.uint8)
    x = enc.renorm(*enc.encode(st), level=mix.packed_input_need() + SHIFTROWS_DEPTH)
    x = pipe.shift_rows(*x)
    fl = RENORM_FLOOR
    gl = fl + LUT2_DEPTH + enc.PACK_DEPTH
    times = {}

    def step(name, f):
        E.sync()
        l0 = launch_count()
        t0 = time.perf_counter()
        r = f()
        flat, todo = [], [r]
        while todo:
            v = todo.pop()
            if isinstance(v, (tuple, list)):
                todo.extend(v)
            else:
                flat.append(v)
        E.settle(*flat)
        E.sync()
        dt = (time.perf_counter() - t0) * 1e3
        a = times.setdefault(name, [0.0, 0, 0])
        a[0] += dt
        a[1] += launch_count() - l0
        a[2] += 1
        return r

    for _ in range(reps + 1):
        if _ == 1:
            times.clear()
        ct_hi, ct_lo = x
        s1 = -4 * mix.stride
        (rh1,), (rl1,) = step("rot r1 (pair)", lambda: rot_pair(ctx, ct_hi, ct_lo, [s1]))
        p1 = step("pack r1", lambda: enc.pack(rh1, rl1))
        p0 = step("pack x", lambda: enc.pack(ct_hi, ct_lo))
        t = step("XOR4(x, r1)", lambda: mix._xor_ct(p0, p1, fl))
        u = step("renorm_unpack u", lambda: enc.renorm_unpack(t, level=gl))
        g = step("gf_mult_2(u) pair", lambda: mix.gf_mult_2(*u, out_level=fl + enc.PACK_DEPTH))
        two = step("pack + renorm 2u", lambda: enc.renorm_packed(enc.pack(*g), level=NEED_XOR))
        (vh,), (vl,) = step("rot R^2 u (pair)", lambda: rot_pair(ctx, u[0], u[1], [2 * s1]))
        pv = step("pack R^2 u", lambda: enc.pack(vh, vl))
        w0 = step("XOR4(R^2 u, r1)", lambda: mix._xor_ct(pv, p1, fl))
        w = step("renorm w", lambda: enc.renorm_packed(w0, level=NEED_XOR))
        acc = step("XOR4(2u, w)", lambda: mix._xor_ct(two, w, fl))
        step("renorm to level 0", lambda: enc.renorm_packed(acc, level=NEED_BOOTSTRAP))
    out = {k: {"ms": round(v[0] / v[2], 3), "launches": v[1] / v[2]} for k, v in times.items()}
    out["total"] = {"ms": round(sum(v["ms"] for v in out.values()), 3), "launches": sum(v["launches"] for v in out.values())}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
