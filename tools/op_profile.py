"""Synchronised wall time of the AES steps' building blocks at the levels one C2 round uses
(mean of 10 repetitions): renorm pair, XOR4 pair at the floor, GF multiplier pair, SubBytes
(without renorm), the six MixColumns rotations, bootstrap pair -- where a round's time goes
below the step level of tools/step_profile.py."""
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "aes-implementation-fhe_amd")]

from aes_keyschedule import load_all_coeffs  # noqa: E402
from engine_context import EngineContext  # noqa: E402
from mixcol_final import MixColFinal  # noqa: E402
from state_encoder import StateEncoder  # noqa: E402
from sub_bytes_lut import SubBytesLUT  # noqa: E402
from utils import LUT2_DEPTH, NEED_BOOTSTRAP, NEED_GF, NEED_SUBBYTES, NEED_XOR, RENORM_FLOOR, bootstrap2, pair  # noqa: E402
from xor4_lut import XOR4LUT  # noqa: E402


def main(reps=10):
    ctx = EngineContext(signature=1, max_level=17, concurrent="--concurrent" in sys.argv)
    E = ctx.engine
    co = load_all_coeffs()
    enc = StateEncoder(ctx)
    xor4 = XOR4LUT(ctx, co["xor4"])
    mix = MixColFinal(ctx, xor4)
    sb = SubBytesLUT(ctx, co["sub_hi"], co["sub_lo"])
    st = np.arange(16, dtype=np.uint8)
    a = enc.encode(st)
    b = enc.encode(st[::-1].copy())
    ax, bx = enc.renorm(*a, level=NEED_XOR), enc.renorm(*b, level=NEED_XOR)
    ag = enc.renorm(*a, level=NEED_GF)
    asb = enc.renorm(*a, level=NEED_SUBBYTES)
    res = {}

    def timed(name, fn):
        fn()
        E.sync()
        t = time.perf_counter()
        for _ in range(reps):
            out = fn()
        E.sync()
        res[name] = round((time.perf_counter() - t) * 1e3 / reps, 3)
        return out

    fl = RENORM_FLOOR
    x = timed("xor4_pair@floor", lambda: pair(ctx, lambda: xor4.apply(ax[0], bx[0], fl), lambda: xor4.apply(ax[1], bx[1], fl)))
    if hasattr(xor4, "apply_pair"):
        timed("xor4.apply_pair@floor", lambda: xor4.apply_pair(ax[0], bx[0], ax[1], bx[1], fl))
    timed("xor4_single@floor", lambda: xor4.apply(ax[0], bx[0], fl))
    timed("renorm_pair->NEED_XOR", lambda: enc.renorm(*x, level=NEED_XOR))
    timed("gf2_pair", lambda: mix.gf_mult_2(*ag, out_level=fl + LUT2_DEPTH))
    timed("subbytes(no renorm)", lambda: sb.apply(*asb, out_level=fl))
    timed("rotations_x6", lambda: pair(ctx, lambda: [mix._col_shift_rowmajor(ag[0], k) for k in (1, 2, 3)],
                                       lambda: [mix._col_shift_rowmajor(ag[1], k) for k in (1, 2, 3)]))
    z = enc.renorm(*x, level=NEED_BOOTSTRAP)
    timed("bootstrap_pair", lambda: bootstrap2(ctx, *z))
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
