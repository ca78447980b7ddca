"""Level consumption and cost of the AES LUT steps vs the level they run at: output levels
of XOR4 / GF-multiplier / SubBytes from a fresh input, and the wall time of an XOR4 pair
and a GF pair when the inputs are first dropped to a lower level (decoded bytes checked)."""
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "aes-implementation-fhe_amd")]

from aes_keyschedule import load_all_coeffs  # noqa: E402
from engine_context import EngineContext  # noqa: E402
from mixcol_final import MixColFinal  # noqa: E402
from oracle import aes_plain as A  # noqa: E402
from state_encoder import StateEncoder  # noqa: E402
from sub_bytes_lut import SubBytesLUT  # noqa: E402
from utils import pair  # noqa: E402
from xor4_lut import XOR4LUT  # noqa: E402


def main():
    ctx = EngineContext(signature=1, max_level=17)
    E = ctx.engine
    co = load_all_coeffs()
    enc = StateEncoder(ctx)
    xor4 = XOR4LUT(ctx, co["xor4"])
    mix = MixColFinal(ctx, xor4)
    sb = SubBytesLUT(ctx, co["sub_hi"], co["sub_lo"])
    rng = np.random.default_rng(0)
    s1, s2 = rng.integers(0, 256, 16, dtype=np.uint8), rng.integers(0, 256, 16, dtype=np.uint8)
    a, b = enc.encode(s1), enc.encode(s2)
    x = xor4.apply(a[0], b[0])
    g = mix.gf_mult_2(*a)
    s = sb.apply(*a)
    print(f"fresh {a[0].level}: xor4 -> {x.level}, gf2 -> {g[0].level}, subbytes -> {s[0].level}", flush=True)

    def timed(fn, reps=5):
        fn()
        E.sync()
        t = time.perf_counter()
        for _ in range(reps):
            out = fn()
        E.sync()
        return (time.perf_counter() - t) / reps * 1e3, out

    for lv in (17, 12, 9, 7, 5):
        da = (E.level_down(a[0], lv), E.level_down(a[1], lv)) if lv < a[0].level else a
        db = (E.level_down(b[0], lv), E.level_down(b[1], lv)) if lv < b[0].level else b
        E.sync()
        try:
            ms, out = timed(lambda: pair(ctx, lambda: xor4.apply(da[0], db[0]), lambda: xor4.apply(da[1], db[1])))
            ok = np.array_equal(enc.decode(*out), s1 ^ s2)
            ms2, out2 = timed(lambda: mix.gf_mult_2(*da))
            ok2 = np.array_equal(enc.decode(*out2), A.GF_MUL[2][s1])
            print(f"inputs at {lv}: xor4 pair {ms:.2f} ms (out {out[0].level}, ok {ok}); gf2 pair {ms2:.2f} ms "
                  f"(out {out2[0].level}, ok {ok2})", flush=True)
        except RuntimeError as e:
            print(f"inputs at {lv}: {e}", flush=True)


if __name__ == "__main__":
    main()
