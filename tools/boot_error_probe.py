"""Bootstrap slot-error anatomy (N = 2^16, bootstrappable set): for several inputs -- zeros,
random |z| <= 1, the constant 1, a Zeta16 state encoding -- the max / rms slot error of
bootstrap(encrypt(z)) and the least-squares complex gain g (out ~ g z): a gain error shows as
|g - 1|, noise as the rms of out - g z.  Usage: python3 tools/boot_error_probe.py [LIB.so]"""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "aes-implementation-fhe_amd")]

import mi355x_ckks  # noqa: E402


def main():
    if len(sys.argv) > 1:
        mi355x_ckks.load_library(Path(sys.argv[1]))
    from engine_context import EngineContext
    ctx = EngineContext(signature=1, max_level=17, seed=0xB007)
    E = ctx.engine
    S = E.slot_count
    rng = np.random.default_rng(9)
    st = np.ones(S, np.complex128)
    st[:: S // 16][:16] = np.exp(-2j * np.pi * rng.integers(0, 16, 16) / 16)
    inputs = {"zeros": np.zeros(S, np.complex128),
              "random": np.exp(2j * np.pi * rng.random(S)) * rng.random(S),
              "unit_random_phase": np.exp(2j * np.pi * rng.random(S)),
              "ones": np.ones(S, np.complex128),
              "zeta16_state": st}
    out = {"boot_info": E.boot_info()}
    for name, z in inputs.items():
        o = ctx.decrypt(ctx.bootstrap(ctx.encrypt(z)))
        d = o - z
        g = complex(np.vdot(z, o) / np.vdot(z, z)) if np.any(z) else 1.0
        r = o - g * z
        out[name] = {"max_err": float(np.abs(d).max()), "rms_err": float(np.sqrt(np.mean(np.abs(d) ** 2))),
                     "gain_re": g.real, "gain_im": g.imag, "rms_after_gain": float(np.sqrt(np.mean(np.abs(r) ** 2))),
                     "max_after_gain": float(np.abs(r).max())}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
