"""Where the bootstrap's noise floor comes from: two independent encryptions of the SAME slots
are bootstrapped up to a stage (aesfhe_debug_boot_stage) and decrypted; the rms of their
difference / sqrt(2) is the noise one bootstrap has added by that stage, free of the integer
overflows I (removed by EvalMod) that make the raw stages incomparable.
Stages: 1 scaled level-0 input, 8 EvalMod(real), 10 recombined (before SlotToCoeff), 11 output."""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "aes-implementation-fhe_amd")]


def main():
    from engine_context import EngineContext
    ctx = EngineContext(signature=1, max_level=17, seed=0xB007)
    E = ctx.engine
    S = E.slot_count
    rng = np.random.default_rng(3)
    out = {"boot_info": E.boot_info()}
    for name, z in (("zeros", np.zeros(S, np.complex128)), ("random", np.exp(2j * np.pi * rng.random(S)) * rng.random(S))):
        a, b = ctx.encrypt(z), ctx.encrypt(z)
        res = {"fresh_noise_rms": float(np.sqrt(np.mean(np.abs(ctx.decrypt(a) - ctx.decrypt(b)) ** 2) / 2))}
        for s in (1, 8, 10, 11):
            oa = E.debug_boot_stage(a, s) if s < 11 else E.bootstrap(a)
            ob = E.debug_boot_stage(b, s) if s < 11 else E.bootstrap(b)
            da, db = ctx.decrypt(oa), ctx.decrypt(ob)
            res[f"stage{s}"] = {"level": oa.level, "noise_rms": float(np.sqrt(np.mean(np.abs(da - db) ** 2) / 2)),
                                "value_rms": float(np.sqrt(np.mean(np.abs(da) ** 2)))}
        out[name] = res
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
