"""Precision of the stacked C3 path by members per packed bootstrap (aesfhe_set_stack_pack): one debug
encrypt of a stack of `pairs` one-state pairs on the bench's C2 set, bench.measure_precision over every
logged stage (every pair of the stack), and the bytes checked.  usage: python3 tools/pack_precision.py
[pairs] [packs...]  (GPU; default 16 pairs, packs 1 2 4 8 16)"""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "aes-implementation-fhe_amd")]

from aes_keyschedule import expand_aes128_key, load_all_coeffs  # noqa: E402
from bench import measure_precision  # noqa: E402
from engine_context import EngineContext  # noqa: E402
from oracle import aes_plain  # noqa: E402
from pipeline import AESPipeline  # noqa: E402


def main():
    pairs = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    packs = [int(a) for a in sys.argv[2:]] or [1, 2, 4, 8, 16]
    ctx = EngineContext(signature=1, boot_fresh_level=7, dnum=4, seed=0xC3C3)
    E = ctx.engine
    pipe = AESPipeline(ctx, load_all_coeffs(), use_hard_renorm_between_steps=True, pairs=pairs)
    rng = np.random.default_rng(33)
    rks = expand_aes128_key(rng.integers(0, 256, 16).astype(np.uint8))
    st = rng.integers(0, 256, (pairs, 16), dtype=np.uint8)
    out = {"pairs": pairs}
    for g in packs:
        E.set_stack_pack(g)
        got = pipe.encoder.decode(*pipe.encrypt(st, rks)).reshape(-1, 16)
        ok = all(np.array_equal(got[j], aes_plain.ref_encrypt(s, rks)) for j, s in enumerate(st))
        p = measure_precision(pipe, ctx, rks, st, f"one stack of {pairs} pairs, {g} members per bootstrap")
        out[f"pack{g}"] = {"verified": bool(ok), "max_slot_angle_error_rad": p["max_slot_angle_error_rad"],
                           "worst_stage": p["worst_stage"], "margin_factor": p["margin_factor"]}
        print(g, out[f"pack{g}"], flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
