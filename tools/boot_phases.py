"""Phase breakdown of the sparse-slot bootstrap (with per-class HBM rooflines per phase: algorithmic
bytes over the in-kernel span, and over span + boundary gap) (C2's MixColumns final bootstrap: one packed
ciphertext, period P = 32): wall time (synchronised) and kernel launches of the bootstrap run up
to each debug stage (aesfhe_debug_boot_stage_sparse), and the per-phase differences.
usage: python tools/boot_phases.py [P] [FRESH_LEVEL DNUM] > out.json   (default: the engine's set, 17 / 5;
bench.py's C2 set is 9 / 4)"""
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "aes-implementation-fhe_amd")]

from engine_context import EngineContext  # noqa: E402
from mi355x_ckks import KERNEL_IDS, launch_count  # noqa: E402

# stop_after codes of bootstrap_l0 (engine.hip) in execution order, packed sparse form
STAGES = [(1, "level-0 scaling"), (2, "dense->sparse key switch"), (3, "ModRaise"), (12, "sparse->dense key switch"),
          (4, "trace to the subring"), (5, "CoeffToSlot"), (9, "conjugate fold"), (10, "EvalMod"), (99, "SlotToCoeff + level drop")]


def main():
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    reps = 5
    fresh = int(sys.argv[2]) if len(sys.argv) > 2 else None
    dnum = int(sys.argv[3]) if len(sys.argv) > 3 else None
    ctx = EngineContext(signature=1, max_level=17, boot_fresh_level=fresh, dnum=dnum)
    E = ctx.engine
    z = np.exp(2j * np.pi * np.random.default_rng(0).random(P))
    ct = E.intt(ctx.encrypt(np.tile(z, E.slot_count // P)))
    cum, kcum, rcum = {}, {}, {}
    for code, name in STAGES:
        run = (lambda: E.bootstrap_sparse(ct, P)) if code == 99 else (lambda: E.debug_boot_stage_sparse(ct, code, P))
        run()
        E.sync()
        t, n0 = time.perf_counter(), launch_count()
        for _ in range(reps):
            run()
        E.sync()
        cum[name] = ((time.perf_counter() - t) * 1e3 / reps, (launch_count() - n0) / reps)
        # launches per kernel class (engine profiler, every launch timed: a separate pass)
        E.profile(list(KERNEL_IDS), every=1)
        E.kernel_stats(reset=True)
        run()
        E.sync()
        gaps = E.kernel_gaps()  # read before kernel_stats(reset) clears them
        ks = E.kernel_stats(reset=True)
        kcum[name] = {k: v["launches"] for k, v in ks.items()}
        # per class: span ms (in-kernel clock, or dispatch events for element-wise kernels), the
        # boundary gaps accounted to the class, algorithmic bytes
        rcum[name] = {k: (v["ms"], gaps.get(k, (0, 0.0))[1], v["bytes"]) for k, v in ks.items()}
        E.profile(())
    out, prev, kprev, rprev = {}, (0.0, 0.0), {}, {}
    for _, name in STAGES:
        ms, ln = cum[name]
        kc = {k: v - kprev.get(k, 0) for k, v in kcum[name].items() if v - kprev.get(k, 0)}
        roof = {}
        for k, (sp, gp, by) in rcum[name].items():
            p0 = rprev.get(k, (0.0, 0.0, 0.0))
            dsp, dgp, dby = sp - p0[0], gp - p0[1], by - p0[2]
            if dsp > 0 and dby > 0 and kc.get(k):
                # a phase's class figures are differences of two separately profiled runs: a difference below
                # their run-to-run spread (a negative gap, or more bytes than 8 TB/s could move in the span) is
                # reported without fractions instead of as a frac > 1
                if dgp < 0 or dby / (dsp * 1e-3) > 8e12:
                    roof[k] = {"span_ms": round(dsp, 4), "GB": round(dby / 1e9, 4), "launches": kc[k],
                               "frac": None, "note": "below the resolution of the two runs' difference"}
                    continue
                roof[k] = {"span_ms": round(dsp, 4), "gap_ms": round(dgp, 4), "GB": round(dby / 1e9, 4),
                           "frac_span": round(dby / (dsp * 1e-3) / 8e12, 3),
                           "frac": round(dby / ((dsp + dgp) * 1e-3) / 8e12, 3)}
        out[name] = {"ms": round(ms - prev[0], 3), "launches": ln - prev[1], "cumulative_ms": round(ms, 3), "by_class": kc,
                     "roofline_by_class": roof}
        prev, kprev, rprev = (ms, ln), kcum[name], rcum[name]
    print(json.dumps({"period": P, "reps": reps, "fresh_level": ctx.engine.fresh_level, "dnum": ctx.engine.dnum, "phases": out}, indent=1))


if __name__ == "__main__":
    main()
