"""Per-primitive timings on the bench parameter set (bootstrappable N = 2^16):
NTT / inverse NTT vs row count, key switch / rescale / mul+relin+rescale vs level."""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "aes-implementation-fhe_amd")]

from engine_context import EngineContext  # noqa: E402


def main():
    E = EngineContext(signature=1, max_level=17).engine
    res = {}
    row_bytes = 4 * E.n
    for op in ("ntt", "intt"):
        for rows in (1, 2, 8, 20, 40, 80, 160):
            us = E.bench_op(op, rows, 200)
            res[f"{op}_{rows}"] = {"us": us, "GBps_2pass": 4 * rows * row_bytes / us / 1e3}
    for op in ("keyswitch", "rescale", "mul_relin_rescale"):
        for lv in sorted({2, 10, 17, 25, E.L}):
            res[f"{op}_L{lv}"] = {"us": E.bench_op(op, lv, 50), "limbs": E.nl(lv)}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
