"""NTT / inverse NTT time per launch vs row count on the bench parameter set (bootstrappable
N = 2^16), for the block-size switch AESFHE_NTT_SMALL_ROWS (set in the environment)."""
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "aes-implementation-fhe_amd")]

from engine_context import EngineContext  # noqa: E402


def main():
    E = EngineContext(signature=1, max_level=17).engine
    top = 4 * (E.n_q + E.n_p)
    out = {"small_rows": os.environ.get("AESFHE_NTT_SMALL_ROWS", "default")}
    for op in ("ntt", "intt"):
        out[op] = {r: round(E.bench_op(op, r, 200), 2) for r in (4, 8, 12, 16, 20, 24, 30, 32, 36, 40, 44, 48, 56, 64, 72, 80, 96, 120, 160) if r <= top}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
