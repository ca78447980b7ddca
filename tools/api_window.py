"""Run the C2 encrypt twice (warm-up), sleep 0.5 s, run it once more (serial pipeline), for a
rocprofv3 --hip-trace run; `--summarize DIR` then reports the HIP API calls of the last
encrypt only (everything after the last idle gap > 0.3 s): counts, total and mean host time."""
import csv
import json
import sys
import time
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "aes-implementation-fhe_amd")]


def summarize(d):
    rows = []
    for f in Path(d).rglob("*hip_api_trace.csv"):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"]))
        f.unlink()
    rows.sort()
    cut = 0
    for i in range(1, len(rows)):
        if rows[i][0] - rows[i - 1][1] > 3e8:
            cut = i
    sel = rows[cut:]
    tot, cnt = defaultdict(float), defaultdict(int)
    for s, e, fn in sel:
        tot[fn] += e - s
        cnt[fn] += 1
    span = (sel[-1][1] - sel[0][0]) / 1e6
    out = {"span_ms": span, "api_ms_total": sum(tot.values()) / 1e6,
           "calls": {k: [cnt[k], round(tot[k] / 1e6, 2), round(tot[k] / cnt[k] / 1e3, 2)] for k in sorted(tot, key=lambda k: -tot[k])}}
    print(json.dumps(out, indent=1))


def main():
    import numpy as np
    from aes_keyschedule import expand_aes128_key, load_all_coeffs
    from engine_context import EngineContext
    from mixcol_final import MixColFinal
    from pipeline import AESPipeline
    from xor4_lut import XOR4LUT
    coeffs = load_all_coeffs()
    ctx = EngineContext(signature=1, max_level=17, thread_count=1, seed=0x5EED, lazy=True, concurrent=False)
    pipe = AESPipeline(ctx, coeffs, mixcolumns=MixColFinal(ctx, XOR4LUT(ctx, coeffs["xor4"])), use_hard_renorm_between_steps=True)
    rks = expand_aes128_key(np.arange(16, dtype=np.uint8))
    st = np.arange(16, dtype=np.uint8)
    for _ in range(2):
        pipe.encrypt(st, rks)
    ctx.engine.sync()
    hi, lo = pipe.encoder.encode(st)
    ctx.engine.sync()
    time.sleep(0.5)
    out = pipe.encrypt_ct(hi, lo, rks) if hasattr(pipe, "encrypt_ct") else pipe.encrypt(st, rks)
    ctx.engine.sync()


if __name__ == "__main__":
    summarize(sys.argv[2]) if len(sys.argv) > 2 and sys.argv[1] == "--summarize" else main()
