"""Kernel breakdown of one AES step op for rocprofv3 --kernel-trace: one XOR4 at the renorm
floor (the most frequent op) or, with OP=sub, one SubBytes (no renorm) from its input level.
run mode repeats it after a marker gap; analyse mode reports per kernel family calls / us per
op and the NTT launches' row counts (Grid_Size / 4096 at N = 2^16).
usage: xor4_trace.py run [ITERS] [OP] | xor4_trace.py analyse OUT.json DIR ITERS"""
import csv
import os
import json
import re
import sys
import time
from collections import Counter, defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "aes-implementation-fhe_amd")]


def run(iters, op="xor4"):
    import numpy as np
    from aes_keyschedule import load_all_coeffs
    from engine_context import EngineContext
    from state_encoder import StateEncoder
    from utils import NEED_XOR, RENORM_FLOOR
    from xor4_lut import XOR4LUT
    ctx = EngineContext(signature=1, max_level=17, concurrent=False)
    E = ctx.engine
    enc = StateEncoder(ctx, periodic=True)
    xor4 = XOR4LUT(ctx, load_all_coeffs()["xor4"])
    st = np.arange(16, dtype=np.uint8)
    a = enc.renorm(*enc.encode(st), level=NEED_XOR)
    b = enc.renorm(*enc.encode(st[::-1].copy()), level=NEED_XOR)
    fn = lambda: xor4.apply(a[0], b[0], RENORM_FLOOR)
    if op == "sub":
        from sub_bytes_lut import SubBytesLUT
        from utils import NEED_SUBBYTES
        sb = SubBytesLUT(ctx, *[load_all_coeffs()[k] for k in ("sub_hi", "sub_lo")])
        x = enc.renorm(*enc.encode(st), level=NEED_SUBBYTES + (os.environ.get('AESFHE_SB_BIV', '1') != '0'))
        fn = lambda: sb.apply(*x, out_level=RENORM_FLOOR)
    fn()
    E.sync()
    time.sleep(0.1)
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    E.sync()
    print(json.dumps({"op": op, "iters": iters, "ms_per_op": (time.perf_counter() - t) * 1e3 / iters}), flush=True)


def analyse(out, d, iters):
    rows = []
    for f in Path(d).rglob("*kernel_trace.csv"):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])))
        f.unlink()
    rows.sort()
    start, end_max = 0, rows[0][1]
    for i in range(1, len(rows)):
        if rows[i][0] - end_max > 50_000_000:
            start = i
        end_max = max(end_max, rows[i][1])
    sel = rows[start:]
    fam = defaultdict(lambda: [0, 0])
    ntt_rows = Counter()
    for s, e, n, g in sel:
        n2 = n.replace("(anonymous namespace)::", "")
        m = re.match(r"(?:void )?(k_[a-z0-9_]+)(<[^>]*>)?", n2)
        k = (m.group(1) + (m.group(2) or "")) if m else n2[:40]
        fam[k][0] += 1
        fam[k][1] += e - s
        if "k_ntt" in n2:
            ntt_rows[(m.group(1), g // 4096)] += 1
    span = sel[-1][1] - sel[0][0]
    res = {"iters": iters, "launches_per_op": len(sel) / iters, "span_us_per_op": span / 1e3 / iters,
           "kernel_us_per_op": sum(e - s for s, e, _, _ in sel) / 1e3 / iters,
           "families": {k: {"calls": v[0] / iters, "us": round(v[1] / 1e3 / iters, 2), "avg_us": round(v[1] / 1e3 / v[0], 2)}
                        for k, v in sorted(fam.items(), key=lambda kv: -kv[1][1])},
           "ntt_rows": {f"{k[0]}:{k[1]}": v / iters for k, v in sorted(ntt_rows.items())}}
    Path(out).write_text(json.dumps(res, indent=1))
    print(json.dumps({k: v for k, v in res.items() if k not in ("families", "ntt_rows")}))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(int(sys.argv[2]) if len(sys.argv) > 2 else 20, sys.argv[3] if len(sys.argv) > 3 else "xor4")
    else:
        analyse(sys.argv[2], sys.argv[3], int(sys.argv[4]))
