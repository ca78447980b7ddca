"""GPU timeline of encrypt rounds (C2 bench workload, both branch streams).

run:      python tools/round_timeline.py run [ROUNDS] [--concurrent]
          one warm round, a 100 ms host pause (a marker gap in the trace), then ROUNDS rounds
analyse:  python tools/round_timeline.py analyse OUT.json DIR
          reads DIR's rocprofv3 --kernel-trace CSV, keeps the kernels after the last gap
          > 50 ms, and reports: span, busy time (union of kernel intervals), summed kernel
          time (sum / busy = mean concurrency of the two branch streams), idle gaps by size,
          and per-kernel-family time; deletes the CSV afterwards.
"""
import csv
import json
import re
import sys
import time
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "aes-implementation-fhe_amd")]


def run(rounds):
    import numpy as np
    from aes_keyschedule import expand_aes128_key, load_all_coeffs
    from engine_context import EngineContext
    from pipeline import AESPipeline
    ctx = EngineContext(signature=1, max_level=17, seed=0x5EED, concurrent="--concurrent" in sys.argv)
    E = ctx.engine
    pipe = AESPipeline(ctx, load_all_coeffs(), use_hard_renorm_between_steps=True)
    np.random.seed(7)
    rks = expand_aes128_key(np.random.randint(0, 256, 16, dtype=np.uint8))
    st = np.random.randint(0, 256, 16, dtype=np.uint8)
    rk = pipe._prepare_round_keys(rks)
    ct = pipe._ark_renorm(pipe.encoder.encode(st), rk[0], level=pipe.need_sub)
    c = pipe.encrypt_round(ct, rk[1], r=1)  # warm: keys, plaintext encodings, bootstrap plan
    if pipe.packed_xor:
        for r in range(2, 10):
            pipe._packed_round_key(r)  # encrypted once per key schedule (the first encrypt's cost)
    E.sync()
    time.sleep(0.1)
    t = time.perf_counter()
    for r in range(rounds):
        c = pipe.encrypt_round(c, rk[2 + r % 8], r=2 + r % 8)
    host = (time.perf_counter() - t) * 1e3 / rounds  # enqueue time: the host returns before the GPU ends
    E.sync()
    ms = (time.perf_counter() - t) * 1e3 / rounds
    print(json.dumps({"rounds": rounds, "wall_ms_per_round": ms, "host_enqueue_ms_per_round": host}), flush=True)


def family(name):
    name = name.replace("(anonymous namespace)::", "")
    m = re.match(r"(?:void )?(k_[a-z0-9_]+)", name)
    return m.group(1) if m else name[:40]


def analyse(out, d):
    rows = []
    for f in Path(d).rglob("*kernel_trace.csv"):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                rows.append((int(row["Start_Timestamp"]), int(row["End_Timestamp"]), family(row["Kernel_Name"]),
                             row.get("Queue_Id", "")))
        f.unlink()
    rows.sort()
    # the timed rounds: after the last gap > 50 ms
    start = 0
    end_max = rows[0][1]
    for i in range(1, len(rows)):
        if rows[i][0] - end_max > 50_000_000:
            start = i
        end_max = max(end_max, rows[i][1])
    sel = rows[start:]
    busy, total = 0, 0
    gaps = []
    cs, ce = sel[0][0], sel[0][1]
    fam = defaultdict(lambda: [0, 0])
    queues = defaultdict(int)
    for s, e, n, q in sel:
        total += e - s
        fam[n][0] += 1
        fam[n][1] += e - s
        queues[q] += e - s
    last = sel[0][2]  # the kernel whose end closes the busy interval
    by_pair = defaultdict(lambda: [0, 0])
    for s, e, n, _ in sel[1:]:
        if s > ce:
            busy += ce - cs
            gaps.append(s - ce)
            if s - ce >= 20_000:  # idle >= 20 us: which kernels it sits between
                k = f"{last} -> {n}"
                by_pair[k][0] += 1
                by_pair[k][1] += s - ce
            cs, ce = s, e
            last = n
        elif e >= ce:
            ce, last = e, n
    busy += ce - cs
    span = max(e for _, e, _, _ in sel) - sel[0][0]
    hist = {}
    for lo, hi in [(0, 1e3), (1e3, 5e3), (5e3, 2e4), (2e4, 1e5), (1e5, 1e6), (1e6, 1e12)]:
        g = [x for x in gaps if lo <= x < hi]
        hist[f"{lo/1e3:g}-{hi/1e3:g}us"] = {"count": len(g), "ms": round(sum(g) / 1e6, 3)}
    res = {
        "launches": len(sel), "span_ms": span / 1e6, "busy_ms": busy / 1e6, "idle_ms": (span - busy) / 1e6,
        "kernel_sum_ms": total / 1e6, "mean_concurrency_when_busy": total / busy,
        "gaps": hist,
        "per_queue_ms": {k: v / 1e6 for k, v in queues.items()},
        "gaps_over_20us_by_neighbours": {k: {"count": v[0], "ms": round(v[1] / 1e6, 3)}
                                         for k, v in sorted(by_pair.items(), key=lambda kv: -kv[1][1])[:25]},
        "families": {k: {"calls": v[0], "ms": round(v[1] / 1e6, 3), "avg_us": round(v[1] / v[0] / 1e3, 2)}
                     for k, v in sorted(fam.items(), key=lambda kv: -kv[1][1])},
    }
    Path(out).write_text(json.dumps(res, indent=1))
    print(json.dumps({k: v for k, v in res.items() if k != "families"}))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(int(sys.argv[2]) if len(sys.argv) > 2 and sys.argv[2].isdigit() else 3)
    else:
        analyse(sys.argv[2], sys.argv[3])
