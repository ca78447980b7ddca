"""Per-kernel launch counts and average durations inside the bench's timed region, from a
rocprofv3 --kernel-trace CSV of `AESFHE_MARK_TIMED=1 python3 bench.py ...` (bench.py idles 250 ms
on each side of the timed region): the launches between the last two idle gaps > 200 ms.  The
comparison for the bench line's live `roofline.avg_us` (which covers only the timed region),
beside the whole-process --stats summary.
usage: python tools/trace_window.py OUT.json DIR"""
import csv
import json
import re
import sys
from collections import defaultdict
from pathlib import Path


def family(name):
    name = name.replace("(anonymous namespace)::", "")
    m = re.match(r"(?:void )?(k_[a-z0-9_]+)", name)
    return m.group(1) if m else name[:40]


def main(out, d):
    rows = []
    for f in Path(d).rglob("*kernel_trace.csv"):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                rows.append((int(row["Start_Timestamp"]), int(row["End_Timestamp"]), family(row["Kernel_Name"])))
    rows.sort()
    gaps = []  # indices i where an idle gap > 200 ms precedes launch i
    end_max = rows[0][1]
    for i in range(1, len(rows)):
        if rows[i][0] - end_max > 200_000_000:
            gaps.append(i)
        end_max = max(end_max, rows[i][1])
    if len(gaps) < 2:
        raise SystemExit(f"expected two idle gaps around the timed region, found {len(gaps)}")
    sel = rows[gaps[-2]:gaps[-1]]
    fam = defaultdict(lambda: [0, 0])
    for s, e, n in sel:
        fam[n][0] += 1
        fam[n][1] += e - s
    res = {"window": "launches between the last two idle gaps > 200 ms (bench.py AESFHE_MARK_TIMED=1: the timed region)",
           "launches": len(sel), "span_ms": (max(e for _, e, _ in sel) - sel[0][0]) / 1e6,
           "kernels": {k: {"calls": v[0], "avg_us": round(v[1] / v[0] / 1e3, 3), "total_ms": round(v[1] / 1e6, 3)}
                       for k, v in sorted(fam.items(), key=lambda kv: -kv[1][1])}}
    Path(out).write_text(json.dumps(res, indent=1))
    print(json.dumps({k: res[k] for k in ("launches", "span_ms")}))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
