"""Timeline summary of a rocprofv3 --kernel-trace CSV: GPU busy time (union of kernel
intervals), span, idle gaps by size, launches; then deletes the (large) CSV.
Usage: python tools/trace_gaps.py OUT.json DIR"""
import csv
import json
import sys
from pathlib import Path


def main():
    out, d = Path(sys.argv[1]), Path(sys.argv[2])
    iv = []
    for f in d.rglob("*kernel_trace.csv"):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                iv.append((int(row["Start_Timestamp"]), int(row["End_Timestamp"])))
        f.unlink()
    iv.sort()
    busy = 0
    gaps = []
    cur_s, cur_e = iv[0]
    for s, e in iv[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            gaps.append(s - cur_e)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    span = iv[-1][1] - iv[0][0]
    hist = {}
    for lo, hi in [(0, 1e3), (1e3, 5e3), (5e3, 2e4), (2e4, 1e5), (1e5, 1e6), (1e6, 1e12)]:
        sel = [g for g in gaps if lo <= g < hi]
        hist[f"{lo/1e3:g}-{hi/1e3:g}us"] = {"count": len(sel), "ms": sum(sel) / 1e6}
    res = {"launches": len(iv), "span_ms": span / 1e6, "busy_ms": busy / 1e6, "idle_ms": (span - busy) / 1e6, "gaps": hist}
    out.write_text(json.dumps(res, indent=1))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
