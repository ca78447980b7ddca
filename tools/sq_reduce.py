"""Reduce a rocprofv3 --pmc pass of SQ counters to per-kernel-family wave-time shares.

SQ_WAVE_CYCLES = SQ_WAIT_ANY (parked: s_waitcnt / barrier) + SQ_WAIT_INST_ANY (issue stall) +
SQ_ACTIVE_INST_ANY (issuing), all in quad-cycles (MI355X_MICROARCH.md, PMC section); the
family's share of each says whether its waves wait on memory or issue instructions, and
SQ_INSTS_VALU / SQ_INSTS_LDS per wave what they issue.  Usage:
  python tools/sq_reduce.py OUT.json DIR     (deletes the CSVs after reading)"""
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


def main():
    out, d = Path(sys.argv[1]), Path(sys.argv[2])
    acc = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for f in d.rglob("*counter_collection.csv"):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = family(row["Kernel_Name"])
                acc[k][row["Counter_Name"]] += float(row["Counter_Value"])
                disp[k].add(row.get("Dispatch_Id", ""))
        f.unlink()
    res = {}
    for k, c in acc.items():
        wc = c.get("SQ_WAVE_CYCLES", 0.0) or 1.0
        waves = c.get("SQ_WAVES", 0.0) or 1.0
        res[k] = {"dispatches": len(disp[k]),
                  "wait_any_share": c.get("SQ_WAIT_ANY", 0.0) / wc,
                  "wait_inst_any_share": c.get("SQ_WAIT_INST_ANY", 0.0) / wc,
                  "active_inst_any_share": c.get("SQ_ACTIVE_INST_ANY", 0.0) / wc,
                  "active_inst_valu_share": c.get("SQ_ACTIVE_INST_VALU", 0.0) / wc,
                  "wait_inst_lds_share": c.get("SQ_WAIT_INST_LDS", 0.0) / wc,
                  "valu_insts_per_wave": c.get("SQ_INSTS_VALU", 0.0) / waves,
                  "lds_insts_per_wave": c.get("SQ_INSTS_LDS", 0.0) / waves,
                  "wave_cycles_per_wave": 4.0 * wc / waves,
                  "wave_cycles_total": 4.0 * wc}
    res = dict(sorted(res.items(), key=lambda kv: -kv[1]["wave_cycles_total"]))
    out.write_text(json.dumps(res, indent=1))
    print(json.dumps({k: {a: round(b, 3) for a, b in v.items()} for k, v in list(res.items())[:12]}))


if __name__ == "__main__":
    main()
