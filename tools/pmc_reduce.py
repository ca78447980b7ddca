"""Reduce a rocprofv3 --pmc counter_collection.csv to per-kernel mean HBM bytes per launch.

gfx950 corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports half the bytes of
wide coalesced reads -> x2; WRITE_SIZE is exact.  Both counters are in KB.  Usage:
  python tools/pmc_reduce.py [--source=LABEL] [--alg=STATS.json] OUT.json DIR [DIR ...]   (one DIR per --pmc pass)
Deletes the (large) CSVs after reading so gpurun can copy the result back.  A DIR that is an earlier
OUT.json re-aggregates its per-kernel entries (after a change of the kernel -> class map below; with
--refetch also after a kernel joined FETCH_AS_IS: its FETCH bytes halved back)."""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

SCALE = {"FETCH_SIZE": 2 * 1024.0, "WRITE_SIZE": 1024.0}
# WRITE_SIZE from its raw TCC requests when the derived counter cannot be collected (on this image a
# WRITE_SIZE pass over the whole bench crawls): bytes = 64 x WRREQ_64B + 32 x (WRREQ - WRREQ_64B),
# rocprofv3's own derivation of WRITE_SIZE
RAW_WRITE = ("TCC_EA0_WRREQ_sum", "TCC_EA0_WRREQ_64B_sum")
# kernels whose bulk reads are 4 B per lane in 64-B segments (not 16-B-per-lane streaming):
# FETCH_SIZE counts those bytes as they are.  Calibrated with tools/ntt_pmc_calib.py (plain
# 160-row NTTs): pass 1 (16-B-per-lane-equivalent coalesced reads) FETCH x2 = 1.03 x its
# WRITE bytes, pass 2 (p[j + 16 k] dword reads) FETCH x2 = 2.36 x WRITE, i.e. FETCH x1 =
# 1.18 x WRITE = its data plus twiddle pairs.  The finish variant's cur / add reads are
# 16 B per lane, so its total is a lower bound.
# k_ntt2_fwd8 (round 6, 8 residues per thread) reads its rows the same way (p[t + 32 k]: 128 B per
# 32-lane half); its finish mode's cur / add reads are 16 B per lane (a lower bound again)
FETCH_AS_IS = ("ntt2_fwd", "ntt2_fwd8")


REFETCH = False


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "").split("(")[0]
    for pre in ("k_", "void k_"):
        if name.startswith(pre):
            return name[len(pre):]
    return name


def main():
    global REFETCH
    src = alg = None
    args = sys.argv[1:]
    while args and args[0].startswith("--"):
        if args[0].startswith("--source="):
            src = args[0].split("=", 1)[1]
        elif args[0] == "--refetch":
            REFETCH = True
        elif args[0].startswith("--alg="):  # the probe's own engine kernel_stats (algorithmic bytes)
            alg = json.loads(Path(args[0].split("=", 1)[1]).read_text())
        args = args[1:]
    out, dirs = Path(args[0]), args[1:]
    acc = defaultdict(lambda: defaultdict(float))
    cnt = defaultdict(lambda: defaultdict(int))
    for d in dirs:
        for f in ([] if d.endswith(".json") else Path(d).rglob("*counter_collection.csv")):
            with open(f) as fh:
                head = [next(fh, "") for _ in range(3)]
                out.with_suffix(".sample.txt").write_text("".join(head))
                fh.seek(0)
                for row in csv.DictReader(fh):
                    c = row["Counter_Name"]
                    k = short(row["Kernel_Name"])
                    sc = SCALE.get(c, 1.0)
                    if c == "FETCH_SIZE" and k.split("<")[0] in FETCH_AS_IS:
                        sc = 1024.0
                    acc[k][c] += float(row["Counter_Value"]) * sc
                    cnt[k][c] += 1
            f.unlink()
    for k in acc:  # the raw write requests -> WRITE_SIZE bytes
        if all(c in acc[k] for c in RAW_WRITE):
            w, w64 = acc[k].pop(RAW_WRITE[0]), acc[k].pop(RAW_WRITE[1])
            acc[k]["WRITE_SIZE"] = 64.0 * w64 + 32.0 * (w - w64)
            cnt[k]["WRITE_SIZE"] = cnt[k].pop(RAW_WRITE[0])
            cnt[k].pop(RAW_WRITE[1], None)
    res = {}
    for d in dirs:
        if d.endswith(".json"):
            old = {k: dict(v) for k, v in json.loads(Path(d).read_text()).items() if isinstance(v, dict) and "fetch_size_bytes" in v}
            for k, v in old.items():  # --refetch: entries reduced with x2 before FETCH_AS_IS named them
                if REFETCH and k.split("<")[0] in FETCH_AS_IS:
                    v["fetch_size_bytes"] /= 2.0
                    v["bytes_per_launch"] = v["fetch_size_bytes"] + v.get("write_size_bytes", 0.0)
            res.update(old)
            if src is None:
                src = json.loads(Path(d).read_text()).get("_source")
    for k in acc:
        per = {c: acc[k][c] / cnt[k][c] for c in acc[k]}
        res[k] = {"bytes_per_launch": sum(per.values()), "launches": max(cnt[k].values()),
                  **{c.lower() + "_bytes": v for c, v in per.items()}}
    # aggregate template instances under the engine's kernel ids (launch-weighted)
    ids = {"ntt1_fwd": "ntt_cols_fwd", "ntt2_fwd": "ntt_rows_fwd", "ntt2_inv": "ntt_rows_inv", "ntt1_inv": "ntt_cols_inv",
           "ntt2_fwd8": "ntt_rows_fwd", "ntt2_inv8": "ntt_rows_inv",
           "key_inner": "key_inner", "key_inner_sum": "key_inner", "key_inner_multi": "key_inner", "ntt2_ki": "key_inner", "ntt2_ki8": "key_inner",
           "base_convert": "base_convert", "bx_cols": "base_convert", "lin_mac": "lin_mac"}
    agg = {}
    for k, v in list(res.items()):
        kid = ids.get(k.split("<")[0])
        if kid and kid != k:
            a = agg.setdefault(kid, {"bytes": 0.0, "launches": 0})
            a["bytes"] += v["bytes_per_launch"] * v["launches"]
            a["launches"] += v["launches"]
    for kid, a in agg.items():
        res[kid] = {"bytes_per_launch": a["bytes"] / max(a["launches"], 1), "launches": a["launches"]}
    if alg:  # traffic per launch over algorithmic bytes per launch, same launches
        for kid, v in alg.items():
            if kid in res and v.get("launches"):
                a_b = v["bytes"] / v["launches"]
                res[kid]["algorithmic_bytes_per_launch"] = a_b
                res[kid]["traffic_over_algorithmic"] = res[kid]["bytes_per_launch"] / a_b if a_b else None
    if src:
        res["_source"] = src
    out.write_text(json.dumps(res, indent=1))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
