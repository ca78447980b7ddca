"""Kernel launches of one C2 encrypt by C-ABI entry point and kernel name (AESFHE_CENSUS=1,
aesfhe_launch_census): which engine call issues which kernels -- the map for fusing launches away.
usage: AESFHE_CENSUS=1 python tools/op_kernel_census.py > out.json"""
import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "aes-implementation-fhe_amd")]

from aes_keyschedule import expand_aes128_key, load_all_coeffs  # noqa: E402
from engine_context import EngineContext  # noqa: E402
from mi355x_ckks import launch_census  # noqa: E402
from pipeline import AESPipeline  # noqa: E402


def short(k: str) -> str:
    k = k.replace("(anonymous namespace)::", "").split("(")[0]
    return k.split("<")[0]


def main():
    if os.environ.get("AESFHE_CENSUS") != "1":
        raise SystemExit("run with AESFHE_CENSUS=1 (read at library load)")
    ctx = EngineContext(signature=1, max_level=17)
    pipe = AESPipeline(ctx, load_all_coeffs(), use_hard_renorm_between_steps=True)
    rng = np.random.default_rng(7)
    rks = expand_aes128_key(rng.integers(0, 256, 16).astype(np.uint8))
    st = rng.integers(0, 256, 16).astype(np.uint8)
    pipe.encrypt(st, rks)  # warmup: keys, tables, LUT constants
    ctx.engine.sync()
    launch_census(reset=True)
    pipe.encrypt(st, rks)
    ctx.engine.sync()
    cen = launch_census(reset=True)
    by_op = {op: sum(v.values()) for op, v in cen.items()}
    by_kernel: dict = {}
    for op, v in cen.items():
        for k, n in v.items():
            by_kernel[short(k)] = by_kernel.get(short(k), 0) + n
    out = {"launches": sum(by_op.values()),
           "by_entry": dict(sorted(by_op.items(), key=lambda kv: -kv[1])),
           "by_kernel": dict(sorted(by_kernel.items(), key=lambda kv: -kv[1])),
           "by_entry_kernel": {op: dict(sorted(((short(k), n) for k, n in v.items()), key=lambda kv: -kv[1]))
                               for op, v in sorted(cen.items(), key=lambda kv: -sum(kv[1].values()))}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
