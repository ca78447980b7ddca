"""NTT / inverse NTT time per call (both passes, back-to-back calls incl. the launch gaps) vs row
count, for block-size configurations of the two passes: AESFHE_NTT_P1_NT (column pass, 512 / 256
threads), AESFHE_NTT_P2_NT / AESFHE_NTT_P2I_NT (row pass forward / inverse, 512 / 256 / 128).
Each configuration runs in its own process (the switches are read once per process).
usage: python tools/ntt_grid_sweep.py > out.json"""
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
ROWS = list(range(2, 130, 2))
CONFIGS = [{"AESFHE_NTT_P1_NT": p1, "AESFHE_NTT_P2_NT": p2, "AESFHE_NTT_P2I_NT": p2}
           for p1 in ("512", "256") for p2 in ("256", "128")]

WORKER = r"""
import json, sys
sys.path[:0] = [sys.argv[1], sys.argv[1] + "/aes-implementation-fhe_amd"]
from mi355x_ckks import Engine
E = Engine(log_n=16, max_level=30, dnum=3, seed=1, allow_insecure=True)
rows = [int(x) for x in sys.argv[2].split(",")]
top = 4 * 32
print(json.dumps({op: {r: round(E.bench_op(op, r, 100), 3) for r in rows if r <= top} for op in ("ntt", "intt")}))
"""


def main():
    out = {"what": __doc__.split("\n")[0], "rows": ROWS, "runs": []}
    for cfg in CONFIGS:
        env = dict(os.environ, **cfg)
        r = subprocess.run([sys.executable, "-c", WORKER, str(ROOT), ",".join(map(str, ROWS))], env=env, capture_output=True,
                           text=True, timeout=300)
        if r.returncode != 0:
            out["runs"].append({"config": cfg, "error": r.stderr[-2000:]})
            break
        out["runs"].append({"config": cfg, **json.loads(r.stdout.strip().splitlines()[-1])})
        print(json.dumps(cfg), file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
