"""The N > 1 path of bench.py on CPU: torch.distributed.run with world size 2 over gloo
(one process per rank, 127.0.0.1 rendezvous), exercising the process group, the shared-seed
key broadcast, one CKKS engine per rank (the CPU oracle at N = 2^13 running AddRoundKey),
per-rank state sharding, barrier, max-over-ranks timing and the single rank-0 JSON line."""
import json
import socket
import subprocess
import sys

from conftest import ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_bench_two_ranks_gloo():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr=127.0.0.1",
           f"--master-port={_free_port()}", str(ROOT / "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--dry-run"]
    import os
    env = dict(os.environ, OMP_NUM_THREADS="2")
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1  # rank 0 only
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["dry_run"] and rec["value"] is None
    assert rec["outputs"] == 4
    assert rec["ark_exact_per_rank"] == [True, True]  # each rank's engine decoded state ^ key exactly
    assert rec["same_keys_on_every_rank"]  # the broadcast seed gave every rank one key set
    a, b = rec["first_byte_per_rank"]
    import numpy as np
    sys.path.insert(0, str(ROOT))
    import bench
    assert [a, b] == [int(bench.rank_states(r, 2)[1][0]) for r in (0, 1)]  # each rank owns its states
