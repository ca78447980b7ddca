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


def test_bench_eight_ranks_gloo_sharding():
    """World size 8 (the C4 / C5 node shape) on CPU: every rank gets 1024 / 8 = 128 C5 states
    (bench.c5_states_per_rank, REF/main.py:121-140's batch intent), its own distinct C3/C4 batch and C5
    share (per-rank seeds), and ONE key fingerprint across all eight ranks."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=8", "--master-addr=127.0.0.1",
           f"--master-port={_free_port()}", str(ROOT / "bench.py"), "--gpus", "8", "--steps", "1", "--warmup", "0",
           "--dry-run", "--c5-states", "1024", "--batch-states", "1024"]
    import os
    env = dict(os.environ, OMP_NUM_THREADS="1")
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 8 and rec["outputs"] == 8
    assert rec["ark_exact_per_rank"] == [True] * 8
    assert rec["same_keys_on_every_rank"] and len(rec["key_fingerprints"]) == 1
    assert rec["c5_states_per_rank"] == [128] * 8 and rec["c5_input_rows_per_rank"] == [128] * 8
    assert rec["c5_states_total"] == 1024
    assert len(set(rec["batch_digest_per_rank"])) == 8  # distinct C3/C4 batches per rank
    assert len(set(rec["c5_digest_per_rank"])) == 8     # distinct C5 shares per rank
    assert len(set(rec["first_byte_per_rank"])) > 1


def test_split_arithmetic():
    sys.path.insert(0, str(ROOT))
    import bench
    assert [bench.c5_states_per_rank(1024, w) for w in (1, 2, 4, 8)] == [1024, 512, 256, 128]
    assert bench.c5_states_per_rank(1000, 8) == 125 and bench.c5_states_per_rank(3, 8) == 1
    b, c5 = bench.batch_inputs(3, 1024, 2, 128)
    assert len(b) == 3 and all(x.shape == (1024, 16) for x in b)
    assert len(c5) == 3 and all(x.shape == (128, 16) for x in c5)
    b2, c52 = bench.batch_inputs(3, 1024, 2, 128)
    assert all((x == y).all() for x, y in zip(b + c5, b2 + c52))  # seeded per rank: reproducible
    b4, _ = bench.batch_inputs(4, 1024, 2, 128)
    assert not (b4[1] == b[1]).all()
    _, none = bench.batch_inputs(0, 128, 1, 128)
    assert none is None  # the C5 share equals the batch: run_batch decrypts the batch's own outputs
