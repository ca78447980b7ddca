#!/usr/bin/env python
"""bench.py -- homomorphic AES-128 encryption throughput on MI355X.

Workload (BASELINE.json configs[1], "C2"): full 10-round AES-128 encryption
(AESPipeline.encrypt, REF/pipeline.py:123-188) of one packed 16-byte state per ciphertext
pair at N = 2^16, secret-key renorm between steps on (as the reference harness,
REF/test/test_aes_pipeline_roundtrip.py:132), synthetic random states, FIPS key schedule
from a seed-7 master key.  One "step" = one full encryption of one state on every rank.

Metric: homomorphic AES-128 rounds/sec (enc) = 10 * states / wall time, summed over ranks
(independent states shard across GPUs with no collective -- weak scaling).

Launch: python bench.py [--gpus N --steps K --warmup W]; N > 1 under
torch.distributed.run (one process per GPU; RANK/LOCAL_RANK/WORLD_SIZE from the env).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
PKG = ROOT / "aes-implementation-fhe_amd"
for _p in (str(ROOT), str(PKG)):
    if _p not in sys.path:
        sys.path.insert(0, _p)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
# VALU roofline of the NTT passes: u32 VALU issue rate measured on this chip with
# tools/valu_rate.hip (v_mul_lo_u32 / v_mul_hi_u32 / v_min_u32 all at ~3.85e13 lane-instr/s,
# i.e. the 32-bit multiplies are NOT quarter rate on gfx950) over the VALU instructions per
# radix-2 butterfly in the row pass's ISA.  Round 6 runs the 8-residue form k_ntt2_fwd8 (AESFHE_NTT_FWD8,
# default since): 451 v_* lines per thread for its 32 butterflies (plain mode; hipcc --save-temps,
# k_ntt2_fwd8<8, 0>), against 676 for k_ntt2_fwd<8, 0, 256>'s 64 -- more indexing per butterfly, twice the
# blocks and half the serial work per thread
VALU_LANE_INSTR_PER_S = 3.85e13
NTT_VALU_INSTR_PER_BFLY = 451.0 / 32.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--kernel", default="ntt_rows_fwd", help="kernel id timed live for the roofline (the dominant kernel)")
    ap.add_argument("--kernel2", default="key_inner", help="secondary kernel id reported as roofline_secondary")
    ap.add_argument("--eager-steps", type=int, default=1,
                    help="the per-primitive drop-in leg (VERDICT r3 item 7): C2 through EngineContext with REF's own call "
                         "sequence -- eager relinearise/rescale after every product, per-term LUT product loops (no fused "
                         "LUT kernels), the reference slot layout with full-slot bootstraps; 0 = skip")
    ap.add_argument("--deferred-steps", type=int, default=1,
                    help="REF's own call sequence through EngineContext (per-term LUT loops, reference slot layout) with the "
                         "engine's default deferred evaluation (VERDICT r4 item 6); 0 = skip")
    ap.add_argument("--profile-all", action="store_true", help="time every kernel id (diagnostic; slower)")
    ap.add_argument("--profile-every", type=int, default=32,
                    help="time one launch in N of the roofline kernels (live sample over the timed region)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--ref-layout", action="store_true",
                    help="the reference's slot layout (byte i at slot i*N/32, full-slot bootstraps) instead of the periodic "
                         "one (sparse-slot bootstraps, DESIGN.md 4b); A/B only")
    ap.add_argument("--no-final-bootstrap", action="store_true",
                    help="diagnostic only: skip MixColFinal's final bootstrap (not the benchmark workload)")
    ap.add_argument("--eager", action="store_true", help="relinearise and rescale after every product (no deferred evaluation)")
    ap.add_argument("--serial", action="store_true",
                    help="hi/lo halves on one stream, batched (the default since round 3; kept for old command lines)")
    ap.add_argument("--concurrent", action="store_true",
                    help="A/B only: hi/lo halves on two HIP streams (each half batching its own products)")
    ap.add_argument("--dry-run", action="store_true",
                    help="the N-rank host path on CPU (process group, shared-seed key broadcast, sharding, barrier, "
                         "max-over-ranks, rank-0 line) with one CPU oracle engine per rank running AddRoundKey (config C1 "
                         "shape at N=2^13) in place of the GPU engine; prints value null -- a test harness, not a measurement")
    ap.add_argument("--seed", type=int, default=None,
                    help="key seed shared by every rank (default: drawn from os.urandom on rank 0 and broadcast)")
    ap.add_argument("--c5-states", type=int, default=1024,
                    help="BASELINE config 5: total states of the enc->dec round trip, split evenly across ranks")
    ap.add_argument("--batch-states", type=int, default=1024,
                    help="secondary measurement (BASELINE configs 3/4): this many independent states per rank, "
                         "slot-packed into one ciphertext pair (SURVEY.md 8(f)1); 0 = skip")
    ap.add_argument("--batch-steps", type=int, default=3)
    ap.add_argument("--pair-states", type=int, default=1024,
                    help="BASELINE config 3 literally (1024 ciphertext pairs hi/lo, ONE state each): this many pairs "
                         "per rank as stacked ciphertexts (DESIGN.md 3.16), --pair-stack per stack; 0 = skip")
    ap.add_argument("--pair-stack", type=int, default=64,
                    help="pairs per stack: --pair-states pairs run as ceil(pair-states / pair-stack) stacks in turn")
    ap.add_argument("--packed-pairs", type=int, default=4,
                    help="multi-pair slot-packed batch: this many stacked ciphertext pairs of 2048 states each per rank; 0 = skip")
    ap.add_argument("--pair-steps", type=int, default=1, help="timed steps of the one-state multi-pair leg (C3 literally)")
    ap.add_argument("--packed-pair-steps", type=int, default=3, help="timed steps of the slot-packed multi-pair leg")
    ap.add_argument("--fresh-level", type=int, default=7,
                    help="fresh level of the C2 context's bootstrappable set (EngineContext(boot_fresh_level=)): 7, the most "
                         "any step of the strict pipeline needs between renorms / bootstraps at the renorm floor 1 "
                         "(utils.RENORM_FLOOR), puts the bootstrap's double-prime region 10 primes lower (DESIGN.md 3.1); the "
                         "true-FHE leg has its own set (--fhe-fresh-level), the REF-call legs keep the engine's 17")
    ap.add_argument("--dnum", type=int, default=4, help="key-switching digits of the C2 context (4: the shorter chain leaves "
                                                         "room under the 128-bit bound; the engine's default set uses 5)")
    ap.add_argument("--folded-steps", type=int, default=5,
                    help="timed steps of the 'folded' leg: C2 with the renorm folds on (utils.RenormFolds; the headline is strict)")
    ap.add_argument("--true-fhe-steps", type=int, default=2,
                    help="SURVEY.md 8(f)3 line beside the headline: C2 encrypts with every secret-key renorm replaced "
                         "by bootstrap + homomorphic Zeta16 snap (AESPipeline(true_fhe=True)); 0 = skip")
    ap.add_argument("--fhe-fresh-level", type=int, default=11,
                    help="fresh level of the true-FHE leg's context: one depth-4 snap + the 7 levels of the deepest step "
                         "between renorms at the renorm floor 1 (ShiftRows -> GF multipliers / XOR4s, nibble-bivariate "
                         "SubBytes), DESIGN.md 8")
    ap.add_argument("--fhe-dnum", type=int, default=4, help="key-switching digits of the true-FHE leg's context")
    ap.add_argument("--no-batch-roundtrip", dest="batch_roundtrip", action="store_false",
                    help="skip the decrypt leg of the batch (BASELINE config 5)")
    ap.add_argument("--whole-stats", default=None,
                    help="with AESFHE_PROFILE_FROM_START=<ids>: keep the engine's per-kernel accounting from the first "
                         "launch on (no reset, every launch) and write it to this JSON file -- the algorithmic bytes of "
                         "exactly the launches a whole-process rocprofv3 --pmc pass counts")
    ap.add_argument("--traffic-json", default=str(Path(__file__).resolve().parent / "profiles" / "r6_pmc_traffic_bench_final.json"),
                    help="per-kernel-class HBM / algorithmic byte ratios from rocprofv3 --pmc passes over this bench's own "
                         "C2 leg (tools/gpu_task.sh pmcbench; FETCH_SIZE and raw TCC write requests, separate runs)")
    ap.add_argument("--detail-json", default="gpurun_out/bench_detail.json",
                    help="the full per-leg / per-class record (prose included) is written here; stdout carries the compact "
                         "line (<= 12 KB) that names this file; '' = do not write it")
    return ap.parse_args()


def dist_setup(want: int):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # AESFHE_FORCE_DIST=1 (under torch.distributed.run): the process group even for one rank, so the
    # RCCL path (key broadcast, barriers, max-over-ranks, all_gather) runs on a one-GPU box
    if world > 1 or (os.environ.get("AESFHE_FORCE_DIST") == "1" and "MASTER_PORT" in os.environ):
        import torch
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # AESFHE_DIST_BACKEND=gloo rehearses N ranks on fewer GPUs (ranks share a device,
        # local % device_count); the real N-GPU run is one rank per GPU over RCCL ("nccl")
        backend = os.environ.get("AESFHE_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        ndev = torch.cuda.device_count()
        if ndev:
            local = local % ndev
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend=backend, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend=backend)
        return rank, world, local, dist
    if want > 1:
        raise SystemExit("--gpus > 1 must be launched with torch.distributed.run (one process per GPU)")
    return 0, 1, 0, None


def shared_seed(dist, seed: int | None):
    """One key set for the whole job: rank 0 draws a 256-bit ChaCha20 key from
    os.urandom (or takes the integer --seed) and broadcasts it once, before any timed region;
    every rank then derives identical keys.  This is the only collective outside the timing
    barriers and the max-over-ranks.  Returns the 32-byte key, or the int seed if one was given."""
    if seed is not None:
        return int(seed)
    key = os.urandom(32)
    if dist is None:
        return key
    import torch
    gpu = dist.get_backend() == "nccl"
    dev = torch.device("cuda", torch.cuda.current_device()) if gpu else torch.device("cpu")
    t = torch.tensor(list(key), dtype=torch.uint8, device=dev)
    dist.broadcast(t, src=0)
    return bytes(t.cpu().tolist())


def all_gather_ints(dist, vals):
    """rank-ordered list of every rank's small int list (host bookkeeping after timing)"""
    if dist is None:
        return [list(vals)]
    import torch
    gpu = dist.get_backend() == "nccl"
    dev = torch.device("cuda", torch.cuda.current_device()) if gpu else torch.device("cpu")
    t = torch.tensor(list(vals), dtype=torch.int64, device=dev)
    got = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(got, t)
    return [[int(x) for x in g.cpu().tolist()] for g in got]


def barrier(dist):
    if dist is not None:
        dist.barrier()


def max_over_ranks(dist, x: float) -> float:
    if dist is None:
        return x
    import torch
    gpu = dist.get_backend() == "nccl"
    dev = torch.device("cuda", torch.cuda.current_device()) if gpu else torch.device("cpu")
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def boot_tallies(ctx, period: int | None) -> dict:
    """the engine's per-level work tallies (aesfhe_level_counters) of ONE C2 MixColumns final
    bootstrap: the sparse form at the pipeline's period (tools/boot_phases.py's input), or the
    full-slot one for the reference layout; read after the timed legs, for the CPU baseline"""
    E = ctx.engine
    P = period or E.slot_count
    z = np.exp(2j * np.pi * np.random.default_rng(0).random(P))
    ct = E.intt(ctx.encrypt(np.tile(z, E.slot_count // P)))
    E.sync()
    E.reset_counters()
    if period:
        E.bootstrap_sparse(ct, period)
    else:
        E.bootstrap(ct)
    E.sync()
    return {"tallies": E.level_counters(), "level_limbs": list(E.level_limbs), "dnum": E.dnum, "log_n": E.log_n}


def cpu_baseline(coeffs, boot: dict | None = None) -> dict:
    """The C oracle CPU CKKS engine (oracle/ckks_cpu.py over oracle/ckks_oracle.c: Shoup / Barrett
    modular products, OpenMP over OMP_NUM_THREADS host threads), timed live on this host
    (tools/cpu_round.py): BASELINE config 1 in full (AddRoundKey at N = 2^15), then ONE FULL middle
    round of the C2 encrypt at N = 2^16 (SubBytes, renorm, ShiftRows, MixColumns without its final
    bootstrap, AddRoundKey, renorm), checked against the byte model, plus MixColumns' final
    bootstrap as a replay of its work (boot: the GPU engine's per-level tallies of one such
    bootstrap; cpu_round.boot_replay times one key switch / product / diagonal product per level
    on the oracle and multiplies by the counts -- the oracle has no bootstrap plan).  Budget:
    ~1.5 min on 16 host threads; nothing is read from a file."""
    sys.path.insert(0, str(ROOT / "tools"))
    import cpu_round
    c1 = cpu_round.c1(coeffs)
    c2 = cpu_round.c2_round(coeffs, full=True)
    round_s = c2["round_s"]
    br = cpu_round.boot_replay(boot["tallies"], boot["level_limbs"], boot["dnum"], boot["log_n"]) if boot else None
    total_s = round_s + (br["boot_s"] if br else 0.0)
    boot_txt = (f"; plus MixColumns' final bootstrap MODELED, not computed: {br['boot_s']:.1f} s = a replay of its work on the "
                f"oracle (the GPU engine's per-level tallies of one C2 final bootstrap: {br['ops']['key_switch']} key switches, "
                f"{br['ops'].get('product', 0)} products, {br['ops'].get('diagonal', 0)} diagonal products in Q.P over levels "
                f"{br['levels'][0]}-{br['levels'][-1]}; one operation per kind and level timed live ({br['sampled_s']:.1f} s) times "
                f"its count; every hoisted rotation replayed as a full key switch, so the model leans pessimistic for the CPU); "
                f"value_measured_no_boot = the measured round alone"
                ) if br else "; MixColumns' final bootstrap excluded (no tallies)"
    out = {"value": 1.0 / total_s, "unit": "rounds/s", "cores": cpu_round.threads(), "kind": "port",
           "sample": f"C oracle on the host, timed live: config 1 (AddRoundKey, N=2^15) in full {c1['ark_s']:.2f} s "
                     f"(exact: {c1['exact']}); one full middle round of C2 at N=2^16 {round_s:.1f} s without its final bootstrap "
                     f"(exact: {c2['exact']}; " + ", ".join(f"{k} {v:.1f} s" for k, v in c2["steps_s"].items()) + ")" + boot_txt,
           "c1_ark_s": c1["ark_s"], "c2_round_s": total_s, "c2_round_no_boot_s": round_s, "c2_steps_s": c2["steps_s"],
           "value_measured_no_boot": 1.0 / round_s, "value_kind": "measured round + modeled bootstrap" if br else "measured round"}
    if br:
        out["c2_boot_modeled_s"] = br["boot_s"]
        out["c2_boot_by_kind_s"] = br["by_kind_s"]
    return out


class _NoFinalBootstrap:
    """Diagnostic wrapper: MixColFinal without its final bootstrap."""

    def __init__(self, mix):
        self.mix = mix
        self.layout = mix.layout

    def __call__(self, ct_hi, ct_lo, **kw):
        return self.mix(ct_hi, ct_lo, do_final_bootstrap=False)


def empty_pools(E) -> None:
    """empty the engine's pools of zero encryptions (aesfhe_renorm_pool) before a timed
    region: every re-encryption a timed renorm uses is then made inside that region"""
    f = getattr(E, "renorm_pool", None)
    if f is not None:
        f(-1)


def _progress(ctx, every_s: float = 30.0):
    """stderr heartbeat with real progress (bootstraps done), for long profiled runs."""
    import threading
    t0 = time.perf_counter()

    def run():
        while True:
            time.sleep(every_s)
            print(f"[bench] {time.perf_counter() - t0:.0f}s bootstraps={ctx.bootstrap_stats()['count']}",
                  file=sys.stderr, flush=True)

    threading.Thread(target=run, daemon=True).start()


def state_slots(pipe, ctx, ct, packed: bool) -> np.ndarray:
    """decrypted slot values of every state of a (stacked) ciphertext: (hi | lo of a packed one)"""
    from utils import conj_sum
    enc = pipe.encoder
    out = []
    ct = conj_sum(ctx, ct)  # a folded-renorm input logged unsummed (utils.ConjSum): its value s1 + conj(s2)
    for c in (ctx.unstack(ct) if enc.pairs > 1 else [ct]):
        z = ctx.decrypt(c)
        out.append(enc._take(z).ravel())
        if packed:
            out.append(enc._take(z[enc.layout.period:]).ravel())
    return np.concatenate(out)


def measure_precision(pipe, ctx, rks, state, what: str) -> dict:
    """CKKS precision of a bench leg, measured after its timed region on one more input of the
    leg's own shape: the largest angular deviation of ANY state slot (every state of the batch,
    every pair of a stack) from its Zeta16 codeword over every logged stage of one encrypt (debug
    dict of the production path), against the decode margin pi/16 -- bytes are
    exact while it stays below (REF/utils.py:15-19, REF/state_encoder.py:30-38)."""
    E = ctx.engine
    dbg = {}
    pipe.encrypt(state, rks, debug=dbg)
    worst, where, nslots = 0.0, None, 0
    for tag, entry in dbg.items():
        cts = [(entry["ct_packed"], True)] if "ct_packed" in entry else [(entry["ct_hi"], False), (entry["ct_lo"], False)]
        for c, packed in cts:
            z = state_slots(pipe, ctx, c, packed)
            nslots = max(nslots, z.size)
            ang = np.angle(z) * 16 / (2 * np.pi)
            dev = float(np.abs(ang - np.rint(ang)).max() * 2 * np.pi / 16)
            if dev > worst:
                worst, where = dev, tag
    deltas = E.scales()
    margin = float(np.pi / 16)
    return {"log2_delta_fresh": float(np.log2(deltas[E.fresh_level])), "log2_delta_level0": float(np.log2(deltas[0])),
            "max_slot_angle_error_rad": worst, "worst_stage": where, "decode_margin_rad": margin,
            "margin_factor": margin / worst if worst > 0 else None, "stages_checked": len(dbg),
            "state_slots_per_stage": nslots,
            "note": f"slot error = angular distance of every state slot to the nearest 16th root of unity, over every "
                    f"logged stage of one encrypt of {what} (renorm / XOR4 / GF / SubBytes / bootstrap outputs)"}


def rank_states(rank: int, n: int):
    """Independent synthetic states of one rank (weak scaling: each rank owns its own)."""
    rng = np.random.default_rng(2025 + rank)
    return [rng.integers(0, 256, 16).astype(np.uint8) for _ in range(n)]


def c5_states_per_rank(total: int, world: int) -> int:
    """BASELINE config 5's split: `total` enc->dec states over `world` ranks, ceil(total / world)
    each (1024 over 8 MI355X = 128 per GPU; REF/main.py:121-140's batch intent)"""
    return max(1, -(-total // world))


def batch_inputs(rank: int, B: int, steps: int, B5: int | None = None):
    """the batch leg's inputs of one rank: 1 + steps arrays of (B, 16) states (warmup first), then,
    when the C5 share B5 differs from B, 1 + steps arrays of (B5, 16) -- one seeded stream per rank,
    so every rank encrypts its own states"""
    rng = np.random.default_rng(4096 + rank)
    batches = [rng.integers(0, 256, (B, 16), dtype=np.uint8) for _ in range(1 + steps)]
    c5 = [rng.integers(0, 256, (B5, 16), dtype=np.uint8) for _ in range(1 + steps)] if B5 and B5 != B else None
    return batches, c5


# kernel classes timed live (one launch in --profile-every): the roofline kernels and the classes
# whose fractions VERDICT r3 weak #2 tabulates
PROF_KIDS = ["ntt_rows_fwd", "ntt_cols_fwd", "ntt_rows_inv", "ntt_cols_inv", "base_convert", "key_inner", "lin_mac"]


class Leg:
    """Live accounting of one timed leg: the algorithmic bytes and launches of
    EVERY launch (engine counters), and, for the sampled launches of PROF_KIDS, their in-kernel
    span and the boundary gap before them (the previous launch's drain + this one's dispatch ramp,
    include/aesfhe.h aesfhe_kernel_gaps) -- span + gap is the dispatch-inclusive duration that
    rocprofv3 --kernel-trace reports for the same launches."""

    def __init__(self, E):
        import mi355x_ckks
        self.E, self.m = E, mi355x_ckks

    def start(self):
        self.E.kernel_stats(reset=True)  # flushes (device sync) and zeroes spans and gaps
        self.alg0, self.l0 = self.m.alg_bytes(), self.m.launch_count()
        return self

    def stop(self):
        self.alg1, self.l1 = self.m.alg_bytes(), self.m.launch_count()
        self.work = self.E.kernel_work()
        self.gaps = self.E.kernel_gaps()
        self.stats = self.E.kernel_stats(reset=True)
        return self

    def bytes_by_class(self):
        return {k: self.alg1[k][0] - self.alg0[k][0] for k in self.alg1}

    def launches_by_class(self):
        return {k: self.alg1[k][1] - self.alg0[k][1] for k in self.alg1}

    def kernel(self, kid: str):
        """(launches, span us, gap us or None, gaps measured, bytes per launch, butterflies per launch)"""
        ks = self.stats.get(kid)
        if not ks or ks["launches"] == 0:
            return None
        n = ks["launches"]
        gn, gms = self.gaps.get(kid, (0, 0.0))
        return n, ks["ms"] / n * 1e3, (gms / gn * 1e3 if gn else None), gn, ks["bytes"] / n, self.work.get(kid, 0.0) / n

    def roofline(self, kid: str, tj: dict, every: int, note: str) -> dict | None:
        """HBM roofline of one kernel class at its DISPATCH-INCLUSIVE average duration (span + gap,
        comparable with rocprofv3's average for the same launches); frac_span keeps the in-kernel span"""
        k = self.kernel(kid)
        if k is None:
            return None
        n, span_us, gap_us, gn, bpl, _ = k
        dur_us = span_us + (gap_us if gap_us is not None else 0.0)
        achieved = bpl / (dur_us * 1e-6) / 1e9
        t = tj.get(kid)
        traffic = None
        if t and t.get("traffic_over_algorithmic"):  # measured HBM / algorithmic ratio applied to this leg's launches
            traffic = t["traffic_over_algorithmic"] * bpl
        return {"kernel": kid, "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                "traffic_over_algorithmic": t.get("traffic_over_algorithmic") if t else None,
                "traffic_source": tj.get("_source") if t else None,
                "timed_launches": n, "sampled_every": every, "avg_us": dur_us, "avg_us_span": span_us, "avg_us_gap": gap_us,
                "gaps_measured": gn, "frac_span": bpl / (span_us * 1e-6) / 1e9 / HBM_PEAK_GBS,
                "timing": "avg_us = in-kernel span (first block start -> last block end, s_memrealtime) + the boundary gap "
                          "before the launch (previous launch's last block end -> this launch's first block start), both "
                          "measured live on the sampled launches: the dispatch-inclusive duration rocprofv3 reports",
                "bytes_per_launch": bpl, "note": note}

    def valu_roofline(self, kid: str) -> dict | None:
        k = self.kernel(kid)
        if k is None or not k[5]:
            return None
        n, span_us, gap_us, gn, bpl, bfly = k
        dur_us = span_us + (gap_us if gap_us is not None else 0.0)
        achieved = bfly / (dur_us * 1e-6)
        peak = VALU_LANE_INSTR_PER_S / NTT_VALU_INSTR_PER_BFLY
        return {"kernel": kid, "bound": "valu", "achieved": achieved, "peak": peak, "unit": "butterfly/s", "frac": achieved / peak,
                "butterflies_per_launch": bfly, "avg_us": dur_us,
                "note": "peak = measured u32 VALU issue rate (tools/valu_rate.hip) / VALU instructions per butterfly in the "
                        "kernel's ISA; at the dispatch-inclusive duration"}

    def step(self, elapsed: float, steps: int, tj: dict, every: int) -> dict:
        """whole-leg roofline: algorithmic bytes of every launch / this leg's wall time / 8 TB/s, plus
        the per-class fractions of the sampled classes and launches per step"""
        b, n = self.bytes_by_class(), self.launches_by_class()
        tot = sum(b.values())
        return {"bound": "hbm", "achieved": tot / elapsed / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": tot / elapsed / 1e9 / HBM_PEAK_GBS, "algorithmic_bytes_per_step": tot / steps,
                "launches_per_step": (self.l1 - self.l0) / steps,
                "bytes_per_step_by_class": {k: v / steps for k, v in b.items() if v},
                "launches_per_step_by_class": {k: v / steps for k, v in n.items() if v},
                "classes": {k: r for k in PROF_KIDS if (r := self.roofline(k, tj, every, "per-class fraction (live sample)"))},
                "note": "sum over every kernel launch of the leg's timed steps of its algorithmic bytes (each operand word "
                        "read once, each result word written once; DESIGN.md 5) / wall time / 8 TB/s; classes at the "
                        "dispatch-inclusive duration"}


def run_pairs(ctx, coeffs, rks, args, rank, world, dist, pairs: int, states: int, stack: int, steps_n: int, workload: str,
              tj: dict) -> dict:
    """Multi-pair batch: `pairs` independent ciphertext pairs of `states` states each
    per rank, run as stacked ciphertexts of `stack` pairs (AESPipeline(pairs=...)), one after the
    other; full 10-round encrypt with renorm and final bootstraps.  Whole-job blocks/s = states
    encrypted by all ranks / max time; every pair's output checked against the plaintext AES.
    Warmup: ONE stack of each shape (every stack of a shape runs the same launches)."""
    from oracle import aes_plain  # checker only, after the timed region
    from pipeline import AESPipeline
    if 2 * 16 * states > ctx.engine.slot_count:  # no packed form for this state count: the pair path's levels
        ctx = full_levels(ctx)
    chunks = [min(stack, pairs - i) for i in range(0, pairs, stack)]
    pipes = {c: AESPipeline(ctx, coeffs, use_hard_renorm_between_steps=True, states=states, pairs=c) for c in set(chunks)}
    rng = np.random.default_rng(8192 + rank)
    shape = lambda c: (c, 16) if states == 1 else (c, states, 16)  # noqa: E731
    warm = {c: rng.integers(0, 256, shape(c), dtype=np.uint8) for c in set(chunks)}
    steps = [[rng.integers(0, 256, shape(c), dtype=np.uint8) for c in chunks] for _ in range(steps_n)]
    E = ctx.engine
    for c, b in warm.items():  # warmup: masks, LUT constants, codec buffers, stacked keys
        pipes[c].encrypt(b, rks)
    E.sync()
    empty_pools(E)
    leg = Leg(E).start()
    barrier(dist)
    t0 = time.perf_counter()
    outs = [[pipes[c].encrypt(b, rks) for c, b in zip(chunks, st)] for st in steps]
    E.sync()
    barrier(dist)
    elapsed = time.perf_counter() - t0
    leg.stop()
    elapsed = max_over_ranks(dist, elapsed)
    ok = True
    for st, ot in zip(steps, outs):
        for c, b, o in zip(chunks, st, ot):
            got = pipes[c].encoder.decode(*o).reshape(-1, 16)
            ok &= all(np.array_equal(got[j], aes_plain.ref_encrypt(s, rks)) for j, s in enumerate(b.reshape(-1, 16)))
    ok = all(r[0] for r in all_gather_ints(dist, [int(ok)]))
    blocks = pairs * states * steps_n * world
    c0 = chunks[0]
    return {"workload": workload, "pairs_per_rank": pairs, "states_per_pair": states, "pairs_per_stack": stack,
            "stacks_per_step": len(chunks), "steps": steps_n, "n_gpus": world,
            "blocks_per_s": blocks / elapsed, "rounds_per_s": 10.0 * blocks / elapsed,
            "ms_per_step": elapsed / steps_n * 1e3, "ms_per_pair": elapsed / (steps_n * pairs) * 1e3,
            "verified_against_plaintext_model": bool(ok),
            "roofline_step": leg.step(elapsed, steps_n, tj, args.profile_every),
            # one-state pairs: a debug-logged stack of 64 would decrypt ~16k stage ciphertexts, so a stack of
            # 16 (every member of its MixColumns bootstraps packed into one, as in the stacks of 64:
            # aesfhe_set_stack_pack)
            "precision": (pair_precision(ctx, coeffs, rks, rng) if states == 1 else
                          measure_precision(pipes[c0], ctx, rks, warm[c0], f"one stack of {c0} pairs x {states} states"))
            if rank == 0 else None}


def pair_precision(ctx, coeffs, rks, rng, pairs: int = 16) -> dict:
    """measure_precision of the one-state stacked path on a stack of `pairs` pairs"""
    from pipeline import AESPipeline
    pipe = AESPipeline(ctx, coeffs, use_hard_renorm_between_steps=True, pairs=pairs)
    st = rng.integers(0, 256, (pairs, 16), dtype=np.uint8)
    pipe.encrypt(st, rks)  # warm: the stack's plaintext caches
    return measure_precision(pipe, ctx, rks, st, f"one stack of {pairs} one-state pairs")


def run_batch(ctx, coeffs, rks, args, rank, world, dist, tj: dict) -> dict:
    """BASELINE configs 3/4: `--batch-states` independent states per rank under one shared
    key, slot-packed in one ciphertext pair (state b in slots i*stride + b), full 10-round
    encrypt with renorm and final bootstraps.  Whole-job blocks/s = states x ranks / max time."""
    from oracle import aes_plain  # checker only, after the timed region
    from pipeline import AESPipeline
    B = args.batch_states
    B5 = c5_states_per_rank(args.c5_states, world)
    pipe = AESPipeline(ctx, coeffs, use_hard_renorm_between_steps=True, states=B)
    batches, ins5 = batch_inputs(rank, B, args.batch_steps, B5 if args.batch_roundtrip else None)
    E = ctx.engine
    pipe.encrypt(batches[0], rks)  # warmup: masks, LUT constants, FFT buffers
    E.sync()
    empty_pools(E)
    leg = Leg(E).start()
    barrier(dist)
    t0 = time.perf_counter()
    outs = [pipe.encrypt(b, rks) for b in batches[1:]]
    E.sync()
    barrier(dist)
    elapsed = time.perf_counter() - t0
    leg.stop()
    elapsed = max_over_ranks(dist, elapsed)
    ok = True
    for b, o in zip(batches[1:], outs):
        got = pipe.encoder.decode(*o)
        ok &= all(np.array_equal(got[j], aes_plain.ref_encrypt(b[j], rks)) for j in range(B))
    ok = all(r[0] for r in all_gather_ints(dist, [int(ok)]))
    rt = None
    if args.batch_roundtrip:
        # BASELINE config 5: enc -> dec of --c5-states states in total, split across the ranks
        # (1024 = 128 per GPU at N = 8); decrypt inserts InvMixColumns
        if ins5 is None:  # same shape as the batch leg: decrypt its outputs
            pipe5, ins5, outs5, enc_s = pipe, batches[1:], outs, elapsed
        else:
            pipe5 = AESPipeline(ctx, coeffs, use_hard_renorm_between_steps=True, states=B5)
            pipe5.encrypt(ins5[0], rks)  # warmup of the new shape
            ins5 = ins5[1:]
            E.sync()
            barrier(dist)
            t1 = time.perf_counter()
            outs5 = [pipe5.encrypt(b, rks) for b in ins5]
            E.sync()
            barrier(dist)
            enc_s = max_over_ranks(dist, time.perf_counter() - t1)
        pipe5.decrypt(*outs5[0], rks)  # warmup of the decrypt-only constants (InvSubBytes, InvMixColumns)
        E.sync()
        leg5 = Leg(E).start()
        barrier(dist)
        t1 = time.perf_counter()
        backs = [pipe5.decrypt(*o, rks) for o in outs5]
        E.sync()
        barrier(dist)
        dec_s = time.perf_counter() - t1
        leg5.stop()
        dec_s = max_over_ranks(dist, dec_s)
        exact = all(np.array_equal(pipe5.encoder.decode(*bk), b) for bk, b in zip(backs, ins5))
        exact = all(r[0] for r in all_gather_ints(dist, [int(exact)]))
        rt = {"workload": f"C5: enc->dec round trip (InvMixColumns + bootstrap + snap) of {B5 * world} states, "
                          f"{B5} per GPU slot-packed in one ciphertext pair",
              "states_per_rank": B5, "enc_ms_per_step": enc_s / args.batch_steps * 1e3,
              "dec_ms_per_step": dec_s / args.batch_steps * 1e3,
              "roundtrip_blocks_per_s": B5 * args.batch_steps * world / (enc_s + dec_s),
              "roundtrip_bit_exact": bool(exact),
              "roofline_step_dec": leg5.step(dec_s, args.batch_steps, tj, args.profile_every)}
    blocks = B * args.batch_steps * world
    return {"workload": f"C3/C4: {B} independent states per GPU slot-packed in one ciphertext pair (SURVEY.md 8(f)1), "
                        f"full AES-128 encrypt, N=2^16, renorm on, shared key",
            "states_per_rank_per_step": B, "steps": args.batch_steps, "n_gpus": world,
            "blocks_per_s": blocks / elapsed, "rounds_per_s": 10.0 * blocks / elapsed,
            "ms_per_step": elapsed / args.batch_steps * 1e3, "verified_against_plaintext_model": bool(ok),
            "roofline_step": leg.step(elapsed, args.batch_steps, tj, args.profile_every),
            "precision": measure_precision(pipe, ctx, rks, batches[0], f"{B} slot-packed states") if rank == 0 else None,
            **({"roundtrip": rt} if rt else {})}


def run_folded(ctx, coeffs, rks, args, rank, world, dist, mix_layout, strict_value: float) -> dict:
    """The C2 workload with the secret-key renorm allowed to fold AES work into its decrypt -> snap ->
    re-encrypt (utils.RenormFolds: ShiftRows as a slot permutation, the conjugate-split LUTs' S1 +
    conj(S2), the hi | lo pack and unpack).  NOT the reference's workload -- its renorm is the identity
    on the message (REF/pipeline.py:65-69) -- reported beside the strict headline with the delta."""
    from mixcol_final import MixColFinal
    from oracle import aes_plain  # checker only, after the timed region
    from pipeline import AESPipeline
    from utils import RENORM_TALLY, renorm_folds
    from xor4_lut import XOR4LUT
    with renorm_folds(True) as folds:
        xor4 = XOR4LUT(ctx, coeffs["xor4"])
        pipe = AESPipeline(ctx, coeffs, mixcolumns=MixColFinal(ctx, xor4, layout=mix_layout), use_hard_renorm_between_steps=True,
                           periodic=mix_layout.periodic)
        sts = rank_states(rank + 5000, 1 + args.folded_steps)
        pipe.encrypt(sts[0], rks)
        ctx.engine.sync()
        import mi355x_ckks
        empty_pools(ctx.engine)
        l0 = mi355x_ckks.launch_count()
        r0 = dict(RENORM_TALLY)
        barrier(dist)
        t0 = time.perf_counter()
        outs = [pipe.encrypt(s, rks) for s in sts[1:]]
        ctx.engine.sync()
        barrier(dist)
        elapsed = time.perf_counter() - t0
        l1 = mi355x_ckks.launch_count()
        folds_on = dict(conj=folds.conj, sr=folds.sr, pack=folds.pack, unpack=folds.unpack)
    elapsed = max_over_ranks(dist, elapsed)
    ok = all(np.array_equal(pipe.encoder.decode(*o), aes_plain.ref_encrypt(s, rks)) for s, o in zip(sts[1:], outs))
    ok = all(r[0] for r in all_gather_ints(dist, [int(ok)]))
    steps = args.folded_steps
    rps = 10.0 * steps * world / elapsed
    return {"workload": "C2 with the renorm folds on (not REF's workload: the renorm computes ShiftRows, conjugations, "
                        "pack/unpack on the decrypted message)", "folds": folds_on,
            "rounds_per_s": rps, "ms_per_step": elapsed / steps * 1e3, "steps": steps,
            "delta_vs_strict": rps / strict_value - 1.0 if strict_value else None,
            "launches_per_encrypt": (l1 - l0) / steps,
            "secret_key_renorms_per_encrypt": (RENORM_TALLY["ciphertexts"] - r0["ciphertexts"]) / steps,
            "verified_against_plaintext_model": bool(ok)}


_CTX17 = {}


def full_levels(ctx):
    """ctx itself when its fresh level covers the reference pair path, else ONE extra context (same seed, its
    own keys), made once: for the pair path of a state count too large for the packed form, whose deepest
    step between renorms is ShiftRows -> GF multipliers -> XOR4 (utils.NEED_SR_MIX levels: 12 at the renorm
    floor 1), on a bootstrappable set with that fresh level and 4 digits (AESFHE_PAIR_SET_17=1: the engine's
    default 17 / 5 set, round 5's)"""
    from utils import NEED_SR_MIX
    fresh, dnum = (17, 5) if os.environ.get("AESFHE_PAIR_SET_17") == "1" else (max(NEED_SR_MIX, 1), 4)
    if ctx.engine.fresh_level >= fresh:
        return ctx
    return fhe_context(ctx, fresh, dnum)


def fhe_context(ctx, fresh: int, dnum: int):
    """ctx itself when it has the bootstrappable set (fresh, dnum), else ONE extra context with it (same
    seed, its own keys), made once per set: the true-FHE leg's (--fhe-fresh-level / --fhe-dnum) and the
    pair path's (full_levels)"""
    E = ctx.engine
    if E.fresh_level == fresh and E.dnum == dnum:
        return ctx
    key = ("fhe", fresh, dnum)
    if key not in _CTX17:
        from engine_context import EngineContext
        _CTX17[key] = EngineContext(signature=1, boot_fresh_level=fresh, dnum=dnum, thread_count=1, device_id=E.device_id,
                                    seed=E.seed, lazy=E.lazy)
    return _CTX17[key]


def run_true_fhe(ctx, coeffs, rks, args, rank, world, dist, tj: dict) -> dict:
    """the C2 workload with no secret key between encryption and decryption --
    every renorm point is a bootstrap + homomorphic Zeta16 snap (zeta16_noise_reducer.py), XOR4
    normalised by 1/256.  One state per rank per step, checked after the timed region."""
    from oracle import aes_plain  # checker only, after the timed region
    from pipeline import AESPipeline
    # one snap + the deepest step between renorms (7 levels at the renorm floor 1): the --fhe-fresh-level set (11 / 4)
    ctx = fhe_context(ctx, args.fhe_fresh_level, args.fhe_dnum)
    pipe = AESPipeline(ctx, coeffs, use_hard_renorm_between_steps=False, true_fhe=True)
    sts = rank_states(rank + 1000, 1 + args.true_fhe_steps)
    pipe.encrypt(sts[0], rks)  # warmup: snap constants, normalised XOR4 coefficient sets
    ctx.engine.sync()
    leg = Leg(ctx.engine).start()
    barrier(dist)
    b0 = ctx.bootstrap_stats()
    t0 = time.perf_counter()
    outs = [pipe.encrypt(s, rks) for s in sts[1:]]
    ctx.engine.sync()
    barrier(dist)
    elapsed = time.perf_counter() - t0
    leg.stop()
    elapsed = max_over_ranks(dist, elapsed)
    b1 = ctx.bootstrap_stats()
    nboot = (b1["count"] - b0["count"]) / args.true_fhe_steps
    ncalls = (b1["calls"] - b0["calls"]) / args.true_fhe_steps
    ok = all(np.array_equal(pipe.encoder.decode(*o), aes_plain.ref_encrypt(s, rks)) for s, o in zip(sts[1:], outs))
    ok = all(r[0] for r in all_gather_ints(dist, [int(ok)]))
    done = args.true_fhe_steps * world
    snaps = pipe.snapper.max_snaps
    return {"workload": "C2 in true-FHE mode: every secret-key renorm replaced by bootstrap + depth-4 Zeta16 snap "
                        + ("(one snap per renorm, nibble-bivariate SubBytes" if snaps == 1 else "(two snaps where the next step is an XOR4")
                        + "; MixColumns' paired renorms share one quad bootstrap); no secret key between encryption and decryption",
            "params": {"fresh_level": ctx.engine.fresh_level, "dnum": ctx.engine.dnum, "log2_pq": round(ctx.engine.log_pq, 1),
                       "max_snaps": snaps},
            "rounds_per_s": 10.0 * done / elapsed, "ms_per_step": elapsed / args.true_fhe_steps * 1e3,
            "bootstraps_per_encrypt": nboot, "bootstrap_calls_per_encrypt": ncalls, "steps": args.true_fhe_steps, "verified_against_plaintext_model": bool(ok),
            "roofline_step": leg.step(elapsed, args.true_fhe_steps, tj, args.profile_every),
            "precision": measure_precision(pipe, ctx, rks, sts[0], "one state, true-FHE") if rank == 0 else None}


def run_ref_calls(coeffs, rks, args, rank, world, dist, local, seed, tj: dict, lazy: bool) -> dict:
    """The per-primitive drop-in path: C2 through a SEPARATE EngineContext that issues the
    reference's own call sequence -- every LUT as REF's per-term product loop (fused_luts=False:
    REF/xor4_lut.py:71-73, REF/sub_bytes_lut.py:66-71, REF/mixcol_final.py:80-91), the reference
    slot layout (byte i at slot i*N/32) with full-slot bootstraps (REF/mixcol_final.py:158-162).
    lazy=False: every call executed when it is made, every ct x ct product relinearised and rescaled at
    once (REF/engine_context.py:65-68, VERDICT r3 item 7: no deferred calls, no deferred evaluation);
    lazy=True: the engine's defaults under the same calls -- deferred call sequences
    and deferred evaluation.  The throughput a caller gets by
    swapping the import line and changing nothing else."""
    from engine_context import EngineContext
    from oracle import aes_plain  # checker only, after the timed region
    from pipeline import AESPipeline
    ctx = EngineContext(signature=1, max_level=17, thread_count=1, device_id=local, seed=seed, lazy=lazy, fused_luts=False,
                        defer_calls=lazy)
    pipe = AESPipeline(ctx, coeffs, use_hard_renorm_between_steps=True, periodic=False)
    steps = args.deferred_steps if lazy else args.eager_steps
    sts = rank_states(rank + (4000 if lazy else 3000), 1 + steps)
    E = ctx.engine
    pipe.encrypt(sts[0], rks)  # warmup: plaintext constants of the per-term loops
    E.sync()
    E.profile(PROF_KIDS, every=args.profile_every)
    empty_pools(E)
    leg = Leg(E).start()
    E.reset_counters()
    barrier(dist)
    t0 = time.perf_counter()
    outs = [pipe.encrypt(s, rks) for s in sts[1:]]
    E.sync()
    barrier(dist)
    elapsed = time.perf_counter() - t0
    leg.stop()
    counters = E.counters()
    E.profile(())
    elapsed = max_over_ranks(dist, elapsed)
    ok = all(np.array_equal(pipe.encoder.decode(*o), aes_plain.ref_encrypt(s, rks)) for s, o in zip(sts[1:], outs))
    ok = all(r[0] for r in all_gather_ints(dist, [int(ok)]))
    done = steps * world
    out = {"workload": "C2 through EngineContext with the reference's call sequence: per-term LUT product loops, reference "
                       "slot layout, full-slot bootstraps, " + ("deferred relinearise/rescale (engine default)" if lazy else
                                                                "every call executed as made, eager relinearise + rescale per product"),
           "rounds_per_s": 10.0 * done / elapsed, "ms_per_step": elapsed / steps * 1e3,
           "steps": steps, "verified_against_plaintext_model": bool(ok),
           "op_counts_per_round": {k: v / (10.0 * steps) for k, v in counters.items()},
           "launches_per_encrypt": (leg.l1 - leg.l0) / steps,
           "roofline_step": leg.step(elapsed, steps, tj, args.profile_every)}
    del pipe, ctx
    return out


# ---------------------------------------------------------------------------------------------
# The stdout line.  The driver parses ONE JSON line; round 4's grew to 83 KB (every per-class dict
# repeated two prose paragraphs) and was not parsed.  The full per-leg detail goes to a side file
# (--detail-json); stdout carries numbers only, every prose note once under "notes".
LINE_MAX_BYTES = 12_000
CLASS_FIELDS = ["frac", "avg_us", "avg_us_span", "avg_us_gap", "MB_per_launch", "launches_per_step"]
NOTES = {
    "timing": "avg_us = in-kernel span + boundary gap before the launch, live on 1 launch in --profile-every per class over the "
              "timed region: the dispatch-inclusive duration rocprofv3 --kernel-trace reports (DESIGN.md 5)",
    "classes": "roofline_step.classes[k] = [" + ", ".join(CLASS_FIELDS) + "]; frac = algorithmic bytes/launch / avg_us / 8 TB/s",
    "algorithmic_bytes": "each operand word read once, each result word written once (DESIGN.md 5); roofline_step.frac = "
                         "all launches' bytes / wall time / 8 TB/s",
    "traffic": "roofline.traffic = rocprofv3 --pmc HBM-side bytes / algorithmic bytes of the class x this launch's bytes",
    "precision": "max angular error of any state slot vs its Zeta16 codeword over all stages of one encrypt; margin pi/16",
    "parity": "every timed output of every leg decoded and checked against FIPS-197 AES after the timed region; residues "
              "bit-exact vs the C oracle in tests/",
    "evaluation": "deferred relin/rescale, fused LUT kernels, batched key switches, periodic layout + sparse bootstraps (DESIGN.md 3-4)",
}


def _sig(x, n: int = 4):
    """x rounded to n significant digits (floats only; ints and None unchanged)"""
    if isinstance(x, bool) or x is None or isinstance(x, int):
        return x
    if isinstance(x, float):
        if x == 0.0 or x != x:
            return x
        from math import floor, log10
        return float(round(x, n - 1 - int(floor(log10(abs(x))))))
    return x


def _compact_classes(rs: dict) -> dict:
    out = {}
    per_step = rs.get("launches_per_step_by_class", {})
    for k, c in (rs.get("classes") or {}).items():
        out[k] = [_sig(c.get("frac"), 3), _sig(c.get("avg_us"), 4), _sig(c.get("avg_us_span"), 4), _sig(c.get("avg_us_gap"), 3),
                  _sig(c["bytes_per_launch"] / 1e6 if c.get("bytes_per_launch") else None, 4), _sig(per_step.get(k), 5)]
    return out


def _traffic_ratios(rs: dict | None) -> dict:
    return {k: _sig(c.get("traffic_over_algorithmic"), 3) for k, c in ((rs or {}).get("classes") or {}).items()
            if c.get("traffic_over_algorithmic")}


def _compact_step(rs: dict | None, classes: bool = True) -> dict | None:
    if not rs:
        return None
    out = {"frac": _sig(rs.get("frac"), 4), "achieved_GBs": _sig(rs.get("achieved"), 5),
           "GB_per_step": _sig(rs.get("algorithmic_bytes_per_step", 0) / 1e9, 5), "launches_per_step": _sig(rs.get("launches_per_step"), 6)}
    if classes:
        out["classes"] = _compact_classes(rs)
    return out


def _compact_roof(r: dict | None) -> dict | None:
    if not r:
        return None
    keep = ("kernel", "bound", "achieved", "peak", "unit", "frac", "traffic", "traffic_over_algorithmic", "avg_us", "avg_us_span",
            "avg_us_gap", "frac_span", "bytes_per_launch", "timed_launches", "butterflies_per_launch")
    return {k: _sig(r[k], 5) for k in keep if k in r}


def _compact_precision(p: dict | None) -> dict | None:
    if not p:
        return None
    return {"margin_factor": _sig(p.get("margin_factor"), 3), "max_err_rad": _sig(p.get("max_slot_angle_error_rad"), 3),
            "worst_stage": p.get("worst_stage"), "log2_delta_fresh": _sig(p.get("log2_delta_fresh"), 4),
            "slots_per_stage": p.get("state_slots_per_stage"), "stages": p.get("stages_checked")}


def _compact_leg(d: dict) -> dict:
    """one secondary leg: its throughput, verification, step roofline (with per-class arrays), precision"""
    num = ("blocks_per_s", "rounds_per_s", "ms_per_step", "ms_per_pair", "steps", "pairs_per_rank", "states_per_pair",
           "pairs_per_stack", "states_per_rank_per_step", "bootstraps_per_encrypt", "launches_per_encrypt", "delta_vs_strict",
           "secret_key_renorms_per_encrypt")
    out = {k: _sig(d[k], 5) for k in num if k in d}
    out["verified"] = d.get("verified_against_plaintext_model")
    if d.get("folds") is not None:
        out["folds"] = d["folds"]
    if d.get("roofline_step") is not None:
        out["roofline_step"] = _compact_step(d.get("roofline_step"))
    if d.get("precision"):
        out["precision"] = _compact_precision(d["precision"])
    rt = d.get("roundtrip")
    if rt:
        out["roundtrip"] = {"states_per_rank": rt.get("states_per_rank"),
                            "roundtrip_blocks_per_s": _sig(rt.get("roundtrip_blocks_per_s"), 5),
                            "enc_ms_per_step": _sig(rt.get("enc_ms_per_step"), 5), "dec_ms_per_step": _sig(rt.get("dec_ms_per_step"), 5),
                            "bit_exact": rt.get("roundtrip_bit_exact"),
                            "roofline_step_dec": _compact_step(rt.get("roofline_step_dec"))}
    return out


LEG_NOTES = {
    "batch": "C3/C4 shape: --batch-states states per GPU slot-packed in one ciphertext pair, full encrypt",
    "batch.roundtrip": "C5: enc->dec round trip of --c5-states states split over the ranks, bit-exact check",
    "batch_pairs": "C3 literally: --pair-states one-state ciphertext pairs per GPU, stacked --pair-stack per operand",
    "batch_packed_pairs": "--packed-pairs slot-packed pairs of 2048 states stacked into one operand",
    "folded": "C2 with the renorm folds on (ShiftRows / conjugations / pack / unpack computed inside the secret-key renorm): "
              "NOT REF's workload; delta_vs_strict against the headline value, whose renorms are the identity on the message",
    "true_fhe": "C2 with every secret-key renorm replaced by bootstrap + homomorphic Zeta16 snap",
    "eager_ref_calls": "C2 via EngineContext with REF's call sequence, eager relin/rescale, reference slot layout",
    "deferred_ref_calls": "C2 via EngineContext with REF's call sequence (per-term loops), deferred evaluation on",
}
LEG_KEYS = ("batch", "folded", "batch_pairs", "batch_packed_pairs", "true_fhe", "eager_ref_calls", "deferred_ref_calls")


def compact_line(full: dict, detail_path: str | None = None) -> dict:
    """The driver's stdout line from the full bench record: every contract key, the roofline /
    roofline_step / cpu_baseline objects as numbers, each leg's value and step fraction, and the
    prose once under `notes` (VERDICT r4 'do this' 1: <= 12 KB)."""
    line = {k: full[k] for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                                 "scaling", "vs_baseline", "dtype", "data") if k in full}
    line["value"] = _sig(line.get("value"), 6)
    line["ms_per_step"] = _sig(line.get("ms_per_step"), 6)
    cfg = full.get("config", {})
    line["config"] = {k: cfg[k] for k in ("workload", "log_n", "params", "states_per_rank_per_step", "parallelism", "blocks_per_s",
                                          "verified_against_plaintext_model") if k in cfg}
    line["config"]["blocks_per_s"] = _sig(line["config"].get("blocks_per_s"), 6)
    r = _compact_roof(full.get("roofline"))
    if r is not None:
        r["traffic_source"] = "see notes.traffic_source"
    line["roofline"] = r
    line["roofline_secondary"] = _compact_roof(full.get("roofline_secondary"))
    line["roofline_valu"] = _compact_roof(full.get("roofline_valu"))
    line["roofline_step"] = _compact_step(full.get("roofline_step"))
    if line["roofline_step"]:
        line["roofline_step"]["traffic_over_algorithmic"] = _traffic_ratios(full.get("roofline_step"))
    line["launches_per_encrypt"] = _sig(full.get("launches_per_encrypt"), 6)
    if full.get("secret_key_renorms_per_encrypt") is not None:
        line["secret_key_renorms_per_encrypt"] = {k: _sig(v, 5) for k, v in full["secret_key_renorms_per_encrypt"].items()}
    line["precision"] = _compact_precision(full.get("precision"))
    for k in LEG_KEYS:
        if full.get(k) is not None:
            line[k] = _compact_leg(full[k])
    cb = full.get("cpu_baseline")
    if cb:
        line["cpu_baseline"] = {k: _sig(cb[k], 5) if k != "sample" else cb[k] for k in
                                ("value", "unit", "cores", "kind", "value_kind", "value_measured_no_boot", "sample", "c1_ark_s", "c2_round_s",
                                 "c2_round_no_boot_s", "c2_boot_modeled_s") if k in cb}
    notes = dict(NOTES)
    ts = (full.get("roofline") or {}).get("traffic_source")
    if ts:
        notes["traffic_source"] = ts
    notes["legs"] = {k: v for k, v in LEG_NOTES.items() if full.get(k.split(".")[0]) is not None}
    line["notes"] = notes
    if detail_path:
        line["detail_file"] = detail_path
    return line


def emit_line(full: dict, detail_path: str | None) -> str:
    """write the full record to detail_path (if given) and return the compact stdout line; a line that
    would exceed LINE_MAX_BYTES drops the per-class arrays of the secondary legs, then the notes"""
    if detail_path:
        try:
            p = Path(detail_path)
            p.parent.mkdir(parents=True, exist_ok=True)
            p.write_text(json.dumps(full, indent=1))
        except OSError as e:  # a read-only tree must not lose the line
            print(f"[bench] detail file not written: {e}", file=sys.stderr)
            detail_path = None
    line = compact_line(full, detail_path)
    s = json.dumps(line)
    if len(s) > LINE_MAX_BYTES:
        for k in LEG_KEYS:
            for rs in (line.get(k, {}).get("roofline_step"), (line.get(k, {}).get("roundtrip") or {}).get("roofline_step_dec")):
                if rs:
                    rs.pop("classes", None)
        s = json.dumps(line)
    if len(s) > LINE_MAX_BYTES:
        line["notes"] = {"see": detail_path}
        s = json.dumps(line)
    return s


def dry_run(args, rank, world, dist):
    """The N > 1 host path with a real engine per rank, on CPU: one oracle CKKS engine per rank
    (oracle/ckks_cpu.py, N = 2^13) keyed by the broadcast seed, AddRoundKey on the rank's own
    states under one shared round key, decoded and checked per rank."""
    from add_round_key import AddRoundKey, default_xor4_coeffs
    from oracle.ckks_cpu import OracleContext
    from state_encoder import StateEncoder
    from xor4_lut import XOR4LUT
    seed = shared_seed(dist, args.seed)
    ctx = OracleContext(log_n=13, max_level=6, seed=seed)
    enc = StateEncoder(ctx)
    ark = AddRoundKey(XOR4LUT(ctx, default_xor4_coeffs()))
    np.random.seed(7)
    key = np.random.randint(0, 256, 16, dtype=np.uint8)
    states = rank_states(rank, args.warmup + args.steps)
    kc = enc.encode(key)
    for i in range(args.warmup):
        ark(*enc.encode(states[i]), *kc)
    barrier(dist)
    t0 = time.perf_counter()
    outs = [ark(*enc.encode(states[i]), *kc) for i in range(args.warmup, args.warmup + args.steps)]
    barrier(dist)
    elapsed = max_over_ranks(dist, time.perf_counter() - t0)
    ok = all(np.array_equal(enc.decode(*o), states[args.warmup + j] ^ key) for j, o in enumerate(outs))
    sk = ctx.eng.p.secret()
    fp = int(np.bitwise_xor.reduce((sk[:64].astype(np.int64) + 2) * np.arange(1, 65)))  # secret-key fingerprint
    # the sharding of the batch legs (no engine work): each rank's own C3/C4 batch and C5 share, the
    # same functions run_batch uses -- digests show the ranks' inputs are distinct
    import zlib
    B5 = c5_states_per_rank(args.c5_states, world)
    batches, ins5 = batch_inputs(rank, max(1, args.batch_states), args.batch_steps, B5)
    c5_in = ins5[1:] if ins5 is not None else batches[1:]
    dig = lambda arrs: zlib.crc32(b"".join(a.tobytes() for a in arrs))  # noqa: E731
    rows = all_gather_ints(dist, [int(states[args.warmup][0]), int(ok), fp, B5, int(c5_in[0].shape[0]), dig(batches[1:]),
                                  dig(c5_in)])
    if rank == 0:
        print(json.dumps({"metric": "homomorphic AES-128 rounds/sec (enc) at N=2^16", "value": None, "dry_run": True,
                          "engine": "CPU oracle per rank (N=2^13, AddRoundKey)", "n_gpus": world, "steps": args.steps,
                          "warmup": args.warmup, "elapsed_max_s": elapsed,
                          "first_byte_per_rank": [r[0] for r in rows], "ark_exact_per_rank": [bool(r[1]) for r in rows],
                          "same_keys_on_every_rank": len({r[2] for r in rows}) == 1, "outputs": len(outs) * world,
                          "key_fingerprints": sorted({r[2] for r in rows}),
                          "c5_states_per_rank": [r[3] for r in rows], "c5_input_rows_per_rank": [r[4] for r in rows],
                          "c5_states_total": sum(r[4] for r in rows),
                          "batch_digest_per_rank": [r[5] for r in rows], "c5_digest_per_rank": [r[6] for r in rows]}),
              flush=True)
    if dist is not None:
        dist.destroy_process_group()


def main():
    args = parse()
    rank, world, local, dist = dist_setup(args.gpus)
    if args.dry_run:
        return dry_run(args, rank, world, dist)

    from aes_keyschedule import expand_aes128_key, load_all_coeffs
    from engine_context import EngineContext
    from mixcol_final import MixColFinal
    from oracle import aes_plain  # checker only: verifies the ciphertext after the timed region
    from pipeline import AESPipeline
    from xor4_lut import XOR4LUT

    coeffs = load_all_coeffs()
    signature = 2 if args.no_final_bootstrap else 1
    seed = shared_seed(dist, args.seed)  # one key set for every rank (broadcast once, untimed)
    ctx = EngineContext(signature=signature, max_level=17, thread_count=1, device_id=local, seed=seed, lazy=not args.eager,
                        concurrent=args.concurrent and not args.serial, boot_fresh_level=args.fresh_level, dnum=args.dnum)
    xor4 = XOR4LUT(ctx, coeffs["xor4"])
    from state_encoder import SlotLayout
    layout = SlotLayout(ctx.engine.slot_count, 1, periodic=not args.ref_layout)
    mix = MixColFinal(ctx, xor4, layout=layout)
    if args.no_final_bootstrap:
        mix = _NoFinalBootstrap(mix)
    pipe = AESPipeline(ctx, coeffs, mixcolumns=mix, use_hard_renorm_between_steps=True, periodic=layout.periodic)

    np.random.seed(7)
    key = np.random.randint(0, 256, 16, dtype=np.uint8)
    rks = expand_aes128_key(key)
    states = rank_states(rank, args.warmup + args.steps)

    E = ctx.engine
    _progress(ctx)
    for i in range(args.warmup):
        pipe.encrypt(states[i], rks)
    E.sync()
    import mi355x_ckks
    tj = json.loads(Path(args.traffic_json).read_text()) if args.traffic_json and Path(args.traffic_json).exists() else {}
    every = 1 if args.profile_all else args.profile_every
    # the sampled kernel classes (PROF_KIDS: the roofline kernels and the per-class fractions)
    kernels = list(mi355x_ckks.KERNEL_IDS) if args.profile_all else list(dict.fromkeys([args.kernel, args.kernel2] + PROF_KIDS))
    # --whole-stats: the launch sequence of a rocprofv3 --pmc pass (no sampled profiler, no precision
    # pass).  With AESFHE_PROFILE_FROM_START the engine's accounting of every launch since start-up is
    # written there (the algorithmic bytes of the counter pass's launches); without it (the counter pass
    # itself: no in-kernel timestamps under the counters) nothing is written
    whole = bool(args.whole_stats)
    account = whole and bool(os.environ.get("AESFHE_PROFILE_FROM_START"))
    pre = {}
    if whole:  # whole-process accounting: keep the from-start configuration, fold the pre-timed part in
        pre = E.kernel_stats(reset=True) if account else {}
    else:
        E.profile(kernels, every=every)
        # one profiled, untimed encrypt allocates the profiler's clock slots outside the timing
        pipe.encrypt(states[0], rks)
        E.sync()
    E.reset_counters()

    outs = []
    E.sync()
    empty_pools(E)
    leg = Leg(E).start() if not whole else None
    barrier(dist)
    # AESFHE_MARK_TIMED=1: a 250 ms idle gap on each side of the timed region (outside the timing),
    # so tools/trace_window.py can pick the timed launches out of a rocprofv3 kernel trace
    mark = os.environ.get("AESFHE_MARK_TIMED") == "1"
    if mark:
        time.sleep(0.25)
    from utils import FOLDS, RENORM_TALLY
    alg0, launches0 = mi355x_ckks.alg_bytes(), mi355x_ckks.launch_count()
    ren0 = dict(RENORM_TALLY)
    t0 = time.perf_counter()
    for i in range(args.warmup, args.warmup + args.steps):
        outs.append(pipe.encrypt(states[i], rks))
    E.sync()
    barrier(dist)
    elapsed = time.perf_counter() - t0
    alg1, launches1 = mi355x_ckks.alg_bytes(), mi355x_ckks.launch_count()
    renorms = {"ciphertexts": (RENORM_TALLY["ciphertexts"] - ren0["ciphertexts"]) / args.steps,
               "calls": (RENORM_TALLY["calls"] - ren0["calls"]) / args.steps,
               "reference_pairs": 48, "reference_ciphertexts": 96, "strict": not FOLDS.any}
    if mark:
        time.sleep(0.25)
    counters = E.counters()
    if account:
        stats = E.kernel_stats(reset=True)
        tot = {k: {f: pre.get(k, {}).get(f, 0) + v.get(f, 0) for f in ("launches", "ms", "bytes")} for k, v in stats.items()}
        Path(args.whole_stats).write_text(json.dumps(tot, indent=1))
    elif not whole:
        leg.stop()
    elapsed = max_over_ranks(dist, elapsed)
    launches_per_encrypt = (launches1 - launches0) / args.steps
    # (a --whole-stats run skips it: its rocprofv3 --pmc pass must count exactly the accounted launches)
    precision = measure_precision(pipe, ctx, rks, states[0], "one C2 state") if rank == 0 and not whole else None

    batch = run_batch(ctx, coeffs, rks, args, rank, world, dist, tj) if args.batch_states > 0 else None
    pairs_c3 = run_pairs(ctx, coeffs, rks, args, rank, world, dist, args.pair_states, 1, max(1, args.pair_stack), args.pair_steps,
                         f"C3 literally: {args.pair_states} ciphertext pairs (hi/lo) per GPU with ONE state each "
                         f"(REF/state_encoder.py:17-28), stacked {args.pair_stack} pairs per operand (DESIGN.md 3.16), full "
                         f"AES-128 encrypt, N=2^16, renorm on, shared key", tj) if args.pair_states > 0 else None
    pairs_packed = run_pairs(ctx, coeffs, rks, args, rank, world, dist, args.packed_pairs, 2048, args.packed_pairs,
                             args.packed_pair_steps,
                             f"{args.packed_pairs} x 2048 states per GPU: {args.packed_pairs} slot-packed ciphertext pairs stacked "
                             f"into one operand (DESIGN.md 3.9 + 3.16), full AES-128 encrypt, N=2^16, renorm on, shared key",
                             tj) if args.packed_pairs > 0 else None
    folded = (run_folded(ctx, coeffs, rks, args, rank, world, dist, layout, 10.0 * args.steps * world / elapsed)
              if args.folded_steps > 0 and not args.no_final_bootstrap and not whole else None)
    true_fhe = (run_true_fhe(ctx, coeffs, rks, args, rank, world, dist, tj)
                if args.true_fhe_steps > 0 and not args.no_final_bootstrap else None)
    E.profile(())
    eager = run_ref_calls(coeffs, rks, args, rank, world, dist, local, seed, tj, lazy=False) if args.eager_steps > 0 else None
    deferred = run_ref_calls(coeffs, rks, args, rank, world, dist, local, seed, tj, lazy=True) if args.deferred_steps > 0 else None

    # correctness of the timed outputs (outside the timed region)
    ok = all(np.array_equal(pipe.encoder.decode(*o), aes_plain.ref_encrypt(states[args.warmup + j], rks))
             for j, o in enumerate(outs))
    ok = all(r[0] for r in all_gather_ints(dist, [int(ok)]))  # every rank's outputs verified

    states_done = args.steps * world
    value = 10.0 * states_done / elapsed
    if whole:
        roof = dict(roofline=None, roofline_secondary=None, roofline_valu=None, roofline_step=None)
    else:
        roof = dict(
            roofline=leg.roofline(args.kernel, tj, every, "dominant kernel by time (NTT pass 2 incl. fused rescale/ModDown "
                                                          "epilogue); VALU / latency-bound: ~11.8 VALU instructions per lazy "
                                                          "butterfly, u32 multiplies at full rate (DESIGN.md 5)"),
            roofline_secondary=leg.roofline(args.kernel2, tj, every, "key-switch inner product: HBM-bound"),
            roofline_valu=leg.valu_roofline(args.kernel),
            # whole-step roofline: algorithmic bytes of EVERY launch of the timed steps
            roofline_step=leg.step(elapsed, args.steps, tj, every))

    line = {
        "metric": "homomorphic AES-128 rounds/sec (enc) at N=2^16",
        "value": value,
        "unit": "rounds/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32 (RNS residues, 30-bit primes; CKKS scale Delta ~ 2^29.9 on the single-prime levels, see precision)",
        "data": "synthetic random 16-byte states, FIPS key schedule of a seed-7 master key",
        "config": {"workload": "C2: full AES-128 encrypt (10 rounds), 1 packed state per ciphertext pair, "
                               "N=2^16, renorm on (strict: every secret-key renorm the identity on the message, as REF's)" + ("" if not args.no_final_bootstrap else ", FINAL BOOTSTRAP SKIPPED"),
                   "log_n": 16, "states_per_rank_per_step": 1, "parallelism": f"replicas x{world}",
                   "params": {"fresh_level": ctx.engine.fresh_level, "dnum": ctx.engine.dnum, "log2_pq": round(ctx.engine.log_pq, 1),
                              "top_limbs": int(ctx.engine.level_limbs[-1]), "security_bound_log2_pq": 1772},
                   "slot_layout": ("reference (byte i at slot i*N/32; full-slot bootstraps)" if args.ref_layout else
                                   "periodic (the 16-slot state block repeated; MixColumns' final bootstraps as "
                                   "sparse-slot bootstraps, DESIGN.md 4b)"),
                   "evaluation": "eager (relinearise + rescale after every product)" if args.eager else
                   ("optimised evaluation, same module interfaces and outputs: deferred relinearisation/rescale "
                    "(DESIGN.md 3.7), fused LUT kernels with one relinearisation per LUT, XOR4/GF LUTs over a conjugate "
                    "split, SubBytes by baby-step giant-step (3.8), XOR chain as a tree (6), hoisted column rotations, "
                    "inputs dropped to the renorm floor before renormalised steps (3.11), batched products (3.12); "
                    "the engine op counts per round are in op_counts_per_round; REF's own call sequence through the "
                    "same engine is the eager_ref_calls leg"),
                   "blocks_per_s": states_done / elapsed, "verified_against_plaintext_model": bool(ok)},
        "parity": "decoded bytes verified against FIPS-197 AES (oracle/aes_plain.py) for every timed output of every leg; "
                  "engine residues bit-exact against the C oracle (oracle/ckks_oracle.c) in tests/test_gpu_parity.py; "
                  "raw-ciphertext parity with the reference's desilofhe engine is unpinnable (closed binary, absent)",
        **roof,
        "launches_per_encrypt": launches_per_encrypt,
        # secret-key renorms (decrypt -> snap -> re-encrypt) per encrypt, in ciphertexts; REF: 48 pairs
        # (REF/pipeline.py:123-188).  strict: every renorm is the identity on the message (utils.RenormFolds)
        "secret_key_renorms_per_encrypt": renorms,
        "precision": precision,
        "op_counts_per_round": {k: v / (10.0 * args.steps) for k, v in counters.items()},
    }
    if batch is not None:
        line["batch"] = batch
    if pairs_c3 is not None:
        line["batch_pairs"] = pairs_c3
    if pairs_packed is not None:
        line["batch_packed_pairs"] = pairs_packed
    if folded is not None:
        line["folded"] = folded
    if true_fhe is not None:
        line["true_fhe"] = true_fhe
    if eager is not None:
        line["eager_ref_calls"] = eager
    if deferred is not None:
        line["deferred_ref_calls"] = deferred
    if rank == 0:
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(coeffs, boot_tallies(ctx, 2 * layout.period if layout.periodic else None))
        print(emit_line(line, args.detail_json or None), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
