"""CPU baseline on the C oracle (oracle/ckks_oracle.c through oracle/ckks_cpu.OracleContext,
OpenMP over OMP_NUM_THREADS host threads), measured, not extrapolated:

  C1  BASELINE config 1 in full: AddRoundKey (2 XOR4 LUTs) on one state at N = 2^15
      (REF/main.py:44-69: np.random.seed(0), state then key);
  C2  one middle round r = 1 of the C2 encrypt at N = 2^16 (SubBytes, renorm, ShiftRows,
      MixColumns, AddRoundKey, renorm; REF/pipeline.py:142-151) with the build's AES modules
      in the reference's per-term product form (the oracle has no fused LUT op), the
      MixColumns final bootstrap timed apart by boot_replay (its work replayed on the oracle).

Prints one JSON object; bench.py's cpu_baseline leg runs C1 and the C2 SubBytes step (a
bounded sample) and tools/cpu_round.py --full the whole middle round (profiles/)."""
from __future__ import annotations

import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
for _p in (str(ROOT), str(ROOT / "aes-implementation-fhe_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)


def threads() -> int:
    return int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))


def c1(coeffs) -> dict:
    """config 1 in full: ARK = XOR4(hi, k_hi), XOR4(lo, k_lo) at N = 2^15, checked"""
    from add_round_key import AddRoundKey
    from oracle.ckks_cpu import OracleContext
    from state_encoder import StateEncoder
    from xor4_lut import XOR4LUT
    ctx = OracleContext(log_n=15, max_level=17, seed=7)
    enc = StateEncoder(ctx)
    ark = AddRoundKey(XOR4LUT(ctx, coeffs["xor4"]))
    np.random.seed(0)
    state = np.random.randint(0, 256, 16, dtype=np.uint8)
    key = np.random.randint(0, 256, 16, dtype=np.uint8)
    s, k = enc.encode(state), enc.encode(key)
    ark(*s, *k)  # warm: key-switching keys
    t0 = time.perf_counter()
    out = ark(*s, *k)
    dt = time.perf_counter() - t0
    return {"ark_s": dt, "exact": bool(np.array_equal(enc.decode(*out), state ^ key))}


def c2_round(coeffs, full: bool = True) -> dict:
    """one middle round at N = 2^16 (full) or only its SubBytes + renorm step (sample)"""
    from aes_keyschedule import expand_aes128_key
    from mixcol_final import MixColFinal
    from oracle import aes_plain
    from oracle.ckks_cpu import OracleContext
    from pipeline import AESPipeline
    ctx = OracleContext(log_n=16, max_level=17, seed=7)
    pipe = AESPipeline(ctx, coeffs, use_hard_renorm_between_steps=True)
    mix = MixColFinal(ctx, pipe.xor4)
    np.random.seed(7)
    key = np.random.randint(0, 256, 16, dtype=np.uint8)
    pt = np.random.randint(0, 256, 16, dtype=np.uint8)
    rks = expand_aes128_key(key)
    rk = pipe._prepare_round_keys(rks)
    s0 = pt ^ rks[0]
    ct = pipe.encoder.encode(s0)
    pipe.xor4.apply(*ct[:1], *rk[1][:1])  # warm: relinearisation / conjugation keys
    steps = {}
    t = time.perf_counter()
    ct = pipe._renorm_pair(*pipe.sub_bytes(*ct))
    steps["subbytes+renorm"] = time.perf_counter() - t
    want = aes_plain.SBOX[s0]
    if full:
        t = time.perf_counter()
        ct = pipe.shift_rows(*ct)
        steps["shiftrows"] = time.perf_counter() - t
        t = time.perf_counter()
        ct = mix(*ct, do_final_bootstrap=False)
        steps["mixcolumns (no final bootstrap)"] = time.perf_counter() - t
        t = time.perf_counter()
        ct = pipe._renorm_pair(*pipe.add_round_key(*ct, *rk[1]))
        steps["addroundkey+renorm"] = time.perf_counter() - t
        want = aes_plain.ref_mix_columns(aes_plain.shift_rows(want)) ^ rks[1]
    return {"steps_s": steps, "round_s": sum(steps.values()),
            "exact": bool(np.array_equal(pipe.encoder.decode(*ct), want))}


def boot_replay(tallies: dict, level_limbs, dnum: int, log_n: int = 16) -> dict:
    """MixColumns' final bootstrap on the C oracle, as a replay of its work: the GPU engine's
    per-level tallies of one C2 final bootstrap (aesfhe_level_counters: key switches of one
    polynomial, ct x ct products, linear-transform diagonal products) and, for every (kind, level)
    that occurs, ONE such operation timed live on the oracle over the same bootstrappable chain
    (oracle.keyswitch / tensor + rescale / mul_poly on random residues and a random key: the same
    arithmetic as real data), times its count.  The oracle's key switch is the textbook one
    (ModUp, inner product, ModDown per call), so the replay does not hoist rotations that share an
    input; the oracle has no bootstrap plan of its own, so no bootstrapped ciphertext comes out --
    this times the bootstrap's work, it does not compute one."""
    from oracle.ckks_cpu import OracleParams
    limbs = [int(x) for x in level_limbs]
    L = len(limbs) - 1
    L1 = max(l for l in range(L + 1) if limbs[l] == l + 2)
    O = OracleParams(log_n=log_n, max_level=L1, dnum=dnum, seed=11, boot_double=L - L1)
    if [O.nl(l) for l in range(L + 1)] != limbs:
        raise RuntimeError("boot_replay: the oracle chain does not match the engine's limbs per level")
    n = O.n
    rng = np.random.default_rng(5)

    def rand(*shape):  # residues below every 30-bit prime of the chain
        return rng.integers(0, 1 << 29, shape, dtype=np.uint32)

    key = rand(O.dnum, 2, O.n_ks + O.n_p, n)
    O.keyswitch(0, rand(O.nl(0), n), key)  # warm: OpenMP pool, tables

    def t_ks(l):
        d = rand(O.nl(l), n)
        t = time.perf_counter()
        O.keyswitch(l, d, key)
        return time.perf_counter() - t

    def t_mul(l):
        nl = O.nl(l)
        a, b, out = rand(2, nl, n), rand(2, nl, n), np.zeros((3, nl, n), np.uint32)
        t = time.perf_counter()
        O._L.orc_tensor(O.h, l, a, b, out)
        if nl - O.nl(l - 1) == 2:
            O.rescale2(l, out[:2])
        else:
            O.rescale(l, out[:2])
        return time.perf_counter() - t

    def t_pt(l):
        # k_lin_mac forms the diagonal products in Q.P (the special primes too)
        nl = O.nl(l) + O.n_p
        pt, x = rand(nl, n), rand(2, nl, n)
        t = time.perf_counter()
        O.mul_poly(pt, x)
        return time.perf_counter() - t

    timers = {"key_switch": t_ks, "product": t_mul, "diagonal": t_pt}
    by_kind, sampled, ops = {}, 0.0, {}
    for kind, per_level in tallies.items():
        tot = 0.0
        for l, cnt in sorted(per_level.items()):
            dt = timers[kind](int(l))
            sampled += dt
            tot += dt * cnt
        by_kind[kind] = tot
        ops[kind] = int(sum(per_level.values()))
    return {"boot_s": sum(by_kind.values()), "by_kind_s": by_kind, "ops": ops, "sampled_s": sampled,
            "levels": sorted({int(l) for v in tallies.values() for l in v})}


def _heartbeat(every_s: float = 45.0):
    """stderr progress line for long runs (a silent run is taken to be hung on the GPU box)"""
    import threading
    t0 = time.perf_counter()

    def run():
        while True:
            time.sleep(every_s)
            print(f"[cpu_round] {time.perf_counter() - t0:.0f}s", file=sys.stderr, flush=True)

    threading.Thread(target=run, daemon=True).start()


def main():
    from aes_keyschedule import load_all_coeffs
    _heartbeat()
    co = load_all_coeffs()
    full = "--full" in sys.argv
    out = {"threads": threads(), "c1": c1(co), "c2": c2_round(co, full)}
    if full:
        out["c2_rounds_per_s_no_bootstrap"] = 1.0 / out["c2"]["round_s"]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
