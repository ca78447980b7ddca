"""Zeta16 nibble codec (REF/utils.py:4-19).

A nibble v is carried as the 16th root of unity ζ^v, ζ = e^{-2πi/16}; decoding reads
only the phase, so any positive real magnitude (e.g. XOR4's 256×)
decodes to the same nibble.
"""
import os

import numpy as np


class ZetaEncoder:
    @staticmethod
    def to_zeta(arr: np.ndarray, modulus: int) -> np.ndarray:
        k = np.asarray(arr) % modulus
        return np.exp(-2j * np.pi * k / modulus)

    @staticmethod
    def from_zeta(z_arr: np.ndarray, modulus: int) -> np.ndarray:
        turns = -np.angle(z_arr) * modulus / (2 * np.pi)
        return np.mod(np.rint(turns), modulus).astype(np.uint8)


# Level management for LUT steps whose result is renormalised right away:
# the renorm decrypts at any level, so such a step may run on inputs dropped to the lowest
# level that still leaves its output at RENORM_FLOOR.  Depths are those of the fused forms
# from canonical inputs (measured: fresh level 17 -> 12 for XOR4 / GF multipliers, -> 4 for
# SubBytes).
# 1 since round 6 (2 before): every renormalised step ends one level lower, so its whole evaluation runs on
# one limb fewer and the C2 set's fresh level drops to 8 (bench.py --fresh-level): C2 97.5-98.0 -> 101.9-102.3
# rounds/s, precision margin 322-360x -> 337-423x (profiles/r6_renorm_floor_ab.txt).  0 is too low for the
# fused LUT sums (the per-term loops take over: 45.5 rounds/s).  AESFHE_RENORM_FLOOR overrides (A/B runs)
RENORM_FLOOR = int(os.environ.get("AESFHE_RENORM_FLOOR", "1"))
LUT2_DEPTH = 5       # bivariate nibble LUT (XOR4, GF multipliers): basis 3 + product + coefficient
SUBBYTES_DEPTH = 13  # lift, b = hi * L(lo), baby/giant steps (sub_bytes_lut.py)
SHIFTROWS_DEPTH = 1  # masked rotations (shift_rows.py)
# the level each renorm re-encrypts at = what the step after it needs (engine renorm `level`)
NEED_XOR = RENORM_FLOOR + LUT2_DEPTH                 # an XOR4 whose result is renormalised
NEED_GF = NEED_XOR + LUT2_DEPTH                      # GF multipliers feeding such an XOR4
NEED_SUBBYTES = RENORM_FLOOR + SUBBYTES_DEPTH        # (Inv)SubBytes, then renorm
NEED_SR_MIX = NEED_GF + SHIFTROWS_DEPTH              # ShiftRows -> MixColumns
NEED_SR_ARK = NEED_XOR + SHIFTROWS_DEPTH             # ShiftRows -> AddRoundKey (last round)
NEED_ISR_ISB = NEED_SUBBYTES + SHIFTROWS_DEPTH       # InvShiftRows -> InvSubBytes
NEED_BOOTSTRAP = 0                                   # bootstrapping starts from level 0


class ConjSum:
    """s1 + conj(s2) left unsummed for a secret-key renorm that folds the conjugation into its
    decryption (aesfhe_renorm_packed_conj / _unpack_conj): a conjugate-split LUT
    whose result is renormalised right away needs no conjugation key switch.  Only the renorms
    (StateEncoder.renorm_packed / renorm_unpack) take one; conj_sum() materialises it."""
    __slots__ = ("s1", "s2")

    def __init__(self, s1, s2):
        self.s1, self.s2 = s1, s2


class RenormFolds:
    """Which AES work the secret-key renorm may fold into its decrypt -> snap -> re-encrypt.

    The reference's renorm is the identity on the message: decrypt, snap every slot to the nearest
    Zeta16 codeword, re-encrypt (REF/pipeline.py:65-69, REF/mixcol_final.py:104-106).  Each fold
    below makes the engine's renorm compute a function of the decrypted message instead:

    - ``conj``: a conjugate-split LUT's S1 + conj(S2) summed after the decryption (the reference
      conjugates by key switch, REF/xor4_lut.py:57-59);
    - ``sr``: (Inv)ShiftRows as a slot permutation of the snap (the reference rotates masked rows,
      REF/shift_rows.py:39-56);
    - ``pack``: the hi | lo packing written by the renorm's encoder (homomorphic: two mask products);
    - ``unpack``: the packed state gathered into its (hi, lo) pair by the renorm's encoder
      (homomorphic: one rotation and a mask product, StateEncoder.unpack).

    Strict (the default; the bench's headline): none of them, so every renorm is the identity on
    the message and all AES work between encryption and decryption is homomorphic.
    AESFHE_RENORM_FOLDS=1 (or ``set_all(True)``, the bench's secondary ``folded`` leg) enables
    them; AESFHE_CONJ_RENORM / AESFHE_SR_RENORM / AESFHE_PACK_RENORM / AESFHE_UNPACK_RENORM=0 then
    switch one off (A/B).  Read at call time, so a process can run both forms."""

    def __init__(self):
        self.set_all(os.environ.get("AESFHE_RENORM_FOLDS", "0") == "1")

    def set_all(self, on: bool) -> None:
        env = lambda k: os.environ.get(k, "1") != "0"  # noqa: E731
        self.conj = bool(on) and env("AESFHE_CONJ_RENORM")
        self.sr = bool(on) and env("AESFHE_SR_RENORM")
        self.pack = bool(on) and env("AESFHE_PACK_RENORM")
        self.unpack = bool(on) and env("AESFHE_UNPACK_RENORM")

    @property
    def any(self) -> bool:
        return self.conj or self.sr or self.pack or self.unpack

    def state(self):
        return (self.conj, self.sr, self.pack, self.unpack)

    def restore(self, st) -> None:
        self.conj, self.sr, self.pack, self.unpack = st


FOLDS = RenormFolds()


class renorm_folds:
    """``with renorm_folds(True): ...`` -- the folds switched for the block (bench.py's folded leg)"""

    def __init__(self, on: bool):
        self.on = on

    def __enter__(self):
        self._st = FOLDS.state()
        FOLDS.set_all(self.on)
        return FOLDS

    def __exit__(self, *exc):
        FOLDS.restore(self._st)
        return False


# Secret-key renorm tally (ciphertexts decrypted and re-encrypted; a stack of P members counts P):
# the bench reports it per encrypt beside the reference's 48 pairs (REF/pipeline.py:123-188)
RENORM_TALLY = {"calls": 0, "ciphertexts": 0}


def tally_renorm(ctx, *cts) -> None:
    RENORM_TALLY["calls"] += 1
    members = getattr(getattr(ctx, "engine", None), "members", None)
    for c in cts:
        RENORM_TALLY["ciphertexts"] += members(c) if members is not None and hasattr(c, "handle") else 1


def takes_kw(fn, *names) -> bool:
    """whether callable fn accepts every keyword in `names` (checked by signature, so a TypeError
    raised inside an evaluation is never mistaken for a missing keyword)"""
    import inspect
    try:
        params = inspect.signature(fn).parameters
    except (TypeError, ValueError):
        return False
    if any(p.kind is inspect.Parameter.VAR_KEYWORD for p in params.values()):
        return True
    return all(n in params for n in names)


def conj_sum(ctx, x):
    """a ConjSum as one ciphertext (s1 + conj(s2)); anything else unchanged"""
    return ctx.add(x.s1, ctx.conjugate(x.s2)) if isinstance(x, ConjSum) else x
# SubBytes-AddRoundKey fusion (sub_bytes_ark.py): SubBytes + the key product and its
# coefficient, then the (Inv)ShiftRows it is fused across, down to level 1 (the renorm reads
# any level; the fused step has no room for the usual floor below the fresh level 17)
SUB_ARK_DEPTH = SUBBYTES_DEPTH + 2
NEED_SUB_ARK_SR = 1 + SHIFTROWS_DEPTH + SUB_ARK_DEPTH


def drop_to(ctx, ct, level):
    """ct at `level` if it sits higher (exact-scale level drop, no rescale noise), else ct"""
    if level is None or level < 0:
        return ct
    down = getattr(ctx, "level_down", None)
    lv = getattr(ct, "level", None)
    if down is None or lv is None or lv <= level:
        return ct
    return down(ct, level)


def pair(ctx, fa, fb, shared=(), fork=False):
    """(fa(), fb()) -- the hi / lo halves of an AES step, run concurrently on two HIP streams
    when the context supports it (EngineContext.run_parallel); `shared` ciphertexts read by
    both halves are settled first.  Results are identical to the sequential order.  fork=True:
    on two streams even in a one-stream context (halves made of whole bootstraps)."""
    run = getattr(ctx, "run_parallel", None)
    if run is None:
        return fa(), fb()
    if shared:
        ctx.engine.settle(*shared)
    a, b = run(fa, fb, force=True) if fork else run(fa, fb)
    return a, b


def bootstrap2(ctx, a, b, period=None):
    """(bootstrap(a), bootstrap(b)) of the hi / lo halves (REF/mixcol_final.py:158-162): one
    batched engine bootstrap when the context has it (identical results, shared key and
    diagonal reads), else the two calls on the two branch streams.  `period`:
    the messages' slot period in the periodic layout -> the sparse-slot bootstrap (§4b)"""
    sparse = getattr(ctx, "bootstrap_pair_sparse", None)
    if period is not None and sparse is not None:
        return sparse(ctx.to_intt(a), ctx.to_intt(b), period)
    both = getattr(ctx, "bootstrap_pair", None)
    if both is not None and os.environ.get("AESFHE_BOOT_PAIR", "1") != "0":  # "0": A/B measurements
        return both(ctx.to_intt(a), ctx.to_intt(b))
    return pair(ctx, lambda: ctx.bootstrap(ctx.to_intt(a)), lambda: ctx.bootstrap(ctx.to_intt(b)))


def bootstrap1(ctx, ct, period=None):
    """bootstrap(ct); `period` < slot count: the message's slot period -> the sparse-slot bootstrap"""
    sparse = getattr(ctx.engine, "bootstrap_sparse", None)
    if period is not None and period < ctx.engine.slot_count and sparse is not None:
        return sparse(ctx.to_intt(ct), period)
    return ctx.bootstrap(ctx.to_intt(ct))


def stacked_pair(ctx, f, a, b):
    """(f(a), f(b)) for ONE function of one ciphertext applied to both halves: a and b stacked
    into a two-member operand (include/aesfhe.h aesfhe_stack), so every launch of f covers both
    halves' rows -- when the engine stacks and the halves would not fork onto
    two streams; else utils.pair.  Results identical either way (tests/test_gpu_stacked.py);
    AESFHE_STACK_HALVES=0 keeps the two separate calls (A/B runs)."""
    E = getattr(ctx, "engine", ctx)
    if _STACK_HALVES and not can_fork(ctx) and getattr(E, "stack", None) is not None:
        out = E.unstack(f(E.stack([a, b])))
        return out[0], out[1]
    return pair(ctx, lambda: f(a), lambda: f(b), shared=(a, b))


def stacked_many(ctx, f, cts):
    """[f(c) for c in cts] as ONE stacked evaluation (stacked_pair's rule for more members),
    else pairwise"""
    cts = list(cts)
    E = getattr(ctx, "engine", ctx)
    if _STACK_HALVES and not can_fork(ctx) and getattr(E, "stack", None) is not None:
        return list(E.unstack(f(E.stack(cts))))
    out = []
    for i in range(0, len(cts) - 1, 2):
        out.extend(stacked_pair(ctx, f, cts[i], cts[i + 1]))
    if len(cts) % 2:
        out.append(f(cts[-1]))
    return out


def can_fork(ctx) -> bool:
    """two independent halves would run on two streams (utils.pair): then each half batches
    its own products; otherwise both halves' products go into shared batches"""
    f = getattr(ctx, "can_fork", None)
    return bool(f()) if f is not None else False


def mul_many(ctx, pairs):
    """[ctx.multiply(a, b) for a, b in pairs] as one batched engine call when the context has
    it (identical results)"""
    pairs = list(pairs)
    f = getattr(ctx, "multiply_many", None)
    if f is not None and len(pairs) > 1:
        return f(pairs)
    return [ctx.multiply(a, b) for a, b in pairs]


def rot_many(ctx, ct, steps):
    """[ctx.rotate(ct, s) for s in steps], hoisted when the context has it (same results)"""
    steps = list(steps)
    f = getattr(ctx, "rotate_many", None)
    if f is not None and len(steps) > 1:
        return f(ct, steps)
    return [ctx.rotate(ct, s) for s in steps]


# heterogeneous batched key switch (EngineContext.rotate_multi); "0": the
# per-half hoisted rotations on the two branch streams (A/B measurements)
_MULTI = os.environ.get("AESFHE_GALOIS_MULTI", "1") != "0"
_STACK_HALVES = os.environ.get("AESFHE_STACK_HALVES", "1") != "0"


def rotate_multi(ctx, items):
    """[ctx.rotate(ct, s) for ct, s in items] -- different ciphertexts, different steps -- as ONE
    batched engine call when the context has it (same results); steps 0 return the canonical
    input (its deferred rescale shared with the batch)"""
    items = list(items)
    f = getattr(ctx, "rotate_multi", None)
    if f is not None and _MULTI and len(items) > 1:
        return f(items)
    return [ctx.rotate(ct, s) if s else ct for ct, s in items]


def rot_pair(ctx, ct_hi, ct_lo, steps):
    """(rot_many(hi, steps), rot_many(lo, steps)) -- the column shifts of both nibble halves
    (REF/mixcol_final.py:124-154) -- as one rotate_multi when available, else per half on the
    two branch streams"""
    steps = list(steps)
    if getattr(ctx, "rotate_multi", None) is not None and _MULTI:
        r = ctx.rotate_multi([(ct_hi, s) for s in steps] + [(ct_lo, s) for s in steps])
        return r[:len(steps)], r[len(steps):]
    return pair(ctx, lambda: rot_many(ctx, ct_hi, steps), lambda: rot_many(ctx, ct_lo, steps))


def conj_many(ctx, cts):
    """[ctx.conjugate(c) for c in cts], batched like mul_many"""
    cts = list(cts)
    f = getattr(ctx, "conjugate_many", None)
    if f is not None and len(cts) > 1:
        return f(cts)
    return [ctx.conjugate(c) for c in cts]


def fused_lut(ctx, key, coeffs, a, b=None, c0: complex = 0j, owner=None):
    """The LUT sum sum_{p,q} C[p,q] a[p] b[q] (b given) or c0 + sum_k C[k] a[k] as one engine
    call, or None when the context has no fused form or the elements sit too
    low for it -- the caller then runs the reference's per-term product loop.  `owner`: the
    module object holding the coefficients (the device set is evicted once it is collected)."""
    if not getattr(ctx, "fused_luts", False):
        return None
    try:
        return ctx.lut_eval(ctx.lut(key, coeffs, c0, owner=owner), a, b)
    except RuntimeError as e:
        if "level" in str(e):
            return None
        raise
