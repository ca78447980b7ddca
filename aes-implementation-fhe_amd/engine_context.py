"""EngineContext -- drop-in of the reference adapter (REF/engine_context.py:6-204) over
the MI355X engine (mi355x_ckks, a ctypes binding of libaesfhe.so).

Same constructor keywords, same methods, same error-string behaviour; the AES round
modules only ever talk to this object.  Extra keywords: ``log_n`` (N = 2^log_n, default
2^16 as in the reference harness; config 1 of BASELINE.json uses 2^15), ``dnum`` and
``seed`` (key material; drawn from ``os.urandom`` when None, pinned only by tests, smoke and
multi-rank runs that share one key set), ``lazy`` (deferred relinearisation),
``concurrent`` (hi / lo halves on two HIP streams; off by default: the batched forms
on one stream are faster), ``fused_luts`` (one-kernel LUT sums,
DESIGN.md §3.8), ``allow_insecure`` (parameter sets above the 128-bit bound, for small
test / smoke sets only) and ``enc_nonce`` (the per-process nonce of the encryption
randomness, include/aesfhe.h aesfhe_set_enc_nonce; random unless pinned).
"""
from __future__ import annotations

import hashlib
import threading
import weakref
import time

import numpy as np

from mi355x_ckks import Ciphertext, Engine, Plaintext

_SIG_DEFAULT_LEVEL = 17


class EngineContext:
    def __init__(self, signature: int, *, max_level: int = 17, use_bootstrap: bool = True,
                 use_multiparty: bool = False, mode: str = "cpu", device_id: int = 0,
                 thread_count: int | None = None, log_n: int = 16, dnum: int | None = None, seed: int | bytes | None = None,
                 lazy: bool = True, concurrent: bool = False, fused_luts: bool = True, allow_insecure: bool = False,
                 enc_nonce: int | None = None, defer_calls: bool | None = None, boot_fresh_level: int | None = None):
        # REF/engine_context.py:17-42: signature selects the engine constructor form.  boot_fresh_level
        # (an extension; REF's signature 1 takes the engine's default, 17): the fresh level of the
        # bootstrappable set -- the bootstrap's double-prime region sits above it, so a pipeline that never
        # needs more levels between its renorms / bootstraps runs every bootstrap on fewer limbs
        if signature == 1:
            kw = dict(use_bootstrap=use_bootstrap, max_level=boot_fresh_level or _SIG_DEFAULT_LEVEL)
        elif signature == 2:
            kw = dict(max_level=max_level)
        elif signature == 3:
            kw = dict(max_level=_SIG_DEFAULT_LEVEL)
        else:
            raise ValueError(f"Unsupported signature: {signature}")
        self.signature = signature
        self.engine = Engine(mode=mode, use_multiparty=use_multiparty, thread_count=thread_count or 0,
                             device_id=device_id, log_n=log_n, dnum=dnum, seed=seed, lazy=lazy,
                             concurrent=concurrent, allow_insecure=allow_insecure, enc_nonce=enc_nonce, defer_calls=defer_calls, **kw)
        eng = self.engine
        # REF/engine_context.py:44-50
        self.secret_key = eng.create_secret_key()
        self.public_key = eng.create_public_key(self.secret_key)
        self.relinearization_key = eng.create_relinearization_key(self.secret_key)
        self.conjugation_key = eng.create_conjugation_key(self.secret_key)
        self.rotation_key = eng.create_rotation_key(self.secret_key)
        self.bootstrap_key = eng.create_bootstrap_key(self.secret_key)
        self._bs_count = 0  # ciphertexts refreshed
        self._bs_calls = 0  # bootstrap calls (a pair / quad call on periodic messages: one packed bootstrap)
        self._bs_total_s = 0.0
        self.fused_luts = bool(fused_luts)
        self._init_lut_cache()

    # -------------------------------------------------------------- codec
    def encrypt(self, data: np.ndarray):
        return self.engine.encrypt(data, self.public_key)

    def decrypt(self, ct) -> np.ndarray:
        return self.engine.decrypt(ct, self.secret_key)

    def encode(self, vec: np.ndarray):
        return self.engine.encode(vec)

    # -------------------------------------------------------------- arithmetic
    def multiply(self, a, b):
        """ct x ct -> relinearised product; otherwise ct x plaintext/scalar (REF :65-68)."""
        if isinstance(a, Ciphertext) and isinstance(b, Ciphertext):
            return self.engine.multiply(a, b, self.relinearization_key)
        return self.engine.multiply(a, b)

    def add(self, a, b):
        return self.engine.add(a, b)

    def sub(self, a, b):
        return self.engine.subtract(a, b)

    def _full(self, val):
        if np.isscalar(val):
            return np.full(self.engine.slot_count, val, dtype=np.complex128)
        return np.asarray(val, dtype=np.complex128)

    def add_plain(self, ct, val):
        """Scalar or vector plaintext addition; complex values go through encode (REF :76-98)."""
        if np.iscomplexobj(val):
            return self.engine.add(ct, self.engine.encode(self._full(val)))
        try:
            return self.engine.add_plain(ct, float(val))
        except (TypeError, ValueError):
            return self.engine.add(ct, self.engine.encode(self._full(val)))

    def multiply_plain(self, ct, val):
        """Scalar (real or complex) or vector plaintext product (REF :106-125)."""
        if np.isscalar(val):
            if np.iscomplexobj(val):
                return self.engine.multiply(ct, self.engine.encode(self._full(val)))
            return self.engine.multiply(ct, float(val))
        arr = np.asarray(val)
        return self.engine.multiply(ct, self.engine.encode(arr.astype(np.complex128 if np.iscomplexobj(arr) else np.float64)))

    def make_power_basis(self, ct, degree: int):
        return self.engine.make_power_basis(ct, degree, self.relinearization_key)

    def conjugate(self, ct):
        return self.engine.conjugate(ct, self.conjugation_key)

    # batched variants (include/aesfhe.h aesfhe_mul_many / aesfhe_conjugate_many): independent
    # products / conjugations stacked into shared launches; results equal the separate calls
    def multiply_many(self, pairs):
        return self.engine.multiply_many(pairs)

    def conjugate_many(self, cts):
        return self.engine.conjugate_many(cts)

    # stacked ciphertexts (multi-pair batches, include/aesfhe.h aesfhe_stack)
    def stack(self, cts):
        """n single ciphertexts -> one stack; every op then runs on all members at once"""
        return self.engine.stack(cts)

    def unstack(self, ct):
        return self.engine.unstack(ct)

    def rotate_multi(self, items):
        """[rotate(ct, s) for ct, s in items] -- different ciphertexts, different steps -- as one
        heterogeneous batched key switch (include/aesfhe.h aesfhe_galois_multi)"""
        return self.engine.rotate_multi(items)

    def galois_multi(self, items):
        """[(ct, g)]: rotations / conjugations by Galois element, batched (aesfhe_galois_multi)"""
        return self.engine.galois_multi(items)

    def rotate_many(self, ct, steps):
        """[rotate(ct, s) for s in steps], hoisted (one ModUp)"""
        return self.engine.rotate_many(ct, steps)

    def rotate(self, ct, steps: int):
        """np.roll(slots, steps) semantics."""
        return self.engine.rotate(ct, self.rotation_key, steps)

    def relinearize(self, ct):
        """Relinearise degree-2 ciphertexts; a degree-1 ciphertext comes back as is (REF :134-145)."""
        try:
            return self.engine.relinearize(ct, self.relinearization_key)
        except RuntimeError as err:
            if "should have 3 polynomials" in str(err):
                return ct
            raise

    # -------------------------------------------------------------- bootstrap
    def bootstrap(self, ct):
        t0 = time.perf_counter()
        out = self.engine.bootstrap(ct, self.relinearization_key, self.conjugation_key, self.bootstrap_key)
        self._bs_count += 1
        self._bs_calls += 1
        self._bs_total_s += time.perf_counter() - t0
        return out

    def bootstrap_pair(self, a, b):
        """(bootstrap(a), bootstrap(b)) as one batched bootstrap of two stacked ciphertexts
        (engine-side: each key switch reads its key, each linear transform its diagonals once
        for both); the same results as two bootstrap calls"""
        t0 = time.perf_counter()
        out = self.engine.bootstrap_pair(a, b)
        self._bs_count += 2
        self._bs_calls += 1
        self._bs_total_s += time.perf_counter() - t0
        return out

    def bootstrap_pair_scaled(self, a, b, gain: float, period=None):
        """(gain * bootstrap(a), gain * bootstrap(b)), gain in (0, 1] at no extra level (the
        true-FHE renorm, zeta16_noise_reducer.BootstrapSnap); `period`: sparse-slot form"""
        t0 = time.perf_counter()
        if period is not None:
            out = self.engine.bootstrap_pair_sparse(a, b, period, gain)
        else:
            out = self.engine.bootstrap_pair_scaled(a, b, gain)
        self._bs_count += 2
        self._bs_calls += 1
        self._bs_total_s += time.perf_counter() - t0
        return out

    def bootstrap_quad_scaled(self, cts, gain: float, period: int):
        """[gain * bootstrap(c) for c in cts] for four `period`-periodic ciphertexts as ONE bootstrap
        at period 4 * period (monomial quad packing)"""
        t0 = time.perf_counter()
        out = self.engine.bootstrap_quad_sparse(cts, period, gain)
        self._bs_count += 4
        self._bs_calls += 1
        self._bs_total_s += time.perf_counter() - t0
        return out

    def bootstrap_pair_sparse(self, a, b, period: int):
        """bootstrap_pair of two messages whose slots repeat with period `period` (the periodic
        state layout, state_encoder.SlotLayout): the sparse-slot bootstrap"""
        t0 = time.perf_counter()
        out = self.engine.bootstrap_pair_sparse(a, b, period)
        self._bs_count += 2
        self._bs_calls += 1
        self._bs_total_s += time.perf_counter() - t0
        return out

    def bootstrap_stats(self):
        n = self._bs_count
        return {"count": n, "calls": self._bs_calls, "total_s": self._bs_total_s, "avg_s": self._bs_total_s / n if n else 0.0}

    def reset_bootstrap_stats(self):
        self._bs_count = 0
        self._bs_calls = 0
        self._bs_total_s = 0

    # -------------------------------------------------------------- representation
    def to_ntt(self, x):
        return self.engine.ntt(x)

    def to_intt(self, x):
        return self.engine.intt(x)

    def make_power_basis_safe(self, ct, deg):
        """Retry after INTT on an "NTT" complaint, bootstrap on a level complaint (REF :180-195)."""
        try:
            return self.engine.make_power_basis(ct, deg, self.relinearization_key)
        except RuntimeError as err:
            msg = str(err)
            if "NTT" in msg:
                return self.engine.make_power_basis(self.to_intt(ct), deg, self.relinearization_key)
            if "level" in msg or "positive" in msg:
                fresh = self.bootstrap(self.to_intt(ct))
                return self.engine.make_power_basis(fresh, deg, self.relinearization_key)
            raise

    def bootstrap_safe(self, ct):
        return self.engine.bootstrap(self.to_intt(ct), self.relinearization_key, self.conjugation_key,
                                     self.bootstrap_key)

    # -------------------------------------------------------------- MI355X extras
    def can_fork(self) -> bool:
        """whether run_parallel branches would run concurrently (False inside a branch)"""
        return self.engine.can_fork()

    def run_parallel(self, *fns, force: bool = False):
        """Independent branches (e.g. the hi and lo nibble halves of an AES step) on separate
        HIP streams; sequential when the context was built with concurrent=False, unless
        `force` (Engine.parallel)."""
        return self.engine.parallel(*fns, force=force)

    def level_down(self, ct, level: int):
        """the same message at a lower level (exact scale; used by utils.drop_to)"""
        return self.engine.level_down(ct, level)

    def renorm_pair(self, hi, lo, states: int = 1, level=None):
        """Device-side Zeta16 secret-key renorm of a (hi, lo) state pair (REF/pipeline.py:65-69);
        `states` > 1: that many slot-packed states per pair (StateEncoder);
        `level`: re-encrypt at that level instead of the fresh one."""
        return self.engine.renorm_pair(hi, lo, states, level)

    def renorm_periodic(self, hi, lo, period: int, level=None, conj=None):
        """renorm_pair for the periodic state layout (state_encoder.SlotLayout);
        conj: the pair whose conjugates are added first (hi + conj(c_hi), lo + conj(c_lo))"""
        if conj is not None:
            return self.engine.renorm_periodic(hi, lo, period, level, conj=conj)
        return self.engine.renorm_periodic(hi, lo, period, level)

    def renorm_unpack_perm(self, packed, period: int, perm, level=None, conj=None):
        """renorm_unpack with a byte permutation folded in (both halves)"""
        return self.engine.renorm_unpack_perm(packed, period, perm, level, conj=conj)

    def renorm_periodic_perm(self, hi, lo, period: int, perm, level=None, conj=None):
        """renorm_periodic with a byte permutation folded in (output slot i <- input slot perm[i])"""
        return self.engine.renorm_periodic_perm(hi, lo, period, perm, level, conj=conj)

    def renorm_pack(self, hi, lo, period: int, level=None, conj=None):
        """renorm of a period-16 state pair straight into the packed form (StateEncoder.pack's layout);
        conj: the pair whose conjugates are added first"""
        return self.engine.renorm_pack(hi, lo, period, level, conj=conj)

    def renorm_single(self, ct, level=None, period=None, conj=None):
        """renorm of one packed-state ciphertext, every slot snapped; period: the
        packed period when known (2 x the state period); conj: renormalise ct + conj(conj)"""
        if conj is not None:
            return self.engine.renorm_single(ct, level, period, conj=conj)
        return self.engine.renorm_single(ct, level, period)

    def renorm_unpack(self, packed, period: int, level=None, conj=None):
        """renorm of a packed hi | lo state (2 period-periodic) into its (hi, lo) pair;
        conj: renormalise packed + conj(conj)"""
        if conj is not None:
            return self.engine.renorm_unpack(packed, period, level, conj=conj)
        return self.engine.renorm_unpack(packed, period, level)

    def _init_lut_cache(self):
        self._luts = {}                                  # digest -> LookupTable
        self._lut_pinned = set()                         # digests requested without an owner
        self._lut_refs = {}                              # digest -> live owners holding it
        self._lut_owned = weakref.WeakKeyDictionary()    # owner -> digests it holds
        self._lut_lock = threading.RLock()               # RLock: an owner's finalizer may run in a GC pass inside the lock
        self._lut_gen = 0                                # bumped by clear_luts: older owners' finalizers do nothing

    def lut(self, key, coeffs, c0: complex = 0j, owner=None):
        """Engine-side coefficient set of a LUT polynomial, created once per coefficient CONTENT
        (a digest of the coefficients, their shape and c0).  `key` is the caller's label only: a
        label built from id() can be inherited by a new object with other coefficients once the old
        one is collected (the stale-set failure of DESIGN_HISTORY.md §B), and keying by content lets every
        module with the same set share one device copy.
        `owner` (the SubBytes / XOR4 / GF module object using the set): the set is evicted, and its
        device memory released (aesfhe_lut_free), once every owner holding it has been collected
        (weakref.finalize); sets requested without an owner stay for the context's lifetime."""
        arr = np.ascontiguousarray(coeffs, dtype=np.complex128)
        digest = hashlib.blake2b(arr.tobytes() + repr(arr.shape).encode() + np.complex128(c0).tobytes(), digest_size=16).digest()
        with self._lut_lock:
            t = self._luts.get(digest)
            if t is None:
                t = self._luts[digest] = self.engine.lut_create(coeffs, c0)
            if owner is None:
                self._lut_pinned.add(digest)
            else:
                held = self._lut_owned.get(owner)
                if held is None:
                    held = self._lut_owned[owner] = set()
                    weakref.finalize(owner, self._release_owner, weakref.ref(self), held, self._lut_gen).atexit = False
                if digest not in held:
                    held.add(digest)
                    self._lut_refs[digest] = self._lut_refs.get(digest, 0) + 1
            return t

    @staticmethod
    def _release_owner(ctx_ref, held, gen=0):
        """finalizer of a LUT owner: drop its references, evict the sets nobody holds any more.
        An owner registered before the last clear_luts (older generation) holds nothing."""
        ctx = ctx_ref()
        if ctx is None:
            return
        dead = []
        with ctx._lut_lock:
            if gen != ctx._lut_gen:
                held.clear()
                return
            for d in held:
                n = ctx._lut_refs.get(d, 0) - 1
                if n > 0:
                    ctx._lut_refs[d] = n
                    continue
                ctx._lut_refs.pop(d, None)
                if d not in ctx._lut_pinned:
                    t = ctx._luts.pop(d, None)
                    if t is not None:
                        dead.append(t)
            held.clear()
        free = getattr(ctx.engine, "lut_free", None)
        for t in dead:
            if free is not None:
                free(t)

    def lut_cache_size(self) -> int:
        with self._lut_lock:
            return len(self._luts)

    def clear_luts(self):
        """drop the cached coefficient sets (their device memory is freed with the last reference).
        Every live owner's record is emptied too and a new generation starts: an owner still
        alive from before the clear must not release (lut_free) a set that a later request made
        with the same content -- that set belongs to the new generation's owners only."""
        with self._lut_lock:
            for held in list(self._lut_owned.values()):
                held.clear()
            self._lut_owned = weakref.WeakKeyDictionary()
            self._luts.clear()
            self._lut_pinned.clear()
            self._lut_refs.clear()
            self._lut_gen += 1

    def lut_eval(self, lut, a, b=None):
        """sum C[p,q] a[p] b[q] (or c0 + sum C[k] a[k]) in one fused kernel."""
        return self.engine.lut_eval(lut, a, b)
