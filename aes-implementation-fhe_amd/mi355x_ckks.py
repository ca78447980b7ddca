"""mi355x_ckks -- ctypes binding of libaesfhe.so, the MI355X-native RNS-CKKS engine.

The classes mirror the part of ``desilofhe``'s API that the reference's adapter uses
(REF/engine_context.py:1,17-204): ``Engine``, ``Ciphertext``, ``Plaintext`` and the key
objects, with the same method names and argument meaning, so that
``engine_context.EngineContext`` is a line-for-line drop-in of the reference adapter.

There is no CPU fallback: constructing an ``Engine`` without the HIP library or without
a visible GPU raises ``RuntimeError``.
"""
from __future__ import annotations

import concurrent.futures
import os
import ctypes
import threading
import numbers
from pathlib import Path
from typing import List, Optional

import numpy as np

_PKG = Path(__file__).resolve().parent
_LIB_PATH = _PKG / "libaesfhe.so"
_lib = None

_H = ctypes.c_uint64
_Hp = ctypes.POINTER(ctypes.c_uint64)
_dp = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
_up = np.ctypeslib.ndpointer(dtype=np.uint32, flags="C_CONTIGUOUS")

EXPORTED = [
    "aesfhe_create", "aesfhe_destroy", "aesfhe_last_error", "aesfhe_keygen", "aesfhe_slot_count",
    "aesfhe_max_level", "aesfhe_set_fresh_level", "aesfhe_info", "aesfhe_moduli", "aesfhe_scales", "aesfhe_sync", "aesfhe_free",
    "aesfhe_level", "aesfhe_plaintext", "aesfhe_encrypt", "aesfhe_decrypt", "aesfhe_add", "aesfhe_sub",
    "aesfhe_add_pt", "aesfhe_add_scalar", "aesfhe_mul_scalar", "aesfhe_mul_pt", "aesfhe_mul",
    "aesfhe_relinearize", "aesfhe_rescale", "aesfhe_level_down", "aesfhe_rotate", "aesfhe_conjugate",
    "aesfhe_mul_many", "aesfhe_mul_pt_sum", "aesfhe_renorm_pool", "aesfhe_set_stack_pack", "aesfhe_conjugate_many", "aesfhe_rotate_hoisted",
    "aesfhe_power_basis", "aesfhe_to_ntt", "aesfhe_to_intt", "aesfhe_bootstrap", "aesfhe_bootstrap_pair", "aesfhe_renorm_pair", "aesfhe_renorm_states", "aesfhe_renorm_at",
    "aesfhe_export", "aesfhe_import", "aesfhe_export_secret", "aesfhe_export_pk", "aesfhe_export_ksk",
    "aesfhe_debug_ntt", "aesfhe_debug_keyswitch", "aesfhe_counters", "aesfhe_reset_counters", "aesfhe_level_counters", "aesfhe_bench_op", "aesfhe_set_lazy",
    "aesfhe_streams", "aesfhe_bind_stream", "aesfhe_fork", "aesfhe_join", "aesfhe_settle",
    "aesfhe_profile", "aesfhe_profile_every", "aesfhe_kernel_stats", "aesfhe_kernel_work", "aesfhe_kernel_gaps", "aesfhe_pool_stats", "aesfhe_bootstrap_depth", "aesfhe_debug_bootplan", "aesfhe_debug_sparseplan",
    "aesfhe_debug_boot_stage", "aesfhe_export_sparse", "aesfhe_boot_info", "aesfhe_create_boot", "aesfhe_create_keyed", "aesfhe_bootstrap_sparse", "aesfhe_bootstrap_pair_sparse", "aesfhe_bootstrap_quad_sparse", "aesfhe_renorm_periodic",
    "aesfhe_renorm_single", "aesfhe_renorm_unpack",
    "aesfhe_level_limbs", "aesfhe_debug_lin_group", "aesfhe_debug_lin_group_plain", "aesfhe_lut_create", "aesfhe_lut_eval", "aesfhe_lut_free",
    "aesfhe_bootstrap_scaled", "aesfhe_bootstrap_pair_scaled", "aesfhe_set_enc_nonce", "aesfhe_launch_count", "aesfhe_launch_census",
    "aesfhe_galois_multi", "aesfhe_debug_boot_stage_sparse", "aesfhe_debug_sparse_group", "aesfhe_debug_sparse_group_plain",
    "aesfhe_debug_mono_pack", "aesfhe_debug_mono_split", "aesfhe_alg_bytes", "aesfhe_stack", "aesfhe_unstack", "aesfhe_members",
    "aesfhe_renorm_packed", "aesfhe_renorm_packed_conj", "aesfhe_renorm_unpack_conj", "aesfhe_renorm_periodic_conj", "aesfhe_renorm_pack", "aesfhe_renorm_periodic_perm", "aesfhe_renorm_unpack_perm",
]

# largest log2(PQ) for 128-bit classical security with a ternary secret (HE standard)
SECURITY_LOG_PQ_128 = {13: 218, 14: 438, 15: 881, 16: 1772, 17: 3544}

KERNEL_IDS = ["ntt_cols_fwd", "ntt_rows_fwd", "ntt_rows_inv", "ntt_cols_inv", "base_convert", "key_inner",
              "moddown", "tensor", "rescale", "automorph", "elementwise", "sample", "lin_mac"]
# the __global__ symbol behind each kernel id (for matching rocprofv3 summaries)
KERNEL_SYMBOLS = {"ntt_cols_fwd": "k_ntt_cols_fwd", "ntt_rows_fwd": "k_ntt_rows_fwd", "ntt_rows_inv": "k_ntt_rows_inv",
                  "ntt_cols_inv": "k_ntt_cols_inv", "base_convert": "k_base_convert", "key_inner": "k_key_inner",
                  "moddown": "k_moddown_finish", "tensor": "k_tensor", "automorph": "k_automorph",
                  "lin_mac": "k_lin_mac"}

COUNTER_NAMES = ["mul", "relin", "rot", "conj", "ptmul", "scalar", "rescale", "ntt_rows", "keyswitch",
                 "encrypt", "decrypt", "bootstrap", "add", "lut"]


def load_library(path: Optional[Path] = None):
    """Load (never silently replace) the HIP engine library."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    # AESFHE_LIB: another build of the same library (A/B runs, tools/gpu_ab*.sh)
    p = Path(path) if path else Path(os.environ.get("AESFHE_LIB") or _LIB_PATH)
    if not p.exists():
        raise RuntimeError(f"MI355X engine library missing: {p} (run build_ext.py / __graft_entry__.build())")
    L = ctypes.CDLL(str(p))
    c_int, vp, c_dbl = ctypes.c_int, ctypes.c_void_p, ctypes.c_double
    pp = ctypes.POINTER(ctypes.c_void_p)
    sig = {
        "aesfhe_create": [pp, c_int, c_int, c_int, c_int, ctypes.c_uint64],
        "aesfhe_destroy": [vp], "aesfhe_keygen": [vp], "aesfhe_slot_count": [vp], "aesfhe_max_level": [vp], "aesfhe_set_fresh_level": [vp, c_int],
        "aesfhe_info": [vp, np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")],
        "aesfhe_moduli": [vp, _up], "aesfhe_scales": [vp, _dp], "aesfhe_sync": [vp], "aesfhe_free": [vp, _H],
        "aesfhe_level": [vp, _H, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32)],
        "aesfhe_plaintext": [vp, _dp, _dp, c_int, _Hp],
        "aesfhe_encrypt": [vp, _dp, _dp, c_int, _Hp],
        "aesfhe_decrypt": [vp, _H, _dp, _dp, c_int],
        "aesfhe_add": [vp, _H, _H, _Hp], "aesfhe_sub": [vp, _H, _H, _Hp], "aesfhe_add_pt": [vp, _H, _H, _Hp],
        "aesfhe_add_scalar": [vp, _H, c_dbl, c_dbl, _Hp], "aesfhe_mul_scalar": [vp, _H, c_dbl, c_dbl, _Hp],
        "aesfhe_mul_pt": [vp, _H, _H, _Hp], "aesfhe_mul": [vp, _H, _H, c_int, _Hp],
        "aesfhe_relinearize": [vp, _H, _Hp], "aesfhe_rescale": [vp, _H, _Hp],
        "aesfhe_level_down": [vp, _H, c_int, _Hp], "aesfhe_rotate": [vp, _H, c_int, _Hp],
        "aesfhe_conjugate": [vp, _H, _Hp], "aesfhe_power_basis": [vp, _H, c_int, _Hp],
        "aesfhe_mul_many": [vp, c_int, _Hp, _Hp, _Hp], "aesfhe_conjugate_many": [vp, c_int, _Hp, _Hp],
        "aesfhe_mul_pt_sum": [vp, c_int, _Hp, _Hp, _Hp], "aesfhe_renorm_pool": [vp, c_int], "aesfhe_set_stack_pack": [vp, c_int],
        "aesfhe_rotate_hoisted": [vp, _H, c_int, ctypes.POINTER(c_int), _Hp],
        "aesfhe_to_ntt": [vp, _H, _Hp], "aesfhe_to_intt": [vp, _H, _Hp], "aesfhe_bootstrap": [vp, _H, _Hp],
        "aesfhe_renorm_pair": [vp, _H, _H, _Hp, _Hp],
        "aesfhe_bootstrap_pair": [vp, _H, _H, _Hp, _Hp],
        "aesfhe_renorm_states": [vp, _H, _H, c_int, _Hp, _Hp],
        "aesfhe_renorm_at": [vp, _H, _H, c_int, c_int, _Hp, _Hp],
        "aesfhe_export": [vp, _H, _up, ctypes.c_uint64], "aesfhe_import": [vp, c_int, c_int, _up, _Hp],
        "aesfhe_export_secret": [vp, _up], "aesfhe_export_pk": [vp, _up],
        "aesfhe_export_ksk": [vp, ctypes.c_uint64, _up],
        "aesfhe_debug_ntt": [vp, _up, c_int, c_int, c_int],
        "aesfhe_debug_keyswitch": [vp, c_int, ctypes.c_uint64, _up, _up],
        "aesfhe_counters": [vp, np.ctypeslib.ndpointer(np.uint64, flags="C_CONTIGUOUS"), c_int],
        "aesfhe_bench_op": [vp, c_int, c_int, c_int, ctypes.POINTER(c_dbl)],
        "aesfhe_set_lazy": [vp, c_int],
        "aesfhe_streams": [vp], "aesfhe_bind_stream": [vp, c_int], "aesfhe_fork": [vp], "aesfhe_join": [vp], "aesfhe_settle": [vp, _H],
        "aesfhe_reset_counters": [vp],
        "aesfhe_level_counters": [vp, c_int, np.ctypeslib.ndpointer(np.uint64, flags="C_CONTIGUOUS"), c_int],
        "aesfhe_profile": [vp, ctypes.c_uint32], "aesfhe_profile_every": [vp, c_int],
        "aesfhe_kernel_stats": [vp, _dp, c_int, c_int],
        "aesfhe_kernel_work": [vp, _dp, c_int],
        "aesfhe_kernel_gaps": [vp, _dp, c_int],
        "aesfhe_pool_stats": [vp, np.ctypeslib.ndpointer(np.uint64, flags="C_CONTIGUOUS")],
    }
    sig["aesfhe_bootstrap_depth"] = []
    sig["aesfhe_bootstrap_scaled"] = [vp, _H, c_dbl, _Hp]
    sig["aesfhe_bootstrap_pair_scaled"] = [vp, _H, _H, c_dbl, _Hp, _Hp]
    sig["aesfhe_debug_bootplan"] = [c_int, _dp]
    sig["aesfhe_debug_sparseplan"] = [c_int, c_int, _dp]
    sig["aesfhe_debug_boot_stage"] = [vp, _H, c_int, _Hp]
    sig["aesfhe_export_sparse"] = [vp, _up]
    sig["aesfhe_boot_info"] = [vp, _dp]
    sig["aesfhe_debug_lin_group"] = [vp, _H, c_int, _Hp]
    sig["aesfhe_debug_lin_group_plain"] = [vp, c_int, _dp, _dp, _dp, _dp]
    sig["aesfhe_create_boot"] = [pp, c_int, c_int, c_int, c_int, ctypes.c_uint64]
    sig["aesfhe_renorm_periodic"] = [vp, _H, _H, c_int, c_int, _Hp, _Hp]
    sig["aesfhe_renorm_single"] = [vp, _H, c_int, _Hp]
    sig["aesfhe_renorm_unpack"] = [vp, _H, c_int, c_int, _Hp, _Hp]
    sig["aesfhe_bootstrap_sparse"] = [vp, _H, c_int, c_dbl, _Hp]
    sig["aesfhe_bootstrap_pair_sparse"] = [vp, _H, _H, c_int, c_dbl, _Hp, _Hp]
    sig["aesfhe_bootstrap_quad_sparse"] = [vp, _Hp, c_int, c_dbl, _Hp]
    sig["aesfhe_create_keyed"] = [pp, c_int, c_int, c_int, c_int, ctypes.c_char_p, c_int]
    sig["aesfhe_lut_create"] = [vp, c_int, c_int, _dp, _dp, c_dbl, c_dbl, _Hp]
    sig["aesfhe_lut_eval"] = [vp, _H, _Hp, _Hp, _Hp]
    sig["aesfhe_lut_free"] = [vp, _H]
    sig["aesfhe_level_limbs"] = [vp, np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")]
    sig["aesfhe_set_enc_nonce"] = [vp, ctypes.c_uint64]
    sig["aesfhe_launch_count"] = []
    sig["aesfhe_launch_census"] = [ctypes.c_char_p, ctypes.c_uint64, c_int]
    sig["aesfhe_alg_bytes"] = [_dp, np.ctypeslib.ndpointer(np.uint64, flags="C_CONTIGUOUS"), c_int]
    sig["aesfhe_galois_multi"] = [vp, c_int, _Hp, _Hp, _Hp]
    sig["aesfhe_debug_boot_stage_sparse"] = [vp, _H, c_int, c_int, _Hp]
    sig["aesfhe_debug_sparse_group"] = [vp, _H, c_int, c_int, c_int, _Hp]
    sig["aesfhe_debug_sparse_group_plain"] = [vp, c_int, c_int, c_int, _dp, _dp, _dp, _dp, np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")]
    sig["aesfhe_debug_mono_pack"] = [vp, _H, _H, c_int, _Hp]
    sig["aesfhe_debug_mono_split"] = [vp, _H, c_int, _Hp, _Hp]
    sig["aesfhe_stack"] = [vp, c_int, _Hp, _Hp]
    sig["aesfhe_unstack"] = [vp, _H, c_int, _Hp]
    sig["aesfhe_members"] = [vp, _H, ctypes.POINTER(c_int)]
    sig["aesfhe_renorm_packed"] = [vp, _H, c_int, c_int, _Hp]
    sig["aesfhe_renorm_packed_conj"] = [vp, _H, _H, c_int, c_int, _Hp]
    sig["aesfhe_renorm_periodic_conj"] = [vp, _H, _H, _H, _H, c_int, c_int, _Hp, _Hp]
    sig["aesfhe_renorm_pack"] = [vp, _H, _H, _H, _H, c_int, c_int, _Hp]
    sig["aesfhe_renorm_unpack_perm"] = [vp, _H, _H, np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS"), c_int, c_int, _Hp, _Hp]
    sig["aesfhe_renorm_periodic_perm"] = [vp, _H, _H, _H, _H, np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS"), c_int, c_int, c_int, _Hp, _Hp]
    sig["aesfhe_renorm_unpack_conj"] = [vp, _H, _H, c_int, c_int, _Hp, _Hp]
    for name in EXPORTED:
        fn = getattr(L, name)
        fn.restype = (ctypes.c_char_p if name == "aesfhe_last_error"
                      else ctypes.c_uint64 if name in ("aesfhe_launch_count", "aesfhe_launch_census") else ctypes.c_int)
        fn.argtypes = [vp] if name == "aesfhe_last_error" else sig[name]
    _lib = L
    return L


class _Context:
    """Owns one aesfhe_ctx; destroyed when the last object referring to it dies."""

    def __init__(self, log_n, max_level, dnum, device_id, seed, bootstrappable=False):
        self.lib = load_library()
        ptr = ctypes.c_void_p()
        if isinstance(seed, (bytes, bytearray)):  # the full 256-bit ChaCha20 key
            if len(seed) != 32:
                raise ValueError("a key must be 32 bytes")
            rc = self.lib.aesfhe_create_keyed(ctypes.byref(ptr), log_n, max_level, dnum, device_id, bytes(seed),
                                              int(bootstrappable))
        else:
            create = self.lib.aesfhe_create_boot if bootstrappable else self.lib.aesfhe_create
            rc = create(ctypes.byref(ptr), log_n, max_level, dnum, device_id, seed)
        self.ptr = ptr
        if rc != 0:
            msg = self.lib.aesfhe_last_error(ptr).decode() if ptr.value else "aesfhe_create failed"
            if ptr.value:
                self.lib.aesfhe_destroy(ptr)
            self.ptr = None
            raise RuntimeError(msg)

    def check(self, rc):
        if rc != 0:
            raise RuntimeError(self.lib.aesfhe_last_error(self.ptr).decode())

    def __del__(self):
        if getattr(self, "ptr", None):
            try:
                self.lib.aesfhe_destroy(self.ptr)
            except Exception:
                pass
            self.ptr = None


class _Handle:
    __slots__ = ("_ctx", "handle", "__weakref__")

    def __init__(self, ctx: _Context, handle: int):
        self._ctx = ctx
        self.handle = handle

    def __del__(self):
        ctx = getattr(self, "_ctx", None)
        if ctx is not None and ctx.ptr and self.handle:
            try:
                ctx.lib.aesfhe_free(ctx.ptr, self.handle)
            except Exception:
                pass


class Ciphertext(_Handle):
    """Device-resident RNS-CKKS ciphertext (opaque handle).  `layout`: the AES slot layout
    (state_encoder.SlotLayout) the state encoder tagged it with, unset for plain ciphertexts"""

    __slots__ = ("layout",)

    @property
    def level(self) -> int:
        lv, npoly = ctypes.c_int32(), ctypes.c_int32()
        self._ctx.check(self._ctx.lib.aesfhe_level(self._ctx.ptr, self.handle, ctypes.byref(lv), ctypes.byref(npoly)))
        return lv.value

    @property
    def num_polys(self) -> int:
        lv, npoly = ctypes.c_int32(), ctypes.c_int32()
        self._ctx.check(self._ctx.lib.aesfhe_level(self._ctx.ptr, self.handle, ctypes.byref(lv), ctypes.byref(npoly)))
        return npoly.value


class Plaintext(_Handle):
    """Encoded slot vector; encoded at the level of the ciphertext it meets.  `const`: the value
    of a constant vector (every slot equal; deferred_calls folds it into LUT coefficients)"""

    __slots__ = ("const",)


class LookupTable(_Handle):
    """Coefficient set of a fused LUT evaluation (aesfhe_lut_create)."""

    __slots__ = ("n_a", "n_b")


class _Key:
    def __init__(self, kind: str):
        self.kind = kind


class SecretKey(_Key):
    pass


class PublicKey(_Key):
    pass


class RelinearizationKey(_Key):
    pass


class ConjugationKey(_Key):
    pass


class RotationKey(_Key):
    pass


class BootstrapKey(_Key):
    pass


def _complex_vec(data, n: int):
    a = np.asarray(data)
    if a.ndim == 0:
        a = np.full(n, a.item(), dtype=np.complex128)
    a = a.astype(np.complex128, copy=False).ravel()
    if a.size > n:
        raise ValueError(f"vector of length {a.size} exceeds slot_count {n}")
    re = np.zeros(n)
    im = np.zeros(n)
    re[: a.size] = a.real
    im[: a.size] = a.imag
    return re, im


class Engine:
    """RNS-CKKS engine on one MI355X (desilofhe.Engine-shaped, REF/engine_context.py:17-39).

    ``mode`` and ``thread_count`` are accepted for API compatibility; the engine always
    runs on HIP device ``device_id``.
    """

    def __init__(self, *, mode: str = "gpu", use_bootstrap: bool = False, use_multiparty: bool = False,
                 thread_count: int = 0, device_id: int = 0, max_level: int = 17, log_n: int = 16,
                 dnum: int | None = None, seed: int | None = None, lazy: bool = True, concurrent: bool = False,
                 allow_insecure: bool = False, enc_nonce: int | None = None, defer_calls: bool | None = None):
        if use_multiparty:
            raise ValueError("multiparty key generation is not supported")
        self.mode = mode
        self.use_bootstrap = use_bootstrap
        self.device_id = int(device_id)
        # bootstrappable set: the chain is extended by the bootstrap depth above the fresh level;
        # 5 key-switching digits there (alpha = 9, 10 special primes, log2 PQ = 1699) keep log2 PQ
        # under the 128-bit bound (1772 at N = 2^16); 4 digits would cross it (1790), 6 cost
        # ~5 % more time (more ModUp rows per key switch)
        if dnum is None:
            dnum = int(os.environ.get("AESFHE_BOOT_DNUM", "5")) if use_bootstrap else 3
        # key material and encryption randomness are ChaCha20 blocks under a 256-bit key
        # (DESIGN.md §3.4): 32 bytes from the OS entropy source unless the caller pins it -- an
        # int seed (parity tests, smoke: key words 0-1) or a 32-byte key (multi-rank runs that
        # broadcast one key so every rank holds the same key set)
        if seed is None:
            seed = os.urandom(32)
        self.seed = bytes(seed) if isinstance(seed, (bytes, bytearray)) else int(seed) & 0xFFFFFFFFFFFFFFFF
        self._ctx = _Context(log_n, max_level, dnum, device_id, self.seed, bootstrappable=use_bootstrap)
        L = self._ctx.lib
        # encryption randomness has its own per-process nonce (aesfhe_set_enc_nonce): processes
        # that share the key set (multi-rank jobs) never reuse (v, e); pinned only for tests and
        # bit-exact A/B digests (AESFHE_ENC_NONCE)
        if enc_nonce is None and os.environ.get("AESFHE_ENC_NONCE"):
            enc_nonce = int(os.environ["AESFHE_ENC_NONCE"], 0)
        self.enc_nonce = (int.from_bytes(os.urandom(8), "little") if enc_nonce is None else int(enc_nonce)) & 0xFFFFFFFFFFFFFFFF
        self._ctx.check(L.aesfhe_set_enc_nonce(self._ctx.ptr, self.enc_nonce))
        self.fresh_level = max_level
        self.slot_count = int(L.aesfhe_slot_count(self._ctx.ptr))
        self.max_level = int(L.aesfhe_max_level(self._ctx.ptr))
        info = np.zeros(8, np.int32)
        self._ctx.check(L.aesfhe_info(self._ctx.ptr, info))
        self.n, self.L, self.n_q, self.n_ks, self.n_p, self.alpha, self.dnum, self.log_n = map(int, info)
        limbs = np.zeros(self.L + 1, np.int32)
        self._ctx.check(L.aesfhe_level_limbs(self._ctx.ptr, limbs))
        self.level_limbs = [int(x) for x in limbs]
        # 128-bit security (HE standard, ternary secret): log2(PQ) bound per ring dimension
        self.log_pq = float(np.log2(self.moduli().astype(np.float64)).sum())
        bound = SECURITY_LOG_PQ_128.get(self.log_n)
        if bound is not None and self.log_pq > bound and not allow_insecure:
            raise ValueError(f"parameter set above the 128-bit security bound: log2(PQ) = {self.log_pq:.1f} > {bound} "
                             f"at N = 2^{self.log_n} (allow_insecure=True for test-only sets)")
        self._keys_ready = False
        # AESFHE_PROFILE_FROM_START=kid,kid: engine kernel accounting from the first launch on
        # (key generation included), to match whole-process rocprofv3 --pmc totals (tools/ks_probe.py)
        early = os.environ.get("AESFHE_PROFILE_FROM_START")
        if early:
            self.profile([k for k in early.split(",") if k])
        self.set_lazy(lazy)
        # branches (utils.pair) on their own streams only when asked: since the batched forms of
        # round 3 (one launch for both halves' rows) one stream is faster
        # (C2 57.8 vs 53.1 rounds/s, profiles/r3_serial_ab.json).  AESFHE_CONCURRENT=1 /
        # AESFHE_SERIAL=1 force either mode for every context (A/B runs)
        env = os.environ
        self._serial = env.get("AESFHE_SERIAL") == "1"
        self.concurrent = (bool(concurrent) or env.get("AESFHE_CONCURRENT") == "1") and not self._serial
        self._pool = None
        self._tls = threading.local()
        self._defer_lock = threading.RLock()  # deferred_calls.Deferred.handle: one resolution per object
        # deferred call sequences (deferred_calls.py): products / constant products /
        # sums fused into LUT kernels, rotations and conjugations batched; AESFHE_DEFER_CALLS=0 = off
        if defer_calls is None:
            defer_calls = env.get("AESFHE_DEFER_CALLS", "1") != "0"
        self.defer = bool(defer_calls)
        self._defer_luts = {}

    # ------------------------------------------------------------------ concurrency
    def _executor(self):
        if self._pool is None:
            n_branch = int(self._ctx.lib.aesfhe_streams(self._ctx.ptr)) - 1
            ids = iter(range(1, n_branch + 1))
            lock = threading.Lock()

            def bind():
                with lock:
                    k = next(ids)
                self._tls.worker = True
                self._ctx.check(self._ctx.lib.aesfhe_bind_stream(self._ctx.ptr, k))

            self._pool = concurrent.futures.ThreadPoolExecutor(max_workers=n_branch, initializer=bind,
                                                               thread_name_prefix="aesfhe-stream")
        return self._pool

    def parallel(self, *fns, force: bool = False):
        """Run independent branches concurrently: one host thread and one HIP stream each,
        between aesfhe_fork and aesfhe_join.  Results in order; nested calls and
        concurrent=False run sequentially unless `force` (a call site whose branches are whole
        bootstraps, where two streams pay; AESFHE_SERIAL=1 still wins)."""
        if len(fns) <= 1 or not (self.concurrent or (force and not self._serial)) or getattr(self._tls, "worker", False):
            return [f() for f in fns]
        ex = self._executor()
        self._ctx.check(self._ctx.lib.aesfhe_fork(self._ctx.ptr))
        futs = [ex.submit(f) for f in fns]
        out, err = [], None
        for fu in futs:
            try:
                out.append(fu.result())
            except BaseException as e:  # join before re-raising
                err = err or e
                out.append(None)
        self._ctx.check(self._ctx.lib.aesfhe_join(self._ctx.ptr))
        if err is not None:
            raise err
        return out

    def can_fork(self) -> bool:
        """True when parallel() would really run its branches on separate streams"""
        return bool(self.concurrent) and not getattr(self._tls, "worker", False)

    def settle(self, *cts):
        """Apply deferred work of shared inputs before they are used by parallel branches."""
        for c in cts:
            self._ctx.check(self._ctx.lib.aesfhe_settle(self._ctx.ptr, c.handle))

    def set_lazy(self, on: bool):
        """Deferred relinearisation / rescale of products; False = eager."""
        self.lazy = bool(on)
        self._ctx.check(self._ctx.lib.aesfhe_set_lazy(self._ctx.ptr, int(self.lazy)))

    # ------------------------------------------------------------------ internals
    @property
    def _lib(self):
        return self._ctx.lib

    def _new(self, fn, *args, cls=Ciphertext):
        h = ctypes.c_uint64()
        self._ctx.check(fn(self._ctx.ptr, *args, ctypes.byref(h)))
        return cls(self._ctx, h.value)

    def _ensure_keys(self):
        if not self._keys_ready:
            self._ctx.check(self._lib.aesfhe_keygen(self._ctx.ptr))
            self._keys_ready = True

    # ------------------------------------------------------------------ keys
    def create_secret_key(self):
        self._ensure_keys()
        return SecretKey("secret")

    def create_public_key(self, sk=None):
        self._ensure_keys()
        return PublicKey("public")

    def create_relinearization_key(self, sk=None):
        self._ensure_keys()
        return RelinearizationKey("relin")

    def create_conjugation_key(self, sk=None):
        self._ensure_keys()
        return ConjugationKey("conj")

    def create_rotation_key(self, sk=None):
        """Rotation keys are generated on the device on first use of each rotation amount."""
        self._ensure_keys()
        return RotationKey("rotation")

    def create_bootstrap_key(self, sk=None):
        self._ensure_keys()
        return BootstrapKey("bootstrap")

    # ------------------------------------------------------------------ codec
    def encode(self, vec) -> Plaintext:
        re, im = _complex_vec(vec, self.slot_count)
        p = self._new(self._lib.aesfhe_plaintext, re, im, self.slot_count, cls=Plaintext)
        p.const = complex(re[0], im[0]) if (re == re[0]).all() and (im == im[0]).all() else None
        return p

    def encrypt(self, data, pk=None) -> Ciphertext:
        self._ensure_keys()
        re, im = _complex_vec(data, self.slot_count)
        return self._new(self._lib.aesfhe_encrypt, re, im, self.slot_count)

    def decrypt(self, ct: Ciphertext, sk=None) -> np.ndarray:
        re = np.zeros(self.slot_count)
        im = np.zeros(self.slot_count)
        self._ctx.check(self._lib.aesfhe_decrypt(self._ctx.ptr, ct.handle, re, im, self.slot_count))
        return re + 1j * im

    # ------------------------------------------------------------------ arithmetic
    # With defer_calls (the default) products, constant products, sums involving them, rotations
    # and conjugations come back as deferred ciphertexts (deferred_calls.py): the work is issued
    # when a result is needed, fused / batched.  The _raw_* forms are the undeferred calls.
    @staticmethod
    def _has_level(x) -> bool:
        """a deferred operand, or a ciphertext above level 0 (a product / non-integer constant
        product of it can be formed)"""
        from deferred_calls import Deferred
        return isinstance(x, Deferred) or x.level > 0

    @staticmethod
    def _settled(x):
        """a deferred operand that was already resolved acts as its result"""
        r = getattr(x, "_res", None)
        return r if r is not None else x

    def add(self, a, b):
        if self.defer:
            from deferred_calls import Deferred, TermSum, constant_of
            a, b = self._settled(a), self._settled(b)
            if isinstance(a, TermSum) and not isinstance(b, Ciphertext):
                c = constant_of(b)
                if c is not None:
                    return TermSum(self, a.c0 + c, a.bil, a.lin)
            if isinstance(b, Ciphertext) and (isinstance(a, Deferred) or isinstance(b, Deferred)):
                if isinstance(a, TermSum):
                    return a.plus(b)
                if isinstance(b, TermSum):
                    return b.plus(a)
                return TermSum(self, 0j, (), [(a, 1.0 + 0j, []), (b, 1.0 + 0j, [])])
        return self._raw_add(a, b)

    def _raw_add(self, a, b):
        if isinstance(b, Ciphertext):
            return self._new(self._lib.aesfhe_add, a.handle, b.handle)
        if isinstance(b, Plaintext):
            return self._new(self._lib.aesfhe_add_pt, a.handle, b.handle)
        if isinstance(b, numbers.Number):
            v = complex(b)
            return self._new(self._lib.aesfhe_add_scalar, a.handle, v.real, v.imag)
        return self._raw_add(a, self.encode(b))

    def subtract(self, a, b):
        if self.defer and isinstance(b, Ciphertext):
            from deferred_calls import Deferred, TermSum
            a, b = self._settled(a), self._settled(b)
            if isinstance(a, Deferred) or isinstance(b, Deferred):
                if isinstance(a, TermSum):
                    return a.plus(b, -1.0)
                neg = b.scaled(-1.0, -1.0) if isinstance(b, TermSum) else TermSum(self, 0j, (), [(b, -1.0 + 0j, [-1.0])])
                return neg.plus(a)
        if isinstance(b, Ciphertext):
            return self._raw_sub(a, b)
        if isinstance(b, numbers.Number):
            return self.add(a, -complex(b))
        return self.add(a, self.encode(-np.asarray(b, dtype=np.complex128)))

    def _raw_sub(self, a, b):
        return self._new(self._lib.aesfhe_sub, a.handle, b.handle)

    def add_plain(self, ct, val):
        return self.add(ct, complex(val) if np.isscalar(val) else val)

    def multiply(self, a, b, relinearization_key=None):
        if isinstance(a, (Plaintext, numbers.Number)) and isinstance(b, Ciphertext):
            a, b = b, a
        if self.defer and isinstance(a, Ciphertext):
            from deferred_calls import TermSum, constant_of
            a, b = self._settled(a), self._settled(b)
            if isinstance(b, Ciphertext):
                # a plain operand without a level to spend raises now, as the undeferred call does
                # (REF's callers see the "level" error at the call that caused it)
                if relinearization_key is not None and self._has_level(a) and self._has_level(b):
                    return TermSum(self, 0j, [(a, b, 1.0 + 0j, [])])
            else:
                c = constant_of(b)
                if c is not None:
                    if isinstance(a, TermSum):
                        return a.scaled(b, c)
                    if (c.real.is_integer() and c.imag.is_integer()) or self._has_level(a):
                        return TermSum(self, 0j, (), [(a, c, [b])])
        return self._raw_mul(a, b, relinearization_key is not None)

    def _raw_mul(self, a, b, relin: bool = True):
        if isinstance(a, Ciphertext) and isinstance(b, Ciphertext):
            return self._new(self._lib.aesfhe_mul, a.handle, b.handle, 1 if relin else 0)
        if isinstance(b, Plaintext):
            return self._new(self._lib.aesfhe_mul_pt, a.handle, b.handle)
        if isinstance(b, numbers.Number):
            v = complex(b)
            return self._new(self._lib.aesfhe_mul_scalar, a.handle, v.real, v.imag)
        return self._raw_mul(a, self.encode(b))

    # -- the deferred-call machinery's entry points (deferred_calls.py)
    def _raw(self, op, *args):
        if op == "add":
            return self._raw_add(*args)
        if op == "add_scalar":
            return self._raw_add(args[0], complex(args[1]))
        if op == "mul":
            return self._raw_mul(args[0], args[1], True)
        if op == "mul_by":
            return self._raw_mul(args[0], args[1])
        if op == "mul_many":
            return self.multiply_many(args[0])
        raise ValueError(op)

    def _raw_lut(self, C, fa, fb, c0=0j):
        """one fused LUT over the factors (bivariate: C[p, q] fa[p] fb[q]; univariate: c0 + C[k] fa[k]),
        the coefficient set created once per content"""
        from deferred_calls import lut_key
        key = lut_key(C, c0)
        t = self._defer_luts.get(key)
        if t is None:
            if len(self._defer_luts) >= 4096:  # bounded: call sites with ever-new coefficients
                for old in self._defer_luts.values():
                    self.lut_free(old)
                self._defer_luts.clear()
            t = self._defer_luts[key] = self.lut_create(C, c0)
        return self.lut_eval(t, fa, fb)

    def _gal_pending(self):
        lst = getattr(self._tls, "gal", None)
        if lst is None:
            lst = self._tls.gal = []
        return lst

    def _flush_gal(self, target):
        """resolve every live pending rotation / conjugation of this thread: one galois_multi
        (a lone one: its own undeferred call); returns target's result"""
        from deferred_calls import real
        lst = self._gal_pending()
        live = [g for g in (w() for w in lst) if g is not None and g._res is None]
        lst.clear()
        if target is not None and target not in live:
            live.append(target)
        if not live:
            return None
        if len(live) == 1:
            outs = [live[0].raw()]
        else:
            outs = self.galois_multi([(real(g.src), g.g) for g in live])
        res = None
        for g, o in zip(live, outs):
            g._res = o
            g._release_operands()
            if g is target:
                res = o
        return res

    def relinearize(self, ct, relinearization_key=None):
        return self._new(self._lib.aesfhe_relinearize, ct.handle)

    def rescale(self, ct):
        return self._new(self._lib.aesfhe_rescale, ct.handle)

    def level_down(self, ct, level: int):
        return self._new(self._lib.aesfhe_level_down, ct.handle, int(level))

    def make_power_basis(self, ct, degree: int, relinearization_key=None) -> List[Ciphertext]:
        out = (ctypes.c_uint64 * int(degree))()
        self._ctx.check(self._lib.aesfhe_power_basis(self._ctx.ptr, ct.handle, int(degree), out))
        return [Ciphertext(self._ctx, out[i]) for i in range(int(degree))]

    def conjugate(self, ct, conjugation_key=None):
        if self.defer:
            from deferred_calls import GalPending
            return GalPending(self, ct, self.galois_conj, lambda: self._new(self._lib.aesfhe_conjugate, ct.handle))
        return self._new(self._lib.aesfhe_conjugate, ct.handle)

    # batched variants (include/aesfhe.h): results equal the separate calls
    def multiply_many(self, pairs) -> List[Ciphertext]:
        """[a * b (relinearised, rescaled) for a, b in pairs] as one batched engine call"""
        pairs = list(pairs)
        n = len(pairs)
        if n == 0:
            return []
        H = ctypes.c_uint64 * n
        a, b, out = H(*[p[0].handle for p in pairs]), H(*[p[1].handle for p in pairs]), H()
        self._ctx.check(self._lib.aesfhe_mul_many(self._ctx.ptr, n, a, b, out))
        return [Ciphertext(self._ctx, out[i]) for i in range(n)]

    def renorm_pool(self, size: int = -1) -> None:
        """the renorm's pool of zero encryptions (aesfhe_renorm_pool): size per refill (0: off, the
        per-renorm encryption; -1: keep), every pool emptied"""
        self._ctx.check(self._lib.aesfhe_renorm_pool(self._ctx.ptr, int(size)))

    def set_stack_pack(self, members: int) -> None:
        """members per packed bootstrap of a stacked periodic ciphertext (aesfhe_set_stack_pack;
        1 = every member its own bootstrap)"""
        self._ctx.check(self._lib.aesfhe_set_stack_pack(self._ctx.ptr, int(members)))

    def mul_pt_sum(self, pairs) -> Ciphertext:
        """sum of ct * pt over 1..8 (ciphertext, non-constant plaintext) pairs as one engine call
        (aesfhe_mul_pt_sum: one kernel); the same value as the separate products summed"""
        pairs = list(pairs)
        n = len(pairs)
        H = ctypes.c_uint64 * n
        c = H(*[self._settled(p[0]).handle for p in pairs])
        q = H(*[p[1].handle for p in pairs])
        out = ctypes.c_uint64()
        self._ctx.check(self._lib.aesfhe_mul_pt_sum(self._ctx.ptr, n, c, q, ctypes.byref(out)))
        return Ciphertext(self._ctx, out.value)

    def rotate_many(self, ct, steps) -> List[Ciphertext]:
        """[rotate(ct, s) for s in steps] with one hoisted ModUp (np.roll semantics each)"""
        steps = [int(x) for x in steps]
        n = len(steps)
        if n == 0:
            return []
        st, out = (ctypes.c_int * n)(*steps), (ctypes.c_uint64 * n)()
        self._ctx.check(self._lib.aesfhe_rotate_hoisted(self._ctx.ptr, ct.handle, n, st, out))
        return [Ciphertext(self._ctx, out[i]) for i in range(n)]

    def galois_multi(self, items) -> List[Ciphertext]:
        """[(ct, g)] -> [ct through X -> X^g, key-switched] for odd g < 2N (aesfhe_galois_multi):
        rotations (g = galois_rotate(steps)) and conjugations (g = galois_conj) of different
        ciphertexts as one batched key switch per level; same results as the separate calls"""
        items = list(items)
        n = len(items)
        if n == 0:
            return []
        H = ctypes.c_uint64 * n
        src, gal, out = H(*[c.handle for c, _ in items]), H(*[int(g) for _, g in items]), H()
        self._ctx.check(self._lib.aesfhe_galois_multi(self._ctx.ptr, n, src, gal, out))
        return [Ciphertext(self._ctx, out[i]) for i in range(n)]

    # ---------------------------------------------------------------- stacked ciphertexts
    def stack(self, cts) -> Ciphertext:
        """n single ciphertexts -> ONE stacked ciphertext of n members (aesfhe_stack): every op
        then runs on all members at once; operands of one op are stacks of one size"""
        cts = list(cts)
        H = ctypes.c_uint64 * len(cts)
        out = ctypes.c_uint64()
        self._ctx.check(self._lib.aesfhe_stack(self._ctx.ptr, len(cts), H(*[c.handle for c in cts]), ctypes.byref(out)))
        return Ciphertext(self._ctx, out.value)

    def unstack(self, ct) -> List[Ciphertext]:
        """the members of a stack as single ciphertexts (aesfhe_unstack)"""
        n = self.members(ct)
        out = (ctypes.c_uint64 * n)()
        self._ctx.check(self._lib.aesfhe_unstack(self._ctx.ptr, ct.handle, n, out))
        return [Ciphertext(self._ctx, out[i]) for i in range(n)]

    @staticmethod
    def direct32() -> bool:
        """whether the engine's renorm has the direct period-32 codec (csrc/engine.hip direct32_: off
        with AESFHE_RENORM_DIRECT32=0, read the same way), which a slot-permuting unpack needs"""
        v = os.environ.get("AESFHE_RENORM_DIRECT32")
        if v is None:
            return True
        import re
        m = re.match(r"\s*[+-]?\d+", v)
        return not (m is None or int(m.group()) == 0)

    def members(self, ct) -> int:
        m = ctypes.c_int()
        self._ctx.check(self._lib.aesfhe_members(self._ctx.ptr, ct.handle, ctypes.byref(m)))
        return m.value

    def rotate_multi(self, items) -> List[Ciphertext]:
        """[(ct, steps)] -> [np.roll(slots(ct), steps)] as one galois_multi"""
        return self.galois_multi([(c, self.galois_rotate(s)) for c, s in items])

    def conjugate_many(self, cts) -> List[Ciphertext]:
        cts = list(cts)
        n = len(cts)
        if n == 0:
            return []
        H = ctypes.c_uint64 * n
        src, out = H(*[c.handle for c in cts]), H()
        self._ctx.check(self._lib.aesfhe_conjugate_many(self._ctx.ptr, n, src, out))
        return [Ciphertext(self._ctx, out[i]) for i in range(n)]

    def rotate(self, ct, rotation_key=None, delta: int = 0):
        """np.roll(slots, delta)."""
        if self.defer and int(delta) % self.slot_count:
            from deferred_calls import GalPending
            d = int(delta)
            return GalPending(self, ct, self.galois_rotate(d), lambda: self._new(self._lib.aesfhe_rotate, ct.handle, d))
        return self._new(self._lib.aesfhe_rotate, ct.handle, int(delta))

    def bootstrap(self, ct, relinearization_key=None, conjugation_key=None, bootstrap_key=None):
        return self._new(self._lib.aesfhe_bootstrap, ct.handle)

    def bootstrap_pair(self, a, b):
        """bootstrap(a), bootstrap(b) as one batched bootstrap (shared key / diagonal reads)"""
        x, y = ctypes.c_uint64(), ctypes.c_uint64()
        self._ctx.check(self._lib.aesfhe_bootstrap_pair(self._ctx.ptr, a.handle, b.handle, ctypes.byref(x), ctypes.byref(y)))
        return Ciphertext(self._ctx, x.value), Ciphertext(self._ctx, y.value)

    def bootstrap_scaled(self, ct, gain: float):
        """gain * bootstrap(ct), gain in (0, 1] folded into the bootstrap's level-0 scaling"""
        return self._new(self._lib.aesfhe_bootstrap_scaled, ct.handle, float(gain))

    def bootstrap_pair_scaled(self, a, b, gain: float):
        x, y = ctypes.c_uint64(), ctypes.c_uint64()
        self._ctx.check(self._lib.aesfhe_bootstrap_pair_scaled(self._ctx.ptr, a.handle, b.handle, float(gain), ctypes.byref(x),
                                                               ctypes.byref(y)))
        return Ciphertext(self._ctx, x.value), Ciphertext(self._ctx, y.value)

    def bootstrap_sparse(self, ct, period: int, gain: float = 1.0):
        """bootstrap of a message whose slots repeat with period `period` (aesfhe_bootstrap_sparse)"""
        return self._new(self._lib.aesfhe_bootstrap_sparse, ct.handle, int(period), float(gain))

    def bootstrap_pair_sparse(self, a, b, period: int, gain: float = 1.0):
        x, y = ctypes.c_uint64(), ctypes.c_uint64()
        self._ctx.check(self._lib.aesfhe_bootstrap_pair_sparse(self._ctx.ptr, a.handle, b.handle, int(period), float(gain),
                                                               ctypes.byref(x), ctypes.byref(y)))
        return Ciphertext(self._ctx, x.value), Ciphertext(self._ctx, y.value)

    def bootstrap_quad_sparse(self, cts, period: int, gain: float = 1.0):
        """four `period`-periodic ciphertexts refreshed by one bootstrap at period 4 * period
        (aesfhe_bootstrap_quad_sparse), gain * each"""
        cts = list(cts)
        if len(cts) != 4:
            raise ValueError("bootstrap_quad_sparse takes four ciphertexts")
        H = ctypes.c_uint64 * 4
        inp, out = H(*[c.handle for c in cts]), H()
        self._ctx.check(self._lib.aesfhe_bootstrap_quad_sparse(self._ctx.ptr, inp, int(period), float(gain), out))
        return [Ciphertext(self._ctx, out[m]) for m in range(4)]
    def debug_boot_stage(self, ct, stage: int):
        return self._new(self._lib.aesfhe_debug_boot_stage, ct.handle, int(stage))

    def debug_boot_stage_sparse(self, ct, stage: int, period: int):
        return self._new(self._lib.aesfhe_debug_boot_stage_sparse, ct.handle, int(stage), int(period))

    def debug_sparse_group(self, ct, period: int, which: int, pair: bool = False):
        return self._new(self._lib.aesfhe_debug_sparse_group, ct.handle, int(period), int(which), int(pair))

    def debug_sparse_group_plain(self, period: int, which: int, z: np.ndarray, pair: bool = False):
        """(host model of debug_sparse_group on the first dn slots of z, tiled; dn, #CtS groups,
        #groups)"""
        z = np.asarray(z, np.complex128)
        re, im = np.ascontiguousarray(z.real), np.ascontiguousarray(z.imag)
        ore, oim, info = np.zeros(self.slot_count), np.zeros(self.slot_count), np.zeros(3, np.int32)
        self._ctx.check(self._lib.aesfhe_debug_sparse_group_plain(self._ctx.ptr, int(period), int(which), int(pair), re, im, ore, oim,
                                                                  info))
        return ore + 1j * oim, int(info[0]), int(info[1]), int(info[2])

    def debug_mono_pack(self, a, b, period: int):
        return self._new(self._lib.aesfhe_debug_mono_pack, a.handle, b.handle, int(period))

    def debug_mono_split(self, m, period: int):
        x, y = ctypes.c_uint64(), ctypes.c_uint64()
        self._ctx.check(self._lib.aesfhe_debug_mono_split(self._ctx.ptr, m.handle, int(period), ctypes.byref(x), ctypes.byref(y)))
        return Ciphertext(self._ctx, x.value), Ciphertext(self._ctx, y.value)

    def debug_lin_group(self, ct, which: int):
        return self._new(self._lib.aesfhe_debug_lin_group, ct.handle, int(which))

    def debug_lin_group_plain(self, which: int, z: np.ndarray) -> np.ndarray:
        """bootstrap linear-transform group `which` (CoeffToSlot 0.., then SlotToCoeff) applied
        to slot values on the host: the plan model of debug_lin_group"""
        z = np.asarray(z, np.complex128)
        re, im = np.ascontiguousarray(z.real), np.ascontiguousarray(z.imag)
        ore, oim = np.zeros(self.slot_count), np.zeros(self.slot_count)
        self._ctx.check(self._lib.aesfhe_debug_lin_group_plain(self._ctx.ptr, int(which), re, im, ore, oim))
        return ore + 1j * oim

    def export_sparse(self) -> np.ndarray:
        out = np.zeros((self.n_q + self.n_p, self.n), np.uint32)
        self._ctx.check(self._lib.aesfhe_export_sparse(self._ctx.ptr, out))
        return out

    def boot_info(self) -> dict:
        self._ensure_keys()
        out = np.zeros(11)
        self._ctx.check(self._lib.aesfhe_boot_info(self._ctx.ptr, out))
        return dict(zip(["s_bt", "k1", "top", "K", "r", "deg", "d2s_log_modulus", "sparse_h", "d2s_special_primes",
                         "d2s_base_limbs", "msg_bits"], out.tolist()))

    def ntt(self, ct):
        return self._new(self._lib.aesfhe_to_ntt, ct.handle)

    def intt(self, ct):
        return self._new(self._lib.aesfhe_to_intt, ct.handle)

    def renorm_pair(self, hi, lo, states: int = 1, level=None):
        """secret-key Zeta16 renorm of a (hi, lo) pair holding `states` slot-packed AES states,
        re-encrypted at `level` (None = the fresh level)"""
        a, b = ctypes.c_uint64(), ctypes.c_uint64()
        if level is not None:
            rc = self._lib.aesfhe_renorm_at(self._ctx.ptr, hi.handle, lo.handle, int(states), int(level), ctypes.byref(a),
                                            ctypes.byref(b))
        elif states == 1:
            rc = self._lib.aesfhe_renorm_pair(self._ctx.ptr, hi.handle, lo.handle, ctypes.byref(a), ctypes.byref(b))
        else:
            rc = self._lib.aesfhe_renorm_states(self._ctx.ptr, hi.handle, lo.handle, int(states), ctypes.byref(a), ctypes.byref(b))
        self._ctx.check(rc)
        return Ciphertext(self._ctx, a.value), Ciphertext(self._ctx, b.value)

    def renorm_periodic(self, hi, lo, period: int, level=None, conj=None):
        """secret-key renorm of a pair in the periodic layout (aesfhe_renorm_periodic); conj: the
        pair (c_hi, c_lo) whose conjugates are added first (aesfhe_renorm_periodic_conj)"""
        a, b = ctypes.c_uint64(), ctypes.c_uint64()
        lv = -1 if level is None else int(level)
        if conj is not None:
            self._ctx.check(self._lib.aesfhe_renorm_periodic_conj(self._ctx.ptr, hi.handle, lo.handle, conj[0].handle, conj[1].handle,
                                                                  int(period), lv, ctypes.byref(a), ctypes.byref(b)))
        else:
            self._ctx.check(self._lib.aesfhe_renorm_periodic(self._ctx.ptr, hi.handle, lo.handle, int(period), lv, ctypes.byref(a),
                                                             ctypes.byref(b)))
        return Ciphertext(self._ctx, a.value), Ciphertext(self._ctx, b.value)

    def renorm_unpack_perm(self, packed, period: int, perm, level=None, conj=None):
        """aesfhe_renorm_unpack with a byte permutation folded in (aesfhe_renorm_unpack_perm): output byte
        i of both halves <- input byte perm[i]; conj: a conjugate partner of packed"""
        a, b = ctypes.c_uint64(), ctypes.c_uint64()
        p = np.ascontiguousarray(perm, np.int32)
        if p.shape != (16,):
            raise ValueError("renorm_unpack_perm: 16 entries")
        self._ctx.check(self._lib.aesfhe_renorm_unpack_perm(self._ctx.ptr, packed.handle, 0 if conj is None else conj.handle, p, int(period),
                                                            -1 if level is None else int(level), ctypes.byref(a), ctypes.byref(b)))
        return Ciphertext(self._ctx, a.value), Ciphertext(self._ctx, b.value)

    def renorm_periodic_perm(self, hi, lo, period: int, perm, level=None, conj=None, pack: bool = False):
        """the periodic pair renorm with a byte permutation folded in (aesfhe_renorm_periodic_perm):
        output slot i <- input slot perm[i]; conj: the pair's conjugate partners; pack: ONE packed output"""
        a, b = ctypes.c_uint64(), ctypes.c_uint64()
        c0, c1 = (0, 0) if conj is None else (conj[0].handle, conj[1].handle)
        p = np.ascontiguousarray(perm, np.int32)
        if p.shape != (16,):
            raise ValueError("renorm_periodic_perm: 16 entries")
        self._ctx.check(self._lib.aesfhe_renorm_periodic_perm(self._ctx.ptr, hi.handle, lo.handle, c0, c1, p, int(bool(pack)), int(period),
                                                              -1 if level is None else int(level), ctypes.byref(a), ctypes.byref(b)))
        if pack:
            return Ciphertext(self._ctx, a.value)
        return Ciphertext(self._ctx, a.value), Ciphertext(self._ctx, b.value)

    def renorm_pack(self, hi, lo, period: int, level=None, conj=None):
        """secret-key renorm of a period-16 state pair into ONE packed period-32 ciphertext
        (aesfhe_renorm_pack); conj: the pair (c_hi, c_lo) whose conjugates are added first"""
        c0, c1 = (0, 0) if conj is None else (conj[0].handle, conj[1].handle)
        return self._new(self._lib.aesfhe_renorm_pack, hi.handle, lo.handle, c0, c1, int(period), -1 if level is None else int(level))

    def renorm_single(self, ct, level=None, period=None, conj=None):
        """secret-key renorm of one ciphertext, every slot snapped (aesfhe_renorm_single); period:
        the message's slot period when known (aesfhe_renorm_packed: period 32 skips the FFT codec);
        conj: a ciphertext whose conjugate is added first (aesfhe_renorm_packed_conj, period needed)"""
        if conj is not None:
            if not period:
                raise ValueError("renorm_single: a conjugate partner needs the period")
            return self._new(self._lib.aesfhe_renorm_packed_conj, ct.handle, conj.handle, int(period), -1 if level is None else int(level))
        if period:
            return self._new(self._lib.aesfhe_renorm_packed, ct.handle, int(period), -1 if level is None else int(level))
        return self._new(self._lib.aesfhe_renorm_single, ct.handle, -1 if level is None else int(level))

    def renorm_unpack(self, packed, period: int, level=None, conj=None):
        """secret-key renorm of a packed hi | lo state into its (hi, lo) pair (aesfhe_renorm_unpack);
        conj: a ciphertext whose conjugate is added first (aesfhe_renorm_unpack_conj)"""
        a, b = ctypes.c_uint64(), ctypes.c_uint64()
        lv = -1 if level is None else int(level)
        if conj is not None:
            self._ctx.check(self._lib.aesfhe_renorm_unpack_conj(self._ctx.ptr, packed.handle, conj.handle, int(period), lv,
                                                                ctypes.byref(a), ctypes.byref(b)))
        else:
            self._ctx.check(self._lib.aesfhe_renorm_unpack(self._ctx.ptr, packed.handle, int(period), lv, ctypes.byref(a), ctypes.byref(b)))
        return Ciphertext(self._ctx, a.value), Ciphertext(self._ctx, b.value)

    def sync(self):
        self._ctx.check(self._lib.aesfhe_sync(self._ctx.ptr))

    # ------------------------------------------------------------------ fused LUT evaluation
    def lut_create(self, coeffs, c0: complex = 0j) -> LookupTable:
        """coeffs: (n_a, n_b) matrix of a bivariate LUT sum_{p,q} C[p,q] A_p B_q, or a vector of
        a univariate one c0 + sum_k C[k] A_k."""
        c = np.asarray(coeffs, dtype=np.complex128)
        c2 = c.reshape(c.shape[0], 1) if c.ndim == 1 else c
        re, im = np.ascontiguousarray(c2.real), np.ascontiguousarray(c2.imag)
        h = ctypes.c_uint64()
        c0 = complex(c0)
        self._ctx.check(self._lib.aesfhe_lut_create(self._ctx.ptr, c2.shape[0], c2.shape[1] if c.ndim == 2 else 1,
                                                    np.ascontiguousarray(re, np.float64), np.ascontiguousarray(im, np.float64),
                                                    c0.real, c0.imag, ctypes.byref(h)))
        t = LookupTable(self._ctx, h.value)
        t.n_a, t.n_b = c2.shape[0], (c2.shape[1] if c.ndim == 2 else 1)
        return t

    def lut_eval(self, lut: LookupTable, a, b=None) -> Ciphertext:
        """One fused kernel for the LUT sum over the element ciphertexts a[p] (b[q]); a / b are
        sequences or dicts index -> Ciphertext (missing = unused).  Raises RuntimeError with
        "level" in the message when the elements are too low for the fused form."""
        def handles(x, n):
            arr = (ctypes.c_uint64 * n)()
            items = x.items() if isinstance(x, dict) else enumerate(x)
            for k, ct in items:
                if ct is not None and 0 <= k < n:
                    arr[k] = ct.handle
            return arr
        self._ensure_keys()
        ha = handles(a, lut.n_a)
        hb = handles(b, lut.n_b) if lut.n_b > 1 else None
        return self._new(self._lib.aesfhe_lut_eval, lut.handle, ha, hb)

    def lut_free(self, lut: LookupTable):
        """release a LUT's device coefficient set now (otherwise: when the handle is collected)"""
        h, lut.handle = lut.handle, 0
        if h:
            self._ctx.check(self._lib.aesfhe_lut_free(self._ctx.ptr, h))

    # ------------------------------------------------------------------ raw access (tests)
    def moduli(self) -> np.ndarray:
        out = np.zeros(self.n_q + self.n_p, np.uint32)
        self._ctx.check(self._lib.aesfhe_moduli(self._ctx.ptr, out))
        return out

    def scales(self) -> np.ndarray:
        out = np.zeros(self.L + 1, np.float64)
        self._ctx.check(self._lib.aesfhe_scales(self._ctx.ptr, out))
        return out

    def export(self, ct: Ciphertext) -> np.ndarray:
        npoly = ct.num_polys
        out = np.zeros((npoly, self.nl(ct.level), self.n), np.uint32)
        self._ctx.check(self._lib.aesfhe_export(self._ctx.ptr, ct.handle, out, out.size))
        return out

    def import_ct(self, data: np.ndarray, level: int) -> Ciphertext:
        self._ensure_keys()
        data = np.ascontiguousarray(data, np.uint32)
        return self._new(self._lib.aesfhe_import, int(level), int(data.shape[0]), data)

    def export_secret(self) -> np.ndarray:
        self._ensure_keys()
        out = np.zeros((self.n_q + self.n_p, self.n), np.uint32)
        self._ctx.check(self._lib.aesfhe_export_secret(self._ctx.ptr, out))
        return out

    def export_pk(self) -> np.ndarray:
        self._ensure_keys()
        out = np.zeros((2, self.n_q, self.n), np.uint32)
        self._ctx.check(self._lib.aesfhe_export_pk(self._ctx.ptr, out))
        return out

    def export_ksk(self, galois: int) -> np.ndarray:
        self._ensure_keys()
        if galois == 2 * self.n + 1:  # dense -> sparse bootstrapping key: [2][q0, q1 + P' limbs][N]
            info = self.boot_info()
            out = np.zeros((1, 2, int(info["d2s_base_limbs"]) + int(info["d2s_special_primes"]), self.n), np.uint32)
        else:
            out = np.zeros((self.dnum, 2, self.n_ks + self.n_p, self.n), np.uint32)
        self._ctx.check(self._lib.aesfhe_export_ksk(self._ctx.ptr, int(galois), out))
        return out

    def debug_ntt(self, rows: np.ndarray, first_prime: int, inverse: bool = False) -> np.ndarray:
        d = np.ascontiguousarray(rows, np.uint32).copy()
        self._ctx.check(self._lib.aesfhe_debug_ntt(self._ctx.ptr, d, d.shape[0], int(first_prime), int(inverse)))
        return d

    def nl(self, level: int) -> int:
        """limbs of a ciphertext at `level` (level -1: the single bootstrapping limb)"""
        return 1 if level == -1 else self.level_limbs[level]

    def debug_keyswitch(self, level: int, galois: int, d: np.ndarray) -> np.ndarray:
        self._ensure_keys()
        out = np.zeros((2, self.nl(level), self.n), np.uint32)
        self._ctx.check(self._lib.aesfhe_debug_keyswitch(self._ctx.ptr, int(level), int(galois),
                                                         np.ascontiguousarray(d, np.uint32), out))
        return out

    def counters(self) -> dict:
        out = np.zeros(len(COUNTER_NAMES), np.uint64)
        self._ctx.check(self._lib.aesfhe_counters(self._ctx.ptr, out, len(COUNTER_NAMES)))
        return dict(zip(COUNTER_NAMES, map(int, out)))

    def reset_counters(self):
        self._ctx.check(self._lib.aesfhe_reset_counters(self._ctx.ptr))

    LEVEL_TALLIES = ("key_switch", "product", "diagonal")

    def level_counters(self) -> dict:
        """{kind: {level: count}} since reset_counters (aesfhe_level_counters): key switches of one
        polynomial, ct x ct products (their key switch under key_switch), plaintext-diagonal products"""
        out = {}
        for k, name in enumerate(self.LEVEL_TALLIES):
            v = np.zeros(64, np.uint64)
            self._ctx.check(self._lib.aesfhe_level_counters(self._ctx.ptr, k, v, 64))
            out[name] = {int(l): int(c) for l, c in enumerate(v) if c}
        return out

    BENCH_OPS = {"ntt": 0, "intt": 1, "keyswitch": 2, "rescale": 3, "mul_relin_rescale": 4}

    def bench_op(self, op: str, arg: int, iters: int = 50) -> float:
        """microseconds per back-to-back iteration of one primitive (aesfhe_bench_op)"""
        self._ensure_keys()
        us = ctypes.c_double(0.0)
        self._ctx.check(self._lib.aesfhe_bench_op(self._ctx.ptr, self.BENCH_OPS[op], int(arg), int(iters), ctypes.byref(us)))
        return us.value

    def profile(self, kernels=(), every: int = 1):
        """Enable HIP-event timing for the named kernel ids (see KERNEL_IDS); () disables.
        every > 1 times one launch in `every` of each (a live sample, less overhead)."""
        mask = 0
        for k in kernels:
            mask |= 1 << KERNEL_IDS.index(k)
        self._ctx.check(self._lib.aesfhe_profile_every(self._ctx.ptr, int(every)))
        self._ctx.check(self._lib.aesfhe_profile(self._ctx.ptr, mask))

    def kernel_work(self) -> dict:
        """butterflies of the timed NTT launches per kernel id (read before kernel_stats resets)"""
        out = np.zeros(len(KERNEL_IDS))
        self._ctx.check(self._lib.aesfhe_kernel_work(self._ctx.ptr, out, len(KERNEL_IDS)))
        return {k: float(out[i]) for i, k in enumerate(KERNEL_IDS)}

    def pool_stats(self) -> dict:
        """{"bytes": device bytes the buffer pools hold, "oom_retries": allocations retried after
        releasing the cached free lists} (aesfhe_pool_stats)"""
        out = np.zeros(2, np.uint64)
        self._ctx.check(self._lib.aesfhe_pool_stats(self._ctx.ptr, out))
        return {"bytes": int(out[0]), "oom_retries": int(out[1])}

    def kernel_gaps(self) -> dict:
        """{kernel id: (gaps, total ms)}: the boundary gap before the launch issued right after a
        sampled one (drain + dispatch ramp), by that launch's id (read before kernel_stats resets)"""
        out = np.zeros(2 * len(KERNEL_IDS))
        self._ctx.check(self._lib.aesfhe_kernel_gaps(self._ctx.ptr, out, len(KERNEL_IDS)))
        return {k: (int(out[2 * i]), float(out[2 * i + 1])) for i, k in enumerate(KERNEL_IDS) if out[2 * i] > 0}

    def kernel_stats(self, reset: bool = True) -> dict:
        out = np.zeros(3 * len(KERNEL_IDS))
        self._ctx.check(self._lib.aesfhe_kernel_stats(self._ctx.ptr, out, len(KERNEL_IDS), int(reset)))
        return {k: {"launches": int(out[3 * i]), "ms": float(out[3 * i + 1]), "bytes": float(out[3 * i + 2])}
                for i, k in enumerate(KERNEL_IDS) if out[3 * i] > 0}

    def galois_rotate(self, steps: int) -> int:
        return pow(5, (-steps) % self.slot_count, 2 * self.n)

    @property
    def galois_conj(self) -> int:
        return 2 * self.n - 1


def launch_count() -> int:
    """kernel launches issued by this process so far (aesfhe_launch_count)"""
    return int(load_library().aesfhe_launch_count())


def launch_census(reset: bool = False) -> dict:
    """{C-ABI entry point: {kernel name: launches}} since start-up / the last reset (AESFHE_CENSUS=1
    at process start; aesfhe_launch_census)"""
    L = load_library()
    need = int(L.aesfhe_launch_census(None, 0, 0))
    buf = ctypes.create_string_buffer(need + 1)
    L.aesfhe_launch_census(buf, need + 1, 1 if reset else 0)
    out: dict = {}
    for line in buf.value.decode().splitlines():
        op, kern, n = line.split("\t")
        out.setdefault(op, {})[kern] = out.get(op, {}).get(kern, 0) + int(n)
    return out


def alg_bytes() -> dict:
    """{kernel id: (algorithmic bytes, launches)} of every launch so far (aesfhe_alg_bytes)"""
    b = np.zeros(len(KERNEL_IDS))
    n = np.zeros(len(KERNEL_IDS), np.uint64)
    load_library().aesfhe_alg_bytes(b, n, len(KERNEL_IDS))
    return {k: (float(b[i]), int(n[i])) for i, k in enumerate(KERNEL_IDS)}


def bootstrap_depth() -> int:
    return int(load_library().aesfhe_bootstrap_depth())


def debug_bootplan(log_n: int = 16) -> np.ndarray:
    """Host self-check of the bootstrap plan (errors of StC, CtS, EvalMod polynomial)."""
    err = np.zeros(3)
    load_library().aesfhe_debug_bootplan(int(log_n), err)
    return err


def debug_sparseplan(n: int, pack: int) -> np.ndarray:
    """host self-check of a sparse bootstrap plan (aesfhe_debug_sparseplan; pack 0 / 1 single /
    2 pair): [StC error, CtS error]"""
    err = np.zeros(2)
    load_library().aesfhe_debug_sparseplan(int(n), int(pack), err)
    return err
