"""oracle/ckks_cpu.py -- TEST INFRASTRUCTURE, NOT PRODUCT CODE.

ctypes front-end of ``oracle/ckks_oracle.c`` (the plain-C CPU restatement of the
RNS-CKKS engine the reference reaches through REF/engine_context.py:56-204), plus
``OracleEngine``: a small CPU CKKS engine with the EngineContext surface
(REF/engine_context.py:56-204) built from those primitives.  It serves

* tests/ as the bit-exact checker of the HIP kernels (same inputs -> same limbs), and
* bench.py's ``cpu_baseline`` leg (the reference's CPU engine, desilofhe, is absent).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import it.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from pathlib import Path

import numpy as np

_HERE = Path(__file__).resolve().parent
_LIB_PATH = _HERE / "_build" / "libckks_oracle.so"
_lib = None

u32p = np.ctypeslib.ndpointer(dtype=np.uint32, flags="C_CONTIGUOUS")
i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
f64p = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")


def build() -> Path:
    """Compile the oracle with its Makefile (gcc only)."""
    subprocess.run(["make", "-s", "-C", str(_HERE)], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not _LIB_PATH.exists():
        build()
    L = ctypes.CDLL(str(_LIB_PATH))
    vp, c_int, c_u64, c_i64, c_dbl = ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64, ctypes.c_int64, ctypes.c_double
    sig = {
        "orc_create": (vp, [c_int, c_int, c_int, c_u64]),
        "orc_create_boot": (vp, [c_int, c_int, c_int, c_int, c_u64]),
        "orc_rescale2": (None, [vp, c_int, c_int, u32p, u32p]),
        "orc_keyswitch_d2s": (None, [vp, c_int, u32p, u32p, u32p]),
        "orc_destroy": (None, [vp]),
        "orc_set_key": (None, [vp, ctypes.c_char_p]),
        "orc_chacha_block": (None, [u32p, c_u64, c_u64, u32p]),
        "orc_info": (None, [vp, i32p]),
        "orc_moduli": (None, [vp, u32p]),
        "orc_deltas": (None, [vp, f64p]),
        "orc_ntt": (None, [vp, i32p, c_int, u32p]),
        "orc_intt": (None, [vp, i32p, c_int, u32p]),
        "orc_embed_inverse": (None, [vp, f64p, f64p, f64p]),
        "orc_embed": (None, [vp, f64p, f64p, f64p]),
        "orc_encode": (None, [vp, f64p, f64p, c_dbl, c_int, u32p]),
        "orc_secret": (None, [vp, i32p]),
        "orc_secret_ntt": (None, [vp, u32p]),
        "orc_gen_pk": (None, [vp, u32p]),
        "orc_gen_ksk": (None, [vp, c_u64, u32p]),
        "orc_rescale": (None, [vp, c_int, c_int, u32p, u32p]),
        "orc_keyswitch": (None, [vp, c_int, u32p, u32p, u32p]),
        "orc_tensor": (None, [vp, c_int, u32p, u32p, u32p]),
        "orc_mul_poly": (None, [vp, c_int, c_int, u32p, u32p, u32p]),
        "orc_mul_limb_consts": (None, [vp, c_int, c_int, u32p, u32p, u32p]),
        "orc_automorph": (None, [vp, c_int, c_u64, c_int, u32p, u32p]),
        "orc_encrypt": (None, [vp, c_int, u32p, u32p, c_u64, u32p]),
        "orc_decrypt_coeffs": (None, [vp, c_int, c_int, u32p, u32p, f64p]),
        "orc_const_residues": (None, [vp, c_i64, c_int, u32p]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


class OracleParams:
    """Parameter set + raw primitives."""

    def __init__(self, log_n: int = 16, max_level: int = 17, dnum: int = 3, seed: int | bytes = 0, boot_double: int = 0):
        """boot_double > 0: the bootstrappable chain (params.cpp), single-prime levels 0..max_level
        and boot_double double-prime levels above (top level max_level + boot_double).
        seed: an int (ChaCha20 key words 0-1, aesfhe_create) or the 32-byte key (aesfhe_create_keyed)"""
        self._L = lib()
        self.L1 = max_level
        key = bytes(seed) if isinstance(seed, (bytes, bytearray)) else None
        if key is not None and len(key) != 32:
            raise ValueError("a key must be 32 bytes")
        s = 0 if key is not None else int(seed) & 0xFFFFFFFFFFFFFFFF
        if boot_double:
            self.h = self._L.orc_create_boot(log_n, max_level, boot_double, dnum, s)
        else:
            self.h = self._L.orc_create(log_n, max_level, dnum, s)
        if key is not None:
            self._L.orc_set_key(self.h, key)
        info = np.zeros(8, np.int32)
        self._L.orc_info(self.h, info)
        self.n, self.L, self.n_q, self.n_ks, self.n_p, self.alpha, self.dnum, self.log_n = map(int, info)
        self.moduli = np.zeros(self.n_q + self.n_p, np.uint32)
        self._L.orc_moduli(self.h, self.moduli)
        self.deltas = np.zeros(self.L + 1, np.float64)
        self._L.orc_deltas(self.h, self.deltas)
        self.slot_count = self.n // 2

    def __del__(self):
        try:
            self._L.orc_destroy(self.h)
        except Exception:
            pass

    # -- raw transforms --------------------------------------------------------------
    def ntt(self, data: np.ndarray, limbs) -> np.ndarray:
        d = np.ascontiguousarray(data, np.uint32).copy()
        ids = np.ascontiguousarray(limbs, np.int32)
        self._L.orc_ntt(self.h, ids, len(ids), d)
        return d

    def intt(self, data: np.ndarray, limbs) -> np.ndarray:
        d = np.ascontiguousarray(data, np.uint32).copy()
        ids = np.ascontiguousarray(limbs, np.int32)
        self._L.orc_intt(self.h, ids, len(ids), d)
        return d

    def embed_inverse(self, z: np.ndarray) -> np.ndarray:
        z = np.asarray(z, np.complex128)
        m = np.zeros(self.n, np.float64)
        self._L.orc_embed_inverse(self.h, np.ascontiguousarray(z.real), np.ascontiguousarray(z.imag), m)
        return m

    def embed(self, m: np.ndarray) -> np.ndarray:
        re = np.zeros(self.slot_count)
        im = np.zeros(self.slot_count)
        self._L.orc_embed(self.h, np.ascontiguousarray(m, np.float64), re, im)
        return re + 1j * im

    def encode(self, z: np.ndarray, scale: float, nl: int) -> np.ndarray:
        z = np.broadcast_to(np.asarray(z, np.complex128), (self.slot_count,))
        out = np.zeros((nl, self.n), np.uint32)
        self._L.orc_encode(self.h, np.ascontiguousarray(z.real), np.ascontiguousarray(z.imag), float(scale), nl, out)
        return out

    # -- keys ------------------------------------------------------------------------------
    def secret(self) -> np.ndarray:
        s = np.zeros(self.n, np.int32)
        self._L.orc_secret(self.h, s)
        return s

    def secret_ntt(self) -> np.ndarray:
        out = np.zeros((self.n_q + self.n_p, self.n), np.uint32)
        self._L.orc_secret_ntt(self.h, out)
        return out

    def gen_pk(self) -> np.ndarray:
        out = np.zeros((2, self.n_q, self.n), np.uint32)
        self._L.orc_gen_pk(self.h, out)
        return out

    def gen_ksk(self, galois: int) -> np.ndarray:
        out = np.zeros((self.dnum, 2, self.n_ks + self.n_p, self.n), np.uint32)
        self._L.orc_gen_ksk(self.h, galois, out)
        return out

    # -- ciphertext primitives (NTT form arrays) ------------------------------------
    def rescale(self, level: int, x: np.ndarray) -> np.ndarray:
        x = np.ascontiguousarray(x, np.uint32)
        npoly = x.shape[0]
        out = np.zeros((npoly, level + 1, self.n), np.uint32)
        self._L.orc_rescale(self.h, level, npoly, x, out)
        return out

    def keyswitch(self, level: int, d: np.ndarray, ksk: np.ndarray) -> np.ndarray:
        out = np.zeros((2, self.nl(level), self.n), np.uint32)
        self._L.orc_keyswitch(self.h, level, np.ascontiguousarray(d, np.uint32), np.ascontiguousarray(ksk, np.uint32), out)
        return out

    def tensor(self, level: int, a: np.ndarray, b: np.ndarray) -> np.ndarray:
        out = np.zeros((3, level + 2, self.n), np.uint32)
        self._L.orc_tensor(self.h, level, np.ascontiguousarray(a, np.uint32), np.ascontiguousarray(b, np.uint32), out)
        return out

    def automorph(self, level: int, g: int, x: np.ndarray) -> np.ndarray:
        x = np.ascontiguousarray(x, np.uint32)
        out = np.zeros_like(x)
        self._L.orc_automorph(self.h, level, g, x.shape[0], x, out)
        return out

    def mul_poly(self, pt: np.ndarray, x: np.ndarray) -> np.ndarray:
        """x (npoly x nl limbs) times the plaintext polynomial pt (nl limbs), elementwise (NTT form)"""
        x = np.ascontiguousarray(x, np.uint32)
        out = np.zeros_like(x)
        self._L.orc_mul_poly(self.h, x.shape[1], x.shape[0], np.ascontiguousarray(pt, np.uint32), x, out)
        return out

    def mul_limb_consts(self, consts: np.ndarray, x: np.ndarray) -> np.ndarray:
        x = np.ascontiguousarray(x, np.uint32)
        out = np.zeros_like(x)
        self._L.orc_mul_limb_consts(self.h, x.shape[1], x.shape[0], np.ascontiguousarray(consts, np.uint32), x, out)
        return out

    def const_residues(self, c: int, nl: int) -> np.ndarray:
        out = np.zeros(nl, np.uint32)
        self._L.orc_const_residues(self.h, int(c), nl, out)
        return out

    def encrypt(self, pt_top: np.ndarray, pk: np.ndarray, ctr: int, fresh_level: int | None = None) -> np.ndarray:
        f = self.L if fresh_level is None else fresh_level
        out = np.zeros((2, f + 2, self.n), np.uint32)
        self._L.orc_encrypt(self.h, f, np.ascontiguousarray(pt_top, np.uint32), np.ascontiguousarray(pk, np.uint32), ctr, out)
        return out

    def decrypt_coeffs(self, level: int, ct: np.ndarray, s_ntt: np.ndarray) -> np.ndarray:
        ct = np.ascontiguousarray(ct, np.uint32)
        out = np.zeros(self.n, np.float64)
        self._L.orc_decrypt_coeffs(self.h, level, ct.shape[0], ct, np.ascontiguousarray(s_ntt, np.uint32), out)
        return out

    def nl(self, level: int) -> int:
        """limbs at a level: l + 2 up to L1, two more per double-prime level above"""
        if level > self.L:  # transient level L + 1 of a top-level encryption
            return self.nl(self.L) + 1
        return level + 2 if level <= self.L1 else self.L1 + 2 + 2 * (level - self.L1)

    def rescale2(self, level: int, x: np.ndarray) -> np.ndarray:
        """double-prime rescale from `level` (drops the two last limbs, one rounding)"""
        x = np.ascontiguousarray(x, np.uint32)
        out = np.zeros((x.shape[0], self.nl(level) - 2, self.n), np.uint32)
        self._L.orc_rescale2(self.h, level, x.shape[0], x, out)
        return out

    def keyswitch_d2s(self, np_d2s: int, d: np.ndarray, ksk: np.ndarray) -> np.ndarray:
        """the bootstrap's dense -> sparse key switch over Q0 P' (d: c1 on q0, q1)"""
        out = np.zeros((2, 2, self.n), np.uint32)
        self._L.orc_keyswitch_d2s(self.h, int(np_d2s), np.ascontiguousarray(d, np.uint32), np.ascontiguousarray(ksk, np.uint32), out)
        return out

    # -- helpers -----------------------------------------------------------------------
    def limbs_mod(self, nl: int) -> np.ndarray:
        return self.moduli[:nl].astype(np.uint64)[:, None]

    def galois_rotate(self, steps: int) -> int:
        """rotate(ct, steps) == np.roll(slots, steps): left rotation by -steps."""
        k = (-steps) % self.slot_count
        return pow(5, k, 2 * self.n)

    @property
    def galois_conj(self) -> int:
        return 2 * self.n - 1


class OracleCiphertext:
    __slots__ = ("data", "level")

    def __init__(self, data: np.ndarray, level: int):
        self.data = data
        self.level = level


class OracleEngine:
    """CPU CKKS engine over the oracle primitives (EngineContext surface,
    REF/engine_context.py:56-204).  Same conventions as the HIP engine
     so that levels, scales and key streams coincide."""

    def __init__(self, log_n: int = 16, max_level: int = 17, dnum: int = 3, seed: int | bytes = 0, fresh_level: int | None = None):
        self.p = OracleParams(log_n, max_level, dnum, seed)
        self.fresh = self.p.L if fresh_level is None else fresh_level
        self.slot_count = self.p.slot_count
        self.s_ntt = self.p.secret_ntt()
        self.pk = self.p.gen_pk()
        self._ksk = {}
        self._enc_ctr = 0

    def ksk(self, g: int) -> np.ndarray:
        if g not in self._ksk:
            self._ksk[g] = self.p.gen_ksk(g)
        return self._ksk[g]

    # -- codec -------------------------------------------------------------------------
    def encrypt(self, z) -> OracleCiphertext:
        p, f = self.p, self.fresh
        pt = p.encode(z, p.deltas[f] * float(p.moduli[f + 2]), f + 3)
        data = p.encrypt(pt, self.pk, self._enc_ctr, f)
        self._enc_ctr += 1
        return OracleCiphertext(data, f)

    def decrypt(self, ct: OracleCiphertext) -> np.ndarray:
        m = self.p.decrypt_coeffs(ct.level, ct.data, self.s_ntt)
        return self.p.embed(m / self.p.deltas[ct.level])

    # -- arithmetic ---------------------------------------------------------------------
    def _mod(self, nl):
        return self.p.limbs_mod(nl)

    def level_down(self, ct: OracleCiphertext, level: int) -> OracleCiphertext:
        """drop limbs to level+1, multiply by round(D_b q / D_a), rescale."""
        if ct.level == level:
            return ct
        p = self.p
        x = np.ascontiguousarray(ct.data[:, : level + 3])
        c = int(round(p.deltas[level] * float(p.moduli[level + 2]) / p.deltas[ct.level]))
        x = p.mul_limb_consts(p.const_residues(c, level + 3), x)
        return OracleCiphertext(p.rescale(level + 1, x), level)

    def _align(self, a, b):
        lv = min(a.level, b.level)
        return self.level_down(a, lv), self.level_down(b, lv)

    def add(self, a, b):
        a, b = self._align(a, b)
        return OracleCiphertext(((a.data.astype(np.uint64) + b.data) % self._mod(a.level + 2)).astype(np.uint32), a.level)

    def sub(self, a, b):
        a, b = self._align(a, b)
        q = self._mod(a.level + 2)
        return OracleCiphertext(((a.data.astype(np.uint64) + q - b.data) % q).astype(np.uint32), a.level)

    def _ntt_scalar(self, re: float, im: float, scale: float, nl: int) -> np.ndarray:
        """NTT image of round(re*scale) + round(im*scale) X^{N/2} (constant slots re+i*im)."""
        p = self.p
        poly = np.zeros((nl, p.n), np.uint32)
        A, B = int(round(re * scale)), int(round(im * scale))
        poly[:, 0] = p.const_residues(A, nl)
        poly[:, p.n // 2] = p.const_residues(B, nl)
        return p.ntt(poly, range(nl))

    def add_plain(self, ct, val: complex):
        p = self.p
        nl = ct.level + 2
        c = self._ntt_scalar(complex(val).real, complex(val).imag, p.deltas[ct.level], nl)
        d = ct.data.copy()
        d[0] = ((d[0].astype(np.uint64) + c) % self._mod(nl)).astype(np.uint32)
        return OracleCiphertext(d, ct.level)

    def multiply_scalar(self, ct, val: complex):
        p = self.p
        v = complex(val)
        nl = ct.level + 2
        if v.imag == 0 and float(v.real).is_integer() and abs(v.real) < 2 ** 20:
            c = p.const_residues(int(v.real), nl)
            return OracleCiphertext(p.mul_limb_consts(c, ct.data), ct.level)
        if ct.level < 1:
            raise RuntimeError("not enough level to multiply (level 0)")
        c = self._ntt_scalar(v.real, v.imag, p.deltas[ct.level], nl)
        x = ((ct.data.astype(np.uint64) * c[None]) % self._mod(nl)).astype(np.uint32)
        return OracleCiphertext(p.rescale(ct.level, x), ct.level - 1)

    def multiply(self, a, b):
        if a.level < 1 or b.level < 1:
            raise RuntimeError("not enough level to multiply (level 0)")
        a, b = self._align(a, b)
        p = self.p
        lv = a.level
        d = p.tensor(lv, a.data, b.data)
        ks = p.keyswitch(lv, d[2], self.ksk(0))
        q = self._mod(lv + 2)
        c = ((d[:2].astype(np.uint64) + ks) % q).astype(np.uint32)
        return OracleCiphertext(p.rescale(lv, c), lv - 1)

    def _galois(self, ct, g):
        p = self.p
        x = p.automorph(ct.level, g, ct.data)
        ks = p.keyswitch(ct.level, x[1], self.ksk(g))
        q = self._mod(ct.level + 2)
        out = ks.copy()
        out[0] = ((ks[0].astype(np.uint64) + x[0]) % q).astype(np.uint32)
        return OracleCiphertext(out, ct.level)

    def rotate(self, ct, steps: int):
        return self._galois(ct, self.p.galois_rotate(steps))

    def conjugate(self, ct):
        return self._galois(ct, self.p.galois_conj)

    def make_power_basis(self, ct, degree: int):
        """x^k at depth ceil(log2 k): x^(2^i) by squaring, x^k = x^(2^t) * x^(k-2^t)."""
        pw = {1: ct}
        for k in range(2, degree + 1):
            t = 1 << (k.bit_length() - 1)
            pw[k] = self.multiply(pw[t // 2], pw[t // 2]) if t == k else self.multiply(pw[t], pw[k - t])
        return [pw[k] for k in range(1, degree + 1)]


class _OraclePt:
    """Level-agnostic plaintext of the oracle engine: slot values, constant flag."""

    __slots__ = ("z", "const")

    def __init__(self, z):
        self.z = np.asarray(z, np.complex128)
        self.const = bool(np.all(self.z == self.z[0]))


class _EngineView:
    def __init__(self, slot_count):
        self.slot_count = slot_count


class OracleContext:
    """EngineContext surface (REF/engine_context.py:56-204) over OracleEngine, so the
    build's AES modules can run on the CPU oracle (tests, cpu_baseline)."""

    def __init__(self, log_n: int = 16, max_level: int = 17, dnum: int = 3, seed: int | bytes = 0):
        self.eng = OracleEngine(log_n, max_level, dnum, seed)
        self.engine = _EngineView(self.eng.slot_count)

    def encrypt(self, data):
        return self.eng.encrypt(np.broadcast_to(np.asarray(data, np.complex128), (self.eng.slot_count,)))

    def decrypt(self, ct):
        return self.eng.decrypt(ct)

    def encode(self, vec):
        return _OraclePt(np.broadcast_to(np.asarray(vec, np.complex128), (self.eng.slot_count,)).copy())

    def _mul_pt(self, ct, pt: _OraclePt):
        if pt.const:
            return self.eng.multiply_scalar(ct, complex(pt.z[0]))
        if ct.level < 1:
            raise RuntimeError("not enough level to multiply (level 0)")
        p = self.eng.p
        enc = p.encode(pt.z, p.deltas[ct.level], ct.level + 2)
        x = ((ct.data.astype(np.uint64) * enc[None]) % p.limbs_mod(ct.level + 2)).astype(np.uint32)
        return OracleCiphertext(p.rescale(ct.level, x), ct.level - 1)

    def multiply(self, a, b):
        if isinstance(a, OracleCiphertext) and isinstance(b, OracleCiphertext):
            return self.eng.multiply(a, b)
        if isinstance(b, _OraclePt):
            return self._mul_pt(a, b)
        return self.eng.multiply_scalar(a, complex(b))

    def multiply_plain(self, ct, val):
        return self.multiply(ct, val if np.isscalar(val) else self.encode(val))

    def add(self, a, b):
        if isinstance(b, _OraclePt):
            if b.const:
                return self.eng.add_plain(a, complex(b.z[0]))
            p = self.eng.p
            enc = p.encode(b.z, p.deltas[a.level], a.level + 2)
            d = a.data.copy()
            d[0] = ((d[0].astype(np.uint64) + enc) % p.limbs_mod(a.level + 2)).astype(np.uint32)
            return OracleCiphertext(d, a.level)
        return self.eng.add(a, b)

    def sub(self, a, b):
        return self.eng.sub(a, b)

    def add_plain(self, ct, val):
        return self.eng.add_plain(ct, complex(val))

    def make_power_basis(self, ct, degree):
        import math
        if ct.level < math.ceil(math.log2(degree)) if degree > 1 else False:
            raise RuntimeError("not enough level for make_power_basis")
        return self.eng.make_power_basis(ct, degree)

    def conjugate(self, ct):
        return self.eng.conjugate(ct)

    def rotate(self, ct, steps):
        return ct if steps % self.eng.slot_count == 0 else self.eng.rotate(ct, steps)

    def relinearize(self, ct):
        return ct

    def bootstrap(self, ct):
        raise RuntimeError("the CPU oracle engine does not bootstrap")

    def to_intt(self, ct):
        return ct

    def to_ntt(self, ct):
        return ct


def chacha_block(key_words, ctr: int, nonce: int) -> np.ndarray:
    """the oracle's ChaCha20 block function (16 output words; tests pin it to RFC 8439 2.3.2)"""
    out = np.zeros(16, np.uint32)
    lib().orc_chacha_block(np.ascontiguousarray(key_words, np.uint32), int(ctr), int(nonce), out)
    return out
