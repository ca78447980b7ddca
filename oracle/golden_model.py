"""oracle/golden_model.py -- TEST INFRASTRUCTURE, NOT PRODUCT CODE.

Ideal-slot (noiseless) numpy restatement of the reference's homomorphic AES round
logic.  A "ciphertext" is its complex slot vector; engine primitives are replaced
by their exact slot semantics:

    rotate(ct, d)  = np.roll(slots, d)        (pinned by ShiftRows)
    conjugate      = np.conj
    power basis    = exact powers x^1..x^deg
    bootstrap      = identity
    renorm         = decode 16 strided slots -> bytes -> re-encode (REF/pipeline.py:65-69)

Each function cites the reference lines it restates.  The model runs at any
slot_count; slot_count = 16 (stride 1) is exact for the 16 state slots because
every rotation the AES modules issue is a multiple of the stride.
"""
from __future__ import annotations

import json
from pathlib import Path

import numpy as np

Z16 = np.exp(-2j * np.pi / 16)   # REF/utils.py:10-12
Z256 = np.exp(-2j * np.pi / 256)  # REF/sub_bytes_lut.py:38


# --------------------------------------------------------------------------------
# codec: REF/utils.py:8-19, REF/state_encoder.py:17-38
# --------------------------------------------------------------------------------
def to_zeta(v):
    return Z16 ** (np.asarray(v) % 16)


def from_zeta(z):
    k = (-np.angle(z) * 16) / (2 * np.pi)
    return np.mod(np.rint(k), 16).astype(np.uint8)


def encode_state(state, sc: int):
    """REF/state_encoder.py:17-28: byte i -> slot i*stride, other slots 1.  A (B, 16) array
    is the slot-packed batch: byte i of state b -> slot i*stride + b."""
    state = np.asarray(state, np.uint8)
    batch = state.reshape(-1, 16)
    stride = sc // 16
    assert batch.shape[0] <= stride
    hi = np.ones(sc, np.complex128)
    lo = np.ones(sc, np.complex128)
    hi[:16 * stride].reshape(16, stride)[:, :batch.shape[0]] = to_zeta(batch.T >> 4)
    lo[:16 * stride].reshape(16, stride)[:, :batch.shape[0]] = to_zeta(batch.T & 15)
    return hi, lo


def decode_state(hi, lo, states: int = 1):
    """REF/state_encoder.py:30-38: read only the 16 strided slots (x `states` packed states)."""
    stride = len(hi) // 16
    take = lambda v: v[:16 * stride].reshape(16, stride)[:, :states].T
    out = ((from_zeta(take(hi)) << 4) | from_zeta(take(lo))).astype(np.uint8)
    return out[0] if states == 1 else out


def renorm(hi, lo, states: int = 1):
    """REF/pipeline.py:65-69 / REF/mixcol_final.py:104-106: decode then re-encode."""
    return encode_state(decode_state(hi, lo, states), len(hi))


# --------------------------------------------------------------------------------
# coefficient files: REF/lut.py:10-62 JSON layout {"entries": [[k,re,im]|[p,q,re,im]]}
# --------------------------------------------------------------------------------
def load_1d(path):
    ent = json.loads(Path(path).read_text())["entries"]
    A = np.zeros(max(int(e[0]) for e in ent) + 1, np.complex128)
    for k, re, im in ent:
        A[int(k)] = complex(re, im)
    return A


def load_2d(path, size=16):
    A = np.zeros((size, size), np.complex128)
    for p, q, re, im in json.loads(Path(path).read_text())["entries"]:
        A[int(p), int(q)] = complex(re, im)
    return A


# --------------------------------------------------------------------------------
# LUT evaluation
# --------------------------------------------------------------------------------
def basis16(x):
    """REF/xor4_lut.py:27-60: 1, x..x^8, conj(x^7)..conj(x^1)."""
    B = [np.ones_like(x)] + [x ** k for k in range(1, 9)]
    B += [np.conj(x ** (16 - k)) for k in range(9, 16)]
    return B


def bivariate(C, x, y, tol=1e-12):
    """REF/xor4_lut.py:63-74 and REF/mixcol_final.py:80-91: sum_{p,q} C[p,q] X^p Y^q."""
    BX, BY = basis16(x), basis16(y)
    out = np.zeros_like(x)
    for p in range(16):
        for q in range(16):
            if abs(C[p, q]) > tol:
                out = out + C[p, q] * BX[p] * BY[q]
    return out


def subbytes(hi, lo, H, Lo, tol=1e-12):
    """REF/sub_bytes_lut.py:46-73: lift lo to zeta256, combine, two 255-term sums."""
    lift = np.fft.ifft(Z256 ** np.arange(16))
    b16 = basis16(lo)
    res_lift = lift[0] + sum(lift[k] * b16[k] for k in range(1, 16) if abs(lift[k]) > tol)
    b = hi * res_lift
    out_h = np.full_like(b, H[0])
    out_l = np.full_like(b, Lo[0])
    for k in range(1, 256):
        bk = b ** k if k <= 128 else np.conj(b ** (256 - k))
        if k < len(H) and abs(H[k]) > tol:
            out_h = out_h + H[k] * bk
        if k < len(Lo) and abs(Lo[k]) > tol:
            out_l = out_l + Lo[k] * bk
    return out_h, out_l


def _row_masks(sc, states=1):
    stride = sc // 16
    M = []
    for r in range(4):
        m = np.zeros(sc)
        for c in range(4):
            m[(r + 4 * c) * stride:(r + 4 * c) * stride + states] = 1.0
        M.append(m)
    return M


def shift_rows(x, inverse=False, states=1):
    """REF/shift_rows.py:39-56 (steps -4r*stride), REF/inv_shiftrows.py:37-47 (+4r*stride)."""
    sc = len(x)
    stride = sc // 16
    out = np.zeros_like(x)
    for r, m in enumerate(_row_masks(sc, states)):
        step = (4 * r * stride) * (1 if inverse else -1)
        out = out + np.roll(x * m, step)
    return out


def col_shift(x, k):
    """REF/mixcol_final.py:101-102: rotate(ct, -4*k*stride)."""
    return np.roll(x, -4 * k * (len(x) // 16))


class Golden:
    """Stage-by-stage golden model of AESPipeline (REF/pipeline.py) over slot vectors."""

    def __init__(self, coeff_dir, renorm_between_steps: bool = True, states: int = 1):
        d = Path(coeff_dir)
        self.xor = load_2d(d / "xor4_coeffs.json")
        self.sb = (load_1d(d / "mod256_to_16_hi.json"), load_1d(d / "mod256_to_16_lo.json"))
        self.isb = (load_1d(d / "inv_mod256_to_16_hi.json"), load_1d(d / "inv_mod256_to_16_lo.json"))
        self.gf = {(m, w): load_2d(d / f"gf_mult{m}_{w}_coeffs.json") for m in (2, 3, 9, 11, 13, 14) for w in ("hi", "lo")}
        self.renorm_between = renorm_between_steps
        self.states = states  # slot-packed states per vector

    def _renorm(self, hi, lo):
        return renorm(hi, lo, self.states)

    def _sr(self, ct, inverse=False):
        return shift_rows(ct[0], inverse, self.states), shift_rows(ct[1], inverse, self.states)

    def _keys(self, rks, sc):
        return [encode_state(np.broadcast_to(np.asarray(k, np.uint8), (self.states, 16)) if self.states > 1 else k, sc)
                for k in rks]

    def xor4(self, a, b):
        return bivariate(self.xor, a, b)

    def ark(self, hi, lo, khi, klo):
        """REF/add_round_key.py:142-144"""
        return self.xor4(hi, khi), self.xor4(lo, klo)

    def gf_mult(self, m, hi, lo):
        return bivariate(self.gf[(m, "hi")], hi, lo), bivariate(self.gf[(m, "lo")], hi, lo)

    def mix_columns(self, hi, lo, log=None):
        """REF/mixcol_final.py:112-165 (renorm after each XOR pair, final bootstrap = id)."""
        r = {k: (col_shift(hi, k), col_shift(lo, k)) for k in (1, 2, 3)}
        two = self.gf_mult(2, hi, lo)
        thr = self.gf_mult(3, *r[1])
        acc = self._renorm(self.xor4(two[0], thr[0]), self.xor4(two[1], thr[1]))
        acc = self._renorm(self.xor4(acc[0], r[2][0]), self.xor4(acc[1], r[2][1]))
        acc = self._renorm(self.xor4(acc[0], r[3][0]), self.xor4(acc[1], r[3][1]))
        if log is not None:
            log.update(two=two, thr=thr)
        return acc

    def inv_mix_columns(self, hi, lo):
        """REF/invmixcolumns_fhe.py:131-170 (use_hard_renorm=True default)."""
        r = {k: (col_shift(hi, k), col_shift(lo, k)) for k in (1, 2, 3)}
        e14 = self.gf_mult(14, hi, lo)
        e11 = self.gf_mult(11, *r[1])
        e13 = self.gf_mult(13, *r[2])
        e9 = self.gf_mult(9, *r[3])
        acc = self._renorm(self.xor4(e14[0], e11[0]), self.xor4(e14[1], e11[1]))
        acc = self._renorm(self.xor4(acc[0], e13[0]), self.xor4(acc[1], e13[1]))
        return self._renorm(self.xor4(acc[0], e9[0]), self.xor4(acc[1], e9[1]))

    def _rn(self, hi, lo):
        return self._renorm(hi, lo) if self.renorm_between else (hi, lo)

    def encrypt(self, state, rks, sc=None, stages=None):
        """REF/pipeline.py:123-188; `stages` collects decoded bytes per step."""
        sc = sc or 16 * self.states
        def tag(name, pair):
            if stages is not None:
                stages[name] = decode_state(*pair, self.states)
        keys = self._keys(rks, sc)
        ct = encode_state(state, sc)
        ct = self._rn(*self.ark(*ct, *keys[0]))
        tag("r0.ark", ct)
        for r in range(1, 10):
            ct = self._rn(*subbytes(*ct, *self.sb))
            tag(f"r{r}.sb", ct)
            ct = self._sr(ct)
            tag(f"r{r}.sr", ct)
            ct = self.mix_columns(*ct)
            tag(f"r{r}.mc", ct)
            ct = self._rn(*self.ark(*ct, *keys[r]))
            tag(f"r{r}.ark", ct)
        ct = self._rn(*subbytes(*ct, *self.sb))
        tag("r10.sb", ct)
        ct = self._sr(ct)
        tag("r10.sr", ct)
        ct = self._rn(*self.ark(*ct, *keys[10]))
        tag("r10.ark", ct)
        return ct

    def decrypt(self, ct, rks, sc=None, with_inv_mix=True):
        """REF/pipeline.py:193-254 with InvMixColumns after ARK (REF/README.md:87-94)."""
        keys = self._keys(rks, sc or len(ct[0]))
        ct = self._rn(*self.ark(*ct, *keys[10]))
        for r in range(9, 0, -1):
            ct = self._sr(ct, True)
            ct = self._rn(*subbytes(*ct, *self.isb))
            ct = self._rn(*self.ark(*ct, *keys[r]))
            if with_inv_mix:
                ct = self.inv_mix_columns(*ct)
        ct = self._sr(ct, True)
        ct = self._rn(*subbytes(*ct, *self.isb))
        return self._rn(*self.ark(*ct, *keys[0]))
