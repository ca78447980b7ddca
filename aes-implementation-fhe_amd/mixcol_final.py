"""MixColFinal: "MixColumns" as GF×2(x) ⊕ GF×3(r1) ⊕ r2 ⊕ r3 (REF/mixcol_final.py:40-165).

r_k = rotate(x, -4k*stride) shifts every row left by k columns under column-first
packing, so the output is out[r,c] = 2a[r,c] ^ 3a[r,c+1] ^ a[r,c+2] ^ a[r,c+3] -- the
reference's orientation, reproduced as is.  GF multipliers are
bivariate LUTs over (hi, lo); each XOR pair is followed by a secret-key renorm and the
result is bootstrapped (do_final_bootstrap, default True).
"""
from __future__ import annotations

import json
import os
from typing import Any, Dict, Tuple

import numpy as np

from lut import COEFF_DIR, ensure_coeffs
from state_encoder import StateEncoder
from xor4_lut import XOR4LUT, SplitLUT2, batched, eval_two, joint_bases, powers, std_basis
from utils import FOLDS, LUT2_DEPTH, takes_kw, NEED_BOOTSTRAP, NEED_XOR, RENORM_FLOOR, bootstrap1, bootstrap2, can_fork, drop_to, fused_lut, pair, rot_many, rot_pair, rotate_multi

# AESFHE_SHARE_R1=0: MixColumns' r1 basis rebuilt in its second XOR4 (A/B runs)
_SHARE_R1 = os.environ.get("AESFHE_SHARE_R1", "1") != "0"
_FHE_FORK = os.environ.get("AESFHE_FHE_FORK", "0") == "1"  # true-FHE MixColumns halves forced onto two streams (A/B: no gain measured)


class _CoeffCache:
    """gf_mult{k}_{hi|lo} plaintext coefficients, encoded once per engine (REF :19-37)."""

    def __init__(self, coeff_dir=COEFF_DIR):
        self.dir = coeff_dir
        self.pt_cache: Dict[Tuple[int, str], Dict[Tuple[int, int], Any]] = {}
        self.mat_cache: Dict[Tuple[int, str], np.ndarray] = {}

    def _entries(self, mult: int, which: str):
        path = ensure_coeffs(self.dir) / f"gf_mult{mult}_{which}_coeffs.json"
        return json.loads(path.read_text(encoding="utf-8"))["entries"]

    def split(self, mult: int, which: str) -> SplitLUT2:
        key = (mult, which, "split")
        if key not in self.mat_cache:
            self.mat_cache[key] = SplitLUT2(self.matrix(mult, which))
        return self.mat_cache[key]

    def matrix(self, mult: int, which: str) -> np.ndarray:
        """the same coefficients as a dense 16 x 16 matrix C[p, q] (fused LUT form)"""
        key = (mult, which)
        if key not in self.mat_cache:
            m = np.zeros((16, 16), np.complex128)
            for p, q, re, im in self._entries(mult, which):
                m[int(p), int(q)] = complex(re, im)
            self.mat_cache[key] = m
        return self.mat_cache[key]

    def load_plaintexts(self, ctx, mult: int, which: str):
        key = (mult, which)
        if key not in self.pt_cache:
            sc = ctx.engine.slot_count
            self.pt_cache[key] = {(p, q): ctx.encode(np.full(sc, complex(re, im), dtype=np.complex128))
                                  for p, q, re, im in self._entries(mult, which)}
        return self.pt_cache[key]


def gf_basis16(ctx, ct) -> Dict[int, Any]:
    """REF/mixcol_final.py:64-77 (bootstrap fallback only; zero via multiply by 0.0)."""
    try:
        pos = ctx.make_power_basis(ct, 8)
    except RuntimeError:
        ct = ctx.bootstrap(ct)
        pos = ctx.make_power_basis(ct, 8)
    basis = {0: ctx.add_plain(ctx.multiply(ct, 0.0), 1.0)}
    basis.update({k: pos[k - 1] for k in range(1, 9)})
    basis.update({k: ctx.conjugate(pos[15 - k]) for k in range(9, 16)})
    return basis


def _gf_sum(ctx, coeffs, bx, by, ct_hi):
    acc = ctx.multiply(ct_hi, 0.0)
    for (p, q), pt in coeffs.items():
        acc = ctx.add(acc, ctx.multiply(ctx.multiply(bx[p], by[q]), pt))
    return acc


def gf_poly_eval(ctx, coeffs, ct_hi, ct_lo) -> Any:
    """Σ c[p,q] X^p Y^q over the hi / lo bases (REF/mixcol_final.py:80-91)."""
    return _gf_sum(ctx, coeffs, gf_basis16(ctx, ct_hi), gf_basis16(ctx, ct_lo), ct_hi)


def gf_eval(ctx, cache: _CoeffCache, mult: int, which: str, ct_hi, ct_lo) -> Any:
    """gf_mult{mult}_{which}(hi, lo): the 2-variable LUT as one fused engine call when the
    context has it, else the reference's product loop."""
    bx, by = gf_basis16(ctx, ct_hi), gf_basis16(ctx, ct_lo)
    out = fused_lut(ctx, ("gf", mult, which), cache.matrix(mult, which), bx, by, owner=cache)
    if out is not None:
        return out
    return _gf_sum(ctx, cache.load_plaintexts(ctx, mult, which), bx, by, ct_hi)


def gf_mult_pair(ctx, cache: _CoeffCache, mult: int, ct_hi, ct_lo, out_level=None, defer_conj: bool = False):
    """(gf_mult{mult}_hi, gf_mult{mult}_lo)(hi, lo).  With a fused-LUT context both LUTs are
    evaluated in the conjugate-split form (xor4_lut.SplitLUT2) over ONE pair
    of bases -- positive powers of hi, standard basis of lo -- instead of four 16-element
    bases; otherwise the reference's per-LUT product loops (REF/mixcol_final.py:80-99).
    out_level: inputs dropped to out_level + LUT2_DEPTH first (utils.drop_to).  defer_conj: the
    batched split form may return utils.ConjSum outputs (for StateEncoder.pack + a renorm)."""
    if out_level is not None:
        ct_hi, ct_lo = drop_to(ctx, ct_hi, out_level + LUT2_DEPTH), drop_to(ctx, ct_lo, out_level + LUT2_DEPTH)
    if getattr(ctx, "fused_luts", False):
        sh, sl = cache.split(mult, "hi"), cache.split(mult, "lo")
        try:
            if batched(ctx) and not can_fork(ctx):  # one pair of bases, batched products (§3.12)
                A, B = joint_bases(ctx, [(ct_hi, sh.need_a | sl.need_a, "pow"), (ct_lo, sh.need_b | sl.need_b, "std")])
            else:
                A, B = pair(ctx, lambda: powers(ctx, ct_hi, sh.need_a | sl.need_a),
                            lambda: std_basis(ctx, ct_lo, sh.need_b | sl.need_b))
        except RuntimeError as e:
            if "level" not in str(e):
                raise
        else:
            if batched(ctx) and not can_fork(ctx):
                out = eval_two(ctx, (sh, ("gf", mult, "hi"), A, B), (sl, ("gf", mult, "lo"), A, B), defer_conj and FOLDS.conj)
                if out is not None:
                    return out
            else:
                out = pair(ctx, lambda: sh.eval(ctx, ("gf", mult, "hi"), A, B), lambda: sl.eval(ctx, ("gf", mult, "lo"), A, B),
                           shared=(*A.values(), *B.values()))
                if out[0] is not None and out[1] is not None:
                    return out
    return pair(ctx, lambda: gf_eval(ctx, cache, mult, "hi", ct_hi, ct_lo),
                lambda: gf_eval(ctx, cache, mult, "lo", ct_hi, ct_lo), shared=(ct_hi, ct_lo))


# AESFHE_MC_GF_LOW: the rot form's GF multiplier pair at the XOR4 level with an extra renorm of its
# packed output (1), or at its own depth above the last XOR4 with no renorm (0)
_MC_GF_LOW = os.environ.get("AESFHE_MC_GF_LOW", "1") != "0"
# AESFHE_MC_HOIST=0: with the strict renorm, the unpack's rotation and R^2 u as separate key switches (A/B)
_MC_HOIST = os.environ.get("AESFHE_MC_HOIST", "1") != "0"
# AESFHE_SR_MC_ENTRY=0: ShiftRows as its own step before MixColumns' first column shift and packs (A/B)
SR_MC_ENTRY = os.environ.get("AESFHE_SR_MC_ENTRY", "1") != "0"
# AESFHE_PT_SUM=0: sr_entry's masked sums as separate plaintext products and additions (A/B)
_PT_SUM = os.environ.get("AESFHE_PT_SUM", "1") != "0"
# strict hoist: MixColumns' GF pair output renormalised as the (hi, lo) pair and packed after its renorm
# instead of packed before it -- the multipliers (and the renormalised input u they read) one level lower,
# so the strict path needs fresh level 7 instead of 8 (AESFHE_GF2_PAIR_RENORM=0: pack, then renorm)
_GF2_PAIR = os.environ.get("AESFHE_GF2_PAIR_RENORM", "1") != "0"


class MixColFinal:
    def __init__(self, ctx, xor4: XOR4LUT, stride: int | None = None, states: int = 1, layout=None):
        self.ctx = ctx
        self.xor4 = xor4
        self.sc = ctx.engine.slot_count
        # states > 1: slot-packed batch; layout.periodic: the periodic layout (state_encoder.py)
        self.enc = StateEncoder(ctx, states, periodic=bool(layout is not None and layout.periodic))
        self.layout = self.enc.layout
        self.stride = stride if stride is not None else self.layout.unit
        self._coeffs = _CoeffCache()
        self._zero = None

    # zero-state pair, built lazily (REF :58-62 builds it eagerly; only _normalize_via_xor_zero uses it)
    def _normalize_via_xor_zero(self, ct, which: str):
        if self._zero is None:
            self._zero = self.enc.encode(np.zeros(16 if self.enc.states == 1 else (self.enc.states, 16), dtype=np.uint8))
        return self._xor_ct(ct, self._zero[0] if which == "hi" else self._zero[1])

    def _basis16(self, ct):
        return gf_basis16(self.ctx, ct)

    def _gf_poly_eval_2var(self, ct_hi, ct_lo, mult: int, which: str):
        return gf_eval(self.ctx, self._coeffs, mult, which, ct_hi, ct_lo)

    def _gf2_renorm_pack(self, u, fl):
        """renorm_packed(pack(GF2(u))): with the packing renorm (StateEncoder.renorm_pack: the
        device encode packs) the multipliers run one level lower, no pack level"""
        enc = self.enc
        if getattr(enc, "pack_renorm_direct", lambda ct=None: False)(u[0]):
            return enc.renorm_pack(*self.gf_mult_2(*u, out_level=fl, defer_conj=True), level=NEED_XOR)
        if self._gf2_pair_renorm():
            return enc.pack(*enc.renorm(*self.gf_mult_2(*u, out_level=fl, defer_conj=True), level=NEED_XOR + enc.PACK_DEPTH))
        return enc.renorm_packed(enc.pack(*self.gf_mult_2(*u, out_level=fl + enc.PACK_DEPTH, defer_conj=True)), level=NEED_XOR)

    def _gf2_pair_renorm(self) -> bool:
        """the GF pair's output renormalised unpacked, packed after (_GF2_PAIR): strict renorms, a periodic
        layout the pair renorm serves"""
        return _GF2_PAIR and not FOLDS.pack and self.enc.renorm_hook is None and self.layout.periodic

    def hoist_input_level(self) -> int:
        """the level the strict hoist's packed renorm hands out (y): the unpack and the GF pair's inputs"""
        gf_in = RENORM_FLOOR + LUT2_DEPTH + (0 if self._gf2_pair_renorm() else self.enc.PACK_DEPTH)
        return gf_in + self.enc.UNPACK_DEPTH

    def gf_mult_2(self, ct_hi, ct_lo, out_level=None, defer_conj: bool = False):
        return gf_mult_pair(self.ctx, self._coeffs, 2, ct_hi, ct_lo, out_level, defer_conj)

    def gf_mult_3(self, ct_hi, ct_lo, out_level=None):
        return gf_mult_pair(self.ctx, self._coeffs, 3, ct_hi, ct_lo, out_level)

    def _col_shift_rowmajor(self, ct, k_up: int):
        return self.ctx.rotate(ct, -4 * k_up * self.stride)

    def _renorm_pair(self, hi, lo, level=None):
        return self.enc.renorm(hi, lo, level)

    def _xor_ct(self, a, b, out_level=None, keep_b=None, defer_conj: bool = False):
        """XOR4(a, b); defer_conj: the result goes straight into a secret-key renorm, which may take
        the split LUT's S1 + conj(S2) unsummed (utils.ConjSum: no conjugation key switch)"""
        kw = {"defer_conj": True} if defer_conj and FOLDS.conj else {}
        if keep_b is not None:
            kw["keep_b"] = keep_b
        if kw and takes_kw(self.xor4.apply, *kw):
            return self.xor4.apply(a, b, out_level, **kw)
        return self.xor4.apply(a, b, out_level)

    def _xor_pair(self, a, b, out_level=None):
        """(XOR4(a_hi, b_hi), XOR4(a_lo, b_lo))"""
        if hasattr(self.xor4, "apply_pair"):
            return self.xor4.apply_pair(a[0], b[0], a[1], b[1], out_level)
        return pair(self.ctx, lambda: self._xor_ct(a[0], b[0], out_level), lambda: self._xor_ct(a[1], b[1], out_level))

    def __call__(self, ct_hi, ct_lo, do_final_bootstrap: bool = True, debug: Dict[str, Any] | None = None):
        steps = [-4 * k * self.stride for k in (1, 2, 3)]  # _col_shift_rowmajor(ct, k), hoisted
        rh, rl = rot_pair(self.ctx, ct_hi, ct_lo, steps)
        rot = {k: (rh[k - 1], rl[k - 1]) for k in (1, 2, 3)}
        return self.mix_rotated((ct_hi, ct_lo), rot, do_final_bootstrap, debug)

    # ---------------------------------------------------------------- packed XOR stage
    def packed_ok(self) -> bool:
        """the packed XOR stage applies: periodic layout with room for hi | lo side by side, the
        secret-key renorm (not true-FHE), fused LUTs and the engine's packed renorms"""
        ctx = self.ctx
        return (self.layout.packable and self.enc.renorm_hook is None and getattr(ctx, "fused_luts", False)
                and getattr(ctx, "renorm_unpack", None) is not None)

    def packed_input_need(self) -> int:
        """the level mix_packed needs on its (ShiftRows') output: NEED_XOR + PACK_DEPTH when the rot
        form's GF multipliers run low (_MC_GF_LOW: every XOR4 input is a pack of the input or of a
        renormalised ciphertext), else NEED_GF + PACK_DEPTH (the GF pair on the input's level chain)"""
        if _MC_GF_LOW and os.environ.get("AESFHE_MC_FORM", "rot") == "rot":
            return NEED_XOR + self.enc.PACK_DEPTH
        return NEED_XOR + LUT2_DEPTH + self.enc.PACK_DEPTH

    def _plain(self, key, make):
        """a slot-vector plaintext encoded once per module (make() -> the vector)"""
        cache = self.__dict__.setdefault("_pt_cache", {})
        if key not in cache:
            cache[key] = self.ctx.encode(make())
        return cache[key]

    def sr_entry(self, x_hi, x_lo, shift):
        """(p0, p1) = (pack(SR(x)), pack(rot(SR(x), s1))) from the pair x BEFORE ShiftRows, ShiftRows
        homomorphic and fused with MixColumns' first column shift and the two packs (the GHS12 form of
        REF/temp/shiftrows_mixcolumns_fused.py:44-258, shiftrows_mixcolumns.py): with R^k x = rot(x, k s1)
        (s1 = -4 unit; R^4 x = x, x being 16-unit-periodic), SR(x) = sum_k rot(m_k, k s1) R^k x over the
        row masks m_k (REF/shift_rows.py:20-56) and rot(SR(x), s1) = sum_k rot(m_k, (k+1) s1) R^(k+1) x.
        The three rotations of each half come from one hoisted key switch (rot_pair: one ModUp per half),
        the packing masks ride in the row masks, so both packed outputs are ONE level of mask products
        below x -- against ShiftRows (6 masked rotations, one level), r1 (2 rotations) and the packs (one
        more level).  Same bytes; the renorm before hands x out one level lower (packed_input_need)."""
        ctx, lay = self.ctx, self.layout
        s1 = -4 * self.stride
        if getattr(shift, "direction", None) != -1 or not lay.same(getattr(shift, "layout", None)) or not lay.packable:
            raise ValueError("sr_entry: ShiftRows of this module's packed periodic layout")
        rh, rl = rot_pair(ctx, x_hi, x_lo, [s1, 2 * s1, 3 * s1])
        R = ((x_hi, *rh), (x_lo, *rl))
        rows = [lay.row_mask(r).real for r in range(4)]
        halves = [lay.half_mask(h).real for h in (0, 1)]

        fused = getattr(getattr(ctx, "engine", None), "mul_pt_sum", None) if _PT_SUM else None

        def masked_sum(tag, shift_k):
            pairs = []
            for h in (0, 1):
                for k in range(4):
                    j = (k + shift_k) % 4
                    pt = self._plain((tag, h, k), lambda: np.roll(rows[k], (k + shift_k) * s1) * halves[h])
                    pairs.append((R[h][j], pt))
            if fused is not None:  # the eight products summed in ONE kernel (aesfhe_mul_pt_sum)
                return fused(pairs)
            terms = [ctx.multiply(c, p) for c, p in pairs]
            while len(terms) > 1:  # a tree of adds (the lazy products combine without rescales)
                terms = [ctx.add(terms[i], terms[i + 1]) if i + 1 < len(terms) else terms[i] for i in range(0, len(terms), 2)]
            return terms[0]

        return masked_sum("sr_p0", 0), masked_sum("sr_p1", 1)

    def mix_packed(self, ct_hi, ct_lo, do_final_bootstrap: bool = True, sr=None, on_sr=None):
        """MixColumns with its XOR stage on packed states (StateEncoder.pack: hi and lo side by side
        in one ciphertext, the XOR4 LUT being the same for both halves): the three XOR pairs of
        mix_rotated become three single XOR4s, their renorms single-ciphertext renorms, and the
        final bootstrap one sparse bootstrap at period 2P.  Returns the PACKED output (the caller's
        AddRoundKey XORs it with a packed round key and unpacks in its renorm).  The GF
        multipliers stay pairs (they mix hi and lo); their outputs and the column shifts are
        packed (one level: inputs one level higher than mix_rotated's).  Default form
        (AESFHE_MC_FORM=rot): with u = x ^ r1, the column shift by two of u is r2 ^ r3 (R^2 x =
        r2, R^2 r1 = r3), so 2x ^ 3 r1 ^ r2 ^ r3 = 2u ^ (r1 ^ R^2 u): one GF multiplier pair on
        the renormalised, unpacked u, one extra rotation pair of u and three single XOR4s, and
        only r1 shifted from the input.  AESFHE_MC_FORM=xtime computes r2 ^ r3 from shifted
        inputs (2 (x ^ r1) ^ (r1 ^ r2 ^ r3), four XOR4s, xtime being GF(2)-linear);
        AESFHE_MC_FORM=2gf keeps the reference's two multiplier pairs (GF2(x), GF3(r1)).  The
        bytes are the same in every form.  sr (rot form): a ShiftRows module -- (ct_hi, ct_lo) is the
        pair BEFORE ShiftRows, which sr_entry fuses with the first column shift and the packs
        (AESFHE_SR_MC_ENTRY=0: the caller runs ShiftRows first); on_sr(p0): a debug hook for pack(SR(x))."""
        ctx, enc = self.ctx, self.enc
        fl = RENORM_FLOOR
        gl = fl + LUT2_DEPTH + enc.PACK_DEPTH
        form = os.environ.get("AESFHE_MC_FORM", "rot")
        if form == "rot":
            s1 = -4 * self.stride
            if sr is not None:
                p0, p1 = self.sr_entry(ct_hi, ct_lo, sr)
            else:
                (rh1,), (rl1,) = rot_pair(ctx, ct_hi, ct_lo, [s1])
                p1, p0 = pair(ctx, lambda: enc.pack(rh1, rl1), lambda: enc.pack(ct_hi, ct_lo), shared=(ct_hi, ct_lo, rh1, rl1))
            if on_sr is not None:
                on_sr(p0)
            if _MC_GF_LOW:
                # the GF multiplier pair five levels lower (inputs at gl instead of gl + LUT2_DEPTH) and its
                # packed output renormalised before the last XOR4: a renorm costs less than the pair's
                # key switches and LUT sums at five more limbs; u at gl serves both branches (round 5).
                # r1 is the second operand of both XOR4s at one level: its drop and std basis built once
                kb = {} if _SHARE_R1 else None
                x = self._xor_ct(p0, p1, fl, kb, defer_conj=True)
                if not FOLDS.unpack and _MC_HOIST and self.enc.layout.packable:
                    # strict renorm: y = renorm(x) packed, then ONE batched key switch of y (aesfhe_galois_multi:
                    # one ModUp of its one source) for the unpack's half swap rot(y, P) and for R^2 u packed,
                    # which within each P-slot half is rot(y, 2 s1) on the first 8 unit slots and
                    # rot(y, 2 s1 + P) on the others -- no rotation waits for the unpack
                    P = self.layout.period
                    y = enc.renorm_packed(x, level=self.hoist_input_level())
                    z, ym, yp = rotate_multi(ctx, [(y, P), (y, 2 * s1), (y, 2 * s1 + P)])  # one source: one ModUp
                    u = enc.unpack(y, z)
                    lowm = lambda: np.tile((np.arange(P) < -2 * s1).astype(np.float64), self.sc // P)  # noqa: E731

                    def r1_r2r3_low():
                        a = self._plain(("r2u", 0), lowm)
                        b = self._plain(("r2u", 1), lambda: 1.0 - lowm())
                        w_pre = ctx.add(ctx.multiply(ym, a), ctx.multiply(yp, b))
                        return enc.renorm_packed(self._xor_ct(w_pre, p1, fl, kb, defer_conj=True), level=NEED_XOR)
                else:
                    u = enc.renorm_unpack(x, level=gl)

                    def r1_r2r3_low():
                        (vh,), (vl,) = rot_pair(ctx, u[0], u[1], [2 * s1])
                        return enc.renorm_packed(self._xor_ct(enc.pack(vh, vl), p1, fl, kb, defer_conj=True), level=NEED_XOR)
                two, w = pair(ctx, lambda: self._gf2_renorm_pack(u, fl),
                              r1_r2r3_low, shared=(*u, p1))
                acc = enc.renorm_packed(self._xor_ct(two, w, fl, defer_conj=True), level=NEED_BOOTSTRAP if do_final_bootstrap else None)
                if do_final_bootstrap:
                    acc = bootstrap1(ctx, acc, 2 * self.layout.period)
                return acc
            u = enc.renorm_unpack(self._xor_ct(p0, p1, fl), level=gl + LUT2_DEPTH)

            def r1_r2r3():
                # R^2 u = r2 ^ r3, shifted at the level its pack + XOR4 need (gl), not u's
                (vh,), (vl,) = rot_pair(ctx, drop_to(ctx, u[0], gl), drop_to(ctx, u[1], gl), [2 * s1])
                return enc.renorm_packed(self._xor_ct(enc.pack(vh, vl), p1, fl), level=NEED_XOR)
            two, w = pair(ctx, lambda: enc.pack(*self.gf_mult_2(*u, out_level=gl)), r1_r2r3, shared=(*u, p1))
            acc = enc.renorm_packed(self._xor_ct(two, w, fl), level=NEED_BOOTSTRAP if do_final_bootstrap else None)
            if do_final_bootstrap:
                acc = bootstrap1(ctx, acc, 2 * self.layout.period)
            return acc
        steps = [-4 * k * self.stride for k in (1, 2, 3)]
        rh, rl = rot_pair(ctx, ct_hi, ct_lo, steps)
        if form == "xtime":
            # 2x ^ 3 r1 ^ r2 ^ r3 = 2 (x ^ r1) ^ (r1 ^ r2 ^ r3) (xtime is GF(2)-linear): ONE GF
            # multiplier pair and four single XOR4s instead of two pairs and three XOR4s
            p1, p0 = pair(ctx, lambda: enc.pack(rh[0], rl[0]), lambda: enc.pack(ct_hi, ct_lo), shared=(ct_hi, ct_lo, *rh, *rl))
            r2, r3 = pair(ctx, lambda: enc.pack(rh[1], rl[1]), lambda: enc.pack(rh[2], rl[2]))
            # r1 (p1) enters two XOR4s: as the second operand of both (XOR is symmetric), its
            # level drop and std basis (conjugate + power chain) are built once (keep_b)
            kb = {} if _SHARE_R1 else None
            u, v = pair(ctx, lambda: enc.renorm_unpack(self._xor_ct(p0, p1, fl, kb), level=gl + LUT2_DEPTH),
                        lambda: enc.renorm_packed(self._xor_ct(r2, r3, fl), level=NEED_XOR), shared=(p1,))
            two, w = pair(ctx, lambda: enc.pack(*self.gf_mult_2(*u, out_level=gl)),
                          lambda: enc.renorm_packed(self._xor_ct(v, p1, fl, kb) if kb is not None else self._xor_ct(p1, v, fl),
                                                    level=NEED_XOR))
            acc = enc.renorm_packed(self._xor_ct(two, w, fl), level=NEED_BOOTSTRAP if do_final_bootstrap else None)
            if do_final_bootstrap:
                acc = bootstrap1(ctx, acc, 2 * self.layout.period)
            return acc
        two, thr = pair(ctx, lambda: self.gf_mult_2(ct_hi, ct_lo, out_level=gl),
                        lambda: self.gf_mult_3(rh[0], rl[0], out_level=gl))
        p2, p3 = pair(ctx, lambda: enc.pack(*two), lambda: enc.pack(*thr), shared=(*two, *thr))
        r2, r3 = pair(ctx, lambda: enc.pack(rh[1], rl[1]), lambda: enc.pack(rh[2], rl[2]), shared=(*rh, *rl))
        x1, x2 = pair(ctx, lambda: enc.renorm_packed(self._xor_ct(p2, p3, fl), level=NEED_XOR),
                      lambda: enc.renorm_packed(self._xor_ct(r2, r3, fl), level=NEED_XOR))
        acc = enc.renorm_packed(self._xor_ct(x1, x2, fl), level=NEED_BOOTSTRAP if do_final_bootstrap else None)
        if do_final_bootstrap:
            acc = bootstrap1(ctx, acc, 2 * self.layout.period)
        return acc

    def mix_rotated(self, x, rot, do_final_bootstrap: bool = True, debug: Dict[str, Any] | None = None):
        """GF2(x) ^ GF3(r1) ^ r2 ^ r3 from the state pair x and its column shifts rot[k] = r_k
        (the rest of __call__; shiftrows_mixcolumns.py supplies ShiftRows-permuted shifts)"""
        log = (lambda k, v: debug.__setitem__(k, v)) if isinstance(debug, dict) else (lambda k, v: None)
        ct_hi, ct_lo = x
        for k in (1, 2, 3):
            log(f"rotc{k}", rot[k])
        log("in", (ct_hi, ct_lo))
        # every XOR pair below is renormalised right away (REF :104-106), so the LUTs run on
        # inputs dropped to the lowest level that leaves their output at RENORM_FLOOR
        fl = RENORM_FLOOR
        # the two GF multiplier pairs are independent: one per branch stream, each batching
        # its own bases and evaluations; in true-FHE mode on two streams even
        # in a one-stream context, with the bootstrap-sized renorms that follow
        fhe = self.enc.renorm_hook is not None
        two, thr = pair(self.ctx, lambda: self.gf_mult_2(ct_hi, ct_lo, out_level=fl + LUT2_DEPTH),
                        lambda: self.gf_mult_3(*rot[1], out_level=fl + LUT2_DEPTH), fork=fhe and _FHE_FORK)
        log("two", two)
        log("thr", thr)
        last = NEED_BOOTSTRAP if do_final_bootstrap else None  # bootstrapped next (from level 0), else fresh
        quad = fhe and getattr(self.enc, "renorm_quad_hook", None) is not None
        if quad:
            # true-FHE with the quad bootstrap (zeta16_noise_reducer.BootstrapSnap.apply_quad): the GF
            # outputs renormalised together (one bootstrap for both pairs), then the tree
            # (2x ^ 3r1) ^ (r2 ^ r3): its two first XOR pairs renormalised together again, so a
            # round's MixColumns takes two quad bootstraps and one pair bootstrap instead of five
            # pair bootstraps.  Every XOR4 still meets two freshly snapped inputs (r2 / r3 come
            # straight from SubBytes' renorm)
            two, thr = self.enc.renorm_two(two, thr, level=NEED_XOR)
            a1 = self._xor_pair(two, thr, fl)
            log("acc1", a1)
            b1 = self._xor_pair(rot[2], rot[3], fl)
            log("r23", b1)
            x1, x2 = self.enc.renorm_two(a1, b1, level=NEED_XOR)
            acc = self._renorm_pair(*self._xor_pair(x1, x2, fl), level=last)
            log("acc3", acc)
            return acc
        if fhe:
            # true-FHE: the GF multipliers amplify their inputs' errors up to ~20x, so their outputs
            # are renormalised (bootstrap + snap) before the first XOR; then the reference's
            # chain, each of r2 / r3 meeting a freshly snapped partner (zeta16_noise_reducer.py)
            two, thr = pair(self.ctx, lambda: self._renorm_pair(*two, level=NEED_XOR),
                            lambda: self._renorm_pair(*thr, level=NEED_XOR), fork=_FHE_FORK)
        if isinstance(debug, dict) or fhe:
            # the reference's chain ((2x ^ 3r1) ^ r2) ^ r3 and its debug keys (REF :127-163): acc1 and
            # acc2 before their renorm, acc3 after it.  True-FHE mode keeps this order: each of r2 / r3
            # meets a freshly snapped partner (the tree's r2 ^ r3 would add two residuals)
            a1 = self._xor_pair(two, thr, fl)
            log("acc1", a1)
            a2 = self._xor_pair(self._renorm_pair(*a1, level=NEED_XOR), rot[2], fl)
            log("acc2", a2)
            acc = self._renorm_pair(*self._xor_pair(self._renorm_pair(*a2, level=NEED_XOR), rot[3], fl), level=last)
        else:
            # out = (2x ^ 3r1) ^ (r2 ^ r3): the chain regrouped (XOR is associative, every XOR pair
            # still renormalised, the same three XOR pairs and renorms), so the first two XOR pairs
            # are independent and run on the two branch streams
            x1, x2 = pair(self.ctx, lambda: self._renorm_pair(*self._xor_pair(two, thr, fl), level=NEED_XOR),
                          lambda: self._renorm_pair(*self._xor_pair(rot[2], rot[3], fl), level=NEED_XOR))
            acc = self._renorm_pair(*self._xor_pair(x1, x2, fl), level=last)
        log("acc3", acc)
        out_hi, out_lo = acc
        # true-FHE mode: the renorm above already is a bootstrap (+ snap), the final one merges in
        if do_final_bootstrap and self.enc.renorm_hook is None:
            out_hi, out_lo = bootstrap2(self.ctx, out_hi, out_lo, self.layout.boot_period)
            log("out", (out_hi, out_lo))
        return out_hi, out_lo
