"""StateEncoder: 16-byte AES state <-> (ct_hi, ct_lo) (REF/state_encoder.py:9-38).

Byte i (column-first order, REF/README.md:103-104) goes to slot i*stride with
stride = slot_count/16; every other slot holds 1+0j.

``states`` > 1 selects the slot-packed layout (the paper's layout in
REF/main.py:121-140): state b of a batch of B <= stride states holds byte i in slot
i*stride + b.  Every rotation the AES modules issue is a multiple of stride, so the B
columns never mix; slots with (j mod stride) >= B hold 1+0j as in the reference.
``encode`` then takes a (B, 16) uint8 array and ``decode`` returns one.

``periodic=True`` (the pipeline's default) packs the same bytes with rotation
unit B instead of stride: byte i of state b in slot i*B + b, and that 16B-slot block repeated
over all slots.  Every AES step is slot-wise or a rotation by a multiple of the unit, so the
message stays 16B-periodic -- a polynomial in the subring Z[X^(N/32B)] -- and the final
bootstraps of MixColumns / InvMixColumns run as sparse-slot bootstraps (aesfhe_bootstrap_pair_sparse,
a trace plus period-sized transforms).  Decoded states are the same in both layouts.

The two layouts are NOT interchangeable on ciphertexts: the encoder tags what it produces with
its layout (``tag_layout``) and ``decode`` / ``renorm`` / ``AESPipeline.decrypt`` refuse a
ciphertext tagged with the other one (``check_layout``).  ``StateEncoder(ctx, B)``
keeps the reference layout; ``AESPipeline`` picks the periodic one where the context has the
sparse bootstrap (its ``layout`` attribute says which).
"""
import os
from typing import Any, Tuple

import numpy as np

from utils import FOLDS, ConjSum, ZetaEncoder, conj_sum, takes_kw, tally_renorm

# AESFHE_RENORM_FRESH=1: ignore renorm target levels (A/B measurements of DESIGN.md §3.11)
_RENORM_FRESH = os.environ.get("AESFHE_RENORM_FRESH") == "1"


class SlotLayout:
    """Where the bytes of B states sit: the reference layout (byte i of state b in slot
    i*stride + b, stride = slot_count/16, every other slot 1) or the periodic one (unit = B, the
    16B-slot block repeated).  `unit` is the rotation unit of ShiftRows / MixColumns."""

    def __init__(self, sc: int, states: int = 1, periodic: bool = False):
        if not 1 <= states <= sc // 16:
            raise ValueError(f"states per ciphertext must be in [1, {sc // 16}], got {states}")
        if periodic and states & (states - 1):
            raise ValueError("the periodic layout needs a power-of-two number of states")
        self.sc, self.states, self.periodic = sc, states, periodic
        self.unit = states if periodic else sc // 16
        self.period = 16 * self.unit

    @property
    def boot_period(self):
        """the slot period a sparse bootstrap may use (None: the full-slot bootstrap)"""
        return self.period if self.period < self.sc else None

    @property
    def renorm_states(self) -> int:
        """the engine renorm's `states` (periodic: every slot holds state data)"""
        return self.sc // 16 if self.periodic else self.states

    def tile(self, block: np.ndarray) -> np.ndarray:
        return np.tile(block, self.sc // self.period)

    def row_mask(self, r: int) -> np.ndarray:
        """ones on row r (bytes r + 4c) of every state"""
        m = np.zeros(self.period, dtype=np.complex128)
        for c in range(4):
            m[(r + 4 * c) * self.unit:(r + 4 * c) * self.unit + self.states] = 1.0
        return self.tile(m)

    @property
    def packable(self) -> bool:
        """hi and lo fit side by side in one ciphertext: the packed form holds the
        hi nibbles in slots (j mod 2P) < P and the lo nibbles in the others (P = period)"""
        return self.periodic and 2 * self.period <= self.sc

    def half_mask(self, which: int) -> np.ndarray:
        """ones on the hi (0) / lo (1) half of every 2P-slot block of the packed form"""
        m = np.zeros(2 * self.period, dtype=np.complex128)
        m[which * self.period:(which + 1) * self.period] = 1.0
        return np.tile(m, self.sc // (2 * self.period))

    def same(self, other) -> bool:
        return other is not None and (self.sc, self.states, self.periodic) == (other.sc, other.states, other.periodic)


def tag_layout(layout: SlotLayout, *cts):
    """mark ciphertexts as holding states in `layout` (checked by check_layout); returns them"""
    for c in cts:
        try:
            c.layout = layout
        except AttributeError:  # a context whose ciphertexts carry no tag (the CPU oracle's)
            pass
    return cts


def check_layout(layout: SlotLayout, *cts) -> None:
    """raise if a ciphertext was tagged with another slot layout (a pair made by an encoder with
    the reference layout decrypts to wrong bytes under the periodic one, and vice versa);
    untagged ciphertexts pass"""
    for c in cts:
        lay = getattr(c, "layout", None)
        if lay is not None and not layout.same(lay):
            raise ValueError(f"ciphertext holds states in the {_describe(lay)} slot layout, "
                             f"this encoder / pipeline uses the {_describe(layout)} one")


def _describe(lay: SlotLayout) -> str:
    return f"{'periodic' if lay.periodic else 'reference'} (states={lay.states})"


class StateEncoder:
    """pairs > 1: a multi-pair batch -- `pairs` independent ciphertext pairs,
    each holding `states` states in this layout, carried as ONE stacked hi and ONE stacked lo
    ciphertext (ctx.stack): encode takes (pairs, states, 16) / (pairs, 16) bytes, decode returns
    them, and every AES module runs on the stacks unchanged."""

    def __init__(self, ctx, states: int = 1, periodic: bool = False, pairs: int = 1):
        self.ctx = ctx
        self.sc = ctx.engine.slot_count
        self.layout = SlotLayout(self.sc, states, periodic)
        self.stride = self.layout.unit  # rotation unit (REF: slot_count / 16)
        self.states = states
        if pairs < 1:
            raise ValueError("pairs must be >= 1")
        if pairs > 1 and getattr(ctx, "stack", None) is None:
            raise ValueError("multi-pair batches need a context with stacked ciphertexts (ctx.stack)")
        self.pairs = pairs
        # set by AESPipeline(true_fhe=True): renorm(hi, lo) -> hook(hi, lo), the bootstrap + snap
        # that replaces the secret-key renorm (zeta16_noise_reducer.BootstrapSnap)
        self.renorm_hook = None
        self.renorm_quad_hook = None  # true-FHE: two pairs per bootstrap (renorm_two)

    def _as_batch(self, state: np.ndarray) -> np.ndarray:
        state = np.asarray(state, dtype=np.uint8)
        if state.shape == (16,) and self.states == 1:
            return state[None, :]
        if state.shape != (self.states, 16):
            raise ValueError(f"expected a ({self.states}, 16) uint8 state array, got {state.shape}")
        return state

    def _pack(self, nibbles: np.ndarray) -> np.ndarray:
        """nibbles (B, 16) -> slot vector; slot i*unit + b <- zeta^nibbles[b, i] (periodic: tiled)"""
        grid = np.ones((16, self.stride), dtype=np.complex128)
        grid[:, :nibbles.shape[0]] = ZetaEncoder.to_zeta(nibbles.astype(np.uint8).T, 16)
        return self.layout.tile(grid.reshape(-1))

    def _take(self, slots: np.ndarray) -> np.ndarray:
        """slot vector -> (B, 16) state slots"""
        return slots[:16 * self.stride].reshape(16, self.stride)[:, :self.states].T

    def _pair_states(self, state: np.ndarray):
        """(pairs, ...) bytes -> the per-pair state arrays; a single pair's shape broadcasts"""
        state = np.asarray(state, dtype=np.uint8)
        one = (16,) if self.states == 1 else (self.states, 16)
        if state.shape == one:
            return [state] * self.pairs
        if state.shape != (self.pairs,) + one:
            raise ValueError(f"expected a {(self.pairs,) + one} uint8 state array, got {state.shape}")
        return list(state)

    def encode(self, state: np.ndarray) -> Tuple[Any, Any]:
        if self.pairs > 1:
            his, los = zip(*[self._encode1(s) for s in self._pair_states(state)])
            return tag_layout(self.layout, self.ctx.stack(his), self.ctx.stack(los))
        return self._encode1(self._pair_states(state)[0])

    def _encode1(self, state):
        st = self._as_batch(state)
        return tag_layout(self.layout, self.ctx.encrypt(self._pack(st >> 4)), self.ctx.encrypt(self._pack(st & 0x0F)))

    def decode(self, ct_hi, ct_lo) -> np.ndarray:
        check_layout(self.layout, ct_hi, ct_lo)
        if self.pairs > 1:
            return np.stack([self._decode1(h, l) for h, l in zip(self.ctx.unstack(ct_hi), self.ctx.unstack(ct_lo))])
        return self._decode1(ct_hi, ct_lo)

    def _decode1(self, ct_hi, ct_lo) -> np.ndarray:
        hi = ZetaEncoder.from_zeta(self._take(self.ctx.decrypt(ct_hi)), 16)
        lo = ZetaEncoder.from_zeta(self._take(self.ctx.decrypt(ct_lo)), 16)
        out = ((hi << 4) | lo).astype(np.uint8)
        return out[0] if self.states == 1 else out

    # ---------------------------------------------------------------- packed form
    PACK_DEPTH = 1  # pack(): one plaintext product

    def pack(self, ct_hi, ct_lo):
        """(hi, lo) -> ONE ciphertext, hi on the first half of every 2P-slot block and lo on the
        second: hi * mask_0 + lo * mask_1 (one level; both halves are P-periodic, so no rotation)"""
        if not self.layout.packable:
            raise ValueError("the packed form needs the periodic layout with 2 * period <= slot count")
        if isinstance(ct_hi, ConjSum) or isinstance(ct_lo, ConjSum):
            # the masks are real: pack(conj a, conj b) = conj(pack(a, b)), so a pair of
            # utils.ConjSum packs into one (both halves' S1 packed, and both S2)
            if not (isinstance(ct_hi, ConjSum) and isinstance(ct_lo, ConjSum)):
                return self.pack(conj_sum(self.ctx, ct_hi), conj_sum(self.ctx, ct_lo))
            return ConjSum(self.pack(ct_hi.s1, ct_lo.s1), self.pack(ct_hi.s2, ct_lo.s2))
        ctx = self.ctx
        if getattr(self, "_half_pts", None) is None:
            self._half_pts = [ctx.encode(self.layout.half_mask(w)) for w in (0, 1)]
        return ctx.add(ctx.multiply(ct_hi, self._half_pts[0]), ctx.multiply(ct_lo, self._half_pts[1]))

    def _packed_slots(self, st: np.ndarray) -> np.ndarray:
        hi, lo = self._pack(st >> 4), self._pack(st & 0x0F)
        return np.where(self.layout.half_mask(0).real > 0.5, hi, lo)

    def encode_packed(self, state: np.ndarray):
        """a state (batch) encrypted directly in the packed form"""
        if self.pairs > 1:
            cts = [self.ctx.encrypt(self._packed_slots(self._as_batch(s))) for s in self._pair_states(state)]
            return tag_layout(self.layout, self.ctx.stack(cts))[0]
        return tag_layout(self.layout, self.ctx.encrypt(self._packed_slots(self._as_batch(self._pair_states(state)[0]))))[0]

    def decode_packed(self, ct) -> np.ndarray:
        check_layout(self.layout, ct)
        if self.pairs > 1:
            return np.stack([self._decode_packed1(c) for c in self.ctx.unstack(ct)])
        return self._decode_packed1(ct)

    def _decode_packed1(self, ct) -> np.ndarray:
        z = self.ctx.decrypt(ct)
        hi = ZetaEncoder.from_zeta(self._take(z), 16)
        lo = ZetaEncoder.from_zeta(self._take(z[self.layout.period:]), 16)
        out = ((hi << 4) | lo).astype(np.uint8)
        return out[0] if self.states == 1 else out

    UNPACK_DEPTH = 1  # unpack(): one mask product after the rotation

    def _fold_conj(self, *cts):
        """the renorm's inputs with any utils.ConjSum summed homomorphically unless the conjugation
        fold is on (FOLDS.conj; strict renorms are the identity on the message)"""
        return tuple(c if FOLDS.conj else conj_sum(self.ctx, c) for c in cts)

    def unpack(self, ct, z=None):
        """the packed state -> its (hi, lo) pair, homomorphically (the inverse of pack): both halves
        are P-periodic inside the 2P-periodic message, so z = rot_P(ct) holds lo where ct holds hi
        and vice versa, and hi = z + m0 (ct - z), lo = ct - m0 (ct - z) -- one rotation and one
        mask product (UNPACK_DEPTH levels), every slot of both outputs as the packed input's.
        z: rot_P(ct) when the caller has it (from a hoisted key switch)"""
        ctx = self.ctx
        if getattr(self, "_half_pts", None) is None:
            self._half_pts = [ctx.encode(self.layout.half_mask(w)) for w in (0, 1)]
        if z is None:
            z = ctx.rotate(ct, self.layout.period)
        t = ctx.multiply(ctx.sub(ct, z), self._half_pts[0])
        return tag_layout(self.layout, ctx.add(z, t), ctx.sub(ct, t))

    def renorm_packed(self, ct, level=None):
        """renorm of a packed state, packed again (ct may be a utils.ConjSum: s1 + conj(s2) renormalised
        with the conjugation folded into the decryption when FOLDS.conj)"""
        (ct,) = self._fold_conj(ct)
        lv = None if _RENORM_FRESH else level
        single = self.ctx.renorm_single
        if isinstance(ct, ConjSum):
            if takes_kw(single, "period", "conj"):
                tally_renorm(self.ctx, ct.s1)
                return single(ct.s1, lv, period=2 * self.layout.period, conj=ct.s2)
            ct = conj_sum(self.ctx, ct)
        tally_renorm(self.ctx, ct)
        if takes_kw(single, "period"):
            return single(ct, lv, period=2 * self.layout.period)
        return single(ct, lv)  # a context whose renorm_single takes no period

    def renorm_perm(self, ct_hi, ct_lo, perm, level=None):
        """renorm(hi, lo) followed by a byte permutation (output byte i <- input byte perm[i]), the
        permutation folded into the device renorm (aesfhe_renorm_periodic_perm; FOLDS.sr, the caller
        checks renorm_perm_ok first).  utils.ConjSum halves are folded as in renorm"""
        if not FOLDS.sr:
            raise RuntimeError("renorm_perm: the ShiftRows fold is off (utils.FOLDS.sr)")
        ct_hi, ct_lo = self._fold_conj(ct_hi, ct_lo)
        conj = None
        if isinstance(ct_hi, ConjSum) and isinstance(ct_lo, ConjSum):
            conj, ct_hi, ct_lo = (ct_hi.s2, ct_lo.s2), ct_hi.s1, ct_lo.s1
        else:
            ct_hi, ct_lo = conj_sum(self.ctx, ct_hi), conj_sum(self.ctx, ct_lo)
        check_layout(self.layout, ct_hi, ct_lo)
        tally_renorm(self.ctx, ct_hi, ct_lo)
        return tag_layout(self.layout, *self.ctx.renorm_periodic_perm(ct_hi, ct_lo, self.layout.period, perm,
                                                                      None if _RENORM_FRESH else level, conj=conj))

    def renorm_unpack_perm(self, ct, perm, level=None):
        """renorm_unpack followed by a byte permutation of both halves, folded into the device renorm
        (aesfhe_renorm_unpack_perm; FOLDS.sr and FOLDS.unpack); the caller checks renorm_perm_ok"""
        if not (FOLDS.sr and FOLDS.unpack):
            raise RuntimeError("renorm_unpack_perm: the ShiftRows / unpack folds are off (utils.FOLDS)")
        (ct,) = self._fold_conj(ct)
        conj = None
        if isinstance(ct, ConjSum):
            conj, ct = ct.s2, ct.s1
        check_layout(self.layout, ct)
        tally_renorm(self.ctx, ct)
        return tag_layout(self.layout, *self.ctx.renorm_unpack_perm(ct, self.layout.period, perm, None if _RENORM_FRESH else level,
                                                                    conj=conj))

    def renorm_perm_ok(self, ct=None) -> bool:
        """whether renorm_perm / renorm_unpack_perm run on this encoder / context (the ShiftRows and
        unpack folds on, one period-16 state pair on the device, the engine's direct period-32 codec)"""
        if not (FOLDS.sr and FOLDS.unpack):
            return False
        if not (getattr(self.ctx, "renorm_periodic_perm", None) is not None and getattr(self.ctx, "renorm_unpack_perm", None) is not None
                and self.pack_renorm_direct(ct, need_pack=False)):
            return False
        direct = getattr(getattr(self.ctx, "engine", None), "direct32", None)
        return direct is None or bool(direct())

    def pack_renorm_direct(self, ct=None, need_pack: bool = True) -> bool:
        """whether renorm_pack runs as the device's packing renorm (FOLDS.pack; then its inputs need no
        pack level); ct: an input of the pair -- a stack of several state pairs takes pack + renorm"""
        if not ((FOLDS.pack or not need_pack) and getattr(self.ctx, "renorm_pack", None) is not None and self.renorm_hook is None
                and self.layout.periodic and self.layout.period == 16 and self.pairs == 1):
            return False
        members = getattr(getattr(self.ctx, "engine", None), "members", None)
        return ct is None or members is None or members(ct.s1 if isinstance(ct, ConjSum) else ct) == 1

    def renorm_pack(self, ct_hi, ct_lo, level=None):
        """renorm_packed(pack(hi, lo)): with the pack fold (FOLDS.pack) and one period-16 state pair the
        device renorm encodes the snapped pair straight into the packed form (aesfhe_renorm_pack: no mask
        products, no pack level; utils.ConjSum halves folded as in renorm); otherwise pack, then renorm"""
        if self.pack_renorm_direct(ct_hi):
            ct_hi, ct_lo = self._fold_conj(ct_hi, ct_lo)
            rp = self.ctx.renorm_pack
            conj = None
            if isinstance(ct_hi, ConjSum) and isinstance(ct_lo, ConjSum):
                conj, ct_hi, ct_lo = (ct_hi.s2, ct_lo.s2), ct_hi.s1, ct_lo.s1
            else:
                ct_hi, ct_lo = conj_sum(self.ctx, ct_hi), conj_sum(self.ctx, ct_lo)
            check_layout(self.layout, ct_hi, ct_lo)
            tally_renorm(self.ctx, ct_hi, ct_lo)
            return tag_layout(self.layout, rp(ct_hi, ct_lo, self.layout.period, None if _RENORM_FRESH else level, conj=conj))[0]
        return self.renorm_packed(self.pack(ct_hi, ct_lo), level)

    def renorm_unpack(self, ct, level=None) -> Tuple[Any, Any]:
        """renorm of a packed state into the (hi, lo) pair at `level`.  Strict (FOLDS.unpack off): the
        packed renorm at level + UNPACK_DEPTH, then the homomorphic unpack; with the fold the device
        renorm's encoder gathers the two halves (aesfhe_renorm_unpack).  ct may be a utils.ConjSum"""
        if not FOLDS.unpack or getattr(self.ctx, "renorm_unpack", None) is None:
            lv = None if level is None else level + self.UNPACK_DEPTH
            return self.unpack(self.renorm_packed(ct, lv))
        (ct,) = self._fold_conj(ct)
        lv = None if _RENORM_FRESH else level
        if isinstance(ct, ConjSum):
            check_layout(self.layout, ct.s1)
            tally_renorm(self.ctx, ct.s1)
            return tag_layout(self.layout, *self.ctx.renorm_unpack(ct.s1, self.layout.period, lv, conj=ct.s2))
        check_layout(self.layout, ct)
        tally_renorm(self.ctx, ct)
        return tag_layout(self.layout, *self.ctx.renorm_unpack(ct, self.layout.period, lv))

    def renorm(self, ct_hi, ct_lo, level=None) -> Tuple[Any, Any]:
        """decode -> re-encode (REF/pipeline.py:65-69), done on the device when available;
        `level`: the level the next step needs (None = fresh), honoured by the device path.
        With a renorm_hook (true-FHE mode) the hook runs instead (it reads `level` as the next step's need).
        hi / lo may be utils.ConjSum (s1 + conj(s2)): the periodic device renorm folds the conjugation
        into its decryption; any other path sums them first."""
        ct_hi, ct_lo = self._fold_conj(ct_hi, ct_lo)
        if isinstance(ct_hi, ConjSum) or isinstance(ct_lo, ConjSum):
            per = getattr(self.ctx, "renorm_periodic", None)
            if (isinstance(ct_hi, ConjSum) and isinstance(ct_lo, ConjSum) and self.renorm_hook is None and self.layout.periodic
                    and per is not None and takes_kw(per, "conj")):
                check_layout(self.layout, ct_hi.s1, ct_lo.s1)
                tally_renorm(self.ctx, ct_hi.s1, ct_lo.s1)
                return tag_layout(self.layout, *per(ct_hi.s1, ct_lo.s1, self.layout.period, None if _RENORM_FRESH else level,
                                                    conj=(ct_hi.s2, ct_lo.s2)))
            ct_hi, ct_lo = conj_sum(self.ctx, ct_hi), conj_sum(self.ctx, ct_lo)
        check_layout(self.layout, ct_hi, ct_lo)
        if self.renorm_hook is None:
            tally_renorm(self.ctx, ct_hi, ct_lo)
        return tag_layout(self.layout, *self._renorm(ct_hi, ct_lo, level))

    def renorm_two(self, p, q, level=None):
        """renorm of two (hi, lo) pairs at one point of a step: in true-FHE mode with a quad hook
        (zeta16_noise_reducer.BootstrapSnap.apply_quad) ONE bootstrap refreshes all four
        ciphertexts; otherwise two renorm calls"""
        if self.renorm_quad_hook is not None:
            ps, qs = self._fold_conj(*p), self._fold_conj(*q)
            if not any(isinstance(c, ConjSum) for c in ps + qs):
                check_layout(self.layout, *ps, *qs)
                a, b = self.renorm_quad_hook(ps, qs, level)
                return tag_layout(self.layout, *a), tag_layout(self.layout, *b)
        return self.renorm(*p, level), self.renorm(*q, level)

    def _renorm(self, ct_hi, ct_lo, level):
        if self.renorm_hook is not None:
            return self.renorm_hook(ct_hi, ct_lo, level)
        per = getattr(self.ctx, "renorm_periodic", None)
        if self.layout.periodic and per is not None:
            return per(ct_hi, ct_lo, self.layout.period, None if _RENORM_FRESH else level)
        fast = getattr(self.ctx, "renorm_pair", None)
        if fast is not None:
            st = self.layout.renorm_states
            if level is not None and not _RENORM_FRESH:
                return fast(ct_hi, ct_lo, states=st, level=level)
            return fast(ct_hi, ct_lo) if st == 1 else fast(ct_hi, ct_lo, states=st)
        return self.encode(self.decode(ct_hi, ct_lo))
