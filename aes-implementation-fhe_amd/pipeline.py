"""AESPipeline: AES-128 round orchestration on CKKS/Zeta16 (REF/pipeline.py:17-254).

Drop-in for the reference class: same constructor, same coefficient keys ('xor4',
'sub_hi', 'sub_lo', 'inv_sub_hi', 'inv_sub_lo'), same step order, optional renorm
between steps, per-stage debug snapshots.

Documented deviation: the shipped decrypt (REF/pipeline.py:230-237)
never applies InvMixColumns, so it cannot invert encrypt.  ``decrypt`` here inserts it
after AddRoundKey as the reference README prescribes (REF/README.md:87-94);
``with_inv_mix_columns=False`` reproduces the shipped order.

``fuse_sub_ark=True`` evaluates SubBytes ⊕ AddRoundKey as one fused LUT per nibble
(sub_bytes_ark.py, SURVEY.md §8(f)4, REF/README.md:133-135): the last encrypt round and every
decrypt round, across the (Inv)ShiftRows between them via permuted round keys; one XOR4 pair
and one renorm fewer per fused step, the same bytes.

``fuse_sr_mc=True`` merges ShiftRows into MixColumns' rotations (shiftrows_mixcolumns.py, the
GHS12 refinement of REF/README.md:137-138): three hoisted rotations per nibble instead of six.

``true_fhe=True`` replaces every secret-key renorm by a bootstrap + homomorphic Zeta16 snap
(zeta16_noise_reducer.BootstrapSnap): the XOR4 coefficients are normalised
by 1/256 (REF/gen/generate_xor4_coeffs.py:17) so every LUT output has unit magnitude,
MixColumns' / InvMixColumns' final bootstraps merge into their last renorm, and decrypt
applies each InvShiftRows before the renorm that precedes InvSubBytes (the snap leaves
exactly SubBytes' 13 levels).  No secret key is used between encryption and decryption.

``packed_xor`` (default: wherever it applies) runs MixColumns' XOR stage and the AddRoundKey
after it on packed states -- hi and lo side by side in ONE ciphertext, the XOR4 LUT being the
same for both halves (MixColFinal.mix_packed): single XOR4s instead of pairs,
single-ciphertext renorms, one sparse bootstrap; the renorm after AddRoundKey unpacks into the
(hi, lo) pair SubBytes reads.  A debug dict logs the packed path's own stages (``packed_xor=False``
runs the reference's pair steps).

``states`` = B > 1 runs B independent AES states per ciphertext pair in the slot-packed
layout (state_encoder.py): ``encrypt`` / ``decrypt`` take and return
(B, 16) arrays through the same step sequence, and a (16,) round key is shared by all B
states (a (B, 16) key array gives each state its own).
"""
from __future__ import annotations

import os
from typing import Any, Dict, List, Optional, Tuple

import numpy as np

from add_round_key import AddRoundKey
from invmixcolumns_fhe import InvMixColumnsFHE
from inv_shiftrows import InvShiftRows
from mixcol_final import MixColFinal
from shift_rows import ShiftRows
from state_encoder import StateEncoder, check_layout, tag_layout
from shift_rows import shift_rows_bytes
from shiftrows_mixcolumns import ShiftRowsMixColumnsFusedEnc
from sub_bytes_ark import SubBytesARK
from sub_bytes_lut import SubBytesLUT
from utils import (pair, FOLDS, SHIFTROWS_DEPTH, NEED_GF, NEED_ISR_ISB, NEED_SR_ARK, NEED_SR_MIX, NEED_SUB_ARK_SR, NEED_SUBBYTES, NEED_XOR,
                   RENORM_FLOOR)
from xor4_lut import XOR4LUT

# AESFHE_KEY_BASIS=0: the packed round keys' XOR4 bases rebuilt in every AddRoundKey (A/B runs)
_KEY_BASIS = os.environ.get("AESFHE_KEY_BASIS", "1") != "0"
# AESFHE_FHE_SB_NIB=0: true-FHE mode keeps the reference's 8 -> 4 (Inv)SubBytes (depth 13, double snaps)
# instead of the nibble-bivariate form (A/B runs)
_FHE_NIB = os.environ.get("AESFHE_FHE_SB_NIB", "1") != "0"


class AESPipeline:
    def __init__(self, ctx, coeffs: Dict[str, Any], *, mixcolumns: MixColFinal | None = None,
                 inv_mixcolumns: InvMixColumnsFHE | None = None, use_hard_renorm_between_steps: bool = False,
                 with_inv_mix_columns: bool = True, states: int = 1, fuse_sub_ark: bool = False,
                 fuse_sr_mc: bool = False, true_fhe: bool = False, periodic: bool | None = None,
                 packed_xor: bool | None = None, pairs: int = 1):
        self.ctx = ctx
        self.states = states
        # pairs > 1: a multi-pair batch -- `pairs` ciphertext pairs of `states` states each, run as
        # ONE stacked pair through every step (state_encoder.StateEncoder)
        self.pairs = pairs
        # periodic layout (state_encoder.SlotLayout): default on where the engine
        # has the sparse-slot bootstrap and the state count is a power of two
        if periodic is None:
            periodic = getattr(ctx, "bootstrap_pair_sparse", None) is not None and states & (states - 1) == 0
            for mod in (mixcolumns, inv_mixcolumns):
                lay = getattr(mod, "layout", None)
                if lay is not None:
                    periodic = lay.periodic
        self.encoder = StateEncoder(ctx, states, periodic=periodic, pairs=pairs)
        self.layout = self.encoder.layout
        self.sc = ctx.engine.slot_count
        self.stride = self.layout.unit
        self.true_fhe = true_fhe
        # true-FHE: unit-magnitude XOR4 (REF/gen/generate_xor4_coeffs.py:17), so the snap sees codewords
        self.xor4 = XOR4LUT(ctx, np.asarray(coeffs["xor4"]) / 256.0 if true_fhe else coeffs["xor4"])
        self.sub = SubBytesLUT(ctx, coeffs["sub_hi"], coeffs["sub_lo"])
        self.isub = SubBytesLUT(ctx, coeffs["inv_sub_hi"], coeffs["inv_sub_lo"]) if "inv_sub_hi" in coeffs else None
        self.shift = ShiftRows(ctx, states=states, layout=self.layout)
        self.invshift = InvShiftRows(ctx, states=states, layout=self.layout)
        self.mix = mixcolumns if mixcolumns is not None else MixColFinal(ctx, self.xor4, states=states, layout=self.layout)
        self.invmix = (inv_mixcolumns if inv_mixcolumns is not None else
                       InvMixColumnsFHE(ctx, self.xor4, states=states, layout=self.layout))
        for mod in (self.mix, self.invmix):
            enc = getattr(mod, "enc", None)
            if enc is not None and getattr(enc, "states", 1) != states:
                raise ValueError("mixcolumns / inv_mixcolumns were built for a different states-per-ciphertext count")
            lay = getattr(mod, "layout", None)
            if lay is not None and not self.layout.same(lay):
                raise ValueError("mixcolumns / inv_mixcolumns were built for a different slot layout")
        self.ark = AddRoundKey(self.xor4)
        self.snapper = None
        self.use_hard_renorm_between_steps = use_hard_renorm_between_steps
        self.with_inv_mix_columns = with_inv_mix_columns
        self._rk_cache: List[Tuple[Any, Any]] | None = None
        self._rk_tag = b""
        self.fuse_sub_ark = fuse_sub_ark
        if fuse_sub_ark:
            self.sbark = SubBytesARK(self.sub, coeffs["xor4"])
            self.isbark = SubBytesARK(self.isub, coeffs["xor4"]) if self.isub is not None else None
        self.srmc = None
        if fuse_sr_mc:
            if not hasattr(self.mix, "mix_rotated"):
                raise TypeError("fuse_sr_mc needs a MixColFinal (mix_rotated) as mixcolumns")
            self.srmc = ShiftRowsMixColumnsFusedEnc(ctx, self.mix, states)
        self._fk_cache: Dict[Tuple[int, int], Tuple[Any, Any]] = {}
        self._fk_tag = b""
        # packed XOR stage of encrypt rounds 1..9; AESFHE_PACKED_XOR=0 for A/B
        if packed_xor is None:
            packed_xor = os.environ.get("AESFHE_PACKED_XOR", "1") != "0"
        self.packed_xor = bool(packed_xor and use_hard_renorm_between_steps and not true_fhe and self.srmc is None
                               and hasattr(self.mix, "packed_ok") and self.mix.packed_ok())
        self._pk_cache: List[Any] | None = None
        self._pk_tag = b""
        self._kb_cache: Dict[int, Dict[str, Any]] = {}  # round -> the packed key's dropped form and std basis
        self._kb_tag = b""
        # the same for decrypt rounds 9..1: AddRoundKey + InvMixColumns (with_inv_mix_columns)
        self.packed_dec = bool(self.packed_xor and with_inv_mix_columns and not fuse_sub_ark
                               and hasattr(self.invmix, "packed_ok") and self.invmix.packed_ok())
        # the level encrypt's renorms hand SubBytes: one above its depth in renorm mode, so that it
        # takes the bivariate giant-step form (sub_bytes_lut._outputs_biv; AESFHE_SB_BIV=0 for A/B)
        self.need_sub = NEED_SUBBYTES
        fresh = getattr(ctx.engine, "fresh_level", None)
        # (Inv)SubBytes in the nibble-bivariate form (sub_bytes_lut: depth LUT2_DEPTH instead of 13) in the
        # secret-key renorm mode: its inputs come from a renorm, so they are handed out 9 levels lower
        for lut in (self.sub, self.isub):
            if lut is not None and not fuse_sub_ark:
                lut.use_nibble = bool(use_hard_renorm_between_steps and not true_fhe or true_fhe and _FHE_NIB)
        if true_fhe:
            from zeta16_noise_reducer import BootstrapSnap
            # one snap per renorm with the nibble-bivariate (Inv)SubBytes, two where the reference's
            # 8 -> 4 form's ~3e-2 output errors need them (zeta16_noise_reducer.BootstrapSnap)
            self.snapper = BootstrapSnap(ctx, period=self.layout.boot_period, max_snaps=1 if self.sub.nibble_on() else 2)
            quad = self.snapper.apply_quad if self.snapper.quad_ok() else None
            for enc in (self.encoder, getattr(self.mix, "enc", None), getattr(self.invmix, "enc", None)):
                if enc is not None:
                    enc.renorm_hook = self.snapper.apply_pair
                    enc.renorm_quad_hook = quad
        if self.sub.nibble_on():
            self.need_sub = RENORM_FLOOR + self.sub.need_depth()
        elif (use_hard_renorm_between_steps and not true_fhe and fresh is not None and getattr(ctx, "fused_luts", False)
                and os.environ.get("AESFHE_SB_BIV", "1") != "0"):
            self.need_sub = min(NEED_SUBBYTES + 1, fresh)
        # InvShiftRows -> InvSubBytes (decrypt): the inverse LUT's depth + the masked rotations
        self.need_isr_isb = (RENORM_FLOOR + self.isub.need_depth() + SHIFTROWS_DEPTH
                             if self.isub is not None and self.isub.nibble_on() else NEED_ISR_ISB)

    # ---------------------------------------------------------------- utils
    def _renorm_pair(self, hi, lo, level=None):
        """renorm between steps; `level` = what the next step needs (utils.NEED_*; None = fresh)"""
        if self.true_fhe or self.use_hard_renorm_between_steps:
            return self.encoder.renorm(hi, lo, level)
        return hi, lo

    def _floor(self) -> Optional[int]:
        """output level a step needs when a renorm follows it (utils.RENORM_FLOOR), else None"""
        if self.true_fhe:
            return 1  # the bootstrap reads any level; decrypt's InvShiftRows needs one above 0
        return RENORM_FLOOR if self.use_hard_renorm_between_steps else None

    def _ark_renorm(self, ct, key_pair, level=None):
        """AddRoundKey then renorm: the XOR4s run on inputs dropped just above the floor"""
        return self._renorm_pair(*self.ark(*ct, *key_pair, out_level=self._floor()), level=level)

    def _sub_renorm(self, ct, inverse: bool = False, level=None):
        lut = self.isub if inverse else self.sub
        if lut is None:
            raise KeyError("inv_sub_hi")
        if self.true_fhe:
            level = NEED_SR_ARK  # true-FHE: SubBytes' ~3e-2 output errors get two snaps (ShiftRows +
            #                      the GF multipliers need 6 levels, MixColumns renormalises after them)
        return self._renorm_pair(*self._sub_apply(ct, defer_conj=True, lut=lut), level=level)

    def _encode_key(self, key_bytes: np.ndarray):
        key_bytes = np.asarray(key_bytes, dtype=np.uint8)
        if self.states > 1 and key_bytes.shape == (16,):
            key_bytes = np.broadcast_to(key_bytes, (self.states, 16))
        assert key_bytes.shape == ((16,) if self.states == 1 else (self.states, 16))
        return self.encoder.encode(key_bytes)

    def _prepare_round_keys(self, round_keys: List[np.ndarray]):
        tag = b"".join(np.ascontiguousarray(k, dtype=np.uint8).tobytes() for k in round_keys)
        if self._rk_cache is None or self._rk_tag != tag:  # encrypted round keys are reused across calls
            self._rk_cache = [self._encode_key(np.asarray(k, dtype=np.uint8)) for k in round_keys]
            self._rk_raw = [np.array(k, dtype=np.uint8) for k in round_keys]
            self._rk_tag = tag
        return self._rk_cache

    def _ark_packed(self, x, r: int, defer_conj: bool = False):
        """AddRoundKey on a packed state: XOR4(x, packed round key r).  The key's level drop and
        std basis (its conjugate and power chain) are built once per key schedule and round and
        reused by every later encrypt / decrypt with the same keys (AESFHE_KEY_BASIS=0: rebuilt
        per call) -- the XOR4 then forms only the state's powers.  defer_conj: the result goes into
        renorm_unpack, which takes the split LUT's S1 + conj(S2) unsummed (utils.ConjSum)"""
        key = self._packed_round_key(r)
        if not _KEY_BASIS:
            return self.xor4.apply(x, key, out_level=self._floor())
        if self._kb_tag != self._rk_tag:
            self._kb_cache, self._kb_tag = {}, self._rk_tag
        if not self._xor4_keep_b():  # an XOR4 without basis sharing (a caller-supplied LUT object)
            return self.xor4.apply(x, key, out_level=self._floor())
        kb = self._kb_cache.setdefault(r, {})
        if defer_conj and FOLDS.conj and self._xor4_defer_ok():
            return self.xor4.apply(x, key, out_level=self._floor(), keep_b=kb, defer_conj=True)
        return self.xor4.apply(x, key, out_level=self._floor(), keep_b=kb)

    def _isr_perm(self, ct, debug):
        """InvShiftRows' byte permutation when the renorm before it can fold it (as _sr_perm)"""
        if not FOLDS.sr or self.true_fhe or not self.use_hard_renorm_between_steps:
            return None
        if not hasattr(self, "_isr_perm_v"):
            sp = getattr(self.invshift, "slot_perm", None)
            self._isr_perm_v = sp() if sp is not None else None
        if self._isr_perm_v is None:
            return None
        ok = getattr(self.encoder, "renorm_perm_ok", None)
        c0 = ct[0].s1 if hasattr(ct[0], "s1") else ct[0]
        return self._isr_perm_v if ok is not None and ok(c0) else None

    def _sr_perm(self, ct, debug):
        """ShiftRows' byte permutation when the renorm before it can fold it (utils.FOLDS.sr: off in the
        strict default; secret-key renorm mode, one period-16 state pair on the device), else None.  A
        debug run keeps the fold and logs what it can (no separate log of the renorm's own output)"""
        if not FOLDS.sr or self.true_fhe or not self.use_hard_renorm_between_steps:
            return None
        if not hasattr(self, "_sr_perm_v"):
            sp = getattr(self.shift, "slot_perm", None)
            self._sr_perm_v = sp() if sp is not None else None
        if self._sr_perm_v is None:
            return None
        ok = getattr(self.encoder, "renorm_perm_ok", None)
        c0 = ct[0].s1 if hasattr(ct[0], "s1") else ct[0]
        return self._sr_perm_v if ok is not None and ok(c0) else None

    def _sr_entry_ok(self) -> bool:
        """ShiftRows runs inside MixColumns' packed entry (MixColFinal.sr_entry): the rot form with its
        GF pair low, this pipeline's own ShiftRows layout (AESFHE_SR_MC_ENTRY=0: a separate step)"""
        from mixcol_final import SR_MC_ENTRY
        return (SR_MC_ENTRY and hasattr(self.mix, "sr_entry") and os.environ.get("AESFHE_MC_FORM", "rot") == "rot"
                and self.layout.packable and getattr(self.shift, "direction", None) == -1)

    def _sub_apply(self, ct, defer_conj: bool = False, lut=None):
        """(Inv)SubBytes (lut, default self.sub) on the pair down to the renorm floor; defer_conj (the
        output goes straight into _renorm_pair): the nibble form may hand over utils.ConjSum halves
        for the folded renorm"""
        lut = self.sub if lut is None else lut
        if defer_conj and FOLDS.conj and self.use_hard_renorm_between_steps and not self.true_fhe:
            import inspect
            try:
                ok = "defer_conj" in inspect.signature(lut.apply).parameters
            except (TypeError, ValueError):
                ok = False
            if ok:
                return lut.apply(*ct, out_level=self._floor(), defer_conj=True)
        return lut.apply(*ct, out_level=self._floor())

    def _xor4_defer_ok(self) -> bool:
        """whether this pipeline's XOR4 takes defer_conj (checked once)"""
        if not hasattr(self, "_defer_ok"):
            import inspect
            try:
                self._defer_ok = "defer_conj" in inspect.signature(self.xor4.apply).parameters
            except (TypeError, ValueError):
                self._defer_ok = False
        return self._defer_ok

    def _xor4_keep_b(self) -> bool:
        """whether this pipeline's XOR4 takes keep_b (checked once; a TypeError raised INSIDE the
        evaluation must surface, not be taken for a missing keyword)"""
        if not hasattr(self, "_keep_b_ok"):
            import inspect
            try:
                self._keep_b_ok = "keep_b" in inspect.signature(self.xor4.apply).parameters
            except (TypeError, ValueError):
                self._keep_b_ok = False
        return self._keep_b_ok

    def _packed_round_key(self, r: int):
        """round key r encrypted in the packed form (after _prepare_round_keys of the same keys)"""
        if self._pk_cache is None or self._pk_tag != self._rk_tag:
            self._pk_cache, self._pk_tag = [None] * len(self._rk_cache), self._rk_tag
        if self._pk_cache[r] is None:
            key = self._rk_raw[r]
            if self.states > 1 and key.shape == (16,):
                key = np.broadcast_to(key, (self.states, 16))
            self._pk_cache[r] = self.encoder.encode_packed(key)
        return self._pk_cache[r]

    def _fused_key(self, round_keys, r: int, direction: int):
        """round key r permuted by ShiftRows (direction -1) / InvShiftRows (+1), encrypted once:
        the key of a SubBytes-AddRoundKey fusion across a ShiftRows (sub_bytes_ark.py)"""
        tag = b"".join(np.ascontiguousarray(k, dtype=np.uint8).tobytes() for k in round_keys)
        if tag != self._fk_tag:
            self._fk_cache, self._fk_tag = {}, tag
        if (r, direction) not in self._fk_cache:
            self._fk_cache[(r, direction)] = self._encode_key(shift_rows_bytes(np.asarray(round_keys[r], np.uint8), direction))
        return self._fk_cache[(r, direction)]

    def _log_packed(self, dbg, tag: str, ct, **meta) -> None:
        """debug snapshot of a packed (hi | lo) state, decoded to bytes"""
        if dbg is None:
            return
        entry = {"ct_packed": ct, "meta": dict(meta, packed=True)}
        try:
            entry["plain"] = self.encoder.decode_packed(ct)
        except Exception as err:
            entry["plain"] = None
            entry["plain_err"] = repr(err)
        dbg[tag] = entry

    def _log_pair(self, dbg, tag: str, ct_hi, ct_lo, **meta) -> None:
        if dbg is None:
            return
        entry = {"ct_hi": ct_hi, "ct_lo": ct_lo, "meta": meta}
        try:
            entry["plain"] = self.encoder.decode(ct_hi, ct_lo)
        except Exception as err:  # keep the snapshot, record why decoding failed
            entry["plain"] = None
            entry["plain_err"] = repr(err)
        dbg[tag] = entry

    # ---------------------------------------------------------------- steps
    def add_round_key(self, ct_hi, ct_lo, key_hi, key_lo):
        return self.ark(ct_hi, ct_lo, key_hi, key_lo)

    def sub_bytes(self, ct_hi, ct_lo):
        return self.sub.apply(ct_hi, ct_lo)

    def inv_sub_bytes(self, ct_hi, ct_lo):
        if self.isub is None:
            raise KeyError("inv_sub_hi")
        return self.isub.apply(ct_hi, ct_lo)

    def shift_rows(self, ct_hi, ct_lo):
        return self.shift.apply(ct_hi, ct_lo)

    def inv_shift_rows(self, ct_hi, ct_lo):
        return self.invshift.apply(ct_hi, ct_lo)

    def mix_columns(self, ct_hi, ct_lo):
        return self.mix(ct_hi, ct_lo)

    def inv_mix_columns(self, ct_hi, ct_lo):
        return self.invmix(ct_hi, ct_lo)

    # ---------------------------------------------------------------- encrypt
    def encrypt_round(self, ct, key_pair, debug=None, r: int = 0, next_level: int | None = None):
        """One middle round r = 1..9: SB, renorm, SR, MC, ARK, renorm (REF :142-151).  With a
        debug dict every step is logged under enc.r{r}.<step> (the names of the reference's
        one-round debug block, REF :154-171)."""
        if next_level is None:
            next_level = self.need_sub
        if self.packed_xor and r > 0:
            # packed XOR stage: MixColumns returns the packed state, AddRoundKey
            # XORs it with the packed round key, its renorm unpacks into the (hi, lo) pair.  A debug
            # dict logs THIS path's stages under the reference's names (the packed ones decoded from
            # the hi | lo halves), so the golden stage test observes the headline path itself.
            ct = self._sub_apply(ct, defer_conj=True)
            self._log_pair(debug, f"enc.r{r}.sub", *ct)
            need = getattr(self.mix, "packed_input_need", None)
            lv = need() if need else NEED_SR_MIX - SHIFTROWS_DEPTH + self.encoder.PACK_DEPTH
            perm = self._sr_perm(ct, debug)
            if perm is not None:  # ShiftRows folded into the renorm (a byte permutation of the snap)
                ct = self.encoder.renorm_perm(*ct, perm, level=lv)
            elif self._sr_entry_ok():
                # ShiftRows homomorphic inside MixColumns' entry (MixColFinal.sr_entry: masked rotations
                # fused with the first column shift and the packs, one level): the renorm hands out lv
                ct = self._renorm_pair(*ct, level=lv)
                self._log_pair(debug, f"enc.r{r}.sub.renorm", *ct)
                log_sr = (lambda p0: self._log_packed(debug, f"enc.r{r}.sr", p0)) if debug is not None else None
                acc = self.mix.mix_packed(*ct, sr=self.shift, on_sr=log_sr)
                self._log_packed(debug, f"enc.r{r}.mc", acc)
                x = self._ark_packed(acc, r, defer_conj=True)
                self._log_packed(debug, f"enc.r{r}.ark", x)
                ct = self.encoder.renorm_unpack(x, level=next_level)
                self._log_pair(debug, f"enc.r{r}.ark.renorm", *ct)
                return ct
            else:
                ct = self._renorm_pair(*ct, level=lv + SHIFTROWS_DEPTH)
                self._log_pair(debug, f"enc.r{r}.sub.renorm", *ct)
                ct = self.shift_rows(*ct)
            self._log_pair(debug, f"enc.r{r}.sr", *ct)
            acc = self.mix.mix_packed(*ct)
            self._log_packed(debug, f"enc.r{r}.mc", acc)
            x = self._ark_packed(acc, r, defer_conj=True)
            self._log_packed(debug, f"enc.r{r}.ark", x)
            ct = self.encoder.renorm_unpack(x, level=next_level)
            self._log_pair(debug, f"enc.r{r}.ark.renorm", *ct)
            return ct
        if debug is None:
            ct = self._sub_renorm(ct, level=NEED_SR_MIX)
            ct = self.srmc(*ct) if self.srmc is not None else self.mix_columns(*self.shift_rows(*ct))
            return self._ark_renorm(ct, key_pair, level=next_level)
        ct = self.sub.apply(*ct, out_level=self._floor())
        self._log_pair(debug, f"enc.r{r}.sub", *ct)
        ct = self._renorm_pair(*ct, level=NEED_SR_MIX)
        self._log_pair(debug, f"enc.r{r}.sub.renorm", *ct)
        if self.srmc is not None:  # ShiftRows and MixColumns merged (shiftrows_mixcolumns.py)
            inner = {}
            ct = self.srmc(*ct, debug=inner)
            self._log_pair(debug, f"enc.r{r}.sr", *inner["sr"])
        else:
            ct = self.shift_rows(*ct)
            self._log_pair(debug, f"enc.r{r}.sr", *ct)
            ct = self.mix_columns(*ct)
        self._log_pair(debug, f"enc.r{r}.mc", *ct)
        ct = self.ark(*ct, *key_pair, out_level=self._floor())
        self._log_pair(debug, f"enc.r{r}.ark", *ct)
        ct = self._renorm_pair(*ct, level=next_level)
        self._log_pair(debug, f"enc.r{r}.ark.renorm", *ct)
        return ct

    def encrypt(self, state: np.ndarray, round_keys: List[np.ndarray], debug: Dict[str, Any] | None = None):
        if debug is not None:
            debug.clear()
        ct = self.encoder.encode(state)
        self._log_pair(debug, "enc.input", *ct)
        rk = self._prepare_round_keys(round_keys)
        ct = self.ark(*ct, *rk[0], out_level=self._floor())
        self._log_pair(debug, "enc.r0.ark", *ct)
        ct = self._renorm_pair(*ct, level=self.need_sub)
        self._log_pair(debug, "enc.r0.renorm", *ct)
        for r in range(1, 10):
            nxt = NEED_SUB_ARK_SR if (self.fuse_sub_ark and r == 9) else self.need_sub
            ct = self.encrypt_round(ct, rk[r], debug, r, next_level=nxt)
        if self.fuse_sub_ark:
            # SR(SB(x)) ^ k10 = SR(SB(x) ^ InvShiftRows(k10)): one fused LUT, then ShiftRows
            ct = self.sbark(*ct, *self._fused_key(round_keys, 10, +1))
            self._log_pair(debug, "enc.final.sub_ark", *ct)
            ct = self.shift_rows(*ct)
            self._log_pair(debug, "enc.final.ark10", *ct)
            ct = self._renorm_pair(*ct)
            self._log_pair(debug, "enc.output", *ct)
            return tag_layout(self.layout, *ct)
        ct = self._sub_apply(ct, defer_conj=True)
        self._log_pair(debug, "enc.final.sub", *ct)
        perm = self._sr_perm(ct, debug)
        if perm is not None:  # ShiftRows folded into the renorm
            ct = self.encoder.renorm_perm(*ct, perm, level=NEED_SR_ARK - SHIFTROWS_DEPTH)
        else:
            ct = self._renorm_pair(*ct, level=NEED_SR_ARK)
            self._log_pair(debug, "enc.final.sub.renorm", *ct)
            ct = self.shift_rows(*ct)
        self._log_pair(debug, "enc.final.sr", *ct)
        ct = self.ark(*ct, *rk[10], out_level=self._floor())
        self._log_pair(debug, "enc.final.ark10", *ct)
        ct = self._renorm_pair(*ct)
        self._log_pair(debug, "enc.output", *ct)
        return tag_layout(self.layout, *ct)

    # ---------------------------------------------------------------- decrypt
    def decrypt(self, ct_hi, ct_lo, round_keys: List[np.ndarray], debug: Dict[str, Any] | None = None):
        check_layout(self.layout, ct_hi, ct_lo)  # a pair from another layout would decrypt to wrong bytes
        if debug is not None:
            debug.clear()
        rk = self._prepare_round_keys(round_keys)
        self._log_pair(debug, "dec.input", ct_hi, ct_lo)
        if self.true_fhe and not self.fuse_sub_ark:
            return self._decrypt_fhe(ct_hi, ct_lo, rk, debug)
        ct = self.ark(ct_hi, ct_lo, *rk[10], out_level=self._floor())
        self._log_pair(debug, "dec.init.ark10", *ct)
        fuse = self.fuse_sub_ark
        if fuse and self.isub is None:
            raise KeyError("inv_sub_hi")
        # InvShiftRows folded into the renorm before it (the packed decrypt: this renorm and every
        # InvMixColumns renorm), as ShiftRows in encrypt (pipeline._sr_perm)
        isr = self._isr_perm(ct, debug) if self.packed_dec and not fuse else None
        if isr is not None:
            ct, isr_done = self.encoder.renorm_perm(*ct, isr, level=self.need_isr_isb - SHIFTROWS_DEPTH), True
        else:
            ct, isr_done = self._renorm_pair(*ct, level=NEED_SUB_ARK_SR if fuse else self.need_isr_isb), False
        self._log_pair(debug, "dec.init.ark10.renorm", *ct)
        for r in range(9, 0, -1):
            if fuse:
                # ISB(ISR(x)) ^ k_r = ISR(ISB(x) ^ ShiftRows(k_r)): one fused LUT, then InvShiftRows
                ct = self.isbark(*ct, *self._fused_key(round_keys, r, -1))
                self._log_pair(debug, f"dec.r{r}.isb_ark", *ct)
                ct = self.inv_shift_rows(*ct)
                ct = self._renorm_pair(*ct, level=NEED_GF if self.with_inv_mix_columns else NEED_SUB_ARK_SR)
                self._log_pair(debug, f"dec.r{r}.ark", *ct)
                if self.with_inv_mix_columns:
                    ct = self._renorm_pair(*self.inv_mix_columns(*ct), level=NEED_SUB_ARK_SR)
                    self._log_pair(debug, f"dec.r{r}.imc", *ct)
                continue
            if self.packed_dec:
                # packed XOR stage: AddRoundKey on the packed state, its renorm
                # unpacking; InvMixColumns' XOR stage packed, unpacked by the renorm after it
                # (a debug dict logs this path's stages under the reference's names)
                if not isr_done:
                    ct = self.inv_shift_rows(*ct)
                isr_done = False
                self._log_pair(debug, f"dec.r{r}.isr", *ct)
                ct = self._sub_renorm(ct, inverse=True, level=NEED_XOR + self.encoder.PACK_DEPTH)
                self._log_pair(debug, f"dec.r{r}.isb", *ct)
                x = self._ark_packed(self.encoder.pack(*ct), r, defer_conj=True)
                need = getattr(self.invmix, "packed_input_need", None)
                ct = self.encoder.renorm_unpack(x, level=need() if need else NEED_GF + self.encoder.PACK_DEPTH)
                self._log_pair(debug, f"dec.r{r}.ark", *ct)
                if isr is not None:
                    ct = self.encoder.renorm_unpack_perm(self.invmix.imc_packed(*ct), isr, level=self.need_isr_isb - SHIFTROWS_DEPTH)
                    isr_done = True
                else:
                    ct = self.encoder.renorm_unpack(self.invmix.imc_packed(*ct), level=self.need_isr_isb)
                self._log_pair(debug, f"dec.r{r}.imc", *ct)
                continue
            ct = self.inv_shift_rows(*ct)
            self._log_pair(debug, f"dec.r{r}.isr", *ct)
            ct = self._sub_renorm(ct, inverse=True, level=NEED_XOR)
            self._log_pair(debug, f"dec.r{r}.isb", *ct)
            ct = self._ark_renorm(ct, rk[r], level=NEED_GF if self.with_inv_mix_columns else self.need_isr_isb)
            self._log_pair(debug, f"dec.r{r}.ark", *ct)
            if self.with_inv_mix_columns:
                # InvSubBytes' LUT needs a clean input, as SubBytes gets one after ARK in encrypt
                ct = self._renorm_pair(*self.inv_mix_columns(*ct), level=self.need_isr_isb)
                self._log_pair(debug, f"dec.r{r}.imc", *ct)
        if fuse:
            ct = self.isbark(*ct, *self._fused_key(round_keys, 0, -1))
            self._log_pair(debug, "dec.final.isb_ark", *ct)
            ct = self.inv_shift_rows(*ct)
            self._log_pair(debug, "dec.final.ark0", *ct)
            ct = self._renorm_pair(*ct)
            self._log_pair(debug, "dec.output", *ct)
            return ct
        if not isr_done:
            ct = self.inv_shift_rows(*ct)
        self._log_pair(debug, "dec.final.isr", *ct)
        if self.isub is None:
            raise KeyError("inv_sub_hi")
        ct = self.isub.apply(*ct, out_level=self._floor())
        self._log_pair(debug, "dec.final.isb", *ct)
        ct = self._renorm_pair(*ct, level=NEED_XOR)
        self._log_pair(debug, "dec.final.isb.renorm", *ct)
        ct = self.ark(*ct, *rk[0], out_level=self._floor())
        self._log_pair(debug, "dec.final.ark0", *ct)
        ct = self._renorm_pair(*ct)
        self._log_pair(debug, "dec.output", *ct)
        return ct

    def _decrypt_fhe(self, ct_hi, ct_lo, rk, debug):
        """decrypt in true-FHE mode: the same steps, each InvShiftRows applied BEFORE the renorm
        (bootstrap + snap) that precedes InvSubBytes -- after the snap exactly InvSubBytes' 13
        levels remain.  InvShiftRows is a masked permutation, so moving it across the renorm
        changes no byte (ISB(ISR(x)) with x renormalised either side)."""
        if self.isub is None:
            raise KeyError("inv_sub_hi")
        fl = self._floor()
        ct = self.ark(ct_hi, ct_lo, *rk[10], out_level=fl)
        self._log_pair(debug, "dec.init.ark10", *ct)
        ct = self._renorm_pair(*self.inv_shift_rows(*ct), level=NEED_SUBBYTES)
        self._log_pair(debug, "dec.r9.isr", *ct)
        for r in range(9, -1, -1):
            # InvSubBytes' output error is ~3e-2: its renorm snaps twice before AddRoundKey's XOR4
            ct = self._renorm_pair(*self.isub.apply(*ct, out_level=fl), level=NEED_XOR)
            self._log_pair(debug, f"dec.r{r}.isb" if r else "dec.final.isb.renorm", *ct)
            ct = self.ark(*ct, *rk[r], out_level=fl)
            if r == 0:
                self._log_pair(debug, "dec.final.ark0", *ct)
                ct = self._renorm_pair(*ct)
                self._log_pair(debug, "dec.output", *ct)
                return ct
            if self.with_inv_mix_columns:
                ct = self._renorm_pair(*ct, level=NEED_GF)
                self._log_pair(debug, f"dec.r{r}.ark", *ct)
                ct = self.invmix(*ct, final_renorm=False)
            ct = self._renorm_pair(*self.inv_shift_rows(*ct), level=NEED_SUBBYTES)
            self._log_pair(debug, f"dec.r{r}.imc" if self.with_inv_mix_columns else f"dec.r{r}.ark", *ct)
