"""The reference's error-driven and debug-driven behaviour on the MI355X engine.

- `make_power_basis_safe` / `bootstrap_safe` on an exhausted ciphertext
  (REF/engine_context.py:180-204);
- XOR4's to_intt -> retry -> bootstrap cascade when its inputs sit too low for a power basis
  (REF/xor4_lut.py:33-51), through the fused split path and through the reference's loop;
- MixColFinal and InvMixColumnsFHE stage by stage under the reference's debug keys
  (REF/mixcol_final.py:127-163,250-297; REF/invmixcolumns_fhe.py:111-134,230-296);
- every debug stage of a full C2 encrypt against tests/golden/stages.json (seeds 0, 7, 42).

Decoded nibbles must be exact; slot values after a bootstrap are within BOOT_TOL.
"""
import json

import numpy as np
import pytest

from conftest import GOLDEN, gpu_context

pytestmark = pytest.mark.gpu

from test_gpu_bootstrap import BOOT_TOL  # noqa: E402  (one tolerance for every bootstrap check)


@pytest.fixture(scope="module")
def ctx():
    return gpu_context(log_n=16, signature=1)


def _exhausted(ctx, z):
    """z encrypted, then multiplied by 0.999 until no level is left"""
    E = ctx.engine
    low = ctx.encrypt(z)
    for _ in range(E.fresh_level):
        low = E.multiply(low, 0.999)
    assert low.level == 0
    return low, z * 0.999 ** E.fresh_level


def test_power_basis_safe_bootstraps_an_exhausted_ciphertext(ctx):
    E = ctx.engine
    rng = np.random.default_rng(21)
    low, zl = _exhausted(ctx, np.exp(2j * np.pi * rng.random(E.slot_count)))
    with pytest.raises(RuntimeError, match="level"):
        ctx.make_power_basis(low, 8)
    n0 = ctx.bootstrap_stats()["count"]
    pb = ctx.make_power_basis_safe(low, 8)
    assert ctx.bootstrap_stats()["count"] == n0 + 1
    assert len(pb) == 8 and pb[0].level == E.fresh_level
    for k in (1, 2, 5, 8):
        assert np.abs(ctx.decrypt(pb[k - 1]) - zl ** k).max() < 2 * k * BOOT_TOL, k


def test_bootstrap_safe_equals_bootstrap(ctx):
    E = ctx.engine
    rng = np.random.default_rng(22)
    z = np.exp(2j * np.pi * rng.random(E.slot_count)) * 0.8
    ct = ctx.encrypt(z)
    a, b = ctx.bootstrap_safe(ct), ctx.bootstrap(ct)
    assert np.array_equal(E.export(a), E.export(b))
    assert np.abs(ctx.decrypt(a) - z).max() < BOOT_TOL


@pytest.mark.parametrize("fused", [True, False], ids=["fused", "loop"])
def test_xor4_bootstrap_cascade(ctx, coeff_dir, fused):
    """inputs at level 1 cannot form x^8: XOR4 must fall back to to_intt, retry, then
    bootstrap both inputs and still return the exact XOR"""
    from aes_keyschedule import load_all_coeffs
    from state_encoder import StateEncoder
    from xor4_lut import XOR4LUT
    co = load_all_coeffs(coeff_dir)
    enc = StateEncoder(ctx)
    xor4 = XOR4LUT(ctx, co["xor4"])
    rng = np.random.default_rng(23)
    a, b = rng.integers(0, 256, 16).astype(np.uint8), rng.integers(0, 256, 16).astype(np.uint8)
    (ah, al), (bh, bl) = enc.encode(a), enc.encode(b)
    ah, bh, al, bl = (ctx.level_down(c, 1) for c in (ah, bh, al, bl))
    with pytest.raises(RuntimeError, match="level"):
        ctx.make_power_basis(ah, 8)
    saved = ctx.fused_luts
    ctx.fused_luts = fused
    try:
        n0 = ctx.bootstrap_stats()["count"]
        hi, lo = xor4.apply(ah, bh), xor4.apply(al, bl)
        assert ctx.bootstrap_stats()["count"] == n0 + 4
    finally:
        ctx.fused_luts = saved
    assert np.array_equal(enc.decode(hi, lo), a ^ b)


def _rot_model(state, k):
    return np.roll(state.reshape(4, 4).T, -k, axis=1).T.reshape(16)


def test_mixcolumns_reference_debug_keys(ctx, coeff_dir):
    """REF/mixcol_final.py:250-297: every stage under the reference's keys, final bootstrap on"""
    from aes_keyschedule import load_all_coeffs
    from mixcol_final import MixColFinal
    from oracle import aes_plain as A
    from state_encoder import StateEncoder
    from xor4_lut import XOR4LUT
    enc = StateEncoder(ctx)
    mc = MixColFinal(ctx, XOR4LUT(ctx, load_all_coeffs(coeff_dir)["xor4"]))
    np.random.seed(0)
    state = np.random.randint(0, 256, 16, dtype=np.uint8)
    dbg = {}
    out = mc(*enc.encode(state), do_final_bootstrap=True, debug=dbg)
    r = {k: _rot_model(state, k) for k in (1, 2, 3)}
    two, thr = A.GF_MUL[2][state], A.GF_MUL[3][r[1]]
    want = {"rotc1": r[1], "rotc2": r[2], "rotc3": r[3], "in": state, "two": two, "thr": thr,
            "acc1": two ^ thr, "acc2": two ^ thr ^ r[2], "acc3": two ^ thr ^ r[2] ^ r[3]}
    for key, exp in want.items():
        assert np.array_equal(enc.decode(*dbg[key]), exp), key
    assert np.array_equal(enc.decode(*out), A.ref_mix_columns(state))
    assert np.array_equal(enc.decode(*dbg["out"]), A.ref_mix_columns(state))
    assert out[0].level == ctx.engine.fresh_level


def test_inv_mixcolumns_stagewise(ctx, coeff_dir):
    """REF/invmixcolumns_fhe.py:174-226 plaintext models and the :230-296 stage checks
    (rotations, mul14 / mul11@r1 / mul13@r2 / mul9@r3, acc1, acc2, final), bootstrap on"""
    from aes_keyschedule import load_all_coeffs
    from invmixcolumns_fhe import InvMixColumnsFHE
    from oracle import aes_plain as A
    from state_encoder import StateEncoder
    from xor4_lut import XOR4LUT
    enc = StateEncoder(ctx)
    imc = InvMixColumnsFHE(ctx, XOR4LUT(ctx, load_all_coeffs(coeff_dir)["xor4"]))
    np.random.seed(0)
    state = np.random.randint(0, 256, 16, dtype=np.uint8)
    dbg = {}
    out = imc(*enc.encode(state), do_final_bootstrap=True, debug=dbg)
    r = {k: _rot_model(state, k) for k in (1, 2, 3)}
    G = A.GF_MUL
    m14, m11, m13, m9 = G[14][state], G[11][r[1]], G[13][r[2]], G[9][r[3]]
    want = {"rotc1": r[1], "rotc2": r[2], "rotc3": r[3], "mul14": m14, "mul11": m11, "mul13": m13, "mul9": m9,
            "acc1": m14 ^ m11, "acc2": m14 ^ m11 ^ m13}
    for key, exp in want.items():
        assert np.array_equal(enc.decode(*dbg[key]), exp), key
    final = m14 ^ m11 ^ m13 ^ m9
    assert np.array_equal(final, A.ref_inv_mix_columns(state))
    assert np.array_equal(enc.decode(*out), final)
    assert np.array_equal(A.ref_mix_columns(enc.decode(*out)), state)
    assert out[0].level == ctx.engine.fresh_level


_STAGE = {"sub": "sb", "sub.renorm": "sb", "sr": "sr", "mc": "mc", "ark": "ark", "ark.renorm": "ark"}
_FINAL = {"enc.final.sub": "r10.sb", "enc.final.sub.renorm": "r10.sb", "enc.final.sr": "r10.sr",
          "enc.final.ark10": "r10.ark", "enc.output": "r10.ark", "enc.r0.ark": "r0.ark", "enc.r0.renorm": "r0.ark"}


@pytest.mark.parametrize("seed,packed", [(0, None), (7, None), (42, None), (7, False)])
def test_encrypt_every_debug_stage_matches_golden(ctx, coeff_dir, seed, packed):
    """Each logged stage of a full C2 encrypt decodes to the bytes of tests/golden/stages.json
    (the byte-level reference model, REF/pipeline.py:123-188, inputs drawn as
    REF/test/test_aes_pipeline_roundtrip.py:136-140).  packed None: the bench's own path (the
    packed XOR stage of rounds 1..9) logs its stages; False: the reference's pair
    steps."""
    from aes_keyschedule import load_all_coeffs
    from pipeline import AESPipeline
    fx = {s["seed"]: s for s in json.loads((GOLDEN / "stages.json").read_text())["seeds"]}[seed]
    pipe = AESPipeline(ctx, load_all_coeffs(coeff_dir), use_hard_renorm_between_steps=True, packed_xor=packed)
    assert pipe.packed_xor == (packed is None)  # the default IS the packed path in renorm mode
    pt = np.array(fx["plaintext"], np.uint8)
    rks = [np.array(k, np.uint8) for k in fx["round_keys"]]
    dbg = {}
    ct = pipe.encrypt(pt, rks, debug=dbg)
    want = {"enc.input": pt}
    for tag, stage in _FINAL.items():
        want[tag] = np.array(fx["stages"][stage], np.uint8)
    for r in range(1, 10):
        for step, stage in _STAGE.items():
            want[f"enc.r{r}.{step}"] = np.array(fx["stages"][f"r{r}.{stage}"], np.uint8)
    assert set(dbg) == set(want)
    bad = [t for t, exp in want.items() if dbg[t]["plain"] is None or not np.array_equal(dbg[t]["plain"], exp)]
    assert not bad, bad
    # the packed path's MixColumns / AddRoundKey outputs are single packed ciphertexts
    assert all(("ct_packed" in dbg[f"enc.r{r}.{k}"]) == (packed is None) for r in range(1, 10) for k in ("mc", "ark"))
    assert np.array_equal(pipe.encoder.decode(*ct), np.array(fx["ciphertext"], np.uint8))


@pytest.mark.parametrize("packed", [None, False])
def test_decrypt_every_debug_stage_matches_byte_model(ctx, coeff_dir, packed):
    """Each logged stage of a full C2 decrypt (REF/pipeline.py:193-254 with InvMixColumns after
    AddRoundKey, README.md:87-94) decodes to the byte model's intermediate state: the packed
    decrypt rounds under the same stage names as the reference's pair steps."""
    from aes_keyschedule import load_all_coeffs
    from oracle import aes_plain as A
    from pipeline import AESPipeline
    fx = {s["seed"]: s for s in json.loads((GOLDEN / "stages.json").read_text())["seeds"]}[7]
    pipe = AESPipeline(ctx, load_all_coeffs(coeff_dir), use_hard_renorm_between_steps=True, packed_xor=packed)
    assert pipe.packed_dec == (packed is None)
    pt = np.array(fx["plaintext"], np.uint8)
    rks = [np.array(k, np.uint8) for k in fx["round_keys"]]
    ct = pipe.encoder.encode(A.ref_encrypt(pt, rks))
    dbg = {}
    back = pipe.decrypt(*ct, rks, debug=dbg)
    s = A.ref_encrypt(pt, rks) ^ rks[10]
    want = {"dec.init.ark10": s}
    for r in range(9, 0, -1):
        want[f"dec.r{r}.isr"] = A.inv_shift_rows(s)
        want[f"dec.r{r}.isb"] = A.INV_SBOX[want[f"dec.r{r}.isr"]]
        want[f"dec.r{r}.ark"] = want[f"dec.r{r}.isb"] ^ rks[r]
        s = want[f"dec.r{r}.imc"] = A.ref_inv_mix_columns(want[f"dec.r{r}.ark"])
    bad = [t for t, exp in want.items() if t not in dbg or dbg[t]["plain"] is None or not np.array_equal(dbg[t]["plain"], exp)]
    assert not bad, bad
    assert np.array_equal(pipe.encoder.decode(*back), pt)


def test_encrypt_debug_stages_with_the_renorm_folds(ctx, coeff_dir):
    """a debug run keeps the renorm folds (utils.RenormFolds, the bench's 'folded' leg) and logs what it
    can: every stage it logs that decodes matches tests/golden/stages.json; the ShiftRows fold leaves
    no separate post-renorm log, and a conjugate-split output (utils.ConjSum) is logged undecoded"""
    from aes_keyschedule import load_all_coeffs
    from pipeline import AESPipeline
    from utils import renorm_folds
    fx = {s["seed"]: s for s in json.loads((GOLDEN / "stages.json").read_text())["seeds"]}[7]
    pt = np.array(fx["plaintext"], np.uint8)
    rks = [np.array(k, np.uint8) for k in fx["round_keys"]]
    with renorm_folds(True):
        pipe = AESPipeline(ctx, load_all_coeffs(coeff_dir), use_hard_renorm_between_steps=True)
        dbg = {}
        ct = pipe.encrypt(pt, rks, debug=dbg)
    want = {"enc.input": pt}
    for tag, stage in _FINAL.items():
        want[tag] = np.array(fx["stages"][stage], np.uint8)
    for r in range(1, 10):
        for step, stage in _STAGE.items():
            want[f"enc.r{r}.{step}"] = np.array(fx["stages"][f"r{r}.{stage}"], np.uint8)
    assert set(dbg) <= set(want) and set(want) - set(dbg) <= {f"enc.r{r}.sub.renorm" for r in range(1, 10)} | {"enc.final.sub.renorm"}
    decoded = [t for t in dbg if dbg[t]["plain"] is not None]
    bad = [t for t in decoded if not np.array_equal(dbg[t]["plain"], want[t])]
    assert not bad, bad
    for r in range(1, 10):  # the steps after a folded renorm decode
        assert all(dbg[f"enc.r{r}.{k}"]["plain"] is not None for k in ("sr", "mc", "ark.renorm"))
    assert np.array_equal(pipe.encoder.decode(*ct), np.array(fx["ciphertext"], np.uint8))
