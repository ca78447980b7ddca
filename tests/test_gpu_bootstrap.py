"""CKKS bootstrapping on the MI355X engine and the pipeline steps that
use it.  Slot tolerances are stated in the asserts; decoded nibbles must be exact."""
import numpy as np
import pytest

from conftest import gpu_context

pytestmark = pytest.mark.gpu

# max |slot error| for |z| <= 1 inputs at N = 2^16: ~2x the measured 2.4e-4 (profiles/r2_boot_error.json;
# DESIGN.md §4).  The decode margin of a Zeta16 slot is pi/16 = 0.196.
BOOT_TOL = 5e-4


@pytest.fixture(scope="module")
def ctx():
    return gpu_context(log_n=16, signature=1)


def test_bootstrap_accuracy_and_level(ctx):
    E = ctx.engine
    S = E.slot_count
    rng = np.random.default_rng(1)
    z = np.exp(2j * np.pi * rng.random(S)) * rng.random(S)
    ct = ctx.encrypt(z)
    out = ctx.bootstrap(ct)
    assert out.level == E.fresh_level
    assert np.abs(ctx.decrypt(out) - z).max() < BOOT_TOL
    # from an exhausted ciphertext (the reference's fallback path, REF/xor4_lut.py:46-51)
    low = ct
    for _ in range(E.fresh_level):
        low = ctx.multiply(low, 1.0 + 0j) if False else E.multiply(low, 0.999)
    assert low.level == 0
    out = ctx.bootstrap(ctx.to_intt(low))
    # 17 rescales of input noise ride along (the bootstrap is linear in its input's error)
    assert np.abs(ctx.decrypt(out) - z * 0.999 ** E.fresh_level).max() < 2 * BOOT_TOL
    assert ctx.bootstrap_stats()["count"] >= 2


def test_bootstrap_zeta16_state(ctx):
    from state_encoder import StateEncoder
    enc = StateEncoder(ctx)
    rng = np.random.default_rng(2)
    state = rng.integers(0, 256, 16).astype(np.uint8)
    hi, lo = enc.encode(state)
    bh, bl = ctx.bootstrap(hi), ctx.bootstrap(lo)
    assert np.array_equal(enc.decode(bh, bl), state)
    sc = E_slots = ctx.engine.slot_count
    z = ctx.decrypt(bh)[:: sc // 16][:16]
    assert np.abs(np.angle(z / np.exp(-2j * np.pi * (state >> 4) / 16))).max() < 2 * BOOT_TOL


def test_mixcolumns_with_final_bootstrap(ctx, coeff_dir):
    from aes_keyschedule import load_all_coeffs
    from mixcol_final import MixColFinal
    from oracle import aes_plain
    from state_encoder import StateEncoder
    from xor4_lut import XOR4LUT
    co = load_all_coeffs(coeff_dir)
    enc = StateEncoder(ctx)
    mc = MixColFinal(ctx, XOR4LUT(ctx, co["xor4"]))
    np.random.seed(0)
    state = np.random.randint(0, 256, 16, dtype=np.uint8)
    out = mc(*enc.encode(state))
    assert out[0].level == ctx.engine.fresh_level
    assert np.array_equal(enc.decode(*out), aes_plain.ref_mix_columns(state))


def test_config2_full_encrypt_and_roundtrip(ctx, coeff_dir):
    """BASELINE config 2 on one state (REF/test/test_aes_pipeline_roundtrip.py:114-163):
    10-round encrypt with renorm + final bootstraps, then decrypt with InvMixColumns."""
    from aes_keyschedule import expand_aes128_key, load_all_coeffs
    from oracle import aes_plain
    from pipeline import AESPipeline
    pipe = AESPipeline(ctx, load_all_coeffs(coeff_dir), use_hard_renorm_between_steps=True)
    np.random.seed(7)
    key = np.random.randint(0, 256, 16, dtype=np.uint8)
    rks = expand_aes128_key(key)
    pt = np.random.randint(0, 256, 16, dtype=np.uint8)
    dbg = {}
    ct = pipe.encrypt(pt, rks, debug=dbg)
    assert np.array_equal(pipe.encoder.decode(*ct), aes_plain.ref_encrypt(pt, rks))
    assert np.array_equal(dbg["enc.r0.ark"]["plain"], pt ^ rks[0])
    back = pipe.decrypt(*ct, rks)
    assert np.array_equal(pipe.encoder.decode(*back), pt)


def test_bootstrap_pair_bit_exact(ctx):
    """The batched pair bootstrap (two stacked ciphertexts, shared key and diagonal reads)
    produces exactly the residues of two single bootstraps."""
    E = ctx.engine
    S = E.slot_count
    rng = np.random.default_rng(4)
    za = np.exp(2j * np.pi * rng.random(S))
    zb = np.exp(2j * np.pi * rng.random(S)) * 0.7
    a, b = ctx.encrypt(za), ctx.encrypt(zb)
    pa, pb = ctx.bootstrap_pair(a, b)
    sa, sb = ctx.bootstrap(a), ctx.bootstrap(b)
    assert pa.level == sa.level == E.fresh_level
    assert np.array_equal(E.export(pa), E.export(sa))
    assert np.array_equal(E.export(pb), E.export(sb))
    assert np.abs(ctx.decrypt(pb) - zb).max() < BOOT_TOL


def test_dense_to_sparse_key_modulus(ctx):
    """The dense -> sparse bootstrapping key is an RLWE sample under the h = 32 sparse
    secret, so it lives modulo Q0 * P' only (Q0 = q0 q1, the level-0 limbs the bootstrap
    starts from; ~120 bits), never on the full Q * P chain.  Checks the width
    and the key equation b + a s_sp = e + (P' mod q_t) s on q0, q1 and e on the P' limbs, with e
    a centred binomial (|e| <= 21)."""
    E = ctx.engine
    info = E.boot_info()
    assert info["sparse_h"] == 32
    assert info["d2s_log_modulus"] < 125.0
    nq, npd = int(info["d2s_base_limbs"]), int(info["d2s_special_primes"])
    assert nq == 2
    key = E.export_ksk(2 * E.n + 1).astype(np.uint64)
    assert key.shape == (1, 2, nq + npd, E.n)
    q = E.moduli().astype(np.uint64)
    primes = list(range(nq)) + [E.n_q + k for k in range(npd)]
    assert abs(sum(np.log2(float(q[p])) for p in primes) - info["d2s_log_modulus"]) < 1e-9
    s_sp = E.export_sparse().astype(np.uint64)
    s = E.export_secret().astype(np.uint64)
    b, a = key[0, 0], key[0, 1]
    for row, p in enumerate(primes):
        qt = q[p]
        r = (b[row] + a[row] * s_sp[p] % qt) % qt
        if row < nq:
            pq = 1
            for k in range(npd):
                pq = pq * int(q[E.n_q + k]) % int(qt)
            r = (r + qt - np.uint64(pq) * s[p] % qt) % qt
        e = E.debug_ntt(r.astype(np.uint32)[None], p, inverse=True)[0].astype(np.int64)
        e = np.where(e > int(qt) // 2, e - int(qt), e)
        assert np.abs(e).max() <= 21, (row, np.abs(e).max())


@pytest.mark.parametrize("period", [16, 1024, 16384])
def test_sparse_bootstrap_periodic_message(ctx, period):
    """aesfhe_bootstrap[_pair]_sparse: an n-periodic message (a subring
    element) refreshed by the trace + small-ring transforms.  The pair is packed into ONE
    2n-periodic message a + X^(N/4n) b, bootstrapped once at gain 1/2 and split by the
    rotation by n slots (the full-slot bootstrap when 2n = slots: period 16384), so its
    error is up to the sum of two slots' bootstrap errors"""
    E = ctx.engine
    S = E.slot_count
    rng = np.random.default_rng(period)
    za = np.tile(np.exp(2j * np.pi * rng.random(period)) * rng.random(period), S // period)
    zb = np.tile(np.exp(2j * np.pi * rng.random(period)), S // period)
    a, b = ctx.encrypt(za), ctx.encrypt(zb)
    pa, pb = E.bootstrap_pair_sparse(a, b, period)
    sa = E.bootstrap_sparse(a, period)
    assert pa.level == pb.level == sa.level == E.fresh_level
    assert np.abs(ctx.decrypt(sa) - za).max() < BOOT_TOL
    assert np.abs(ctx.decrypt(pa) - za).max() < 2 * BOOT_TOL
    assert np.abs(ctx.decrypt(pb) - zb).max() < 2 * BOOT_TOL
    with pytest.raises(RuntimeError, match="period"):
        E.bootstrap_sparse(a, 24)


def test_config2_reference_layout_roundtrip(ctx, coeff_dir):
    """the reference's slot layout (AESPipeline(periodic=False): byte i at slot i*N/32, full-slot
    bootstraps) gives the same ciphertext bytes as the default periodic layout"""
    from aes_keyschedule import expand_aes128_key, load_all_coeffs
    from oracle import aes_plain
    from pipeline import AESPipeline
    co = load_all_coeffs(coeff_dir)
    np.random.seed(11)
    rks = expand_aes128_key(np.random.randint(0, 256, 16, dtype=np.uint8))
    pt = np.random.randint(0, 256, 16, dtype=np.uint8)
    ref = AESPipeline(ctx, co, use_hard_renorm_between_steps=True, periodic=False)
    per = AESPipeline(ctx, co, use_hard_renorm_between_steps=True)
    assert not ref.layout.periodic and per.layout.periodic and per.layout.boot_period == 16
    want = aes_plain.ref_encrypt(pt, rks)
    ct_ref, ct_per = ref.encrypt(pt, rks), per.encrypt(pt, rks)
    assert np.array_equal(ref.encoder.decode(*ct_ref), want)
    assert np.array_equal(per.encoder.decode(*ct_per), want)
    assert np.array_equal(ref.encoder.decode(*ref.decrypt(*ct_ref, rks)), pt)


@pytest.mark.parametrize("states", [1, 4])
def test_periodic_renorm(ctx, states):
    """aesfhe_renorm_periodic: the periodic layout's secret-key renorm (period 16: the direct
    16-slot codec at positions 5^i; other periods: every slot snapped) returns the snapped,
    re-encrypted periodic vector at the requested level"""
    from state_encoder import StateEncoder
    E = ctx.engine
    enc = StateEncoder(ctx, states, periodic=True)
    rng = np.random.default_rng(30 + states)
    st = rng.integers(0, 256, (states, 16), dtype=np.uint8)
    hi, lo = enc.encode(st[0] if states == 1 else st)
    hi, lo = E.multiply(hi, 1.0 + 0.01j), E.multiply(lo, 1.0 - 0.01j)  # a small phase error to snap away
    rh, rl = enc.renorm(hi, lo, level=11)
    assert rh.level == rl.level == 11
    assert np.array_equal(enc.decode(rh, rl), st[0] if states == 1 else st)
    clean_hi, _ = enc.encode(st[0] if states == 1 else st)
    assert np.abs(ctx.decrypt(rh) - ctx.decrypt(clean_hi)).max() < 1e-3
