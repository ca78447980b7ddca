"""True-FHE mode: every secret-key renorm replaced by bootstrap + a
homomorphic Zeta16 snap (zeta16_noise_reducer.py; REF/zeta16_noise_reducter.py:6-57,
REF/gen/generate_xor4_coeffs.py:17).  The snaps must contract slot errors quadratically, and a
C2 encrypt / decrypt with use_hard_renorm_between_steps=False must match the byte-level model
without ever calling the secret-key renorm."""
import numpy as np
import pytest

from conftest import gpu_context

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    return gpu_context(log_n=16, signature=1)


def _perturbed(S, rng, eps):
    k = rng.integers(0, 16, S)
    zeta = np.exp(-2j * np.pi * k / 16)
    e = eps * (rng.standard_normal(S) + 1j * rng.standard_normal(S)) / np.sqrt(2)
    return zeta, zeta * (1 + e)


def test_bootstrap_snap_contracts(ctx):
    """errors of ~2e-2 around the codewords come back as O(eps^2): (30x - 15x^2 conj x + conj x^15)/16
    on u = kappa x (kappa folded into the bootstrap), depth 4 -> output at fresh level - 4; when the
    next step is an XOR4 (level hint <= 8) a second snap (x kappa + snap, 5 levels) follows"""
    from utils import NEED_SUBBYTES
    from zeta16_noise_reducer import SNAP15_DEPTH, BootstrapSnap
    E = ctx.engine
    rng = np.random.default_rng(51)
    za, xa = _perturbed(E.slot_count, rng, 0.02)
    zb, xb = _perturbed(E.slot_count, rng, 0.005)
    bs = BootstrapSnap(ctx)
    ya, yb = bs.apply_pair(ctx.encrypt(xa), ctx.encrypt(xb), level=NEED_SUBBYTES)
    assert ya.level == yb.level == E.fresh_level - SNAP15_DEPTH
    # per slot: |f(x) - zeta| <= 12 |e|^2 + 50 |e|^3 (the polynomial, tests/test_snap.py) + bootstrap error
    for x, z, y in ((xa, za, ya), (xb, zb, yb)):
        e_in, e_out = np.abs(x - z), np.abs(ctx.decrypt(y) - z)
        assert np.all(e_out < 12 * e_in ** 2 + 50 * e_in ** 3 + 1e-3), (e_out.max(), e_in.max())
        assert np.sqrt(np.mean(e_out ** 2)) < 0.2 * np.sqrt(np.mean(e_in ** 2))
    y2, _ = bs.apply_pair(ctx.encrypt(xa), ctx.encrypt(xb))  # level hint None: two snaps
    assert y2.level == E.fresh_level - 2 * SNAP15_DEPTH - 1
    e1 = np.abs(ctx.decrypt(ya) - za)
    e2 = np.abs(ctx.decrypt(y2) - za)
    assert np.all(e2 < 12 * e1 ** 2 + 50 * e1 ** 3 + 1e-3), (e2.max(), e1.max())
    assert np.sqrt(np.mean(e2 ** 2)) < 0.2 * np.sqrt(np.mean(e1 ** 2))


def test_reference_noise_reducer_contracts(ctx):
    """the reference's f(x) = (17x - x^17)/16 with bootstrap_before (REF :6-57), depth 6 as written"""
    from zeta16_noise_reducer import Zeta16NoiseReducer
    E = ctx.engine
    rng = np.random.default_rng(52)
    z, x = _perturbed(E.slot_count, rng, 0.02)
    y = Zeta16NoiseReducer(ctx, bootstrap_before=True).apply(ctx.encrypt(x))
    assert y.level == E.fresh_level - 6  # x^17 at depth 5, its -1/16 scalar one more (REF :48-50)
    e_in, e_out = np.abs(x - z), np.abs(ctx.decrypt(y) - z)
    assert np.all(e_out < 12 * e_in ** 2 + 50 * e_in ** 3 + 1e-3), (e_out.max(), e_in.max())


# every entry point that touches the secret key, on the context AND on the engine underneath it
# (state_encoder's periodic-layout renorms call renorm_periodic / renorm_single / renorm_unpack,
# decode calls decrypt): none may run between encryption of the input and the output
SECRET_KEY_CALLS = ("decrypt", "renorm_pair", "renorm_periodic", "renorm_single", "renorm_unpack")
ENGINE_SECRET_CALLS = SECRET_KEY_CALLS + ("export_secret",)


def _no_secret_renorm(ctx, monkeypatch):
    def refuse(name):
        def f(*a, **k):
            raise AssertionError(f"secret-key call {name} in true-FHE mode")
        return f
    for name in SECRET_KEY_CALLS:
        monkeypatch.setattr(ctx, name, refuse("ctx." + name))
    for name in ENGINE_SECRET_CALLS:
        monkeypatch.setattr(ctx.engine, name, refuse("engine." + name))


def test_guard_covers_every_secret_key_entry(ctx, monkeypatch):
    """the guard itself: each secret-key entry point of the context and the engine raises"""
    x = ctx.encrypt(np.ones(ctx.engine.slot_count))
    _no_secret_renorm(ctx, monkeypatch)
    for name in SECRET_KEY_CALLS:
        with pytest.raises(AssertionError, match=name):
            getattr(ctx, name)(x)
        with pytest.raises(AssertionError, match=name):
            getattr(ctx.engine, name)(x)
    monkeypatch.undo()
    assert np.abs(ctx.decrypt(x) - 1).max() < 1e-3  # restored


def test_true_fhe_config2_encrypt_decrypt(ctx, coeff_dir, monkeypatch):
    from aes_keyschedule import expand_aes128_key, load_all_coeffs
    from oracle import aes_plain as A
    from pipeline import AESPipeline
    pipe = AESPipeline(ctx, load_all_coeffs(coeff_dir), use_hard_renorm_between_steps=False, true_fhe=True)
    np.random.seed(7)
    key = np.random.randint(0, 256, 16, dtype=np.uint8)
    pt = np.random.randint(0, 256, 16, dtype=np.uint8)
    rks = expand_aes128_key(key)
    _no_secret_renorm(ctx, monkeypatch)
    n0 = ctx.bootstrap_stats()["count"]
    ct = pipe.encrypt(pt, rks)
    n_enc = ctx.bootstrap_stats()["count"] - n0
    back = pipe.decrypt(*ct, rks)
    monkeypatch.undo()
    assert np.array_equal(pipe.encoder.decode(*ct), A.ref_encrypt(pt, rks))
    assert np.array_equal(pipe.encoder.decode(*back), pt)
    # renorm points of an encrypt (REF/pipeline.py:123-188 + MixColFinal's three) plus the GF
    # multiplier outputs' renorms of true-FHE MixColumns: 1 + 9 * (5 + 2) + 2 pairs
    assert n_enc == 2 * (1 + 9 * 7 + 2), n_enc


def test_quad_bootstrap_matches_pair_bootstraps(ctx):
    """aesfhe_bootstrap_quad_sparse: four 16-periodic messages through ONE bootstrap at period 64 (two
    monomial packings, three split rotations) come back as the pair bootstraps return them: each
    within the bootstrap error of its input, at the same level"""
    from test_gpu_bootstrap import BOOT_TOL
    E = ctx.engine
    S, P = E.slot_count, 16
    rng = np.random.default_rng(61)
    zs = [np.tile(np.exp(2j * np.pi * rng.random(P)), S // P) for _ in range(4)]
    cts = [ctx.to_intt(ctx.encrypt(z)) for z in zs]
    quad = ctx.bootstrap_quad_scaled(cts, 1.0, P)
    pairs = ctx.bootstrap_pair_scaled(cts[0], cts[1], 1.0, P) + ctx.bootstrap_pair_scaled(cts[2], cts[3], 1.0, P)
    for z, q, p in zip(zs, quad, pairs):
        assert q.level == p.level
        assert np.abs(ctx.decrypt(q) - z).max() < 2 * BOOT_TOL
        assert np.abs(ctx.decrypt(q) - ctx.decrypt(p)).max() < 3 * BOOT_TOL
    with pytest.raises(ValueError):
        ctx.engine.bootstrap_quad_sparse(cts[:3], P)


def test_true_fhe_c2_on_the_bench_set(coeff_dir, monkeypatch):
    """the bench's true-FHE set (bench.py --fhe-fresh-level 11 --fhe-dnum 4): one snap per renorm with
    the nibble-bivariate SubBytes, MixColumns' paired renorms in quad bootstraps; encrypt and decrypt
    are FIPS-197's bytes with no secret-key call, 1 + 9 * 5 + 2 bootstrap calls per encrypt for the
    same 132 refreshed ciphertexts"""
    from aes_keyschedule import expand_aes128_key, load_all_coeffs
    from engine_context import EngineContext
    from oracle import aes_plain as A
    from pipeline import AESPipeline
    c12 = EngineContext(signature=1, boot_fresh_level=11, dnum=4, thread_count=4, seed=0xF12, enc_nonce=0xF12)
    pipe = AESPipeline(c12, load_all_coeffs(coeff_dir), use_hard_renorm_between_steps=False, true_fhe=True)
    assert pipe.snapper.max_snaps == 1 and pipe.encoder.renorm_quad_hook is not None
    rng = np.random.default_rng(12)
    rks = expand_aes128_key(rng.integers(0, 256, 16).astype(np.uint8))
    for _ in range(2):
        pt = rng.integers(0, 256, 16).astype(np.uint8)
        _no_secret_renorm(c12, monkeypatch)
        b0 = c12.bootstrap_stats()
        ct = pipe.encrypt(pt, rks)
        b1 = c12.bootstrap_stats()
        back = pipe.decrypt(*ct, rks)
        monkeypatch.undo()
        assert np.array_equal(pipe.encoder.decode(*ct), A.ref_encrypt(pt, rks))
        assert np.array_equal(pipe.encoder.decode(*back), pt)
        assert b1["count"] - b0["count"] == 2 * (1 + 9 * 7 + 2)
        assert b1["calls"] - b0["calls"] == 1 + 9 * 5 + 2


def test_true_fhe_packed_encrypt(ctx, coeff_dir, monkeypatch):
    """256 slot-packed states (8,192 nibble slots per step through every snap), encrypt and
    decrypt: the error tails of a batch, not just one state"""
    from aes_keyschedule import expand_aes128_key, load_all_coeffs
    from oracle import aes_plain as A
    from pipeline import AESPipeline
    B = 256
    pipe = AESPipeline(ctx, load_all_coeffs(coeff_dir), true_fhe=True, states=B)
    rng = np.random.default_rng(53)
    rks = expand_aes128_key(rng.integers(0, 256, 16).astype(np.uint8))
    pts = rng.integers(0, 256, (B, 16)).astype(np.uint8)
    _no_secret_renorm(ctx, monkeypatch)
    ct = pipe.encrypt(pts, rks)
    back = pipe.decrypt(*ct, rks)
    monkeypatch.undo()
    got = pipe.encoder.decode(*ct)
    bad = [j for j in range(B) if not np.array_equal(got[j], A.ref_encrypt(pts[j], rks))]
    assert not bad, bad[:8]
    assert np.array_equal(pipe.encoder.decode(*back), pts)
