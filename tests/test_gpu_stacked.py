"""Stacked ciphertexts -- multi-pair batches (include/aesfhe.h aesfhe_stack) --
on the MI355X.  A stack of P single ciphertexts is one operand: every op's result, unstacked,
equals the same op on each member bit for bit (raw RNS limbs), with stacks larger than one
key-switch chunk; the LUT sum, the renorm and the bootstraps likewise; and AESPipeline with
`pairs` runs P independent ciphertext pairs (BASELINE config 3: one state per pair) through one
encrypt, every pair's ciphertext decoding to the reference AES."""
import numpy as np
import pytest

from conftest import gpu_context, gpu_engine

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def E():
    return gpu_engine(log_n=16, max_level=17)


@pytest.fixture(scope="module")
def ctx():
    return gpu_context(log_n=16, signature=1)


def _cts(E, n, seed, period=None):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        z = np.exp(2j * np.pi * rng.random(period or E.slot_count))
        out.append(E.encrypt(np.tile(z, E.slot_count // len(z))))
    return out


def _same(E, stack, singles, what):
    got = E.unstack(stack)
    assert len(got) == len(singles), what
    for i, (g, w) in enumerate(zip(got, singles)):
        assert g.level == w.level, (what, i)
        assert np.array_equal(E.export(g), E.export(w)), (what, i)


def test_stack_roundtrip_and_guards(E):
    cs = _cts(E, 5, 1)
    st = E.stack(cs)
    assert E.members(st) == 5 and E.members(cs[0]) == 1
    _same(E, st, cs, "stack/unstack")
    with pytest.raises(RuntimeError):
        E.decrypt(st)  # a stack is decrypted member by member
    with pytest.raises(RuntimeError):
        E.add(st, E.stack(cs[:3]))  # no broadcasting between stacks of different sizes


@pytest.mark.parametrize("n", [2, 11])  # 11: more members than one key-switch chunk at any level
def test_stacked_ops_bit_exact(E, n):
    a, b = _cts(E, n, 10 + n), _cts(E, n, 20 + n)
    A, B = E.stack(a), E.stack(b)
    rng = np.random.default_rng(n)
    pt = E.encode(np.where(rng.random(E.slot_count) < 0.5, 1.0, 0.0))
    _same(E, E.multiply(A, B, "rlk"), [E.multiply(x, y, "rlk") for x, y in zip(a, b)], "ct x ct")
    _same(E, E.multiply(A, A, "rlk"), [E.multiply(x, x, "rlk") for x in a], "square")
    _same(E, E.rotate(A, None, 5), [E.rotate(x, None, 5) for x in a], "rotate")
    _same(E, E.conjugate(A), [E.conjugate(x) for x in a], "conjugate")
    _same(E, E.multiply(A, pt), [E.multiply(x, pt) for x in a], "ct x pt")
    _same(E, E.add_plain(E.multiply(A, 3.0), 0.25), [E.add_plain(E.multiply(x, 3.0), 0.25) for x in a], "scalars")
    _same(E, E.subtract(A, B), [E.subtract(x, y) for x, y in zip(a, b)], "sub")
    _same(E, E.level_down(A, 5), [E.level_down(x, 5) for x in a], "level_down")
    # a deferred tensor stack plus a ciphertext stack (the conjugate-split LUT sum's shape)
    _same(E, E.add(E.multiply(A, B, "rlk"), E.rotate(B, None, 3)),
          [E.add(E.multiply(x, y, "rlk"), E.rotate(y, None, 3)) for x, y in zip(a, b)], "tensor + ct")
    pw_st = E.make_power_basis(A, 5)
    pw = [E.make_power_basis(x, 5) for x in a]
    for k in range(5):
        _same(E, pw_st[k], [p[k] for p in pw], f"power basis x^{k + 1}")


def test_stacked_lut_sums_bit_exact(E):
    n = 3
    a, b = _cts(E, n, 31), _cts(E, n, 32)
    rng = np.random.default_rng(3)
    C = rng.standard_normal((4, 4)) + 1j * rng.standard_normal((4, 4))
    biv = E.lut_create(C)
    uni = E.lut_create(rng.standard_normal(4) + 0j, c0=0.5)
    pa = [E.make_power_basis(x, 3) for x in a]
    pb = [E.make_power_basis(y, 3) for y in b]
    PA = [E.stack([p[k] for p in pa]) for k in range(3)]
    PB = [E.stack([p[k] for p in pb]) for k in range(3)]
    one_a = [E.add_plain(E.multiply(x, 0.0), 1.0) for x in a]
    one_b = [E.add_plain(E.multiply(y, 0.0), 1.0) for y in b]
    el_a = lambda i: [one_a[i]] + pa[i]  # noqa: E731
    el_b = lambda i: [one_b[i]] + pb[i]  # noqa: E731
    st_a, st_b = [E.stack(one_a)] + PA, [E.stack(one_b)] + PB
    _same(E, E.lut_eval(biv, st_a, st_b), [E.lut_eval(biv, el_a(i), el_b(i)) for i in range(n)], "bivariate LUT")
    _same(E, E.lut_eval(uni, st_a), [E.lut_eval(uni, el_a(i)) for i in range(n)], "univariate LUT")


@pytest.mark.parametrize("period", [None, 16])
def test_stacked_renorm_matches_singles(ctx, period):
    """renorm of a stacked pair: every member's snapped state equals its single renorm's (the
    stacked codec is the fp64 FFT one, so the re-encryptions are compared by decoded values)"""
    from state_encoder import StateEncoder
    E = ctx.engine
    P = 5
    enc = StateEncoder(ctx, 1, periodic=period is not None, pairs=P)
    rng = np.random.default_rng(41)
    st = rng.integers(0, 256, (P, 16), dtype=np.uint8)
    hi, lo = enc.encode(st)
    # noisy, off-scale inputs as a LUT leaves them: times 256, one level of products
    hi, lo = E.multiply(hi, 256.0), E.multiply(lo, 256.0)
    rh, rl = enc.renorm(hi, lo)
    assert E.members(rh) == P and E.members(rl) == P
    assert np.array_equal(enc.decode(rh, rl), st)
    one = StateEncoder(ctx, 1, periodic=period is not None)
    for m, (h, l) in enumerate(zip(E.unstack(rh), E.unstack(rl))):
        z = ctx.decrypt(h)
        assert np.abs(np.abs(z) - 1.0).max() < 2e-4  # fresh unit-magnitude codewords in every slot
        assert np.array_equal(one.decode(h, l), st[m])


def test_stacked_bootstraps_bit_exact(ctx):
    """chunks of two members through the pair bootstrap equal the single bootstraps"""
    E = ctx.engine
    P = 3
    a = _cts(E, P, 51, period=32)
    A = E.stack(a)
    _same(E, E.bootstrap_sparse(A, 32), [E.bootstrap_sparse(x, 32) for x in a], "sparse bootstrap")
    b = _cts(E, P, 52, period=16)
    c = _cts(E, P, 53, period=16)
    H, L = E.bootstrap_pair_sparse(E.stack(b), E.stack(c), 16)
    singles = [E.bootstrap_pair_sparse(x, y, 16) for x, y in zip(b, c)]
    _same(E, H, [s[0] for s in singles], "mono pair bootstrap (hi)")
    _same(E, L, [s[1] for s in singles], "mono pair bootstrap (lo)")


@pytest.mark.parametrize("members", [2, 4, 8])
def test_stacked_bootstrap_packing(ctx, members):
    """aesfhe_set_stack_pack: an 8-member stack of period-32 ciphertexts bootstrapped `members` per
    bootstrap (monomial packing over the stack's halves) returns every member
    in its place, within `members` x the single bootstrap's error of it, at the same level"""
    from test_gpu_bootstrap import BOOT_TOL
    E = ctx.engine
    M, P = 8, 32
    rng = np.random.default_rng(70 + members)
    zs = [np.tile(np.exp(2j * np.pi * rng.random(P)), E.slot_count // P) for _ in range(M)]
    st = E.stack([E.encrypt(z) for z in zs])
    try:
        E.set_stack_pack(1)
        ref = E.unstack(E.bootstrap_sparse(st, P))
        E.set_stack_pack(members)
        out = E.unstack(E.bootstrap_sparse(st, P))
    finally:
        E.set_stack_pack(16)
    for z, r, o in zip(zs, ref, out):
        assert o.level == r.level
        assert np.abs(E.decrypt(o) - z).max() < members * BOOT_TOL
    with pytest.raises(RuntimeError):
        E.set_stack_pack(0)


@pytest.mark.parametrize("periodic", [True, False])
def test_pipeline_pairs_encrypt(ctx, coeff_dir, periodic):
    """AESPipeline(pairs=P): P ciphertext pairs with one state each (BASELINE config 3's shape),
    one stacked encrypt; every pair decodes to the reference AES of its own state"""
    from aes_keyschedule import expand_aes128_key, load_all_coeffs
    from oracle import aes_plain as A
    from pipeline import AESPipeline
    P = 3
    pipe = AESPipeline(ctx, load_all_coeffs(coeff_dir), use_hard_renorm_between_steps=True, pairs=P, periodic=periodic)
    rks = expand_aes128_key(np.arange(16, dtype=np.uint8) * 7)
    pts = np.random.default_rng(61).integers(0, 256, (P, 16), dtype=np.uint8)
    ct = pipe.encrypt(pts, rks)
    assert ctx.engine.members(ct[0]) == P
    got = pipe.encoder.decode(*ct)
    want = np.stack([A.ref_encrypt(p, rks) for p in pts])
    assert np.array_equal(got, want), int((got != want).any(axis=1).sum())


@pytest.mark.parametrize("P", [16, 19])
def test_pipeline_many_pairs_encrypt(ctx, coeff_dir, P):
    """BASELINE config 3's shape at a real stack size (VERDICT r4 'do this' 4): P >= 16 one-state
    ciphertext pairs stacked through AESPipeline(pairs=P) in the default periodic layout -- more
    members than one key-switch chunk (ks_chunk <= 8) and, for 19, a ragged last chunk and an odd
    member for the pair bootstrap's chunks of two -- every pair checked against FIPS-197 AES of its
    own state (REF/state_encoder.py:17-28: one state per pair)"""
    from aes_keyschedule import expand_aes128_key, load_all_coeffs
    from oracle import aes_plain as A
    from pipeline import AESPipeline
    pipe = AESPipeline(ctx, load_all_coeffs(coeff_dir), use_hard_renorm_between_steps=True, pairs=P)
    rks = expand_aes128_key(np.arange(16, dtype=np.uint8) * 11 + 3)
    pts = np.random.default_rng(1000 + P).integers(0, 256, (P, 16), dtype=np.uint8)
    ct = pipe.encrypt(pts, rks)
    assert ctx.engine.members(ct[0]) == P and ctx.engine.members(ct[1]) == P
    got = pipe.encoder.decode(*ct)
    want = np.stack([A.ref_encrypt(p, rks) for p in pts])
    bad = np.flatnonzero((got != want).any(axis=1))
    assert bad.size == 0, f"pairs {bad.tolist()} differ"
