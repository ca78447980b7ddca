"""Fused LUT evaluation (aesfhe_lut_eval) against the CPU oracle and against
the reference's per-term product loops.

* bit-exact: the fused kernel's deferred tensor, canonicalised by the engine (rescale,
  relinearise, rescale), equals the oracle's sum_{p,q} C_pq (a_p x b_q) put through the same
  oracle primitives -- the integer constants C_pq = llround(c_pq S(l,2) / (delta_p delta_q))
  restated here from the engine's rule;
* module level: XOR4 / SubBytes through the fused op decode to the same bytes as the
  reference's loops (REF/xor4_lut.py:63-74, REF/sub_bytes_lut.py:46-74) and agree with
  them slot by slot within CKKS rounding.
"""
import math

import numpy as np
import pytest

from conftest import gpu_context, gpu_engine

pytestmark = pytest.mark.gpu

SETS = [(13, 6), (16, 17)]


@pytest.fixture(scope="module", params=SETS, ids=lambda s: f"logn{s[0]}_L{s[1]}")
def pair(request):
    from oracle.ckks_cpu import OracleParams
    log_n, L = request.param
    return gpu_engine(log_n=log_n, max_level=L, seed=0x5EED), OracleParams(log_n=log_n, max_level=L, dnum=3, seed=0x5EED)


def llround(x):
    return int(math.copysign(math.floor(abs(x) + 0.5), x))


def raw_scale(O, l, p):
    """delta_{l-p} times the primes the p owed rescales divide out (engine raw_scale)"""
    sc = float(O.deltas[l - p])
    for j in range(p):
        sc *= float(O.moduli[l - j + 1])  # nl(l) = l + 2: the rescale at level l drops q_{l+1}
    return sc


def ntt_const(O, a, b, nl):
    poly = np.zeros((nl, O.n), np.uint32)
    poly[:, 0] = O.const_residues(a, nl)
    poly[:, O.n // 2] = O.const_residues(b, nl)
    return O.ntt(poly, range(nl)).astype(np.uint64)


def rand_ct(O, level, rng):
    return np.stack([np.stack([rng.integers(0, int(O.moduli[t]), O.n, dtype=np.uint64) for t in range(level + 2)])
                     for _ in range(2)]).astype(np.uint32)


def test_bivariate_lut_bitexact(pair):
    E, O = pair
    rng = np.random.default_rng(21)
    top = min(O.L, 6)
    la, lb = [top, top - 1, top], [top - 1, top, top - 2]
    A = [rand_ct(O, lv, rng) for lv in la]
    B = [rand_ct(O, lv, rng) for lv in lb]
    C = (rng.standard_normal((3, 3)) + 1j * rng.standard_normal((3, 3))) * 3
    C[1, 2] = 0
    C[0, 0] = 0.75  # real coefficient
    lut = E.lut_create(C)
    out = E.lut_eval(lut, [E.import_ct(a, lv) for a, lv in zip(A, la)], [E.import_ct(b, lv) for b, lv in zip(B, lb)])
    l = min(la + lb)
    nl = l + 2
    assert out.level == l - 2
    q = O.limbs_mod(nl).astype(np.uint64)
    s_out = raw_scale(O, l, 2)
    raw = np.zeros((3, nl, O.n), np.uint64)
    for p in range(3):
        for qq in range(3):
            if C[p, qq] == 0:
                continue
            f = s_out / (float(O.deltas[la[p]]) * float(O.deltas[lb[qq]]))
            k = ntt_const(O, llround(C[p, qq].real * f), llround(C[p, qq].imag * f), nl)
            t = O.tensor(l, A[p][:, :nl], B[qq][:, :nl]).astype(np.uint64)
            raw = (raw + t * k % q) % q
    r1 = O.rescale(l, raw.astype(np.uint32)).astype(np.uint64)  # 3-poly tensor: one rescale first
    ks = O.keyswitch(l - 1, r1[2].astype(np.uint32), O.gen_ksk(0)).astype(np.uint64)
    q1 = O.limbs_mod(nl - 1).astype(np.uint64)
    relin = ((r1[:2] + ks) % q1).astype(np.uint32)
    assert np.array_equal(E.export(out), O.rescale(l - 1, relin))


def test_univariate_lut_bitexact(pair):
    E, O = pair
    rng = np.random.default_rng(22)
    top = min(O.L, 6)
    lv = [top, top - 1, top - 1, top]
    X = [rand_ct(O, v, rng) for v in lv]
    C = rng.standard_normal(4) + 1j * rng.standard_normal(4)
    C[2] = 0
    c0 = 0.3 - 0.8j
    lut = E.lut_create(C, c0)
    out = E.lut_eval(lut, [E.import_ct(x, v) if c != 0 else None for x, v, c in zip(X, lv, C)])
    l = min(v for v, c in zip(lv, C) if c != 0)
    nl = l + 2
    assert out.level == l - 1
    q = O.limbs_mod(nl).astype(np.uint64)
    s_out = raw_scale(O, l, 1)
    raw = np.zeros((2, nl, O.n), np.uint64)
    for x, v, c in zip(X, lv, C):
        if c == 0:
            continue
        f = s_out / float(O.deltas[v])
        raw = (raw + x[:, :nl].astype(np.uint64) * ntt_const(O, llround(c.real * f), llround(c.imag * f), nl) % q) % q
    # c0 at the raw scale: round(c0 delta_{l-1}) times the prime the owed rescale divides out
    k0 = ntt_const(O, llround(c0.real * float(O.deltas[l - 1])), llround(c0.imag * float(O.deltas[l - 1])), nl)
    f0 = np.array([int(O.moduli[l + 1]) % int(O.moduli[t]) for t in range(nl)], np.uint64)
    raw[0] = (raw[0] + k0 * f0[:, None] % q) % q
    assert np.array_equal(E.export(out), O.rescale(l, raw.astype(np.uint32)))


def test_lut_level_error_message(pair):
    """too low for the fused form -> a "level" error (the modules then run the product loop)"""
    E, O = pair
    rng = np.random.default_rng(23)
    lut = E.lut_create(np.ones((2, 2)))
    a = [E.import_ct(rand_ct(O, 1, rng), 1) for _ in range(2)]
    with pytest.raises(RuntimeError, match="level"):
        E.lut_eval(lut, a, a)


def test_lut_free(pair):
    """aesfhe_lut_free releases a set (and its per-level constants); a freed handle is refused,
    and so is a ciphertext handle passed as a LUT"""
    E, O = pair
    rng = np.random.default_rng(24)
    top = min(O.L, 6)
    lut = E.lut_create(np.ones(2), 0.5)
    x = [E.import_ct(rand_ct(O, top, rng), top) for _ in range(2)]
    out = E.lut_eval(lut, x)
    h = lut.handle
    E.lut_free(lut)
    assert lut.handle == 0
    lut.handle = h
    with pytest.raises(RuntimeError):
        E.lut_eval(lut, x)
    lut.handle = 0
    with pytest.raises(RuntimeError, match="not a LUT"):
        E._ctx.check(E._lib.aesfhe_lut_free(E._ctx.ptr, out.handle))
    assert out.level == top - 1  # the ciphertext is untouched


def test_lut_cache_same_label_different_sets():
    """a deterministic regression for the stale-coefficient failure -- two
    coefficient sets requested under ONE caller label (as an id() reused after collection would
    produce) get two device sets, and each evaluates to its own polynomial"""
    ctx = gpu_context(log_n=16, signature=2)
    E = ctx.engine
    rng = np.random.default_rng(25)
    z = np.exp(2j * np.pi * rng.random(E.slot_count))
    x = ctx.encrypt(z)
    pb = ctx.make_power_basis(x, 3)
    label = ("sb", 140000000000000)
    c1 = np.array([0.5, -0.25 + 0.1j, 0.3])
    c2 = np.array([-0.2, 0.4, 0.1 - 0.3j])
    l1 = ctx.lut(label, c1, 0.1)
    l2 = ctx.lut(label, c2, 0.1)
    assert l1 is not l2
    for c, lut in ((c1, l1), (c2, l2)):
        out = ctx.decrypt(ctx.lut_eval(lut, pb))
        want = 0.1 + c[0] * z + c[1] * z ** 2 + c[2] * z ** 3
        assert np.abs(out - want).max() < 1e-3


# ---------------------------------------------------------------- module level, fused vs loop
@pytest.fixture(scope="module")
def coeffs(coeff_dir):
    from aes_keyschedule import load_all_coeffs
    return load_all_coeffs(coeff_dir)


def _slots(ctx, ct):
    sc = ctx.engine.slot_count
    return ctx.decrypt(ct)[: 16 * (sc // 16): sc // 16]


def test_xor4_fused_matches_loop(coeffs):
    from state_encoder import StateEncoder
    from xor4_lut import XOR4LUT
    ctx = gpu_context(log_n=16)
    enc = StateEncoder(ctx)
    rng = np.random.default_rng(5)
    a, b = rng.integers(0, 256, 16).astype(np.uint8), rng.integers(0, 256, 16).astype(np.uint8)
    (ah, al), (bh, bl) = enc.encode(a), enc.encode(b)
    x = XOR4LUT(ctx, coeffs["xor4"])
    before = ctx.engine.counters()["lut"]
    fused = x.apply(ah, bh)
    assert ctx.engine.counters()["lut"] == before + 2  # conjugate split: S1 + conj(S2)
    ctx.fused_luts = False
    try:
        loop = x.apply(ah, bh)
    finally:
        ctx.fused_luts = True
    assert fused.level == loop.level
    zf, zl = _slots(ctx, fused), _slots(ctx, loop)
    # the two paths evaluate the same polynomial by different product trees (the fused path's
    # mirrors are powers of conj(b), the loop's conjugations of b's powers), each on freshly
    # encrypted inputs (random per process): both against the exact output 256 zeta^(a ^ b) of the
    # high nibbles, within 5e-4 relative -- 400x inside the decode margin
    # 256 sin(pi / 16) ~ 50
    ideal = 256.0 * np.exp(-2j * np.pi / 16) ** ((a >> 4) ^ (b >> 4))
    ef, el = np.abs(zf - ideal).max(), np.abs(zl - ideal).max()
    print(f"fused / loop vs exact: max |err| {ef:.3g} / {el:.3g} at |z| = 256")
    assert ef < 256 * 5e-4 and el < 256 * 5e-4
    assert np.array_equal(enc.decode(fused, x.apply(al, bl)), a ^ b)


def test_subbytes_fused_matches_loop(coeffs):
    from oracle import aes_plain
    from state_encoder import StateEncoder
    from sub_bytes_lut import SubBytesLUT
    ctx = gpu_context(log_n=16)
    enc = StateEncoder(ctx)
    state = np.arange(0, 256, 17, dtype=np.uint8)[:16]
    sb = SubBytesLUT(ctx, coeffs["sub_hi"], coeffs["sub_lo"])
    hi, lo = enc.encode(state)
    fh, fl = sb.apply(hi, lo)
    ctx.fused_luts = False
    try:
        lh, ll = sb.apply(hi, lo)
    finally:
        ctx.fused_luts = True
    assert (fh.level, fl.level) == (lh.level, ll.level)
    # b = hi * lift(lo) is raised to the 128th power, which amplifies the last-bit difference
    # of the two lifted inputs: the paths agree to the noise level (~1e-3 rms, measured by
    # tools/lut_noise.py: fused 1.03e-3, loop 1.26e-3 rad over 6 states), not bit for bit
    for f, g in ((fh, lh), (fl, ll)):
        assert np.abs(_slots(ctx, f) - _slots(ctx, g)).max() < 2e-2
    assert np.array_equal(enc.decode(fh, fl), aes_plain.SBOX[state])


@pytest.mark.parametrize("mult", [2, 3, 9, 11, 13, 14])
def test_gf_mult_split_matches_loop(mult):
    """GF multipliers: the conjugate-split form over shared bases vs the reference's loops"""
    from mixcol_final import _CoeffCache, gf_mult_pair
    from oracle import aes_plain
    from state_encoder import StateEncoder
    ctx = gpu_context(log_n=16)
    enc = StateEncoder(ctx)
    state = np.random.default_rng(mult).integers(0, 256, 16).astype(np.uint8)
    hi, lo = enc.encode(state)
    cache = _CoeffCache()
    fh, fl = gf_mult_pair(ctx, cache, mult, hi, lo)
    ctx.fused_luts = False
    try:
        lh, ll = gf_mult_pair(ctx, cache, mult, hi, lo)
    finally:
        ctx.fused_luts = True
    assert (fh.level, fl.level) == (lh.level, ll.level)
    for f, g in ((fh, lh), (fl, ll)):
        assert np.abs(_slots(ctx, f) - _slots(ctx, g)).max() < 1e-3
    assert np.array_equal(enc.decode(fh, fl), aes_plain.GF_MUL[mult][state])
