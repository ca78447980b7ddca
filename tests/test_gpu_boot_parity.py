"""Limb-level parity of the bootstrap's building blocks against the CPU oracle, on the
N = 2^13 bootstrappable set (fresh level 3 -> L1 = 5, 13 double-prime levels, dnum 5).

Same parameters and seed on both sides -> identical primes, scales and keys; identical input
limbs -> identical output limbs for:
- a key switch at double-prime levels (the CtS / EvalMod / StC rotations);
- the double-prime rescale (oracle orc_rescale2: both limbs of the pair dropped, one rounding);
- bootstrap stage 1, the level-0 scaling by k1 on the two base limbs Q0 = q0 q1;
- stage 2, the dense -> sparse key switch over Q0 P' (oracle orc_keyswitch_d2s, with the
  engine's exported d2s key; c0 added);
- stage 3, ModRaise: the centred CRT lift of (q0, q1) to every limb of the top level;
- stage 4, the sparse -> dense key switch at the top level (the oracle's generic key switch
  with the exported s2d key).
Stages are produced by aesfhe_debug_boot_stage (engine.hip bootstrap_l0 stop_after).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

LOG_N, FRESH, SEED = 13, 3, 7


@pytest.fixture(scope="module")
def pair():
    from mi355x_ckks import Engine
    from oracle.ckks_cpu import OracleParams
    E = Engine(log_n=LOG_N, use_bootstrap=True, max_level=FRESH, dnum=5, seed=SEED, allow_insecure=True)
    # the engine's chain: L1 = fresh + 2 single-prime levels, then the bootstrap's double-prime levels
    L1 = max(l for l in range(E.L + 1) if E.level_limbs[l] == l + 2)
    O = OracleParams(log_n=LOG_N, max_level=L1, dnum=E.dnum, seed=SEED, boot_double=E.L - L1)
    return E, O


def rand_rows(O, limbs, rng):
    return np.stack([rng.integers(0, int(O.moduli[t]), O.n, dtype=np.uint64) for t in limbs]).astype(np.uint32)


def rand_ct(O, level, npoly, rng):
    return np.stack([rand_rows(O, range(O.nl(level)), rng) for _ in range(npoly)])


def addmod(a, b, q):
    return ((a.astype(np.uint64) + b) % q).astype(np.uint32)


def test_boot_chain_matches(pair):
    E, O = pair
    assert O.L == E.L and O.n_q == E.n_q and O.n_p == E.n_p and O.n_ks == E.n_ks
    assert [O.nl(l) for l in range(O.L + 1)] == E.level_limbs
    assert np.array_equal(E.moduli(), O.moduli)
    assert np.array_equal(E.scales(), O.deltas)


@pytest.mark.parametrize("which", ["relin", "conj", "rot"])
def test_keyswitch_double_prime_levels(pair, which):
    E, O = pair
    g = {"relin": 0, "conj": E.galois_conj, "rot": E.galois_rotate(E.slot_count // 8)}[which]
    key = O.gen_ksk(g)
    assert np.array_equal(E.export_ksk(g), key)
    rng = np.random.default_rng(11)
    for level in sorted({O.L, O.L - 1, O.L1 + 2, O.L1 + 1}):
        d = rand_rows(O, range(O.nl(level)), rng)
        assert np.array_equal(E.debug_keyswitch(level, g, d), O.keyswitch(level, d, key)), level


def test_rescale_double_prime(pair):
    E, O = pair
    rng = np.random.default_rng(12)
    for level in sorted({O.L, O.L - 3, O.L1 + 2, O.L1 + 1}):
        x = rand_ct(O, level, 2, rng)
        got = E.export(E.rescale(E.import_ct(x, level)))
        assert np.array_equal(got, O.rescale2(level, x)), level


def _boot_stages(E, O, seed):
    rng = np.random.default_rng(seed)
    x = rand_ct(O, 0, 2, rng)
    ct = E.import_ct(x, 0)
    return x, [E.export(E.debug_boot_stage(ct, s)) for s in (1, 2, 3, 4)]


@pytest.mark.parametrize("seed", [13, 14])
def test_bootstrap_stages_bitexact(pair, seed):
    E, O = pair
    info = E.boot_info()
    x, (s1, s2, s3, s4) = _boot_stages(E, O, seed)
    q0, q1 = int(O.moduli[0]), int(O.moduli[1])
    Q01 = O.limbs_mod(2)
    # 1. scaling by the integer k1 on (q0, q1)
    k1 = int(info["k1"])
    r = np.array([[k1 % q0], [k1 % q1]], np.uint64)
    assert s1.shape == (2, 2, O.n)
    assert np.array_equal(s1, ((x.astype(np.uint64) * r) % Q01).astype(np.uint32))
    # 2. dense -> sparse over Q0 P' (the exported key is the one the engine switches with)
    npd = int(info["d2s_special_primes"])
    key = E.export_ksk(2 * E.n + 1)[0]
    ks = O.keyswitch_d2s(npd, s1[1], key)
    want2 = np.stack([addmod(ks[0], s1[0], Q01), ks[1]])
    assert np.array_equal(s2, want2)
    # 3. ModRaise: X = x0 + q0 ((x1 - x0) q0^-1 mod q1), centred in (-Q0/2, Q0/2], to every top limb
    top = int(info["top"])
    nlt = O.nl(top)
    co = O.intt(s2.reshape(4, O.n), [0, 1, 0, 1]).reshape(2, 2, O.n).astype(np.int64)
    q0inv = pow(q0, -1, q1)
    X = co[:, 0] + q0 * ((((co[:, 1] - co[:, 0]) % q1) * q0inv) % q1)
    X = np.where(X > (q0 * q1) // 2, X - q0 * q1, X)
    lifted = np.stack([np.stack([(X[p] % int(O.moduli[t])) for t in range(nlt)]) for p in range(2)]).astype(np.uint32)
    want3 = O.ntt(lifted.reshape(2 * nlt, O.n), list(range(nlt)) * 2).reshape(2, nlt, O.n)
    assert s3.shape == (2, nlt, O.n)
    assert np.array_equal(s3, want3)
    # 4. sparse -> dense at the top level
    ks = O.keyswitch(top, s3[1], E.export_ksk(2 * E.n + 3))
    want4 = np.stack([addmod(ks[0], s3[0], O.limbs_mod(nlt)), ks[1]])
    assert np.array_equal(s4, want4)


@pytest.mark.parametrize("which", range(6))
def test_lin_group_matches_plan(pair, which):
    """One hoisted BSGS linear-transform group of the bootstrap (k_lin_mac: baby-step key inner
    products, diagonals in Q*P, giant-step rotations, one ModDown + rescale) against the plan's
    matrix applied to the decrypted input on the host (bootstrap.cpp apply_group_plain).  Groups
    0..2 are CoeffToSlot, run from the top level on the bootstrap's own stage-4 ciphertext
    (ModRaise + sparse -> dense key switch); 3..5 are SlotToCoeff, run further down the same
    chain.  Linear in the message, so the check holds for any input: a wrong diagonal, offset
    or key shows up at the scale of the output.  Measured on MI355X: relative error 1.5e-14 ..
    6.7e-14 (CoeffToSlot), ~6e-16 (SlotToCoeff) -- the double-prime scale's noise."""
    E, _ = pair
    rng = np.random.default_rng(20 + which)
    z = 0.5 * (rng.uniform(-1, 1, E.slot_count) + 1j * rng.uniform(-1, 1, E.slot_count))
    x = E.debug_boot_stage(E.encrypt(z), 4)
    for w in range(which):
        x = E.debug_lin_group(x, w)
    want = E.debug_lin_group_plain(which, E.decrypt(x))
    got = E.decrypt(E.debug_lin_group(x, which))
    scale = np.abs(want).max()
    err = np.abs(got - want).max() / scale
    print(f"group {which}: level {x.level}, max |out| {scale:.3g}, relative error {err:.2e}")
    assert scale > 1e-3
    assert err < 1e-9


def _evalmod_plain(y, K, r, deg):
    """the plan's EvalMod (bootstrap.cpp make_boot_plan + engine.hip eval_mod): the degree-deg
    Chebyshev interpolant of cos(2 pi (K y - 1/4) / 2^r) on [-1, 1], then r double angles"""
    n = deg + 1
    j = np.arange(n)
    f = np.cos(2 * np.pi * (K * np.cos(np.pi * (j + 0.5) / n) - 0.25) / 2.0 ** r)
    c = np.array([(1.0 if k == 0 else 2.0) * np.dot(f, np.cos(np.pi * k * (j + 0.5) / n)) / n for k in range(n)])
    g = np.polynomial.chebyshev.chebval(y, c)
    for _ in range(r):
        g = 2 * g * g - 1
    return g


def test_evalmod_matches_plan(pair):
    """EvalMod on the bootstrap's own CoeffToSlot output (stages 6 / 7: the real and imaginary
    parts, slots in [-1, 1]) against the plan's polynomial on the host: stage 8 (real half alone)
    and stage 10 (both halves stacked in one batched ciphertext, recombined as f(re) + i f(im),
    the production path).  The double angles amplify the input noise 4^r-fold, so the tolerance
    is absolute (outputs lie in [-1, 1]).  Measured on MI355X: 1.2e-11 / 1.5e-11."""
    E, _ = pair
    info = E.boot_info()
    K, r, deg = int(info["K"]), int(info["r"]), int(info["deg"])
    rng = np.random.default_rng(31)
    z = 0.5 * (rng.uniform(-1, 1, E.slot_count) + 1j * rng.uniform(-1, 1, E.slot_count))
    ct = E.encrypt(z)
    re, im = E.decrypt(E.debug_boot_stage(ct, 6)), E.decrypt(E.debug_boot_stage(ct, 7))
    assert np.abs(re.imag).max() < 1e-6 and np.abs(im.imag).max() < 1e-6
    assert np.abs(re.real).max() <= 1.0 and np.abs(im.real).max() <= 1.0
    want_re, want_im = _evalmod_plain(re.real, K, r, deg), _evalmod_plain(im.real, K, r, deg)
    got8 = E.decrypt(E.debug_boot_stage(ct, 8))
    got10 = E.decrypt(E.debug_boot_stage(ct, 10))
    e8 = np.abs(got8 - want_re).max()
    e10 = np.abs(got10 - (want_re + 1j * want_im)).max()
    print(f"EvalMod K {K} r {r} deg {deg}: stage 8 max error {e8:.2e}, stage 10 {e10:.2e}")
    assert e8 < 1e-8 and e10 < 1e-8
