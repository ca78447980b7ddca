"""Batched engine ops (aesfhe_mul_many / aesfhe_conjugate_many) on the MI355X:
every result equals the separate engine call bit for bit (raw RNS limbs), for mixed levels,
squarings, more members than one key-switch chunk (4) and than one batch (8); the batched
power basis and the batched AES building blocks decode exactly."""
import numpy as np
import pytest

from conftest import gpu_context, gpu_engine

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def E():
    return gpu_engine(log_n=16, max_level=17)


def _cts(E, n, seed):
    rng = np.random.default_rng(seed)
    return [E.encrypt(np.exp(2j * np.pi * rng.random(E.slot_count))) for _ in range(n)]


@pytest.mark.parametrize("n", [2, 5, 11])
def test_mul_many_bit_exact(E, n):
    cs = _cts(E, n + 1, n)
    low = E.multiply(cs[0], cs[1], "rlk")  # one level lower: the batch has two level groups
    pairs = [(cs[i], cs[i + 1]) for i in range(n - 1)] + [(cs[0], cs[0]), (low, cs[2])][: max(1, min(2, n - 1))]
    got = E.multiply_many(pairs)
    for (a, b), g in zip(pairs, got):
        want = E.multiply(a, b, "rlk")
        assert g.level == want.level
        assert np.array_equal(E.export(g), E.export(want))


@pytest.mark.parametrize("n", [2, 6])
def test_conjugate_many_bit_exact(E, n):
    cs = _cts(E, n, 100 + n)
    cs[-1] = E.multiply(cs[-1], cs[0], "rlk")  # a second level group
    got = E.conjugate_many(cs)
    for c, g in zip(cs, got):
        assert np.array_equal(E.export(g), E.export(E.conjugate(c)))


def test_power_basis_batched_values(E):
    rng = np.random.default_rng(7)
    z = np.exp(2j * np.pi * rng.random(E.slot_count))
    pb = E.make_power_basis(E.encrypt(z), 16)
    for k in (2, 3, 7, 8, 11, 16):
        # |d(z^k)| = k |dz| on the unit circle: the max slot error grows ~linearly in k (the
        # measured tail at k = 16 is ~2e-3 over 32768 slots)
        err = np.abs(E.decrypt(pb[k - 1]) - z ** k).max()
        assert err < 5e-4 + 2.5e-4 * k, (k, err)


def test_batched_aes_blocks_decode_exactly(coeff_dir):
    """XOR pair, GF multiplier pair and SubBytes through the batched paths"""
    from aes_keyschedule import load_all_coeffs
    from mixcol_final import MixColFinal
    from oracle import aes_plain as A
    from state_encoder import StateEncoder
    from sub_bytes_lut import SubBytesLUT
    from utils import LUT2_DEPTH, RENORM_FLOOR
    from xor4_lut import XOR4LUT
    ctx = gpu_context(log_n=16, signature=1)
    co = load_all_coeffs(coeff_dir)
    enc = StateEncoder(ctx)
    xor4 = XOR4LUT(ctx, co["xor4"])
    mix = MixColFinal(ctx, xor4)
    rng = np.random.default_rng(12)
    s1, s2 = rng.integers(0, 256, 16, dtype=np.uint8), rng.integers(0, 256, 16, dtype=np.uint8)
    a, b = enc.encode(s1), enc.encode(s2)
    x = xor4.apply_pair(a[0], b[0], a[1], b[1], RENORM_FLOOR)
    assert np.array_equal(enc.decode(*x), s1 ^ s2)
    g = mix.gf_mult_3(*a, out_level=RENORM_FLOOR + LUT2_DEPTH)
    assert np.array_equal(enc.decode(*g), A.GF_MUL[3][s1])
    sb = SubBytesLUT(ctx, co["sub_hi"], co["sub_lo"])
    assert np.array_equal(enc.decode(*sb.apply(*a, out_level=RENORM_FLOOR)), A.SBOX[s1])


def test_rotate_hoisted_bit_exact(E):
    """one ModUp for several rotations of one ciphertext equals separate rotations"""
    c = _cts(E, 1, 31)[0]
    s = E.slot_count
    steps = [-(s // 4), -(s // 2), 0, 3 * s // 4, 5]
    got = E.rotate_many(c, steps)
    for st, g in zip(steps, got):
        assert np.array_equal(E.export(g), E.export(E.rotate(c, None, st))), st


@pytest.mark.parametrize("layout", ["shared", "mixed", "lazy"])
def test_galois_multi_bit_exact(E, layout):
    """aesfhe_galois_multi: rotations by different steps and conjugations of
    different ciphertexts in one heterogeneous batched key switch equal the separate calls bit
    for bit -- one shared source (hoisted), several sources at two levels (more than one chunk),
    and deferred ct x pt products owing a rescale (stacked and rescaled together first; their
    conjugations stay deferred, as conjugate() does them).
    An item is (ct, steps) for a rotation, (ct, "conj") for a conjugation."""
    rng = np.random.default_rng({"shared": 1, "mixed": 2, "lazy": 3}[layout])
    cs = _cts(E, 4, 200 + len(layout))
    steps = [1, -8192, 16384, 3, -1, 24576, 5, 7, 2]
    if layout == "shared":
        items = [(cs[0], s) for s in steps[:6]] + [(cs[0], "conj"), (cs[0], 0)]
    elif layout == "mixed":
        low = E.multiply(cs[3], cs[2], "rlk")  # a second level group
        items = [(cs[i % 3], s) for i, s in enumerate(steps)] + [(cs[1], "conj"), (low, "conj"), (low, 4)]
    else:
        masks = [E.encode(np.where(rng.random(E.slot_count) < 0.5, 1.0, 0.0)) for _ in range(4)]
        parts = [E.multiply(cs[i % 2], masks[i]) for i in range(4)]  # deferred products (lazy)
        items = [(p, s) for p, s in zip(parts, [-4, -8, -12, 16384])] + [(parts[0], "conj")]
    gal = [(c, E.galois_conj if a == "conj" else E.galois_rotate(a)) for c, a in items]
    got = E.galois_multi(gal)
    # conjugations first: a deferred input is conjugated as it is (galois_lazy)
    # by both paths, while rotate() resolves its input's handle in place (canonical form)
    wants = {i: E.conjugate(c) for i, (c, a) in enumerate(items) if a == "conj"}
    wants.update({i: E.rotate(c, None, a) for i, (c, a) in enumerate(items) if a != "conj"})
    for i, r in enumerate(got):
        assert r.level == wants[i].level
        assert np.array_equal(E.export(r), E.export(wants[i])), items[i][1]


def test_conjugate_of_deferred_tensor(E):
    """conjugate() of a deferred LUT-like tensor (3 polynomials owing a rescale: a lazy product,
    and the same scaled by a non-integer constant owing two) is done without resolving it
    (engine.hip galois_lazy, keys sigma(s) -> s and sigma(s)^2 -> s summed before one ModDown):
    the slots equal conj of the resolved tensor's within CKKS noise, the owed work stays owed, and
    S1 + conj(S2) adds directly"""
    rng = np.random.default_rng(41)
    z = np.exp(2j * np.pi * rng.random(E.slot_count))
    w = np.exp(2j * np.pi * rng.random(E.slot_count))
    x, y = E.encrypt(z), E.encrypt(w)
    t = E.multiply(x, y, "rlk")          # deferred: 3 polynomials, one rescale owed
    t2 = E.multiply(t, 0.3 + 0.1j)       # deferred constant product: two rescales owed
    for c, want in ((t, z * w), (t2, (0.3 + 0.1j) * z * w)):
        got = E.conjugate(c)
        assert got.level == c.level
        err = np.abs(E.decrypt(got) - np.conj(want)).max()
        assert err < 1e-3, err
    s = E.add(t2, E.conjugate(t2))       # the split-LUT sum: 2 Re(...)
    assert np.abs(E.decrypt(s) - 2 * ((0.3 + 0.1j) * z * w).real).max() < 2e-3
