"""The secret-key renorm of s1 + conj(s2) with the conjugation folded into its decryption
(aesfhe_renorm_packed_conj / aesfhe_renorm_unpack_conj, engine.hip renorm_states' conjugate
partner; utils.ConjSum): a conjugate-split LUT's output renormalised without its conjugation key
switch.  Neither input alone decodes to the state (each carries a garbage half that cancels only in
s1 + conj(s2)); the folded renorm must give the states of renorm(add(s1, conjugate(s2))), on the
packed (period 32) and unpacking forms, and inputs at different levels take the summed path."""
import numpy as np
import pytest

from conftest import gpu_context

pytestmark = pytest.mark.gpu

Z16 = np.exp(-2j * np.pi / 16)


@pytest.fixture(scope="module")
def ctx():
    return gpu_context(log_n=16, signature=1)


@pytest.fixture
def folds_on():
    """the renorm folds switched on for one test (utils.RenormFolds; the default is strict)"""
    from utils import renorm_folds
    with renorm_folds(True) as f:
        yield f


def _split(ctx, seed):
    """(s1, s2, nibbles): s1 + conj(s2) = 256 zeta16^nib (32-periodic, with < pi/32 jitter)"""
    E = ctx.engine
    S = E.slot_count
    rng = np.random.default_rng(seed)
    nib = rng.integers(0, 16, 32)
    z = 256.0 * Z16 ** nib * np.exp(1j * rng.uniform(-np.pi / 32, np.pi / 32, 32))
    d = 200.0 * (rng.standard_normal(32) + 1j * rng.standard_normal(32))
    tile = lambda v: np.tile(v, S // 32)
    s1 = ctx.encrypt(tile(0.5 * z + d))
    s2 = ctx.encrypt(tile(np.conj(0.5 * z - d)))
    return s1, s2, nib


def _close(ctx, a, b):
    za, zb = ctx.decrypt(a), ctx.decrypt(b)
    assert np.abs(za - zb).max() < 4e-4  # two fresh encryptions of the same codewords
    return za


@pytest.mark.parametrize("seed", [1, 2])
def test_packed_conj_renorm_matches_summed(ctx, seed):
    s1, s2, nib = _split(ctx, seed)
    got = ctx.renorm_single(s1, None, period=32, conj=s2)
    want = ctx.renorm_single(ctx.add(s1, ctx.conjugate(s2)), None, period=32)
    z = _close(ctx, got, want)
    assert np.abs(z[:32] - Z16 ** nib).max() < 2e-4
    # either input alone is not the state
    alone = ctx.decrypt(ctx.renorm_single(s1, None, period=32))
    assert np.abs(alone[:32] - Z16 ** nib).max() > 0.1


def test_unpack_conj_renorm_matches_summed(ctx):
    s1, s2, nib = _split(ctx, 3)
    gh, gl = ctx.renorm_unpack(s1, 16, None, conj=s2)
    wh, wl = ctx.renorm_unpack(ctx.add(s1, ctx.conjugate(s2)), 16, None)
    _close(ctx, gh, wh)
    _close(ctx, gl, wl)


def test_conj_partner_at_another_level_takes_the_summed_path(ctx):
    from utils import drop_to
    s1, s2, nib = _split(ctx, 4)
    s2d = drop_to(ctx, s2, s2.level - 2)
    got = ctx.renorm_single(s1, None, period=32, conj=s2d)
    want = ctx.renorm_single(ctx.add(s1, ctx.conjugate(s2d)), None, period=32)
    z = _close(ctx, got, want)
    assert np.abs(z[:32] - Z16 ** nib).max() < 2e-4


def test_pair_conj_renorm_matches_summed(ctx):
    """the periodic pair renorm (SubBytes' nibble LUT pair -> renorm): each channel's partner"""
    E = ctx.engine
    S = E.slot_count
    rng = np.random.default_rng(5)
    outs = []
    for _ in range(2):
        nib = rng.integers(0, 16, 16)
        z = 256.0 * Z16 ** nib
        d = 200.0 * (rng.standard_normal(16) + 1j * rng.standard_normal(16))
        outs.append((ctx.encrypt(np.tile(0.5 * z + d, S // 16)), ctx.encrypt(np.tile(np.conj(0.5 * z - d), S // 16)), nib))
    (h1, h2, nh), (l1, l2, nl_) = outs
    gh, gl = ctx.renorm_periodic(h1, l1, 16, None, conj=(h2, l2))
    wh, wl = ctx.renorm_periodic(ctx.add(h1, ctx.conjugate(h2)), ctx.add(l1, ctx.conjugate(l2)), 16, None)
    zh, zl = _close(ctx, gh, wh), _close(ctx, gl, wl)
    assert np.abs(zh[:16] - Z16 ** nh).max() < 2e-4 and np.abs(zl[:16] - Z16 ** nl_).max() < 2e-4


@pytest.mark.parametrize("with_conj", [False, True])
def test_packing_renorm_matches_pack_then_renorm(ctx, with_conj, folds_on):
    """aesfhe_renorm_pack: the period-16 pair renormalised straight into the packed period-32 form
    (no mask products) equals renorm_packed(pack(hi, lo)), with or without conjugate partners"""
    from state_encoder import StateEncoder
    enc = StateEncoder(ctx, periodic=True)
    assert enc.layout.period == 16 and enc.pack_renorm_direct()
    E = ctx.engine
    S = E.slot_count
    rng = np.random.default_rng(6 + with_conj)
    parts = []
    for _ in range(2):
        nib = rng.integers(0, 16, 16)
        z = 256.0 * Z16 ** nib
        d = 200.0 * (rng.standard_normal(16) + 1j * rng.standard_normal(16)) if with_conj else 0.0 * z
        parts.append((ctx.encrypt(np.tile(0.5 * z + d, S // 16)), ctx.encrypt(np.tile(np.conj(0.5 * z - d), S // 16)), nib))
    (h1, h2, nh), (l1, l2, nl_) = parts
    if with_conj:
        got = ctx.renorm_pack(h1, l1, 16, None, conj=(h2, l2))
        hi, lo = ctx.add(h1, ctx.conjugate(h2)), ctx.add(l1, ctx.conjugate(l2))
    else:
        hi, lo = ctx.add(h1, ctx.conjugate(h2)), ctx.add(l1, ctx.conjugate(l2))
        got = ctx.renorm_pack(hi, lo, 16, None)
    want = enc.renorm_packed(enc.pack(hi, lo), None)
    z = _close(ctx, got, want)
    assert np.abs(z[:16] - Z16 ** nh).max() < 2e-4 and np.abs(z[16:32] - Z16 ** nl_).max() < 2e-4


@pytest.mark.parametrize("with_conj", [False, True])
def test_shift_rows_folded_into_the_renorm(ctx, with_conj, folds_on):
    """aesfhe_renorm_periodic_perm with ShiftRows' byte permutation equals ShiftRows (masked
    rotations) after the renorm, per decoded slot, with or without conjugate partners"""
    from shift_rows import ShiftRows
    from state_encoder import StateEncoder
    enc = StateEncoder(ctx, periodic=True)
    sr = ShiftRows(ctx, layout=enc.layout)
    perm = sr.slot_perm()
    assert perm is not None and enc.renorm_perm_ok()
    E = ctx.engine
    S = E.slot_count
    rng = np.random.default_rng(9 + with_conj)
    parts = []
    for _ in range(2):
        nib = rng.integers(0, 16, 16)
        z = 256.0 * Z16 ** nib
        d = 200.0 * (rng.standard_normal(16) + 1j * rng.standard_normal(16)) if with_conj else 0.0 * z
        parts.append((ctx.encrypt(np.tile(0.5 * z + d, S // 16)), ctx.encrypt(np.tile(np.conj(0.5 * z - d), S // 16)), nib))
    (h1, h2, nh), (l1, l2, nl_) = parts
    hi, lo = ctx.add(h1, ctx.conjugate(h2)), ctx.add(l1, ctx.conjugate(l2))
    if with_conj:
        gh, gl = ctx.renorm_periodic_perm(h1, l1, 16, perm, None, conj=(h2, l2))
    else:
        gh, gl = ctx.renorm_periodic_perm(hi, lo, 16, perm, None)
    wh, wl = sr.apply(*ctx.renorm_periodic(hi, lo, 16, None))
    zh, zl = ctx.decrypt(gh), ctx.decrypt(gl)
    assert np.abs(zh - ctx.decrypt(wh)).max() < 5e-3 and np.abs(zl - ctx.decrypt(wl)).max() < 5e-3
    p = np.asarray(perm)
    assert np.abs(zh[:16] - (Z16 ** nh)[p]).max() < 2e-4 and np.abs(zl[:16] - (Z16 ** nl_)[p]).max() < 2e-4


def test_inv_shift_rows_folded_into_the_unpacking_renorm(ctx):
    """aesfhe_renorm_unpack_perm with InvShiftRows' permutation equals InvShiftRows (masked
    rotations) after renorm_unpack, per decoded slot of both halves"""
    from inv_shiftrows import InvShiftRows
    from state_encoder import StateEncoder
    enc = StateEncoder(ctx, periodic=True)
    isr = InvShiftRows(ctx, layout=enc.layout)
    perm = isr.slot_perm()
    assert perm is not None
    E = ctx.engine
    S = E.slot_count
    rng = np.random.default_rng(12)
    nib = rng.integers(0, 16, 32)
    packed = ctx.encrypt(np.tile(256.0 * Z16 ** nib, S // 32))
    gh, gl = ctx.renorm_unpack_perm(packed, 16, perm, None)
    wh, wl = isr.apply(*ctx.renorm_unpack(packed, 16, None))
    zh, zl = ctx.decrypt(gh), ctx.decrypt(gl)
    assert np.abs(zh - ctx.decrypt(wh)).max() < 5e-3 and np.abs(zl - ctx.decrypt(wl)).max() < 5e-3
    p = np.asarray(perm)
    assert np.abs(zh[:16] - (Z16 ** nib[:16])[p]).max() < 2e-4 and np.abs(zl[:16] - (Z16 ** nib[16:])[p]).max() < 2e-4


@pytest.mark.parametrize("seed", [21, 22])
def test_homomorphic_unpack_matches_the_unpacking_renorm(ctx, seed):
    """StateEncoder.renorm_unpack in the strict default (the packed renorm, then one rotation and a
    mask product) gives the (hi, lo) pair of the engine's gathering renorm (aesfhe_renorm_unpack, the
    fold), slot for slot, at the same level"""
    from state_encoder import StateEncoder
    from utils import FOLDS
    assert not FOLDS.unpack
    enc = StateEncoder(ctx, periodic=True)
    S = ctx.engine.slot_count
    rng = np.random.default_rng(seed)
    nib = rng.integers(0, 16, 32)
    packed = ctx.encrypt(np.tile(256.0 * Z16 ** nib * np.exp(1j * rng.uniform(-np.pi / 32, np.pi / 32, 32)), S // 32))
    hi, lo = enc.renorm_unpack(packed, level=7)
    wh, wl = ctx.renorm_unpack(packed, 16, 7)
    assert hi.level == wh.level == 7 and lo.level == wl.level == 7
    zh, zl = _close(ctx, hi, wh), _close(ctx, lo, wl)
    assert np.abs(zh - np.tile(Z16 ** nib[:16], S // 16)).max() < 2e-4
    assert np.abs(zl - np.tile(Z16 ** nib[16:], S // 16)).max() < 2e-4
