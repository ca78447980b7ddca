"""The secret-key renorm's re-encryption drawn from a pool of zero encryptions (aesfhe_renorm_pool,
engine.hip zero_enc / k_renorm_wtab / k_renorm_combine) against the per-renorm
encryption (pool size 0, the round-5 path): the same snapped message.

- the period-32 packed renorm, the unpacking renorm (two 16-periodic outputs) and the periodic pair
  renorm decode to the same slot values either way (two fresh encryptions of the same codewords: equal
  within the encryption noise), at the requested level, across a pool refill;
- the NTT table of the sparse message (the D-point transform broadcast over runs of N / D) is checked by
  the value it decrypts to: every slot is its snapped codeword;
- a full C2 encrypt + decrypt with the pool on is FIPS-197's bytes.
"""
import numpy as np
import pytest

from conftest import gpu_context

pytestmark = pytest.mark.gpu

Z16 = np.exp(-2j * np.pi / 16)


@pytest.fixture(scope="module")
def ctx():
    return gpu_context(log_n=16, signature=1)


@pytest.fixture
def pool(ctx):
    E = ctx.engine
    yield E
    E.renorm_pool(16)  # the default size, pools emptied


def _noisy(ctx, nib, period, seed):
    S = ctx.engine.slot_count
    rng = np.random.default_rng(seed)
    z = 256.0 * Z16 ** nib * np.exp(1j * rng.uniform(-np.pi / 40, np.pi / 40, nib.size))
    return ctx.encrypt(np.tile(z, S // period))


@pytest.mark.parametrize("size", [1, 3, 16])
def test_packed_renorm_pooled_matches_unpooled(ctx, pool, size):
    S = ctx.engine.slot_count
    nib = np.random.default_rng(size).integers(0, 16, 32)
    x = _noisy(ctx, nib, 32, 100 + size)
    want = np.tile(Z16 ** nib, S // 32)
    pool.renorm_pool(0)
    ref = ctx.decrypt(ctx.renorm_single(x, 7, period=32))
    pool.renorm_pool(size)
    for rep in range(4):  # size 1 and 3: several refills
        got = ctx.renorm_single(x, 7, period=32)
        assert got.level == 7
        z = ctx.decrypt(got)
        assert np.abs(z - want).max() < 2e-4, rep
        assert np.abs(z - ref).max() < 4e-4, rep


def test_unpack_and_pair_renorms_pooled(ctx, pool):
    S = ctx.engine.slot_count
    nib = np.random.default_rng(9).integers(0, 16, 32)
    pool.renorm_pool(2)
    hi, lo = ctx.renorm_unpack(_noisy(ctx, nib, 32, 9), 16, 9)
    assert hi.level == lo.level == 9
    assert np.abs(ctx.decrypt(hi) - np.tile(Z16 ** nib[:16], S // 16)).max() < 2e-4
    assert np.abs(ctx.decrypt(lo) - np.tile(Z16 ** nib[16:], S // 16)).max() < 2e-4
    nh, nl_ = nib[:16], nib[16:]
    gh, gl = ctx.renorm_periodic(_noisy(ctx, nh, 16, 10), _noisy(ctx, nl_, 16, 11), 16, 8)
    assert np.abs(ctx.decrypt(gh) - np.tile(Z16 ** nh, S // 16)).max() < 2e-4
    assert np.abs(ctx.decrypt(gl) - np.tile(Z16 ** nl_, S // 16)).max() < 2e-4
    pool.renorm_pool(0)
    wh, wl = ctx.renorm_periodic(_noisy(ctx, nh, 16, 10), _noisy(ctx, nl_, 16, 11), 16, 8)
    assert np.abs(ctx.decrypt(gh) - ctx.decrypt(wh)).max() < 4e-4


def test_c2_bytes_with_the_pool(ctx, coeff_dir, pool):
    from aes_keyschedule import expand_aes128_key, load_all_coeffs
    from oracle import aes_plain
    from pipeline import AESPipeline
    pool.renorm_pool(16)
    pipe = AESPipeline(ctx, load_all_coeffs(coeff_dir), use_hard_renorm_between_steps=True)
    rng = np.random.default_rng(77)
    rks = expand_aes128_key(rng.integers(0, 256, 16).astype(np.uint8))
    for _ in range(2):
        pt = rng.integers(0, 256, 16).astype(np.uint8)
        ct = pipe.encrypt(pt, rks)
        assert np.array_equal(pipe.encoder.decode(*ct), aes_plain.ref_encrypt(pt, rks))
        assert np.array_equal(pipe.encoder.decode(*pipe.decrypt(*ct, rks)), pt)
