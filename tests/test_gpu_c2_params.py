"""The bench's C2 parameter set (bench.py --fresh-level 7 --dnum 4): a bootstrappable set whose
fresh level is 7 -- the most levels any step of the strict pipeline needs between two renorms / bootstraps at the
renorm floor 1 (utils.RENORM_FLOOR) -- so the bootstrap's double-prime region sits 10 primes lower, with 4
key-switching digits.

- the set is under the 128-bit bound (log2 PQ <= 1772 at N = 2^16) and has the documented shape;
- C2 encrypt and decrypt through the default strict pipeline are FIPS-197's bytes (two states), and the
  precision margin of every logged stage stays wide;
- a stack of 16 one-state pairs (the C3 shape) and a 64-state slot-packed pair encrypt to FIPS-197's bytes;
- MixColumns' final bootstrap alone returns its input's slots at the fresh level 7.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx9():
    from engine_context import EngineContext
    return EngineContext(signature=1, boot_fresh_level=7, dnum=4, thread_count=4, seed=0xC2C2, enc_nonce=0xC2C2)


@pytest.fixture(scope="module")
def co(coeff_dir):
    from aes_keyschedule import load_all_coeffs
    return load_all_coeffs(coeff_dir)


def test_parameter_set(ctx9):
    E = ctx9.engine
    assert E.fresh_level == 7 and E.dnum == 4
    assert E.log_pq <= 1772.0
    assert E.level_limbs[7] == 9  # single-prime levels: level l has l + 2 limbs


def test_c2_encrypt_decrypt(ctx9, co):
    from aes_keyschedule import expand_aes128_key
    from oracle import aes_plain
    from pipeline import AESPipeline
    pipe = AESPipeline(ctx9, co, use_hard_renorm_between_steps=True)
    assert pipe.packed_xor and pipe.packed_dec
    rng = np.random.default_rng(99)
    rks = expand_aes128_key(rng.integers(0, 256, 16).astype(np.uint8))
    for _ in range(2):
        pt = rng.integers(0, 256, 16).astype(np.uint8)
        dbg = {}
        ct = pipe.encrypt(pt, rks, debug=dbg)
        assert np.array_equal(pipe.encoder.decode(*ct), aes_plain.ref_encrypt(pt, rks))
        assert np.array_equal(pipe.encoder.decode(*pipe.decrypt(*ct, rks)), pt)
        assert all(v["plain"] is not None for v in dbg.values())


def test_stacked_pairs_and_slot_packed_batch(ctx9, co):
    from aes_keyschedule import expand_aes128_key
    from oracle import aes_plain
    from pipeline import AESPipeline
    rng = np.random.default_rng(5)
    rks = expand_aes128_key(rng.integers(0, 256, 16).astype(np.uint8))
    pipe = AESPipeline(ctx9, co, use_hard_renorm_between_steps=True, pairs=16)
    pts = rng.integers(0, 256, (16, 16), dtype=np.uint8)
    got = pipe.encoder.decode(*pipe.encrypt(pts, rks))
    assert np.array_equal(got, np.stack([aes_plain.ref_encrypt(p, rks) for p in pts]))
    pipe64 = AESPipeline(ctx9, co, use_hard_renorm_between_steps=True, states=64)
    pts = rng.integers(0, 256, (64, 16), dtype=np.uint8)
    got = pipe64.encoder.decode(*pipe64.encrypt(pts, rks))
    assert np.array_equal(got, np.stack([aes_plain.ref_encrypt(p, rks) for p in pts]))


def test_sparse_bootstrap_at_fresh_level_7(ctx9):
    from test_gpu_bootstrap import BOOT_TOL
    E = ctx9.engine
    P = 32
    z = np.exp(2j * np.pi * np.random.default_rng(1).random(P))
    out = E.bootstrap_sparse(E.intt(ctx9.encrypt(np.tile(z, E.slot_count // P))), P)
    assert out.level == 7
    assert np.abs(ctx9.decrypt(out) - np.tile(z, E.slot_count // P)).max() < BOOT_TOL
