"""The sampling PRF: ChaCha20 with a 256-bit context key, one block per
sample.  The oracle's block function is pinned to the published test vector (RFC 8439 §2.3.2;
its 32-bit counter + 96-bit nonce map onto the original 64/64 layout used here as
counter = 1 | nonce_word0 << 32, nonce = nonce_word1 | nonce_word2 << 32); the engine's device
and host copies (csrc/common.h chacha_u64) are pinned to the oracle through the key parity
tests (tests/test_gpu_parity.py)."""
import numpy as np

from oracle.ckks_cpu import OracleParams, chacha_block

RFC8439_232 = ("e4e7f110 15593bd1 1fdd0f50 c47120a3 c7f4d1c7 0368c033 9aaa2204 4e6cd4c3 "
               "466482d2 09aa9f07 05d7c214 a2028bd9 d19c12b5 b94e16de e883d0cb 4e3c50a2")


def test_chacha20_block_rfc8439():
    key = np.frombuffer(bytes(range(32)), "<u4")
    n0 = int.from_bytes(bytes.fromhex("00000009"), "little")
    n1 = int.from_bytes(bytes.fromhex("0000004a"), "little")
    out = chacha_block(key, 1 | (n0 << 32), n1)
    assert " ".join(f"{x:08x}" for x in out) == RFC8439_232


def test_keyed_and_seeded_contexts():
    """an int seed is the key with words 0-1 set; a 32-byte key changes every sample"""
    seed = 0x1234_5678_9ABC_DEF0
    a = OracleParams(log_n=13, max_level=3, seed=seed)
    b = OracleParams(log_n=13, max_level=3, seed=seed.to_bytes(8, "little") + bytes(24))
    assert np.array_equal(a.secret(), b.secret())
    c = OracleParams(log_n=13, max_level=3, seed=bytes(range(32)))
    sc = c.secret()
    assert not np.array_equal(a.secret(), sc)
    # ternary secret: values in {-1, 0, 1}, each about a third of the coefficients
    counts = np.array([(sc == v).sum() for v in (-1, 0, 1)]) / sc.size
    assert set(np.unique(sc)) <= {-1, 0, 1} and np.abs(counts - 1 / 3).max() < 0.03
