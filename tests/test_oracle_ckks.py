"""CPU checks of the C oracle (oracle/ckks_oracle.c), the checker the GPU parity tests compare
the HIP engine with bit-exactly: its NTT is a negacyclic convolution, its CKKS primitives
decrypt to the right slots, and AddRoundKey (BASELINE config 1) runs on it end to end."""
import json

import numpy as np
import pytest

from conftest import GOLDEN

TOL = 1e-3  # slot error bound at N = 2^13, delta ~ 2^30


@pytest.fixture(scope="module")
def eng():
    from oracle.ckks_cpu import OracleEngine
    return OracleEngine(log_n=13, max_level=6, dnum=3, seed=11)


def negacyclic(a, b, q):
    """exact a * b mod (X^N + 1, q) with python integers (small N only)"""
    n = len(a)
    full = np.convolve(a.astype(object), b.astype(object))
    out = full[:n].copy()
    out[: n - 1] -= full[n:]
    return np.array([int(v) % q for v in out], np.uint64)


def test_oracle_ntt_is_negacyclic_convolution():
    from oracle.ckks_cpu import OracleParams
    p = OracleParams(log_n=13, max_level=2, dnum=1, seed=1)
    q = int(p.moduli[0])
    rng = np.random.default_rng(0)
    a = rng.integers(0, q, p.n).astype(np.uint32)
    b = rng.integers(0, 7, p.n).astype(np.uint32)
    A, B = p.ntt(a[None], [0]), p.ntt(b[None], [0])
    C = (A.astype(np.uint64) * B) % q
    assert np.array_equal(p.intt(C.astype(np.uint32), [0])[0].astype(np.uint64), negacyclic(a, b, q))
    assert np.array_equal(p.intt(A, [0])[0], a)


def test_oracle_prime_chain():
    from oracle.ckks_cpu import OracleParams
    p = OracleParams(log_n=16, max_level=17, dnum=3, seed=0)
    q = p.moduli.astype(np.uint64)
    assert np.all(q > 2 ** 29) and np.all(q < 2 ** 30)
    assert np.all(q % (2 * p.n) == 1)
    assert len(set(q.tolist())) == len(q)


def test_oracle_encrypt_decrypt(eng):
    rng = np.random.default_rng(1)
    z = np.exp(2j * np.pi * rng.random(eng.slot_count))
    assert np.abs(eng.decrypt(eng.encrypt(z)) - z).max() < TOL


def test_oracle_mul_rotate_conjugate(eng):
    rng = np.random.default_rng(2)
    z = np.exp(2j * np.pi * rng.random(eng.slot_count))
    w = np.exp(2j * np.pi * rng.random(eng.slot_count))
    cz, cw = eng.encrypt(z), eng.encrypt(w)
    assert np.abs(eng.decrypt(eng.multiply(cz, cw)) - z * w).max() < TOL
    for steps in (1, -512, 1024):
        assert np.abs(eng.decrypt(eng.rotate(cz, steps)) - np.roll(z, steps)).max() < TOL
    assert np.abs(eng.decrypt(eng.conjugate(cz)) - np.conj(z)).max() < TOL
    assert np.abs(eng.decrypt(eng.multiply_scalar(cz, 0.5 - 0.25j)) - (0.5 - 0.25j) * z).max() < TOL


def test_oracle_power_basis(eng):
    rng = np.random.default_rng(3)
    z = np.exp(2j * np.pi * rng.random(eng.slot_count))
    pw = eng.make_power_basis(eng.encrypt(z), 8)
    for k, c in enumerate(pw, 1):
        assert np.abs(eng.decrypt(c) - z ** k).max() < TOL


def test_config1_add_round_key_on_oracle(coeff_dir):
    """BASELINE config 1: one AddRoundKey (2 XOR4 LUTs) at N = 2^15 on the CPU oracle,
    inputs as REF/main.py:44-46 (tests/golden/stages.json "config1")."""
    from add_round_key import AddRoundKey
    from aes_keyschedule import load_all_coeffs
    from oracle.ckks_cpu import OracleContext
    from state_encoder import StateEncoder
    from xor4_lut import XOR4LUT
    c1 = json.loads((GOLDEN / "stages.json").read_text())["config1"]
    ctx = OracleContext(log_n=15, max_level=8, seed=5)
    enc = StateEncoder(ctx)
    ark = AddRoundKey(XOR4LUT(ctx, load_all_coeffs(coeff_dir)["xor4"]))
    out = ark(*enc.encode(np.array(c1["state"], np.uint8)), *enc.encode(np.array(c1["key"], np.uint8)))
    assert bytes(enc.decode(*out)) == bytes(c1["ark"])
