"""The low-level sparse bootstrap (include/aesfhe.h aesfhe_bootstrap_sparse_floor): when
the caller needs the result only at a low level (MixColumns' final bootstrap before an AddRoundKey
that is renormalised, REF/mixcol_final.py:158-162 + REF/pipeline.py:141-150), ModRaise, the trace
and CoeffToSlot run at the lowest double-prime level and EvalMod + SlotToCoeff on single-prime
levels.  The result must still be the bootstrapped message -- within a bound far inside the Zeta16
decode margin pi/16 -- at a level >= the requested floor, for single, monomial-pair and stacked
inputs, and a whole encrypt through it must give FIPS-197 AES bytes with a precision margin."""
import numpy as np
import pytest

from conftest import gpu_context

pytestmark = pytest.mark.gpu

LOW_TOL = 5e-3  # |slot error| of a unit-magnitude message (pi/16 = 0.196 is the decode margin)


@pytest.fixture(scope="module")
def E():
    return gpu_context(log_n=16, signature=1).engine


def _msg(E, n, rng):
    return np.tile(np.exp(2j * np.pi * rng.integers(0, 16, n) / 16), E.slot_count // n)


@pytest.mark.parametrize("n", [16, 32])
def test_low_single_bootstrap(E, n):
    rng = np.random.default_rng(500 + n)
    z = _msg(E, n, rng)
    ct = E.encrypt(z)
    hi = E.bootstrap_sparse(ct, n)
    lo = E.bootstrap_sparse(ct, n, min_level=7)
    e_hi = np.abs(E.decrypt(hi) - z).max()
    e_lo = np.abs(E.decrypt(lo) - z).max()
    print(f"n={n}: standard level {hi.level} err {e_hi:.2e}; low level {lo.level} err {e_lo:.2e}")
    assert e_hi < 1e-3
    assert e_lo < LOW_TOL
    assert 7 <= lo.level < hi.level


def test_low_pair_and_stack(E):
    rng = np.random.default_rng(77)
    zs = [_msg(E, 16, rng) for _ in range(6)]
    cts = [E.encrypt(z) for z in zs]
    h, l = E.bootstrap_pair_sparse(cts[0], cts[1], 16, min_level=7)
    assert np.abs(E.decrypt(h) - zs[0]).max() < LOW_TOL and np.abs(E.decrypt(l) - zs[1]).max() < LOW_TOL
    assert h.level >= 7
    H, L = E.bootstrap_pair_sparse(E.stack(cts[:3]), E.stack(cts[3:]), 16, min_level=7)
    for m, (a, b) in enumerate(zip(E.unstack(H), E.unstack(L))):
        assert np.abs(E.decrypt(a) - zs[m]).max() < LOW_TOL
        assert np.abs(E.decrypt(b) - zs[3 + m]).max() < LOW_TOL


def test_floor_above_the_low_form_keeps_the_standard_one(E):
    """a floor the low form cannot reach (above its output level) takes the standard bootstrap"""
    rng = np.random.default_rng(5)
    z = _msg(E, 32, rng)
    ct = E.encrypt(z)
    a = E.bootstrap_sparse(ct, 32, min_level=15)
    b = E.bootstrap_sparse(ct, 32)
    assert a.level == b.level
    assert np.array_equal(E.export(a), E.export(b))


def test_encrypt_through_low_bootstraps(coeff_dir):
    """C2 (periodic layout, renorm mode: the pipeline asks for the low form) and a 256-state batch:
    FIPS-197 bytes, and the measured slot error stays >= 4x inside pi/16 over every stage"""
    import bench
    from aes_keyschedule import expand_aes128_key, load_all_coeffs
    from oracle import aes_plain
    from pipeline import AESPipeline
    ctx = gpu_context(log_n=16, signature=1)
    rng = np.random.default_rng(9)
    rks = expand_aes128_key(rng.integers(0, 256, 16).astype(np.uint8))
    for states in (1, 256):
        pipe = AESPipeline(ctx, load_all_coeffs(coeff_dir), use_hard_renorm_between_steps=True, states=states)
        assert pipe._mc_floor is not None
        st = rng.integers(0, 256, (16,) if states == 1 else (states, 16)).astype(np.uint8)
        got = pipe.encoder.decode(*pipe.encrypt(st, rks))
        want = aes_plain.ref_encrypt(st, rks) if states == 1 else np.stack([aes_plain.ref_encrypt(s, rks) for s in st])
        assert np.array_equal(got, want)
        p = bench.measure_precision(pipe, ctx, rks, st, f"{states} states")
        print(states, p["margin_factor"], p["worst_stage"])
        assert p["margin_factor"] >= 4.0, p
