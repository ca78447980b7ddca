"""snapper_1d_z16 on the MI355X engine (REF/snapper_1d_z16.py:17-99, the north_star-named snap).

- zeta16_snap_coeffs.json through Zeta16Snap1D / Zeta16SnapPair: codewords (and codewords with
  small noise) map onto the polynomial's value there, nibbles decode exactly, no bootstrap;
- the reference's bootstrap-on-RuntimeError retries (REF :39-52, :69-74) fire on an exhausted
  ciphertext and the result still decodes exactly;
- the fused LUT sum equals the reference's term loop (within CKKS rounding).
"""
import numpy as np
import pytest

from conftest import gpu_context

pytestmark = pytest.mark.gpu

SNAP_TOL = 5e-3  # CKKS error of x^1..x^8 (depth 3) + the 16-term sum at delta ~ 2^30, max over 2^15 slots


@pytest.fixture(scope="module")
def ctx():
    return gpu_context(log_n=16, signature=1)


def _eval(c, x):
    out = np.zeros_like(x)
    for k, ck in enumerate(c):
        kk = k % 16
        out = out + ck * (x ** kk if kk <= 8 else np.conj(x ** (16 - kk)))
    return out


def _nib(z):
    return np.round(-np.angle(z) * 16 / (2 * np.pi)).astype(int) % 16


@pytest.fixture(scope="module")
def coeffs(coeff_dir):
    from snapper_1d_z16 import load_coeff1d
    return load_coeff1d(coeff_dir / "zeta16_snap_coeffs.json")


def test_snap1d_codewords(ctx, coeffs):
    from snapper_1d_z16 import Zeta16Snap1D, Zeta16SnapPair
    E = ctx.engine
    rng = np.random.default_rng(61)
    k = rng.integers(0, 16, E.slot_count)
    z = np.exp(-2j * np.pi * k / 16)
    x = z * (1 + 0.01 * (rng.standard_normal(E.slot_count) + 1j * rng.standard_normal(E.slot_count)) / np.sqrt(2))
    snap = Zeta16Snap1D(ctx, coeffs)
    n0 = ctx.bootstrap_stats()["count"]
    a, b = Zeta16SnapPair(snap).apply_pair(ctx.encrypt(z), ctx.encrypt(x))
    assert ctx.bootstrap_stats()["count"] == n0 and snap.retries == 0  # enough levels: no retry
    ya, yb = ctx.decrypt(a), ctx.decrypt(b)
    assert np.abs(ya - _eval(coeffs, z)).max() < SNAP_TOL
    assert np.abs(yb - _eval(coeffs, x)).max() < SNAP_TOL
    assert np.array_equal(_nib(ya), k) and np.array_equal(_nib(yb), k)


def test_snap1d_fused_equals_term_loop(ctx, coeffs):
    """the fused univariate LUT (one kernel) against the reference's 16-term loop"""
    from snapper_1d_z16 import Zeta16Snap1D
    E = ctx.engine
    rng = np.random.default_rng(62)
    z = np.exp(-2j * np.pi * rng.integers(0, 16, E.slot_count) / 16)
    ct = ctx.encrypt(z)
    fused = Zeta16Snap1D(ctx, coeffs).apply(ct)
    loop = Zeta16Snap1D(ctx, coeffs)
    loop._sum_fused = lambda basis: None
    ref = loop.apply(ct)
    assert np.abs(ctx.decrypt(fused) - ctx.decrypt(ref)).max() < SNAP_TOL


def test_snap1d_retry_bootstraps_an_exhausted_ciphertext(ctx, coeffs):
    """level 0 input: make_power_basis(ct, 8) raises, the snap bootstraps (REF :41-43) and goes on"""
    from snapper_1d_z16 import Zeta16Snap1D
    from test_gpu_bootstrap import BOOT_TOL
    E = ctx.engine
    rng = np.random.default_rng(63)
    k = rng.integers(0, 16, E.slot_count)
    z = np.exp(-2j * np.pi * k / 16)
    low = ctx.encrypt(z)
    for _ in range(E.fresh_level):
        low = E.multiply(low, 0.999)
    assert low.level == 0
    with pytest.raises(RuntimeError, match="level"):
        ctx.make_power_basis(low, 8)
    snap = Zeta16Snap1D(ctx, coeffs)
    n0 = ctx.bootstrap_stats()["count"]
    y = snap.apply(low)
    assert snap.retries >= 1 and ctx.bootstrap_stats()["count"] >= n0 + 1
    zl = z * 0.999 ** E.fresh_level
    got = ctx.decrypt(y)
    assert np.abs(got - _eval(coeffs, zl)).max() < SNAP_TOL + 16 * BOOT_TOL
    assert np.array_equal(_nib(got), k)


def test_snap1d_bootstrap_before(ctx, coeffs):
    """bootstrap_before=True (REF :64-65): one bootstrap up front, no retry"""
    from snapper_1d_z16 import Zeta16Snap1D
    E = ctx.engine
    rng = np.random.default_rng(64)
    k = rng.integers(0, 16, E.slot_count)
    z = np.exp(-2j * np.pi * k / 16)
    snap = Zeta16Snap1D(ctx, coeffs, bootstrap_before=True)
    n0 = ctx.bootstrap_stats()["count"]
    y = snap.apply(ctx.encrypt(z))
    assert ctx.bootstrap_stats()["count"] == n0 + 1 and snap.retries == 0
    assert np.array_equal(_nib(ctx.decrypt(y)), k)
