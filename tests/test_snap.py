"""The Zeta16 snap polynomials of zeta16_noise_reducer.py on ideal slots (no GPU): fixed points
at every 16th root of unity, vanishing first derivatives (in x and conj x), the second-order
constants behind the GPU tests' 12 |e|^2 + 50 |e|^3 bound, and the kappa folding of Zeta16Snap15."""
import numpy as np

Z = np.exp(-2j * np.pi * np.arange(16) / 16)


def _snap15(x):
    return (30 * x - 15 * x * x * np.conj(x) + np.conj(x) ** 15) / 16


def _ref17(x):
    return (17 * x - x ** 17) / 16


def test_fixed_points_and_contraction():
    rng = np.random.default_rng(0)
    for f in (_snap15, _ref17):
        assert np.abs(f(Z) - Z).max() < 1e-12
        for eps in (1e-3, 1e-2, 3e-2, 7e-2):
            e = eps * np.exp(2j * np.pi * rng.random(4096))
            x = np.tile(Z, 256) * (1 + e)
            err = np.abs(f(x) - np.tile(Z, 256))
            ein = np.abs(x - np.tile(Z, 256))
            assert np.all(err <= 12 * ein ** 2 + 50 * ein ** 3 + 1e-12)


def test_kappa_folding_matches():
    """a1 u + a3 u^2 conj(u) + conj(u)^15 on u = kappa x equals the snap of x"""
    from zeta16_noise_reducer import KAPPA, Zeta16Snap15

    class _C:
        pass

    s = Zeta16Snap15(_C())
    assert abs(s.c15 - 1.0) < 1e-12 and abs(KAPPA ** 15 - 1 / 16) < 1e-15
    rng = np.random.default_rng(1)
    x = np.tile(Z, 64) * (1 + 0.01 * (rng.standard_normal(1024) + 1j * rng.standard_normal(1024)))
    u = KAPPA * x
    g = s.a1 * u + s.a3 * u * u * np.conj(u) + s.c15 * np.conj(u) ** 15
    assert np.abs(g - _snap15(x)).max() < 1e-12


def _snap1d_eval(c, x):
    """sum_k c_k B_k(x), B_k = x^k (k <= 8), conj(x^(16-k)) (k >= 9), k > 15 folded (REF/snapper_1d_z16.py:36-90)"""
    out = np.zeros_like(x)
    for k, ck in enumerate(c):
        kk = k % 16
        out = out + ck * (x ** kk if kk <= 8 else np.conj(x ** (16 - kk)))
    return out


def test_snapper_1d_coefficients_and_codewords(coeff_dir, ref_coeffs):
    """snapper_1d_z16.load_coeff1d on the generated zeta16_snap_coeffs.json equals the reference's
    file (tests/golden/ref_coeff.npz), and every codeword maps onto itself within 1e-2 (the fitted
    polynomial's own residual, REF/gen/make_zeta16_snap_coeffs.py) -- nibbles decode exactly"""
    from snapper_1d_z16 import load_coeff1d
    c = load_coeff1d(coeff_dir / "zeta16_snap_coeffs.json")
    ref = ref_coeffs["zeta16_snap_coeffs"]
    assert c.shape == ref.shape and np.abs(c - ref).max() < 1e-12
    y = _snap1d_eval(c, Z)
    assert np.abs(y - Z).max() < 1e-2
    nib = np.round(-np.angle(y) * 16 / (2 * np.pi)).astype(int) % 16
    assert np.array_equal(nib, np.arange(16))
