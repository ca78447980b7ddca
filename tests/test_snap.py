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


class _Eng:
    """engine stub: fresh level, stack / unstack of tagged members (lists), a slot count"""

    def __init__(self, fresh):
        self.fresh_level = fresh
        self.slot_count = 32768
        self.stacked = []

    def stack(self, cts):
        self.stacked.append(len(cts))
        return list(cts)

    def unstack(self, st):
        return list(st)


class _Ctx:
    def __init__(self, fresh, quad=True):
        self.engine = _Eng(fresh)
        self.bootstrap_pair_scaled = lambda *a, **k: None
        if quad:
            self.bootstrap_quad_scaled = lambda cts, gain, period: [("boot", c) for c in cts]
        self.to_intt = lambda c: c


def test_snap_count_rule():
    """BootstrapSnap: one snap everywhere with max_snaps=1 (the nibble SubBytes' rule, round 6); with 2, a
    second one where the consumer needs <= 8 levels (None / 0: an XOR4 follows) and the fresh level
    leaves snap + 5 + the need"""
    from zeta16_noise_reducer import BootstrapSnap
    one = BootstrapSnap(_Ctx(11), period=16, max_snaps=1)
    assert not any(one._twice(lv) for lv in (None, 0, 6, 7, 8, 13))
    from utils import NEED_XOR
    from zeta16_noise_reducer import DOUBLE_SNAP_MAX_LEVEL as M, SNAP15_DEPTH
    two = BootstrapSnap(_Ctx(17), period=16, max_snaps=2)
    for lv in (None, 0, M - 1, M, M + 1, 13):
        need = lv if lv else NEED_XOR
        assert two._twice(lv) == (need <= M and 17 - 2 * SNAP15_DEPTH - 1 >= need), lv
    assert two._twice(None) and two._twice(M) and not two._twice(M + 1)
    low = BootstrapSnap(_Ctx(NEED_XOR + 2 * SNAP15_DEPTH), period=16, max_snaps=2)  # one level short of two snaps + an XOR4
    assert not any(low._twice(lv) for lv in (None, 0, NEED_XOR, M))


def test_quad_renorm_stacks_four():
    """apply_quad: ONE quad bootstrap of the two pairs and ONE snap over a four-member stack; without
    the context's quad bootstrap (or a period) it falls back to two pair renorms"""
    import utils
    from zeta16_noise_reducer import BootstrapSnap
    ctx = _Ctx(11)
    bs = BootstrapSnap(ctx, period=16, max_snaps=1)
    assert bs.quad_ok()
    calls = []
    bs.snap.apply_scaled = lambda u: calls.append(u) or [("snap", m) for m in u]
    if utils.can_fork(ctx):
        return
    (a, b), (c, d) = bs.apply_quad(("h1", "l1"), ("h2", "l2"))
    assert (a, b, c, d) == tuple(("snap", ("boot", x)) for x in ("h1", "l1", "h2", "l2"))
    assert ctx.engine.stacked == [4] and len(calls) == 1
    assert not BootstrapSnap(_Ctx(11, quad=False), period=16).quad_ok()
    assert not BootstrapSnap(ctx, period=None).quad_ok()


def test_stacked_many_pairs_without_stack():
    """utils.stacked_many: one stacked call when the engine stacks, else pairwise (odd count: the last alone)"""
    import utils

    class _NoStack:
        engine = object()

    got = utils.stacked_many(_NoStack(), lambda x: x * 10 if isinstance(x, int) else x, [1, 2, 3])
    assert got == [10, 20, 30]
