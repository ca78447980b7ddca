"""lut.LUTEvaluator (REF/lut.py:65-90, the reference's generic 1-D LUT over x^1..x^{d/2} plus
conjugate mirrors; unused by the reference's own AES path and by this pipeline, kept for the API
surface) evaluated on the CPU oracle context: a random map of the 16 Zeta16 codewords, decoded
exactly (the restated class works as the reference's would on a drop-in context)."""
import numpy as np

from lut import LUTEvaluator


def test_lut_evaluator_maps_codewords():
    from oracle.ckks_cpu import OracleContext
    ctx = OracleContext(log_n=13, max_level=6, seed=3)
    sc = ctx.engine.slot_count
    z16 = np.exp(2j * np.pi * np.arange(16) / 16)
    rng = np.random.default_rng(0)
    f = rng.integers(0, 16, 16)                     # codeword a -> codeword f[a]
    fv = z16[f]
    c = np.array([np.mean(fv * z16 ** (-k)) for k in range(16)])  # f(zeta^a) = sum_k c_k zeta^(a k)
    # {k: plaintext of a_k} (REF/lut.py:68)
    lut = LUTEvaluator(ctx, {k: ctx.encode(np.full(sc, c[k])) for k in range(16) if abs(c[k]) > 1e-12}, 16)
    a = rng.integers(0, 16, sc)
    out = ctx.decrypt(lut.apply(ctx.encrypt(z16[a])))
    got = np.rint(np.angle(out) * 16 / (2 * np.pi)).astype(int) % 16
    assert np.array_equal(got, f[a])
    assert np.abs(out - fv[a]).max() < 1e-2
