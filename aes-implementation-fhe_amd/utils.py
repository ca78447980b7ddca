"""Zeta16 nibble codec (REF/utils.py:4-19).

A nibble v is carried as the 16th root of unity ζ^v, ζ = e^{-2πi/16}; decoding reads
only the phase, so any positive real magnitude (e.g. XOR4's 256×)
decodes to the same nibble.
"""
import numpy as np


class ZetaEncoder:
    @staticmethod
    def to_zeta(arr: np.ndarray, modulus: int) -> np.ndarray:
        k = np.asarray(arr) % modulus
        return np.exp(-2j * np.pi * k / modulus)

    @staticmethod
    def from_zeta(z_arr: np.ndarray, modulus: int) -> np.ndarray:
        turns = -np.angle(z_arr) * modulus / (2 * np.pi)
        return np.mod(np.rint(turns), modulus).astype(np.uint8)


def pair(ctx, fa, fb, shared=()):
    """(fa(), fb()) -- the hi / lo halves of an AES step, run concurrently on two HIP streams
    when the context supports it (EngineContext.run_parallel); `shared` ciphertexts read by
    both halves are settled first.  Results are identical to the sequential order."""
    run = getattr(ctx, "run_parallel", None)
    if run is None:
        return fa(), fb()
    if shared:
        ctx.engine.settle(*shared)
    a, b = run(fa, fb)
    return a, b


def fused_lut(ctx, key, coeffs, a, b=None, c0: complex = 0j):
    """The LUT sum sum_{p,q} C[p,q] a[p] b[q] (b given) or c0 + sum_k C[k] a[k] as one engine
    call, or None when the context has no fused form or the elements sit too
    low for it -- the caller then runs the reference's per-term product loop."""
    if not getattr(ctx, "fused_luts", False):
        return None
    try:
        return ctx.lut_eval(ctx.lut(key, coeffs, c0), a, b)
    except RuntimeError as e:
        if "level" in str(e):
            return None
        raise
