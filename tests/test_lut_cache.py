"""EngineContext.lut keys its cache by a digest of the coefficient content only: callers
label sets with id(), which Python reuses once an object is collected, and a stale
coefficient set was the cause of an intermittent all-states-wrong packed run.
CPU-only: the engine is replaced by a recorder."""
import threading

import numpy as np

from engine_context import EngineContext


class _Rec:
    def __init__(self):
        self.made = []

    def lut_create(self, coeffs, c0):
        self.made.append((np.array(coeffs), c0))
        return len(self.made)


def _ctx():
    ctx = object.__new__(EngineContext)
    ctx.engine = _Rec()
    ctx._luts = {}
    ctx._lut_lock = threading.Lock()
    return ctx


def test_same_key_different_coefficients_get_different_luts():
    ctx = _ctx()
    a = np.arange(16, dtype=np.complex128)
    b = a[::-1].copy()
    key = ("sb", 12345)  # an id() that a new object may inherit
    t1 = ctx.lut(key, a)
    assert ctx.lut(key, a.copy()) == t1  # same content: cached
    t2 = ctx.lut(key, b)
    assert t2 != t1 and len(ctx.engine.made) == 2
    assert ctx.lut(key, a, c0=1j) not in (t1, t2)  # the constant term is part of the set


def test_cache_is_bounded_by_content():
    """Many short-lived owners of the same coefficient set share one device LUT (no growth)."""
    ctx = _ctx()
    a = np.arange(16, dtype=np.complex128)
    handles = {ctx.lut(("xor4", i), a) for i in range(100)}
    assert len(handles) == 1 and len(ctx._luts) == 1 and len(ctx.engine.made) == 1
    ctx.clear_luts()
    assert not ctx._luts
