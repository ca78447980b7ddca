"""EngineContext.lut keys its cache by the caller's key AND a digest of the coefficients:
callers key by id(), which Python reuses once an object is collected, and a stale
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
