"""EngineContext.lut keys its cache by a digest of the coefficient content only: callers
label sets with id(), which Python reuses once an object is collected, and a stale
coefficient set was the cause of an intermittent all-states-wrong packed run (DESIGN_HISTORY.md §B).
CPU-only: the engine is replaced by a recorder."""
import gc

import numpy as np

from engine_context import EngineContext


class _Rec:
    def __init__(self):
        self.made = []
        self.freed = []

    def lut_create(self, coeffs, c0):
        self.made.append((np.array(coeffs), c0))
        return len(self.made)

    def lut_free(self, t):
        self.freed.append(t)


def _ctx():
    ctx = object.__new__(EngineContext)
    ctx.engine = _Rec()
    ctx._init_lut_cache()
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


class _Owner:  # a SubBytes / XOR4 module stand-in
    pass


def test_sets_are_evicted_when_their_owners_die():
    """weakref.finalize on the owning module: a set is released (aesfhe_lut_free) once every
    owner holding it is gone; a set still held by a live owner, or requested without an owner,
    stays"""
    ctx = _ctx()
    a = np.arange(16, dtype=np.complex128)
    b = a[::-1].copy()
    c = a * 2
    o1, o2 = _Owner(), _Owner()
    ta = ctx.lut("sb", a, owner=o1)
    assert ctx.lut("sb", a, owner=o2) == ta  # shared by two owners
    tb = ctx.lut("sb", b, owner=o1)
    tc = ctx.lut("gf", c)  # pinned
    assert ctx.lut("gf", c, owner=o1) == tc
    assert ctx.lut_cache_size() == 3
    del o1
    gc.collect()
    assert ctx.engine.freed == [tb]  # a is still held by o2, c is pinned
    assert ctx.lut_cache_size() == 2
    del o2
    gc.collect()
    assert sorted(ctx.engine.freed) == sorted([tb, ta]) and ctx.lut_cache_size() == 1
    # a new owner of an evicted set gets a fresh device copy
    o3 = _Owner()
    assert ctx.lut("sb", a, owner=o3) not in (ta, tb, tc)
    assert len(ctx.engine.made) == 4


def test_many_module_generations_stay_bounded():
    """the leak the cache had: every new SubBytes object added a set that lived forever"""
    ctx = _ctx()
    rng = np.random.default_rng(0)
    for _ in range(50):
        o = _Owner()
        ctx.lut("sb", rng.standard_normal(8).astype(np.complex128), owner=o)
        del o
        gc.collect()
    assert ctx.lut_cache_size() == 0 and len(ctx.engine.freed) == 50


def test_clear_with_live_owners_never_frees_a_newer_set():
    """owner A holds digest d; clear_luts(); owner B requests d and gets a
    new set t'.  A's stale record must not release t' when A dies -- B still evaluates with it."""
    ctx = _ctx()
    a = np.arange(16, dtype=np.complex128)
    oa, ob = _Owner(), _Owner()
    t = ctx.lut("sb", a, owner=oa)
    ctx.clear_luts()
    t2 = ctx.lut("sb", a, owner=ob)
    assert t2 != t and ctx.lut_cache_size() == 1
    assert ctx.lut("sb", a, owner=oa) == t2  # A asks again after the clear: shares t'
    del oa
    gc.collect()
    assert t2 not in ctx.engine.freed and ctx.lut_cache_size() == 1  # B still holds t'
    del ob
    gc.collect()
    assert t2 in ctx.engine.freed and ctx.lut_cache_size() == 0


def test_clear_then_old_owner_dies_first():
    """the same with A not asking again: its death after the clear is a no-op"""
    ctx = _ctx()
    a = np.arange(16, dtype=np.complex128)
    oa, ob = _Owner(), _Owner()
    ctx.lut("sb", a, owner=oa)
    ctx.clear_luts()
    t2 = ctx.lut("sb", a, owner=ob)
    del oa
    gc.collect()
    assert ctx.engine.freed == [] and ctx.lut_cache_size() == 1
    del ob
    gc.collect()
    assert ctx.engine.freed == [t2]
