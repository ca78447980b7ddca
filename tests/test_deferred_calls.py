"""The deferral algebra of deferred_calls.py on CPU: mi355x_ckks.Engine's own
public methods (multiply / add / subtract / add_plain / rotate / conjugate) bound to a stub engine
whose ciphertexts are numpy slot vectors and whose raw calls compute them exactly.  REF-shaped
call sequences (REF/xor4_lut.py:71-73, REF/sub_bytes_lut.py:66-71, REF/shift_rows.py:20-50) must
give the values of the same calls undeferred, through the expected fused / batched raw calls."""
import threading

import numpy as np
import pytest

import deferred_calls as D
import mi355x_ckks as M

N = 8


class FakeCt(M.Ciphertext):
    __slots__ = ("v", "lv")

    def __init__(self, v, lv=5):
        self._ctx = None
        self.handle = 1
        self.v = np.asarray(v, np.complex128)
        self.lv = lv

    @property
    def level(self):
        return self.lv


class FakePt(M.Plaintext):
    __slots__ = ("v",)

    def __init__(self, v):
        self._ctx = None
        self.handle = 1
        self.v = np.asarray(v, np.complex128)
        self.const = complex(self.v[0]) if (self.v == self.v[0]).all() else None


class Stub:
    slot_count = N
    galois_conj = 2 * 2 * N - 1

    def __init__(self, defer=True):
        self.defer = defer
        self._ctx = None
        self._tls = threading.local()
        self._defer_luts = {}
        self.log = []

    def galois_rotate(self, steps):
        return 1000 + steps % N

    @staticmethod
    def _val(x):
        return D.real(x).v

    def _apply_gal(self, v, g):
        return np.conj(v) if g == self.galois_conj else np.roll(v, g - 1000)

    # raw calls (the undeferred engine)
    def _raw_add(self, a, b):
        self.log.append("add")
        if isinstance(b, M.Ciphertext):
            return FakeCt(self._val(a) + self._val(b))
        if isinstance(b, M.Plaintext):
            return FakeCt(self._val(a) + b.v)
        return FakeCt(self._val(a) + complex(b))

    def _raw_sub(self, a, b):
        self.log.append("sub")
        return FakeCt(self._val(a) - self._val(b))

    def _raw_mul(self, a, b, relin=True):
        self.log.append("mul")
        gauss = not isinstance(b, M.Ciphertext) and D.constant_of(b) is not None and \
            D.constant_of(b).real.is_integer() and D.constant_of(b).imag.is_integer()
        if not gauss and min(x.level for x in (a, b) if isinstance(x, M.Ciphertext)) < 1:
            raise RuntimeError("not enough level")
        if isinstance(b, M.Ciphertext):
            return FakeCt(self._val(a) * self._val(b))
        if isinstance(b, M.Plaintext):
            return FakeCt(self._val(a) * b.v)
        return FakeCt(self._val(a) * complex(b))

    def multiply_many(self, pairs):
        self.log.append("mul_many")
        return [FakeCt(self._val(a) * self._val(b)) for a, b in pairs]

    def galois_multi(self, items):
        self.log.append(f"galois_multi{len(items)}")
        return [FakeCt(self._apply_gal(self._val(c), g)) for c, g in items]

    def lut_create(self, C, c0):
        return (np.array(C), complex(c0))

    def lut_eval(self, t, a, b=None):
        C, c0 = t
        self.log.append("lut2" if b is not None else "lut1")
        if b is not None:
            return FakeCt(sum(C[p, q] * a[p].v * b[q].v for p in range(len(a)) for q in range(len(b))))
        return FakeCt(c0 + sum(C[k] * a[k].v for k in range(len(a))))

    def encode(self, v):
        return FakePt(v)

    # the real Engine's deferral entry points and public methods, bound to the stub
    _raw = M.Engine._raw
    _raw_lut = M.Engine._raw_lut
    _gal_pending = M.Engine._gal_pending
    _flush_gal = M.Engine._flush_gal
    _settled = staticmethod(M.Engine._settled)
    _has_level = staticmethod(M.Engine._has_level)
    add = M.Engine.add
    subtract = M.Engine.subtract
    add_plain = M.Engine.add_plain
    multiply = M.Engine.multiply

    def rotate(self, ct, key=None, delta=0):
        if self.defer and delta % N:
            return D.GalPending(self, ct, self.galois_rotate(delta), lambda: self._one_gal(ct, self.galois_rotate(delta)))
        return self._one_gal(ct, self.galois_rotate(delta))

    def conjugate(self, ct, key=None):
        if self.defer:
            return D.GalPending(self, ct, self.galois_conj, lambda: self._one_gal(ct, self.galois_conj))
        return self._one_gal(ct, self.galois_conj)

    def _one_gal(self, ct, g):
        self.log.append("gal")
        return FakeCt(self._apply_gal(self._val(ct), g))


def _rand(rng):
    return FakeCt(np.exp(2j * np.pi * rng.random(N)))


def _xor4_like(E, A, B, C):
    """REF/xor4_lut.py:63-74: res = sub(A0, A0); res = add(res, multiply(multiply(A[p], B[q]), pt))"""
    res = E.subtract(A[0], A[0])
    for (p, q), c in C.items():
        pt = E.encode(np.full(N, c))
        res = E.add(res, E.multiply(E.multiply(A[p], B[q], "rlk"), pt))
    return res


@pytest.mark.parametrize("defer", [False, True])
def test_bivariate_loop_value_and_calls(defer):
    rng = np.random.default_rng(1)
    E = Stub(defer)
    A = [_rand(rng) for _ in range(16)]
    B = [_rand(rng) for _ in range(16)]
    C = {(p, q): complex(rng.normal(), rng.normal()) for p in range(16) for q in range(16) if rng.random() < 0.3}
    out = _xor4_like(E, A, B, C)
    want = sum(c * A[p].v * B[q].v for (p, q), c in C.items())
    np.testing.assert_allclose(D.real(out).v, want, atol=1e-9)
    if defer:
        assert E.log.count("lut2") == 1 and "mul" not in E.log  # one fused kernel, no per-term products
        assert E.log.count("add") <= 2  # the zero start and nothing else
    else:
        assert E.log.count("mul") == 2 * len(C)


def test_univariate_loop_with_constant():
    """REF/sub_bytes_lut.py:59-71: res = add_plain(multiply(ct, 0), c0); res = add(res, multiply(b_k, pt_k)),
    b_k partly conjugates (pending) -> one univariate LUT, all conjugates in one batched switch"""
    rng = np.random.default_rng(2)
    E = Stub(True)
    ct = _rand(rng)
    pos = [_rand(rng) for _ in range(8)]
    bk = {k: (pos[k - 1] if k <= 8 else E.conjugate(pos[16 - k - 1])) for k in range(1, 16)}
    cs = {k: complex(rng.normal(), rng.normal()) for k in range(1, 16)}
    res = E.add_plain(E.multiply(ct, 0.0), 0.5 - 0.25j)
    for k in range(1, 16):
        res = E.add(res, E.multiply(bk[k], E.encode(np.full(N, cs[k]))))
    want = 0.5 - 0.25j + sum(cs[k] * (pos[k - 1].v if k <= 8 else np.conj(pos[16 - k - 1].v)) for k in range(1, 16))
    np.testing.assert_allclose(D.real(res).v, want, atol=1e-9)
    assert E.log.count("lut1") == 1 and "galois_multi7" in E.log and "gal" not in E.log


def test_rotation_sum_batches():
    """REF/shift_rows.py:38-50: out = multiply(ct, 0); out = add(out, rotate(multiply(ct, mask), step))"""
    rng = np.random.default_rng(3)
    E = Stub(True)
    ct = _rand(rng)
    masks = [FakePt((rng.random(N) < 0.5).astype(float)) for _ in range(4)]
    out = E.multiply(ct, 0.0)
    for r, m in enumerate(masks):
        part = E.multiply(ct, m)  # a non-constant plaintext: issued at once
        out = E.add(out, E.rotate(part, None, -r) if r else part)
    want = sum(np.roll(ct.v * m.v, -r) for r, m in enumerate(masks))
    np.testing.assert_allclose(D.real(out).v, want, atol=1e-12)
    assert "galois_multi3" in E.log and "gal" not in E.log


def test_lone_ops_reissue_callers_calls():
    rng = np.random.default_rng(4)
    E = Stub(True)
    x, y = _rand(rng), _rand(rng)
    p = E.multiply(E.multiply(x, y, "rlk"), E.encode(np.full(N, 2.0)))
    np.testing.assert_allclose(D.real(p).v, 2 * x.v * y.v)
    assert E.log == ["mul", "mul"]  # product then the plaintext product, as called
    E.log.clear()
    z = E.add_plain(E.multiply(x, 0.0), 1.0)
    np.testing.assert_allclose(D.real(z).v, np.ones(N))
    assert E.log == ["mul", "add"]
    E.log.clear()
    r = E.rotate(x, None, 2)
    np.testing.assert_allclose(D.real(r).v, np.roll(x.v, 2))
    assert E.log == ["gal"]


def test_subtract_and_nested():
    rng = np.random.default_rng(5)
    E = Stub(True)
    a, b, c = _rand(rng), _rand(rng), _rand(rng)
    s = E.subtract(E.multiply(a, b, "rlk"), E.multiply(c, 3.0))
    t = E.multiply(s, c, "rlk")  # a deferred factor of a product
    u = E.subtract(E.conjugate(a), t)
    want_s = a.v * b.v - 3 * c.v
    np.testing.assert_allclose(D.real(u).v, np.conj(a.v) - want_s * c.v, atol=1e-9)
    np.testing.assert_allclose(D.real(s).v, want_s, atol=1e-12)


def test_deferred_is_a_ciphertext_and_level_forces():
    rng = np.random.default_rng(6)
    E = Stub(True)
    x, y = _rand(rng), _rand(rng)
    p = E.multiply(x, y, "rlk")
    assert isinstance(p, M.Ciphertext) and p._res is None
    assert p.handle == 1 and p._res is not None and p.bil is None  # resolved once, operands dropped


def test_resolved_operand_acts_as_its_result():
    """a deferred value used again after it was resolved (SubBytes' ct_b: a product resolved by its
    power basis, then multiplied by 0 for the accumulator) behaves as the plain ciphertext"""
    rng = np.random.default_rng(7)
    E = Stub(True)
    x, y = _rand(rng), _rand(rng)
    b = E.multiply(x, y, "rlk")
    D.real(b)  # resolved (e.g. by make_power_basis)
    z = E.add_plain(E.multiply(b, 0.0), 0.5)
    w = E.add(E.multiply(b, 2.0), z)
    s = E.subtract(w, b)
    np.testing.assert_allclose(D.real(s).v, x.v * y.v + 0.5, atol=1e-12)


def test_level_error_at_the_call():
    """a product of a level-0 ciphertext raises at the multiply call, as undeferred (REF's callers
    branch on the "level" message, REF/engine_context.py:184-195); Gaussian-integer constants need
    no level and stay deferred"""
    rng = np.random.default_rng(8)
    E = Stub(True)
    x = FakeCt(np.exp(2j * np.pi * rng.random(N)), lv=0)
    with pytest.raises(RuntimeError, match="level"):
        E.multiply(x, x, "rlk")
    with pytest.raises(RuntimeError, match="level"):
        E.multiply(x, 0.5)
    z = E.multiply(x, -1j)
    assert isinstance(z, D.TermSum)
    np.testing.assert_allclose(D.real(z).v, -1j * x.v)
