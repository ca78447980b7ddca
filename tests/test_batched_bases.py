"""Host logic of the batched bases (xor4_lut.joint_bases, utils.mul_many / conj_many;
DESIGN.md §3.12) on a numpy slot context: the elements equal x^k / conj(x^(16-q)), every
product of one depth goes into one multiply_many call, the std input is conjugated once (its
mirrors are powers of conj(x), in the same product batches) -- or, with the mirror chain off,
every mirror conjugation goes into one conjugate_many call -- and a context without the batched
ops gets the same values."""
import numpy as np

from xor4_lut import _chain, _depth, joint_bases


class SlotCtx:
    """ciphertext = numpy slot vector; records the batched calls"""

    def __init__(self, batched: bool):
        self.calls = []
        if batched:
            self.multiply_many = self._mm
            self.conjugate_many = self._cm

    def multiply(self, a, b):
        return a * b

    def conjugate(self, a):
        self.calls.append(("conj", 1))
        return np.conj(a)

    def add_plain(self, a, v):
        return a + v

    def _mm(self, pairs):
        self.calls.append(("mul", len(pairs)))
        return [a * b for a, b in pairs]

    def _cm(self, cts):
        self.calls.append(("conj", len(cts)))
        return [np.conj(c) for c in cts]


def _check(ctx, a, b, need_a, need_b):
    A, B = joint_bases(ctx, [(a, need_a, "pow"), (b, need_b, "std")])
    for k in need_a:
        assert np.allclose(A[k], a ** k)
    for q in need_b:
        assert np.allclose(B[q], b ** q if q <= 8 else np.conj(b ** (16 - q)))


def test_joint_bases_values_and_batching():
    rng = np.random.default_rng(0)
    a = np.exp(2j * np.pi * rng.integers(0, 16, 64) / 16)
    b = np.exp(2j * np.pi * rng.integers(0, 16, 64) / 16)
    need_a, need_b = {0, 1, 2, 3, 4, 5, 7}, {0, 1, 3, 5, 9, 11, 13, 15}
    ctx = SlotCtx(batched=True)
    _check(ctx, a, b, need_a, need_b)
    muls = [n for kind, n in ctx.calls if kind == "mul"]
    depths = {_depth(k) for k, _, _ in _chain(need_a) + _chain({q if q <= 8 else 16 - q for q in need_b})}
    assert len(muls) == len(depths)  # one batch per depth, all chains together
    assert [(kind, n) for kind, n in ctx.calls if kind == "conj"] == [("conj", 1)]  # b itself, once
    assert ctx.calls[0] == ("conj", 1)  # before the products
    _check(SlotCtx(batched=False), a, b, need_a, need_b)


def test_joint_bases_mirror_conjugations(monkeypatch):
    """AESFHE_CONJ_CHAIN=0: the mirrors as conjugations of the powers, one conjugate_many"""
    import xor4_lut
    monkeypatch.setattr(xor4_lut, "_CONJ_CHAIN", False)
    rng = np.random.default_rng(1)
    a = np.exp(2j * np.pi * rng.integers(0, 16, 64) / 16)
    b = np.exp(2j * np.pi * rng.integers(0, 16, 64) / 16)
    ctx = SlotCtx(batched=True)
    _check(ctx, a, b, {1, 3, 5, 7}, {1, 3, 5, 7, 9, 11, 13, 15})
    assert [(kind, n) for kind, n in ctx.calls if kind == "conj"] == [("conj", 4)]
