"""Conjugations as reversed reads (engine.hip galois / galois_lazy, AESFHE_CONJ_REV)
against the permuted-copy form (k_automorph first, AESFHE_CONJ_REV=0): the same ciphertext bytes
for conjugate() and conjugate_many() of a canonical ciphertext, a relinearised product still owing
its rescale (2 polynomials, pend > 0) and a lazy 3-polynomial tensor (galois_lazy: the sigma(s) and
sigma(s)^2 key inner products summed before one ModDown) -- the form where the reversed ModUp,
own-digit and c0-addend reads all run."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("logn", [13, 16])
def test_conj_rev_bit_identical(logn, monkeypatch):
    from mi355x_ckks import Engine
    outs = []
    for flag in ("0", "1"):
        monkeypatch.setenv("AESFHE_CONJ_REV", flag)
        E = Engine(log_n=logn, max_level=6 if logn == 13 else 17, dnum=3, seed=0xC0DE, allow_insecure=True, enc_nonce=3)
        rng = np.random.default_rng(17)
        z = np.exp(2j * np.pi * rng.random(E.slot_count))
        w = np.exp(2j * np.pi * rng.random(E.slot_count))
        a, b = E.encrypt(z), E.encrypt(w)
        deferred = E.relinearize(E.multiply(a, b))  # 2 polynomials, rescale still owed (pend > 0)
        lazy = E.multiply(a, b, "rlk")              # the engine's deferred product: a lazy 3-polynomial tensor
        lazy2 = E.multiply(lazy, 0.3 + 0.1j)        # a deferred constant product owing two rescales
        cts = [a, deferred, lazy, lazy2]
        res = [E.export(E.conjugate(c)).tobytes() for c in cts]
        res += [E.export(c).tobytes() for c in E.conjugate_many(cts)]
        got = E.decrypt(E.conjugate(lazy))
        assert np.abs(got - np.conj(z * w)).max() < 1e-3
        outs.append(res)
        del E
    assert len(outs[0]) == 8
    for i, (x, y) in enumerate(zip(outs[0], outs[1])):
        assert x == y, f"ciphertext {i} differs between the permuted-copy and reversed-read conjugations"
