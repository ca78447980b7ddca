"""The column-domain basis extension (ntt.hip k_bx_cols): the INTT's column pass of
the sources, the base conversion and the targets' forward column pass in ONE launch, against the
three separate launches (AESFHE_BX_COLS=0).  Every ModUp / ModDown form that takes it must give
the same ciphertext bytes: relinearisation (ModUp of a tensor's c2 formed from its factors, plain
ModDown), relinearisation fused with its rescale (ModDown by P and the dropped limb), rotations,
conjugations (reversed ModUp input, reversed addend), batched products, a stack wider than one
key-switch chunk, hoisted rotations and a sparse bootstrap (trace, CoeffToSlot, EvalMod at
double-prime levels where the 13-source ModDown keeps the separate launches, SlotToCoeff)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _run(E):
    rng = np.random.default_rng(29)
    zs = [np.exp(2j * np.pi * rng.random(E.slot_count)) for _ in range(6)]
    a, b, c = (E.encrypt(z) for z in zs[:3])
    out = []
    prod = E.multiply(a, b, "rlk")
    out.append(E.relinearize(E.multiply(a, b)))
    out.append(E.add(prod, c))
    out += E.multiply_many([(a, b), (b, c), (a, c)])
    out.append(E.rotate(a, None, 3))
    out += E.rotate_many(a, [1, 2, 5]) if hasattr(E, "rotate_many") else []
    out.append(E.conjugate(a))
    out.append(E.conjugate(prod))
    out += E.conjugate_many([b, E.multiply(c, 0.5 + 0.25j)])
    st = E.stack([E.encrypt(z) for z in zs[:4] + zs[:4] + zs[:2]])
    out.append(E.multiply(st, st, "rlk"))
    out.append(E.conjugate(st))
    P = 32
    z = np.exp(2j * np.pi * rng.random(P))
    out.append(E.bootstrap_sparse(E.encrypt(np.tile(z, E.slot_count // P)), P))
    flat = []
    for x in out:
        flat += E.unstack(x) if E.members(x) > 1 else [x]
    return [E.export(x).tobytes() for x in flat]


def test_bx_cols_bit_identical(monkeypatch):
    from engine_context import EngineContext
    outs = []
    for flag in ("0", "1"):
        monkeypatch.setenv("AESFHE_BX_COLS", flag)
        E = EngineContext(signature=1, max_level=17, log_n=16, seed=0x5EED, enc_nonce=0).engine
        outs.append(_run(E))
        del E
    assert len(outs[0]) == len(outs[1])
    bad = [i for i, (x, y) in enumerate(zip(*outs)) if x != y]
    assert not bad, f"ciphertexts {bad} differ between k_bx_cols and the separate launches"


def test_bx_cols_decrypts(monkeypatch):
    """the fused path decrypts to the right slots: relin, relin + rescale, rotation, conjugation"""
    from mi355x_ckks import Engine
    monkeypatch.setenv("AESFHE_BX_COLS", "1")
    E = Engine(log_n=16, max_level=17, dnum=3, seed=0x5EED, allow_insecure=True, enc_nonce=1)
    rng = np.random.default_rng(5)
    z, w = (np.exp(2j * np.pi * rng.random(E.slot_count)) for _ in range(2))
    a, b = E.encrypt(z), E.encrypt(w)
    assert np.abs(E.decrypt(E.multiply(a, b, "rlk")) - z * w).max() < 1e-3
    assert np.abs(E.decrypt(E.relinearize(E.multiply(a, b))) - z * w).max() < 1e-3
    assert np.abs(E.decrypt(E.rotate(a, None, 5)) - np.roll(z, 5)).max() < 1e-3
    assert np.abs(E.decrypt(E.conjugate(a)) - np.conj(z)).max() < 1e-3
