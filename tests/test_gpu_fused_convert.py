"""Level conversions with their exact-scale constant folded into the limb drop (engine.hip convert
-> drop_limbs(cc): the dropped limbs' INTT multiplies by the constant, the rescale finish multiplies
cur by it) against the separate multiply launch (AESFHE_FUSED_CONVERT=0): the same ciphertext
bytes for level drops across single- and double-prime levels, additions of operands at different
levels (and owing rescales), products aligned by mul_many, and a sparse bootstrap."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _run(E):
    rng = np.random.default_rng(31)
    zs = [np.exp(2j * np.pi * rng.random(E.slot_count)) for _ in range(4)]
    a, b, c, d = (E.encrypt(z) for z in zs)
    top = a.level
    out = [E.level_down(a, lv) for lv in range(top - 1, 0, -3)]
    ab = E.multiply(a, b, "rlk")                      # owes its rescale
    out.append(E.add(ab, E.level_down(c, top - 4)))  # operands at different levels
    out.append(E.add(E.level_down(d, 3), ab))
    out += E.multiply_many([(E.level_down(a, top - 2), b), (c, E.level_down(d, top - 5))])
    P = 32
    z = np.exp(2j * np.pi * rng.random(P))
    out.append(E.bootstrap_sparse(E.encrypt(np.tile(z, E.slot_count // P)), P))
    return [E.export(x).tobytes() for x in out]


def test_fused_convert_bit_identical(monkeypatch):
    from engine_context import EngineContext
    outs = []
    for flag in ("0", "1"):
        monkeypatch.setenv("AESFHE_FUSED_CONVERT", flag)
        E = EngineContext(signature=1, max_level=17, log_n=16, seed=0x5EED, enc_nonce=0).engine
        outs.append(_run(E))
        del E
    assert len(outs[0]) == len(outs[1])
    bad = [i for i, (x, y) in enumerate(zip(*outs)) if x != y]
    assert not bad, f"ciphertexts {bad} differ between the fused and the separate conversion constant"


def test_fused_convert_decrypts(monkeypatch):
    from mi355x_ckks import Engine
    monkeypatch.setenv("AESFHE_FUSED_CONVERT", "1")
    E = Engine(log_n=13, max_level=9, dnum=3, seed=0x5EED, allow_insecure=True, enc_nonce=2)
    rng = np.random.default_rng(3)
    z, w = (np.exp(2j * np.pi * rng.random(E.slot_count)) for _ in range(2))
    a, b = E.encrypt(z), E.encrypt(w)
    for lv in (7, 4, 1):
        assert np.abs(E.decrypt(E.level_down(a, lv)) - z).max() < 1e-3
    assert np.abs(E.decrypt(E.add(E.multiply(a, b, "rlk"), E.level_down(b, 3))) - (z * w + w)).max() < 1e-3
