"""The fused key-switch core (ntt.hip k_ntt2_ki, engine ki_core): the ModUp's forward
row pass, the key inner product and the ModDown INTT's row pass in ONE launch, against the three
separate launches (AESFHE_FUSED_KI=0).  Every key-switch form that takes the fused path must give
the same ciphertext bytes: relinearisation (keyswitch), relinearisation fused with its rescale
(gadget fold), products relinearised from their factors (tensor fold, batched members), rotations
(permuted copy + keyswitch), conjugations (reversed own-digit read) of canonical and deferred
ciphertexts (two summed sources), a stack wider than one key-switch chunk, and a bootstrap."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _run(E, sparse: bool):
    rng = np.random.default_rng(23)
    zs = [np.exp(2j * np.pi * rng.random(E.slot_count)) for _ in range(6)]
    a, b, c = (E.encrypt(z) for z in zs[:3])
    out = []
    prod = E.multiply(a, b, "rlk")                       # lazy product (deferred relinearisation)
    out.append(E.relinearize(E.multiply(a, b)))          # keyswitch (relin_raw)
    out.append(E.add(prod, c))                           # normalize: relin fused with its rescale
    out += E.multiply_many([(a, b), (b, c), (a, c)])     # tensor fold, 3 members
    out.append(E.rotate(a, None, 3))                     # permuted copy + keyswitch
    out.append(E.conjugate(a))                           # reversed own digit
    out.append(E.conjugate(prod))                        # deferred tensor: two summed sources
    out += E.conjugate_many([b, E.multiply(c, 0.5 + 0.25j)])
    st = E.stack([E.encrypt(z) for z in zs[:4] + zs[:4] + zs[:2]])  # 10 members: chunked key switches
    out.append(E.multiply(st, st, "rlk"))
    out.append(E.conjugate(st))
    if sparse:
        P = 32
        z = np.exp(2j * np.pi * rng.random(P))
        out.append(E.bootstrap_sparse(E.encrypt(np.tile(z, E.slot_count // P)), P))
    flat = []
    for x in out:
        flat += E.unstack(x) if E.members(x) > 1 else [x]
    return [E.export(x).tobytes() for x in flat]


@pytest.mark.parametrize("logn", [13, 16])
def test_fused_ki_bit_identical(logn, monkeypatch):
    from engine_context import EngineContext
    from mi355x_ckks import Engine
    outs = []
    for flag in ("0", "1"):
        monkeypatch.setenv("AESFHE_FUSED_KI", flag)
        if logn == 13:
            E = Engine(log_n=13, use_bootstrap=True, max_level=3, dnum=5, seed=11, allow_insecure=True, enc_nonce=0)
        else:
            E = EngineContext(signature=1, max_level=17, log_n=16, seed=0x5EED, enc_nonce=0).engine
        outs.append(_run(E, sparse=True))
        del E
    assert len(outs[0]) == len(outs[1])
    bad = [i for i, (x, y) in enumerate(zip(*outs)) if x != y]
    assert not bad, f"ciphertexts {bad} differ between the fused and the separate key-switch launches"


def test_fused_ki_decrypts(monkeypatch):
    """the fused path decrypts to the right slots: relin, rotation, conjugation"""
    from mi355x_ckks import Engine
    monkeypatch.setenv("AESFHE_FUSED_KI", "1")
    E = Engine(log_n=16, max_level=17, dnum=3, seed=0x5EED, allow_insecure=True, enc_nonce=1)
    rng = np.random.default_rng(5)
    z, w = (np.exp(2j * np.pi * rng.random(E.slot_count)) for _ in range(2))
    a, b = E.encrypt(z), E.encrypt(w)
    assert np.abs(E.decrypt(E.multiply(a, b, "rlk")) - z * w).max() < 1e-3
    assert np.abs(E.decrypt(E.rotate(a, None, 5)) - np.roll(z, 5)).max() < 1e-3
    assert np.abs(E.decrypt(E.conjugate(a)) - np.conj(z)).max() < 1e-3
