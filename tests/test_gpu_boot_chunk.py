"""Stacked bootstraps in chunks (engine.hip boot_stack, AESFHE_BOOT_CHUNK): a stack's members are
bootstrapped chunk by chunk, each chunk one batched bootstrap.  Every member's bootstrap is its own
computation, so the chunk size must not change a single output byte: a 6-member stack of sparse
(period 32) ciphertexts bootstrapped in chunks of 2, 3 and 4 (the last chunk partial) against
members bootstrapped one at a time, and the results decrypt to the inputs."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _boot(chunk, monkeypatch):
    from engine_context import EngineContext
    monkeypatch.setenv("AESFHE_BOOT_CHUNK", str(chunk))
    E = EngineContext(signature=1, max_level=17, log_n=16, seed=0x5EED, enc_nonce=0).engine
    rng = np.random.default_rng(41)
    P = 32
    zs = [np.tile(np.exp(2j * np.pi * rng.random(P)), E.slot_count // P) for _ in range(6)]
    st = E.stack([E.encrypt(z) for z in zs])
    out = E.unstack(E.bootstrap_sparse(st, P))
    got = [E.decrypt(o) for o in out]
    return [E.export(o).tobytes() for o in out], got, zs


def test_boot_chunk_bit_identical(monkeypatch):
    ref, got, zs = _boot(1, monkeypatch)
    for g, z in zip(got, zs):
        assert np.abs(g - z).max() < 1e-2
    for chunk in (2, 3, 4):
        out, _, _ = _boot(chunk, monkeypatch)
        bad = [i for i, (x, y) in enumerate(zip(ref, out)) if x != y]
        assert not bad, f"chunk {chunk}: members {bad} differ from the one-at-a-time bootstrap"
