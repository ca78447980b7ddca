"""Double-hoisted giant steps through the multi-source fused key-switch core (engine.hip
giant_accumulate_many; on by default, AESFHE_FUSED_GIANT=0 restores the separate path): a linear-transform group's rotated
giant steps summed in one k_ntt2_ki launch must give the same ciphertext bytes as the separate
k_key_inner accumulation, on the full-slot bootstrap (the plans with multi-step groups) and the
sparse one.  The launch counts show whether the fused form ran."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _run(flag, monkeypatch):
    monkeypatch.setenv("AESFHE_FUSED_GIANT", flag)
    from engine_context import EngineContext
    from mi355x_ckks import launch_count
    E = EngineContext(signature=1, max_level=17, log_n=16, seed=0x5EED, enc_nonce=0).engine
    rng = np.random.default_rng(43)
    z = np.exp(2j * np.pi * rng.random(E.slot_count))
    P = 32
    zs = np.tile(np.exp(2j * np.pi * rng.random(P)), E.slot_count // P)
    a, b = E.encrypt(z), E.encrypt(zs)
    E.sync()
    n0 = launch_count()
    outs = [E.bootstrap(a), E.bootstrap_sparse(b, P)]
    E.sync()
    n = launch_count() - n0
    return [E.export(o).tobytes() for o in outs], n


def test_fused_giant_bit_identical(monkeypatch):
    ref, n0 = _run("0", monkeypatch)
    got, n1 = _run("1", monkeypatch)
    print(f"launches: separate {n0}, fused giant steps {n1}")
    assert ref == got
    assert n1 <= n0
