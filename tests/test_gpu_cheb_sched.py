"""EvalMod's Chebyshev series as a product schedule (engine.hip cheb_eval_sched; on by default,
AESFHE_CHEB_SCHED=0 restores the Paterson-Stockmeyer recursion cheb_eval_many): the products
T_m r of different recursion depths whose r are ready run as one batched multiply, with the
recursion's own leaves, products and sums, so the bootstrapped ciphertext bytes must be the same
on the full-slot bootstrap (re / im halves stacked) and the sparse one, in fewer launches."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _run(flag, monkeypatch):
    monkeypatch.setenv("AESFHE_CHEB_SCHED", flag)
    from engine_context import EngineContext
    from mi355x_ckks import launch_count
    E = EngineContext(signature=1, max_level=17, log_n=16, seed=0x5EED, enc_nonce=0).engine
    rng = np.random.default_rng(47)
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


def test_cheb_schedule_bit_identical(monkeypatch):
    ref, n0 = _run("0", monkeypatch)
    got, n1 = _run("1", monkeypatch)
    print(f"launches: recursion {n0}, schedule {n1}")
    assert ref == got
    assert n1 < n0
