"""Host-side bootstrap plan (homomorphic DFT factorisation + EvalMod polynomial) against
the canonical embedding; no GPU needed (aesfhe_debug_bootplan)."""
import pytest


@pytest.mark.parametrize("log_n", [10, 13, 16])
def test_bootstrap_plan_factorisation(log_n):
    import build_ext
    import mi355x_ckks
    build_ext.build()
    err = mi355x_ckks.debug_bootplan(log_n)
    assert err[0] < 1e-10   # SlotToCoeff groups == canonical embedding
    assert err[1] < 1e-10   # CoeffToSlot groups == its inverse
    assert err[2] < 1e-9    # Chebyshev approximation of the EvalMod kernel


def test_bootstrap_depth():
    import mi355x_ckks
    assert mi355x_ckks.bootstrap_depth() == 15  # CtS 3 + EvalMod (Chebyshev PS 5 + 4 double angles) + StC 3


@pytest.mark.parametrize("n,pack", [(16, 1), (32, 1), (64, 1), (16, 2), (32, 2), (16, 0), (1024, 0)])
def test_sparse_plan_factorisation(n, pack):
    """the sparse (period-n, small-ring) plans: CoeffToSlot to the bit-reversed coefficient
    halves (pack 1: the 2n-periodic (2 Re | 2 Im) real form; pack 2: a pair's hi and lo in one
    4n-periodic vector), SlotToCoeff back"""
    import build_ext
    import mi355x_ckks
    build_ext.build()
    err = mi355x_ckks.debug_sparseplan(n, pack)
    assert err[0] < 1e-10 and err[1] < 1e-10, err
