"""Shared pytest setup: import paths, the `gpu` marker, engine fixtures."""
import os
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
PKG = ROOT / "aes-implementation-fhe_amd"
for p in (str(ROOT), str(PKG)):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = ROOT / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP engine)")


@pytest.fixture(scope="session")
def ref_coeffs():
    """Reference coefficient fixture (tests/golden/ref_coeff.npz) as dense arrays."""
    z = np.load(GOLDEN / "ref_coeff.npz")
    out = {}
    for key in z.files:
        if not key.endswith("__val"):
            continue
        stem = key[: -len("__val")]
        idx, val = z[stem + "__idx"], z[key]
        if idx.shape[1] == 2:
            A = np.zeros((16, 16), np.complex128)
            for (p, q), v in zip(idx, val):
                A[p, q] = v
        else:
            A = np.zeros(int(idx[:, 0].max()) + 1, np.complex128)
            for (k,), v in zip(idx, val):
                A[k] = v
        out[stem] = A
    return out


@pytest.fixture(scope="session")
def coeff_dir():
    from lut import ensure_coeffs
    return ensure_coeffs()


_engines = {}


def gpu_engine(log_n=16, max_level=17, dnum=3, seed=0x5EED):
    """One engine per parameter set per session (key generation is the slow part)."""
    key = (log_n, max_level, dnum, seed)
    if key not in _engines:
        from mi355x_ckks import Engine
        # parity-test sets: the N = 2^13 one is far above the 128-bit bound (bit-exactness only)
        # the encryption nonce pinned too: a test's noise (and so its error margins) is the same
        # in every run instead of a fresh draw per process
        _engines[key] = Engine(log_n=log_n, max_level=max_level, dnum=dnum, seed=seed, allow_insecure=True, enc_nonce=seed)
    return _engines[key]


_contexts = {}


def gpu_context(log_n=16, signature=2, max_level=17, seed=0x5EED):
    key = (log_n, signature, max_level, seed)
    if key not in _contexts:
        from engine_context import EngineContext
        _contexts[key] = EngineContext(signature=signature, max_level=max_level, thread_count=4, log_n=log_n, seed=seed, enc_nonce=seed)
    return _contexts[key]
