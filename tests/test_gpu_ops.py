"""Slot-level accuracy of every EngineContext primitive on the MI355X engine (numpy
reference of the same op; tolerances in the asserts)."""
import numpy as np
import pytest

from conftest import gpu_engine

pytestmark = pytest.mark.gpu

TOL = 1e-3  # absolute slot error on unit-magnitude inputs at delta ~ 2^30.3


@pytest.fixture(scope="module")
def E():
    return gpu_engine(log_n=16, max_level=17)


@pytest.fixture(scope="module")
def zz(E):
    rng = np.random.default_rng(11)
    z = np.exp(2j * np.pi * rng.random(E.slot_count))
    w = np.exp(2j * np.pi * rng.random(E.slot_count))
    return z, w, E.encrypt(z), E.encrypt(w)


def err(E, ct, ref):
    return np.abs(E.decrypt(ct) - ref).max()


def test_add_sub(E, zz):
    z, w, cz, cw = zz
    assert err(E, E.add(cz, cw), z + w) < TOL
    assert err(E, E.subtract(cz, cw), z - w) < TOL


def test_scalar_and_plain(E, zz):
    z, w, cz, cw = zz
    assert err(E, E.multiply(cz, 0.25 - 0.5j), (0.25 - 0.5j) * z) < TOL
    assert err(E, E.multiply(cz, 3.0), 3 * z) < TOL
    assert err(E, E.add_plain(cz, 0.3), z + 0.3) < TOL
    assert err(E, E.add(cz, 1 + 2j), z + 1 + 2j) < TOL
    mask = (np.arange(E.slot_count) % 7 == 0).astype(float)
    assert err(E, E.multiply(cz, E.encode(mask)), z * mask) < TOL
    assert err(E, E.add(cz, E.encode(w)), z + w) < TOL


def test_mul_rot_conj(E, zz):
    z, w, cz, cw = zz
    p = E.multiply(cz, cw, "rlk")
    assert p.level == E.L - 1
    assert err(E, p, z * w) < TOL
    for steps in (1, -8192, 8192, 16384, 24576):
        assert err(E, E.rotate(cz, None, steps), np.roll(z, steps)) < TOL
    assert err(E, E.conjugate(cz), np.conj(z)) < TOL


def test_power_basis_and_levels(E, zz):
    z = zz[0]
    pb = E.make_power_basis(zz[2], 8)
    assert [c.level for c in pb] == [E.L - int(np.ceil(np.log2(k))) if k > 1 else E.L for k in range(1, 9)]
    for k, c in enumerate(pb, 1):
        assert err(E, c, z ** k) < TOL
    # mixed-level add aligns scales exactly
    assert err(E, E.add(pb[0], pb[7]), z + z ** 8) < 2 * TOL  # both operands' errors add


def test_level_exhaustion_message(E, zz):
    ct = zz[2]
    while ct.level > 0:
        ct = E.multiply(ct, 0.5)
    with pytest.raises(RuntimeError, match="level"):
        E.multiply(ct, ct, "rlk")
    with pytest.raises(RuntimeError, match="level"):
        E.make_power_basis(ct, 8)


def test_relinearize_degree1_message(E, zz):
    with pytest.raises(RuntimeError, match="should have 3 polynomials"):
        E.relinearize(zz[2])
    d2 = E.multiply(zz[2], zz[3])
    assert d2.num_polys == 3
    assert err(E, E.relinearize(d2), zz[0] * zz[1]) < TOL


def test_ntt_roundtrip_representation(E, zz):
    z = zz[0]
    c = E.intt(zz[2])
    assert err(E, c, z) < TOL
    assert err(E, E.multiply(c, 2.0), 2 * z) < TOL
    assert err(E, E.ntt(c), z) < TOL
