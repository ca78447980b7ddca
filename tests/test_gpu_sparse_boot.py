"""Stage-level parity of the sparse-slot bootstrap -- the bootstrap the C2 headline
runs once per round in place of REF's engine.bootstrap calls (REF/mixcol_final.py:158-162,
REF/invmixcolumns_fhe.py:166-168) -- against host models, on the N = 2^13 bootstrappable parity
set and the N = 2^16 production set, periods 16 and 32:

- the radix-4 hoisted trace to the subring (x + rot(x, a) + rot(x, 2a) + rot(x, 3a) per two
  doublings) equals the periodisation of its input: out[j] = sum_k in[(j + k n) mod M];
- every small-ring CoeffToSlot / SlotToCoeff group of the plan (diagonals one period long, tiled)
  equals the plan applied on the host to one period of its input (bootstrap.cpp
  apply_group_plain), the packed real form (1 | -i) folded into CoeffToSlot's last group and the
  half recombination into SlotToCoeff's first included;
- the packed real form w' + conj(w') (stage 9) equals w' + conj(w') of the decrypted stage 5;
- the monomial pair packing z = a + X^k b (k = N / 4n) is exact at the limb level (coefficient
  domain: b shifted negacyclically by k, added to a), and its split (m + rot_n(m),
  X^-k (m - rot_n(m))) equals the same map on the decrypted slots.

Every check is <= 1e-9 relative (slot level, on double-prime levels where the noise is ~2^-50 of
the scale) or bit-exact (integer steps).  Stages come from aesfhe_debug_boot_stage_sparse (12 =
before the trace, 4 = after it, 5 = CoeffToSlot, 9 = packed real form)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REL = 1e-9


def _rel(got, want):
    return np.abs(got - want).max() / max(np.abs(want).max(), 1e-300)


@pytest.fixture(scope="module", params=[13, 16], ids=["logn13", "logn16"])
def E(request):
    from mi355x_ckks import Engine
    if request.param == 13:  # the parity set of test_gpu_boot_parity.py (far above the 128-bit bound)
        return Engine(log_n=13, use_bootstrap=True, max_level=3, dnum=5, seed=7, allow_insecure=True)
    from conftest import gpu_context
    return gpu_context(log_n=16, signature=1).engine


def _periodic(E, n, rng, amp=0.5):
    block = amp * (rng.uniform(-1, 1, n) + 1j * rng.uniform(-1, 1, n))
    return np.tile(block, E.slot_count // n)


@pytest.mark.parametrize("n", [16, 32])
def test_trace_is_the_subring_projection(E, n):
    rng = np.random.default_rng(100 + n)
    ct = E.encrypt(_periodic(E, n, rng))
    before = E.decrypt(E.debug_boot_stage_sparse(ct, 12, n))
    after = E.decrypt(E.debug_boot_stage_sparse(ct, 4, n))
    M = E.slot_count
    want = before.reshape(M // n, n).sum(axis=0)  # out[j] = sum_k in[j + k n]
    want = np.tile(want, M // n)
    err = _rel(after, want)
    print(f"N=2^{E.log_n} n={n}: trace relative error {err:.2e}, |in| {np.abs(before).max():.3g}")
    assert err < REL
    # the overflow's components outside the subring are gone: the result is n-periodic
    assert _rel(after, np.tile(after[:n], M // n)) < REL


@pytest.mark.parametrize("n", [16, 32])
def test_sparse_groups_match_plan(E, n):
    """CoeffToSlot on the bootstrap's own post-trace ciphertext (stage 4), SlotToCoeff on the
    packed real form (stage 9) and then on each previous group's output -- each group against the
    plan applied on the host to one period of its decrypted input"""
    rng = np.random.default_rng(200 + n)
    ct = E.encrypt(_periodic(E, n, rng))
    _, _, n_cts, n_all = E.debug_sparse_group_plain(n, 0, np.zeros(E.slot_count))
    assert n_cts >= 1 and n_all > n_cts
    x = E.debug_boot_stage_sparse(ct, 4, n)
    for w in range(n_all):
        if w == n_cts:
            x = E.debug_boot_stage_sparse(ct, 9, n)  # SlotToCoeff reads the packed real form
        z = E.decrypt(x)
        want, dn, _, _ = E.debug_sparse_group_plain(n, w, z)
        assert _rel(z, np.tile(z[:dn], E.slot_count // dn)) < REL  # the input is dn-periodic
        y = E.debug_sparse_group(x, n, w)
        err = _rel(E.decrypt(y), want)
        print(f"N=2^{E.log_n} n={n} group {w}: period {dn}, level {x.level}, relative error {err:.2e}")
        assert err < REL
        x = y


@pytest.mark.parametrize("n", [16, 32])
def test_packed_real_form(E, n):
    """stage 9 = w' + conj(w') of CoeffToSlot's output w' (stage 5): real, and equal slot-wise"""
    rng = np.random.default_rng(300 + n)
    ct = E.encrypt(_periodic(E, n, rng))
    w = E.decrypt(E.debug_boot_stage_sparse(ct, 5, n))
    v = E.decrypt(E.debug_boot_stage_sparse(ct, 9, n))
    assert _rel(v, w + np.conj(w)) < REL
    assert np.abs(v.imag).max() < REL * np.abs(v).max()


def _negacyclic_shift(x, k, q):
    """coefficients of X^k * x(X) mod (X^N + 1, q), x: [..., N] uint32 residues"""
    y = np.roll(x.astype(np.int64), k, axis=-1)
    y[..., :k] = (q - y[..., :k]) % q
    return y


@pytest.mark.parametrize("n", [16, 32])
def test_mono_pack_is_exact(E, n):
    """z = a + X^k b at level 0, k = N / 4n: bit-exact in the coefficient domain"""
    if E.log_n != 13:
        pytest.skip("limb-level oracle check on the N = 2^13 set")
    from oracle.ckks_cpu import OracleParams
    L1 = max(l for l in range(E.L + 1) if E.level_limbs[l] == l + 2)  # as test_gpu_boot_parity.py
    O = OracleParams(log_n=13, max_level=L1, dnum=E.dnum, seed=7, boot_double=E.L - L1)
    assert np.array_equal(O.moduli, E.moduli())
    rng = np.random.default_rng(400 + n)
    a, b = E.encrypt(_periodic(E, n, rng)), E.encrypt(_periodic(E, n, rng))
    a0, b0 = E.level_down(a, 0), E.level_down(b, 0)
    z = E.export(E.debug_mono_pack(a0, b0, n))
    A, B = E.export(a0), E.export(b0)
    k = E.n // (4 * n)
    nl = E.nl(0)
    limbs = list(range(nl))
    q = O.moduli[:nl].astype(np.int64)[:, None]
    for p in range(2):
        ca = O.intt(A[p], limbs).astype(np.int64)
        cb = O.intt(B[p], limbs).astype(np.int64)
        cz = O.intt(z[p], limbs).astype(np.int64)
        assert np.array_equal(cz, (ca + _negacyclic_shift(cb, k, q)) % q), p


@pytest.mark.parametrize("n", [16, 32])
def test_mono_split_matches_slot_model(E, n):
    """(m + rot_n(m), X^-k (m - rot_n(m))) on a double-prime-level ciphertext (the bootstrap's own
    stage 5) against the same map on its decrypted slots: slot j of X^-k is exp(-i pi k e_j / N),
    e_j = 5^j mod 2N"""
    rng = np.random.default_rng(500 + n)
    m = E.debug_boot_stage_sparse(E.encrypt(_periodic(E, 2 * n, rng)), 5, 2 * n)
    zm = E.decrypt(m)
    hi, lo = E.debug_mono_split(m, n)
    N, M, k = E.n, E.slot_count, E.n // (4 * n)
    e = np.array([pow(5, j, 2 * N) for j in range(M)], np.float64)
    r = np.roll(zm, n)
    want_hi = zm + r
    want_lo = (zm - r) * np.exp(-1j * np.pi * k * e / N)
    assert _rel(E.decrypt(hi), want_hi) < REL
    assert _rel(E.decrypt(lo), want_lo) < REL


@pytest.mark.parametrize("logn", [13, 16])
def test_compact_diagonals_bit_identical(logn, monkeypatch):
    """A sparse plan's diagonals are dn-periodic slot vectors, i.e. subring elements, so their NTT
    rows are runs of N / (2 dn) equal residues and k_lin_mac reads 2 dn residues per limb (engine
    group_pts, LinMacArgs::pt_shift).  The full rows of the same projected diagonals
    (AESFHE_COMPACT_DIAG=0) must give the same sparse bootstraps bit for bit: single at periods 16
    and 32, and the monomial pair at 16 (the C2 MixColumns form)."""
    from engine_context import EngineContext
    from mi355x_ckks import Engine
    outs = []
    for flag in ("0", "1"):
        monkeypatch.setenv("AESFHE_COMPACT_DIAG", flag)  # read when an engine is created
        if logn == 13:
            E = Engine(log_n=13, use_bootstrap=True, max_level=3, dnum=5, seed=7, allow_insecure=True, enc_nonce=0)
        else:
            E = EngineContext(signature=1, max_level=17, log_n=16, seed=0x5EED, enc_nonce=0).engine
        rng = np.random.default_rng(3)
        res = []
        for n in (16, 32):
            ct = E.encrypt(_periodic(E, n, rng))
            res.append(E.export(E.bootstrap_sparse(ct, n)).tobytes())
        a, b = E.encrypt(_periodic(E, 16, rng)), E.encrypt(_periodic(E, 16, rng))
        pa, pb = E.bootstrap_pair_sparse(a, b, 16)
        res += [E.export(pa).tobytes(), E.export(pb).tobytes()]
        outs.append(res)
        del E
    assert all(x == y for x, y in zip(outs[0], outs[1]))


@pytest.mark.parametrize("logn", [13, 16])
def test_fused_relin_epilogue_bit_identical(logn, monkeypatch):
    """Products relinearised straight from their factors (AESFHE_FUSED_TENSOR) and EvalMod's
    2 T^2 - 1 in the relinearisation's finish (AESFHE_FUSED_AFFINE) against the tensor-first,
    lincomb-after forms: the same sparse and full-slot bootstraps bit for bit."""
    from engine_context import EngineContext
    from mi355x_ckks import Engine
    outs = []
    for flag in ("0", "1"):
        monkeypatch.setenv("AESFHE_FUSED_TENSOR", flag)
        monkeypatch.setenv("AESFHE_FUSED_AFFINE", flag)
        if logn == 13:
            E = Engine(log_n=13, use_bootstrap=True, max_level=3, dnum=5, seed=7, allow_insecure=True, enc_nonce=0)
        else:
            E = EngineContext(signature=1, max_level=17, log_n=16, seed=0x5EED, enc_nonce=0).engine
        rng = np.random.default_rng(4)
        res = [E.export(E.bootstrap_sparse(E.encrypt(_periodic(E, 32, rng)), 32)).tobytes()]
        full = E.encrypt(0.5 * np.exp(2j * np.pi * rng.random(E.slot_count)))
        res.append(E.export(E.bootstrap(full)).tobytes())
        outs.append(res)
        del E
    assert all(x == y for x, y in zip(outs[0], outs[1]))
