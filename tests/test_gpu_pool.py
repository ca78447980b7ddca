"""Device memory pool under memory pressure (engine.hip Pool): a failed
allocation releases the cached free lists (after a device sync) and retries once, so a long
mixed-shape session keeps running where it used to fail.  AESFHE_POOL_LIMIT_MB simulates a
smaller HBM for one context; the same op sequence run with and without the cap must give the same
ciphertext bytes, with the release-and-retry path taken under the cap."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _session(E):
    """products, rotations and conjugations down the whole chain: every level's buffer sizes
    pass through the pool's free lists"""
    rng = np.random.default_rng(9)
    z = np.exp(2j * np.pi * rng.random(E.slot_count))
    x = E.encrypt(z)
    outs = []
    for i in range(5):
        y = E.multiply(x, x, "rlk")
        r = E.rotate(y, None, 1 + i)
        c = E.conjugate(r)
        outs += [E.export(y), E.export(r), E.export(c)]
        x = E.add(y, c)
    return outs


def test_pool_release_and_retry(monkeypatch):
    from mi355x_ckks import Engine
    kw = dict(log_n=13, max_level=6, dnum=3, seed=0xB0B, allow_insecure=True, enc_nonce=1)
    monkeypatch.delenv("AESFHE_POOL_LIMIT_MB", raising=False)
    E = Engine(**kw)
    want = _session(E)
    st = E.pool_stats()
    assert st["oom_retries"] == 0
    held = st["bytes"]
    del E
    cap_mb = max(1, int(held * 0.5) >> 20)
    monkeypatch.setenv("AESFHE_POOL_LIMIT_MB", str(cap_mb))
    E = Engine(**kw)
    got = _session(E)
    st = E.pool_stats()
    assert st["oom_retries"] > 0, (held, cap_mb, st)      # the cap forced the release path
    assert st["bytes"] <= cap_mb << 20
    assert all(np.array_equal(a, b) for a, b in zip(want, got))
    del E
