"""The renorm codec's snap inside the encode (engine.hip renorm, kernels.hip snap_block,
AESFHE_SNAP_ENCODE): the encode kernels derive the 32 snapped slot values from the decode's
accumulator themselves and zero the other buffer of a per-stream pair, instead of a k_snap16 launch
that snaps and re-zeroes.  The same arithmetic on the same inputs: one full C2 encrypt (every renorm
form it uses: the periodic, the packed period-32 single and unpack codecs) gives the same ciphertext
bytes with the snap inside the encode and as its own launch, and two encrypts in a row (the
accumulators alternating) too."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _encrypts(flag, monkeypatch):
    monkeypatch.setenv("AESFHE_SNAP_ENCODE", flag)
    from aes_keyschedule import expand_aes128_key, load_all_coeffs
    from engine_context import EngineContext
    from oracle import aes_plain
    from pipeline import AESPipeline
    ctx = EngineContext(signature=1, max_level=17, seed=0x5EED, enc_nonce=0)
    pipe = AESPipeline(ctx, load_all_coeffs(), use_hard_renorm_between_steps=True)
    rng = np.random.default_rng(19)
    rks = expand_aes128_key(rng.integers(0, 256, 16).astype(np.uint8))
    out = []
    for _ in range(2):
        st = rng.integers(0, 256, 16).astype(np.uint8)
        cts = pipe.encrypt(st, rks)
        out += [ctx.engine.export(c).tobytes() for c in cts]
        assert np.array_equal(pipe.encoder.decode(*cts), aes_plain.ref_encrypt(st, rks))
    return out


def test_snap_encode_bit_identical(monkeypatch):
    a = _encrypts("0", monkeypatch)
    b = _encrypts("1", monkeypatch)
    assert len(a) == len(b) == 4
    bad = [i for i, (x, y) in enumerate(zip(a, b)) if x != y]
    assert not bad, f"ciphertexts {bad} differ between the snapping encode and the separate snap"
