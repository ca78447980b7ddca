"""Precision where the error tails are: 2,048 slot-packed states in one ciphertext
pair (the packed-pairs leg's per-pair shape), one full encrypt with renorm and the
final bootstraps.  Every state slot of every logged stage (renorm / XOR4 / GF / SubBytes /
bootstrap outputs) stays within a quarter of the decode margin pi/16 of its Zeta16 codeword
(REF/utils.py:15-19, REF/state_encoder.py:30-38), and the bytes match FIPS-197."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_precision_margin_2048_states():
    import bench
    from aes_keyschedule import expand_aes128_key, load_all_coeffs
    from engine_context import EngineContext
    from oracle import aes_plain
    from pipeline import AESPipeline
    ctx = EngineContext(signature=1, max_level=17, seed=0x5EED, enc_nonce=0)
    rng = np.random.default_rng(11)
    rks = expand_aes128_key(rng.integers(0, 256, 16).astype(np.uint8))
    B = 2048
    pipe = AESPipeline(ctx, load_all_coeffs(), use_hard_renorm_between_steps=True, states=B)
    states = rng.integers(0, 256, (B, 16)).astype(np.uint8)
    got = pipe.encoder.decode(*pipe.encrypt(states, rks))
    bad = [j for j in range(B) if not np.array_equal(got[j], aes_plain.ref_encrypt(states[j], rks))]
    assert not bad, f"{len(bad)} of {B} states wrong, first {bad[:8]}"  # every state's bytes
    p = bench.measure_precision(pipe, ctx, rks, states, f"{B} slot-packed states")
    assert p["state_slots_per_stage"] >= 16 * B
    assert p["margin_factor"] >= 4.0, p
