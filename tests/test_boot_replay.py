"""The CPU baseline's bootstrap replay (tools/cpu_round.boot_replay, bench.py cpu_baseline): per-level
tallies of key switches, products and diagonal products replayed on the C oracle over the same
bootstrappable chain -- one operation per (kind, level) timed, times its count.  Small ring here
(N = 2^13); the bench runs it at N = 2^16 with the GPU engine's tallies of one C2 final bootstrap."""
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "tools"))


def _limbs(L1, nd):
    return [l + 2 for l in range(L1 + 1)] + [L1 + 2 + 2 * k for k in range(1, nd + 1)]


def test_replay_counts_and_time():
    import cpu_round
    tallies = {"key_switch": {0: 1, 6: 5, 5: 2}, "product": {6: 2, 4: 1}, "diagonal": {6: 7}}
    r = cpu_round.boot_replay(tallies, _limbs(4, 2), dnum=3, log_n=13)
    assert r["ops"] == {"key_switch": 8, "product": 3, "diagonal": 7}
    assert r["levels"] == [0, 4, 5, 6]
    assert all(v > 0 for v in r["by_kind_s"].values())
    # one operation per (kind, level) was timed; the total scales them by their counts
    assert r["boot_s"] >= r["sampled_s"] * 0.5
    assert abs(r["boot_s"] - sum(r["by_kind_s"].values())) < 1e-12


def test_replay_refuses_a_different_chain():
    import cpu_round
    bad = _limbs(4, 2)
    bad[-1] += 1  # not a chain the oracle builds
    with pytest.raises(RuntimeError, match="limbs per level"):
        cpu_round.boot_replay({"key_switch": {0: 1}}, bad, dnum=3, log_n=13)
