"""Per-level work tallies (aesfhe_level_counters) of one C2 MixColumns final bootstrap, the input
of the CPU baseline's bootstrap replay (bench.boot_tallies): every key switch the engine counts is
tallied at a level, the bootstrap spans level 0 (the dense -> sparse switch) to its ModRaise level (the trace),
and its EvalMod products and linear-transform diagonals are there."""
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parent.parent


def test_boot_tallies_cover_the_bootstrap():
    sys.path.insert(0, str(ROOT))
    import bench
    from engine_context import EngineContext
    ctx = EngineContext(signature=1, max_level=17)
    b = bench.boot_tallies(ctx, 32)
    E = ctx.engine
    t = b["tallies"]
    # the engine's keyswitch counter plus the baby-step rotations inside k_lin_mac (counted as rotations)
    assert sum(t["key_switch"].values()) >= E.counters()["keyswitch"] > 0
    # level 0: the dense -> sparse switch; the top: the sparse plan's ModRaise level (below the chain's
    # top E.L, which the full-slot plan uses)
    assert min(t["key_switch"]) == 0 and E.L - 4 <= max(t["key_switch"]) <= E.L
    assert sum(t["product"].values()) >= 14  # EvalMod's Chebyshev series and double angles
    assert sum(t["diagonal"].values()) > 0
    assert b["level_limbs"] == list(E.level_limbs) and len(b["level_limbs"]) == E.L + 1
    print(t)
