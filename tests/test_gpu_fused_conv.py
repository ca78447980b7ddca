"""The base conversion fused into the forward NTT (ntt.hip k_ntt1_fwd_conv) is
bit for bit the separate k_base_convert + NTT: every key-switching path's raw output limbs, for
one pinned key set and encryption nonce, hash the same with AESFHE_FUSED_CONV=0 and =3 (ModUps and ModDowns fused)
(two fresh processes: the switch is read once per process)."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu

PROBE = Path(__file__).resolve().parent / "helpers" / "fused_conv_probe.py"


def _digests(fused: bool) -> dict:
    env = dict(os.environ, AESFHE_FUSED_CONV="3" if fused else "0")
    r = subprocess.run([sys.executable, str(PROBE)], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_fused_conversion_bit_exact():
    off, on = _digests(False), _digests(True)
    assert off.keys() == on.keys()
    bad = [k for k in off if off[k] != on[k]]
    assert not bad, bad
