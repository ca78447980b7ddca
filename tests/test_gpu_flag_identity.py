"""Default-on kernel paths against the kernels they replaced: each switch is read once per
process, so every configuration runs in a fresh process.

- the 8-residue fused key-switch core (AESFHE_KI8), the 8-residue inverse row pass (AESFHE_NTT_INV8),
  the conversion sources pre-multiplied in the INTT (AESFHE_CONV_PRE), the 8-residue forward row pass
  (AESFHE_NTT_FWD8, on by default since round 6; its switch-off tested): every
  key-switching path's raw output limbs (tests/helpers/fused_conv_probe.py: relinearisation with and
  without the rescale, rotations, a conjugation, a batched rotation set, a stacked key switch, a sparse
  bootstrap) hash the same as with the default kernels -- bit for bit;
- the sparse -> dense key switch fused into the first trace step (AESFHE_S2D_TRACE): a different
  rounding, so the decrypted post-trace and CoeffToSlot stages of a sparse bootstrap agree with the
  separate form within the bootstrap tolerance.
"""
import json
import os
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HELPERS = Path(__file__).resolve().parent / "helpers"


def _run(probe: str, **env) -> dict:
    e = dict(os.environ, **{k: str(v) for k, v in env.items()})
    r = subprocess.run([sys.executable, str(HELPERS / probe)], env=e, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.fixture(scope="module")
def default_digests():
    return _run("fused_conv_probe.py")


@pytest.mark.parametrize("flag,value", [("AESFHE_KI8", 0), ("AESFHE_NTT_INV8", 0), ("AESFHE_CONV_PRE", 0),
                                        ("AESFHE_NTT_FWD8", 0)])
def test_kernel_switch_bit_identical(default_digests, flag, value):
    other = _run("fused_conv_probe.py", **{flag: value})
    assert other.keys() == default_digests.keys()
    bad = [k for k in other if other[k] != default_digests[k]]
    assert not bad, f"{flag}={value}: {bad}"


def test_s2d_trace_fusion_matches_separate_switch():
    from test_gpu_bootstrap import BOOT_TOL
    on, off = _run("s2d_trace_probe.py", AESFHE_S2D_TRACE=1), _run("s2d_trace_probe.py", AESFHE_S2D_TRACE=0)
    for stage in ("trace", "cts"):
        a = np.array(on[stage][0]) + 1j * np.array(on[stage][1])
        b = np.array(off[stage][0]) + 1j * np.array(off[stage][1])
        scale = max(1.0, float(np.abs(b).max()))
        assert np.abs(a - b).max() <= BOOT_TOL * scale, (stage, float(np.abs(a - b).max()), scale)


def test_bootstrap_after_a_mid_group_failure_is_bit_identical():
    """an error inside a linear-transform group (the test hook fails the first giant-step
    accumulation, after the group took its buffers), then a full bootstrap in the same process: the
    same residues as a clean process's bootstrap of the same input"""
    clean = _run("boot_after_error_probe.py")
    after = _run("boot_after_error_probe.py", AESFHE_TEST_FAIL_GIANT=1)
    assert after["failed_first"] is True
    assert after["digest"] == clean["digest"]
