"""The CPU oracle under AddressSanitizer + UndefinedBehaviorSanitizer: oracle/sanitize_main.c
drives every entry point of oracle/ckks_oracle.c (both chains: plain, and bootstrappable with
the double-prime rescale and the d2s key switch) with the buffer shapes oracle/ckks_cpu.py
passes; any out-of-bounds access, leak or UB aborts the run (-fno-sanitize-recover=all)."""
import subprocess

from conftest import ROOT


def test_oracle_clean_under_asan_ubsan():
    odir = ROOT / "oracle"
    build = subprocess.run(["make", "-s", "-C", str(odir), "sanitize"], capture_output=True, text=True, timeout=300)
    assert build.returncode == 0, build.stderr[-2000:]
    run = subprocess.run([str(odir / "_build" / "oracle_sanitize")], capture_output=True, text=True, timeout=300)
    assert run.returncode == 0, run.stderr[-4000:]
    assert "oracle sanitize run ok" in run.stdout
