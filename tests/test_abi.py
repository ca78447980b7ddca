"""The C-ABI library builds for gfx950, loads, and exports every symbol of include/aesfhe.h."""
import re
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent


def declared_symbols():
    text = (ROOT / "include" / "aesfhe.h").read_text()
    return sorted(set(re.findall(r"\b(aesfhe_[a-z0-9_]+)\s*\(", text)))


def test_header_matches_binding():
    import mi355x_ckks
    assert declared_symbols() == sorted(mi355x_ckks.EXPORTED)


def test_library_exports_all_symbols():
    import mi355x_ckks
    import build_ext
    build_ext.build()
    lib = mi355x_ckks.load_library()
    for name in declared_symbols():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", str(build_ext.LIB)], capture_output=True, text=True, check=True).stdout
    for name in declared_symbols():
        assert re.search(rf"\bT {name}\b", out), name


def test_library_carries_gfx950_code_object():
    import build_ext
    data = Path(build_ext.LIB).read_bytes()
    assert b"gfx950" in data


def test_engine_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    from mi355x_ckks import Engine
    with pytest.raises(RuntimeError, match="HIP device|no CPU fallback|hip"):
        Engine(log_n=12, max_level=4)
