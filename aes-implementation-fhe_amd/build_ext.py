"""Build libaesfhe.so (HIP kernels + C ABI) in-tree for gfx950 with hipcc.

The shared library is a build artefact (git-ignored) that travels to the GPU box with
the repository snapshot; nothing is installed into site-packages.
"""
from __future__ import annotations

import os
import shutil
import subprocess
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
LIB = PKG / "libaesfhe.so"
SOURCES = ["engine.hip", "kernels.hip", "ntt.hip", "params.cpp", "encoder.cpp", "bootstrap.cpp"]
HEADERS = ["common.h", "kernels.h", "launch.h", "params.h", "encoder.h", "bootstrap.h"]
ARCH = os.environ.get("AESFHE_ARCH", "gfx950")


def _hipcc() -> str:
    for cand in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found: cannot build the MI355X engine")


def needs_build() -> bool:
    if not LIB.exists():
        return True
    t = LIB.stat().st_mtime
    deps = [CSRC / s for s in SOURCES + HEADERS] + [PKG.parent / "include" / "aesfhe.h"]
    return any(d.stat().st_mtime > t for d in deps if d.exists())


def build(force: bool = False, verbose: bool = False) -> Path:
    if not force and not needs_build():
        return LIB
    cmd = [_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-o", str(LIB)]
    cmd += [str(CSRC / s) for s in SOURCES]
    if verbose:
        print(" ".join(cmd))
    tmp = LIB.with_suffix(".so.tmp")
    cmd[cmd.index("-o") + 1] = str(tmp)
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force=True, verbose=True))
