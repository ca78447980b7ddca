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


STAMP = LIB.with_suffix(".so.sha256")  # content hash the library was built from (travels with it)


def source_digest() -> str:
    """sha256 over the compiler flags and every source / header the library is built from:
    the rebuild decision never depends on file modification times (a checkout or copy that
    reorders mtimes cannot ship a stale binary)"""
    import hashlib
    h = hashlib.sha256()
    h.update(" ".join(_flags()).encode())
    for d in [CSRC / s for s in SOURCES + HEADERS] + [PKG.parent / "include" / "aesfhe.h"]:
        h.update(d.name.encode() + b"\0")
        h.update(d.read_bytes() if d.exists() else b"<missing>")
    return h.hexdigest()


def needs_build() -> bool:
    if not LIB.exists() or not STAMP.exists():
        return True
    return STAMP.read_text().strip() != source_digest()


def _flags() -> list:
    return [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC"]


def build(force: bool = False, verbose: bool = False) -> Path:
    """Each source is compiled to an object in parallel (no device code crosses translation
    units: engine.hip reaches the kernels only through the host launch wrappers), then linked."""
    if not force and not needs_build():
        return LIB
    flags = _flags()
    digest = source_digest()
    objdir = PKG / "build"
    objdir.mkdir(exist_ok=True)
    objs = [objdir / (s + ".o") for s in SOURCES]

    def compile_one(i: int) -> None:
        cmd = [_hipcc(), *flags, "-c", str(CSRC / SOURCES[i]), "-o", str(objs[i])]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)

    from concurrent.futures import ThreadPoolExecutor
    workers = max(1, min(len(SOURCES), os.cpu_count() or 1, 8))
    with ThreadPoolExecutor(workers) as ex:
        list(ex.map(compile_one, range(len(SOURCES))))
    tmp = LIB.with_suffix(".so.tmp")
    cmd = [_hipcc(), *flags, "-shared", "-o", str(tmp), *map(str, objs)]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB)
    STAMP.write_text(digest + "\n")
    return LIB


if __name__ == "__main__":
    print(build(force=True, verbose=True))
