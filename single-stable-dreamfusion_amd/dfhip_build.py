"""Build the gfx950 kernel library (lib/libdfhip.so) in-tree.

Each csrc/*.hip is compiled by hipcc for gfx950 only and linked into one C-ABI
shared library (declared in include/dfhip.h).  Objects are rebuilt only when a
source or header is newer, and compiled in parallel.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
OBJ = PKG / "build"
LIB = PKG / "lib" / "libdfhip.so"

HEADER = ROOT / "include" / "dfhip.h"

ARCH = os.environ.get("DFHIP_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", shutil.which("hipcc") or "/opt/rocm/bin/hipcc")

def abi_hash(header: Path = HEADER) -> int:
    """dfhip_abi_version() of a library built from `header`: the first 28 bits
    of the SHA-256 of its bytes.  _dfhip.load() recomputes it from the header
    the Python binding was written against and refuses a library that differs
    (a stale library would otherwise be called with another signature)."""
    import hashlib
    return int(hashlib.sha256(header.read_bytes()).hexdigest()[:7], 16)


# -ffp-contract=off: only the explicit fmaf() calls (the reference's nvcc
# contraction sites) fuse; see DESIGN.md "Numerics".
CFLAGS = [
    f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
    "-fno-gpu-rdc", "-mcode-object-version=5", "-Wall", "-Wno-unused-function",
    "-fhip-fp32-correctly-rounded-divide-sqrt", f"-I{ROOT / 'include'}",
    f"-DDFHIP_ABI_HASH={abi_hash():#x}",
    *os.environ.get("DFHIP_EXTRA_CFLAGS", "").split(),  # A/B probe builds (tools only)
]


def _newest_dep() -> float:
    deps = list(CSRC.glob("*.h")) + [ROOT / "include" / "dfhip.h", Path(__file__)]
    return max(p.stat().st_mtime for p in deps)


def _compile(src: Path, dep_time: float, verbose: bool) -> Path:
    obj = OBJ / (src.stem + ".o")
    if obj.exists() and obj.stat().st_mtime >= max(src.stat().st_mtime, dep_time):
        return obj
    cmd = [HIPCC, *CFLAGS, "-c", str(src), "-o", str(obj)]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    return obj


def build(verbose: bool = False, jobs: int | None = None) -> Path:
    OBJ.mkdir(exist_ok=True)
    LIB.parent.mkdir(exist_ok=True)
    srcs = sorted(CSRC.glob("*.hip"))
    dep_time = _newest_dep()
    jobs = jobs or min(len(srcs), max(1, min(8, os.cpu_count() or 1)))
    with ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, dep_time, verbose), srcs))
    if not LIB.exists() or LIB.stat().st_mtime < max(o.stat().st_mtime for o in objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *map(str, objs),
               "-o", str(LIB)]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    return LIB


if __name__ == "__main__":
    print(build(verbose="-v" in sys.argv))
