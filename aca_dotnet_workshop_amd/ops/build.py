"""Build the HIP kernels (``ops/hip/*.hip``) into an in-tree shared library for gfx950.

Plain ``hipcc -shared`` (no torch extension machinery): the kernels expose ``extern "C"``
launchers taking raw device pointers and a ``hipStream_t``; ``ops/gpu.py`` calls them via
ctypes with PyTorch tensors' ``data_ptr()`` and the current stream.  Cross-compiles on a
CPU-only host.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
HIP_DIR = HERE / "hip"
LIB = HERE / "_ttgpu.so"
ARCH = os.environ.get("TT_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise FileNotFoundError("hipcc not found (ROCm is required to build the GPU kernels)")


def sources() -> list[Path]:
    return sorted(HIP_DIR.glob("*.hip"))


def stale() -> bool:
    if not LIB.exists():
        return True
    t = LIB.stat().st_mtime
    return any(s.stat().st_mtime > t for s in sources() + sorted(HIP_DIR.glob("*.h")))


def build_gpu(force: bool = False, verbose: bool = False) -> Path:
    if not force and not stale():
        return LIB
    from ..native.build import build_lock
    with build_lock("ttgpu"):
        if force or stale():
            _compile(verbose)
    return LIB


def _compile(verbose: bool) -> None:
    from ..native.build import _install, _newest, _run_compiler
    tmp = LIB.with_suffix(f".tmp{os.getpid()}.so")
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-shared", "-fPIC", "-Wall",
           *map(str, sources()), "-o", str(tmp)]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    stamp = _newest(sources() + sorted(HIP_DIR.glob("*.h")))  # dated like the sources compiled
    _run_compiler(cmd, tmp)
    _install(tmp, LIB, stamp)


if __name__ == "__main__":
    print(build_gpu(force="--force" in sys.argv, verbose=True))
