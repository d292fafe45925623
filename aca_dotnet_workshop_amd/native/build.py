"""In-tree builder for the native extensions.

* ``_ttnative``  -- C++17 document store + broker engines (g++/clang++, pybind11).
* ``bin/ttsidecar-dataplane`` -- native sidecar data plane executable (epoll HTTP/1.1,
  ``src/dataplane.cpp``), spawned by the Python sidecar when ``TT_SIDECAR_DATAPLANE=native``.
* ``_ttgpu``     -- HIP kernels for gfx950 (see ``aca_dotnet_workshop_amd/ops``), built by
  ``ops/build.py``.

Builds are incremental (skipped when the ``.so`` is newer than every source) and land
next to this file so the driver's gpurun snapshot carries them to the GPU box.
"""
from __future__ import annotations

import os
import subprocess
import sys
import sysconfig
from pathlib import Path

HERE = Path(__file__).resolve().parent
SRC = HERE / "src"


def ext_path(name: str) -> Path:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return HERE / f"{name}{suffix}"


def _stale(target: Path, sources: list[Path]) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(s.stat().st_mtime > t for s in sources)


def build_native(force: bool = False, verbose: bool = False) -> Path:
    import pybind11

    target = ext_path("_ttnative")
    sources = sorted(SRC.glob("*.hpp")) + [SRC / "module.cpp"]
    if not force and not _stale(target, sources):
        return target
    cxx = os.environ.get("CXX", "g++")
    tmp = target.with_suffix(f".tmp{os.getpid()}.so")
    cmd = [cxx, "-O3", "-std=c++17", "-shared", "-fPIC", "-fvisibility=hidden", "-Wall", "-Wno-unused-function",
           f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}", str(SRC / "module.cpp"),
           "-o", str(tmp), "-lpthread"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, target)
    return target


DATAPLANE = HERE / "bin" / "ttsidecar-dataplane"


def build_dataplane(force: bool = False, verbose: bool = False) -> Path:
    sources = [SRC / "dataplane.cpp", SRC / "evhttp.hpp", SRC / "json.hpp", SRC / "httpparse.hpp"]
    if not force and not _stale(DATAPLANE, sources):
        return DATAPLANE
    DATAPLANE.parent.mkdir(exist_ok=True)
    cxx = os.environ.get("CXX", "g++")
    tmp = DATAPLANE.with_name(f".{DATAPLANE.name}.tmp{os.getpid()}")
    cmd = [cxx, "-O2", "-std=c++17", "-Wall", "-Wno-unused-function", str(SRC / "dataplane.cpp"), "-o", str(tmp)]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, DATAPLANE)
    return DATAPLANE


LOADGEN = HERE / "bin" / "ttloadgen"


def build_loadgen(force: bool = False, verbose: bool = False) -> Path:
    """Closed-loop HTTP load generator used by bench.py (src/loadgen.cpp)."""
    sources = [SRC / "loadgen.cpp", SRC / "evhttp.hpp", SRC / "json.hpp", SRC / "httpparse.hpp"]
    if not force and not _stale(LOADGEN, sources):
        return LOADGEN
    LOADGEN.parent.mkdir(exist_ok=True)
    cxx = os.environ.get("CXX", "g++")
    tmp = LOADGEN.with_name(f".{LOADGEN.name}.tmp{os.getpid()}")
    cmd = [cxx, "-O2", "-std=c++17", "-Wall", "-Wno-unused-function", str(SRC / "loadgen.cpp"), "-o", str(tmp)]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, LOADGEN)
    return LOADGEN


if __name__ == "__main__":
    print(build_native(force="--force" in sys.argv, verbose=True))
    print(build_dataplane(force="--force" in sys.argv, verbose=True))
    print(build_loadgen(force="--force" in sys.argv, verbose=True))
