"""In-tree builder for the native extensions.

* ``_ttnative``  -- C++17 document store + broker engines (g++/clang++, pybind11).
* ``bin/ttingress`` -- the environment's native HTTP(S) ingress (``src/ingress.cpp``), spawned by
  ``platform/ingress.py`` (the Container Apps / Envoy edge equivalent).
* ``bin/ttsidecar-dataplane`` -- native sidecar data plane executable (epoll HTTP/1.1,
  ``src/dataplane.cpp``), spawned by the Python sidecar when ``TT_SIDECAR_DATAPLANE=native``.
* ``_ttgpu``     -- HIP kernels for gfx950 (see ``aca_dotnet_workshop_amd/ops``), built by
  ``ops/build.py``.

Builds are incremental (skipped when the ``.so`` is as new as every source: it is dated like the
newest source it was compiled from) and land
next to this file so the driver's gpurun snapshot carries them to the GPU box.
"""
from __future__ import annotations

import contextlib
import fcntl
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


@contextlib.contextmanager
def build_lock(name: str):
    """Serialise concurrent builders (e.g. 8 bench ranks x N sidecars starting at once on a fresh
    checkout): one compiles, the others wait and then find the target fresh."""
    lock_dir = HERE / "bin"
    lock_dir.mkdir(exist_ok=True)
    with open(lock_dir / f".{name}.lock", "w") as fh:
        fcntl.flock(fh, fcntl.LOCK_EX)
        try:
            yield
        finally:
            fcntl.flock(fh, fcntl.LOCK_UN)


def _stale(target: Path, sources: list[Path]) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    # a deployed image ships the built extension without its sources: present means current
    return any(s.exists() and s.stat().st_mtime > t for s in sources)


def _newest(sources: list[Path]) -> float:
    return max((s.stat().st_mtime for s in sources if s.exists()), default=0.0)


def _install(tmp: Path, target: Path, stamp: float) -> None:
    """Move the build into place, dated like the newest source it was compiled from: a source
    saved while the compiler ran is newer than the result, so the next check rebuilds."""
    os.replace(tmp, target)
    if stamp > 0:
        os.utime(target, (stamp, stamp))


def _run_compiler(cmd: list[str], tmp: Path) -> None:
    try:
        subprocess.run(cmd, check=True)
    except BaseException:
        tmp.unlink(missing_ok=True)  # no half-written output left next to the target
        raise


EXE_ONLY_HEADERS: set[str] = set()


def build_native(force: bool = False, verbose: bool = False) -> Path:
    target = ext_path("_ttnative")
    # every header but the executables-only ones -- a change there must not make the
    # extension look stale
    sources = sorted(h for h in SRC.glob("*.hpp") if h.name not in EXE_ONLY_HEADERS) + [SRC / "module.cpp"]
    if not force and not _stale(target, sources):
        return target
    with build_lock("ttnative"):
        if force or _stale(target, sources):
            _compile_native(target, verbose, _newest(sources))
    return target


def _compile_native(target: Path, verbose: bool, stamp: float = 0.0) -> None:
    import pybind11
    cxx = os.environ.get("CXX", "g++")
    tmp = target.with_suffix(f".tmp{os.getpid()}.so")
    # default visibility: the engines' functions are in the dynamic symbol table, so a
    # TT_PC_SAMPLE profile of a process hosting them (the backing) names them (dladdr)
    cmd = [cxx, "-O3", "-std=c++17", "-shared", "-fPIC", "-Wall", "-Wno-unused-function", "-Wno-attributes",
           f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}", str(SRC / "module.cpp"),
           "-o", str(tmp), "-lpthread", "-lssl", "-lcrypto"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    _run_compiler(cmd, tmp)
    _install(tmp, target, stamp)


DATAPLANE = HERE / "bin" / "ttsidecar-dataplane"


def build_dataplane(force: bool = False, verbose: bool = False) -> Path:
    sources = [SRC / "dataplane.cpp", SRC / "evhttp.hpp", SRC / "h2.hpp", SRC / "pb.hpp", SRC / "tls.hpp", SRC / "json.hpp", SRC / "httpparse.hpp",
               SRC / "textutil.hpp", SRC / "pcsample.hpp"]
    return _build_exe(DATAPLANE, SRC / "dataplane.cpp", sources, force, verbose)


def _build_exe(target: Path, main: Path, sources: list[Path], force: bool, verbose: bool,
               threads: bool = False) -> Path:
    if not force and not _stale(target, sources):
        return target
    with build_lock(target.name):
        if not force and not _stale(target, sources):
            return target
        cxx = os.environ.get("CXX", "g++")
        tmp = target.with_name(f".{target.name}.tmp{os.getpid()}")
        # -rdynamic: the executables' own functions resolve in TT_PC_SAMPLE profiles (pcsample.hpp)
        cmd = [cxx, "-O2", "-std=c++17", "-Wall", "-Wno-unused-function", "-rdynamic", str(main), "-o", str(tmp),
               "-lssl", "-lcrypto"] + (["-pthread"] if threads else [])
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        stamp = _newest(sources)
        _run_compiler(cmd, tmp)
        _install(tmp, target, stamp)
    return target


INGRESS = HERE / "bin" / "ttingress"


def build_ingress(force: bool = False, verbose: bool = False) -> Path:
    """The environment's native HTTP(S) ingress (src/ingress.cpp), spawned by platform/ingress.py."""
    sources = [SRC / "ingress.cpp", SRC / "evhttp.hpp", SRC / "tls.hpp", SRC / "json.hpp", SRC / "httpparse.hpp",
               SRC / "textutil.hpp", SRC / "pcsample.hpp"]
    return _build_exe(INGRESS, SRC / "ingress.cpp", sources, force, verbose, threads=True)


LOADGEN = HERE / "bin" / "ttloadgen"


def build_loadgen(force: bool = False, verbose: bool = False) -> Path:
    """Closed-loop HTTP load generator used by bench.py (src/loadgen.cpp)."""
    sources = [SRC / "loadgen.cpp", SRC / "evhttp.hpp", SRC / "tls.hpp", SRC / "json.hpp", SRC / "httpparse.hpp"]
    return _build_exe(LOADGEN, SRC / "loadgen.cpp", sources, force, verbose, threads=True)


if __name__ == "__main__":
    print(build_native(force="--force" in sys.argv, verbose=True))
    print(build_dataplane(force="--force" in sys.argv, verbose=True))
    print(build_loadgen(force="--force" in sys.argv, verbose=True))
    print(build_ingress(force="--force" in sys.argv, verbose=True))
