"""Container images for the three services without Docker -- module 12 ("optimise containers").

The reference's only *measured* numbers are image sizes (reference
docs/aca/12-optimize-containers/index.md:318-326): each ASP.NET service as a status-quo image
(``aspnet:8.0``, 226-239 MB) and a chiseled one (``8.0-jammy-chiseled``, 119-133 MB, no shell,
no package manager, non-root).  Docker is not available here, so this module builds the images
itself and writes them as OCI image-layout archives that ``docker load`` / ``podman load`` accept:

``standard``
    The Python runtime as a language base image ships it: the interpreter, the whole standard
    library (minus test suites / IDLE / Tk / ensurepip) with every extension module, the full
    site-packages distributions the service imports, and the service's package.
``chiseled``
    Only what the service can load.  The closure is the union of
    (a) traces: the service is started under a tracer in EVERY configuration it supports
        (``MODES``: HTTP and gRPC SDK transport, asyncio and native app host, each notifier
        mode, fake and store manager, Dapr and plain-HTTP frontend), probed, and the files it
        mapped or imported are recorded -- interpreter, the shared objects of
        ``/proc/self/maps`` (libc, libpython, the loader, our native host), every module; and
    (b) the static import graph of the service's own package modules (``static_closure``:
        every import statement, including the lazy ones inside functions, followed through
        the package; the third-party and standard-library packages they name are shipped
        whole), so a code path no trace exercised still finds its modules.
    Python files are compiled to sourceless ``.pyc``; plus the package's data files.  No shell,
    no pip, non-root user ``65532``.

Each image is a single gzip layer; ``verify_image`` unpacks it and runs the service inside it
with ``chroot`` (root only) in every mode of ``MODES`` -- and drives the lazily imported paths
(``VERIFY_CALLS``) -- to prove the closure is complete.  ``report`` prints the size table
that docs/modules/12-optimize-containers.md compares with the reference's.
"""
from __future__ import annotations

import gzip
import hashlib
import io
import json
import os
import py_compile
import shutil
import signal
import subprocess
import sys
import stat
import sysconfig
import tarfile
import tempfile
import time
from dataclasses import dataclass, field
from pathlib import Path
from typing import Any

PKG = "aca_dotnet_workshop_amd"
PKG_ROOT = Path(__file__).resolve().parents[1]
SERVICES = {"backend_api": "tasksmanager-backend-api", "processor": "tasksmanager-backend-processor",
            "frontend": "tasksmanager-frontend-webapp"}
PROBE = {"backend_api": "/api/tasks?createdBy=tjoudeh@bitoftech.net", "processor": "/dapr/subscribe",
         "frontend": "/"}
# Every configuration a service supports (env overrides) -- each is traced into the chiseled
# closure and verified inside the image.
MODES: dict[str, list[dict[str, str]]] = {
    "backend_api": [{}, {"TT_APP_HOST": "native"},
                    {"TasksManager__Backend": "store", "Dapr__ApiProtocol": "grpc"},
                    {"TasksManager__Backend": "store", "TT_APP_HOST": "native", "Dapr__ApiProtocol": "grpc"}],
    "processor": [{}, {"TT_APP_HOST": "native"}, {"Dapr__ApiProtocol": "grpc"},
                  {"TasksNotifier__Mode": "sendgrid-api", "SendGrid__Endpoint": "http://127.0.0.1:9"},
                  {"TasksNotifier__Mode": "sendgrid-binding"}],
    "frontend": [{}, {"TT_APP_HOST": "native"}, {"Frontend__BackendMode": "http"}, {"Dapr__ApiProtocol": "grpc"}],
}
# Requests that reach code paths importing modules lazily (a notifier mode's client, ...):
# (mode index, method, path, body) -- run by verify_image after the probe.
_TASK = json.dumps({"taskId": "00000000-0000-4000-8000-000000000001", "taskName": "probe", "taskCreatedBy": "a@b.c",
                    "taskCreatedOn": "2030-01-01T00:00:00", "taskDueDate": "2030-01-02T00:00:00",
                    "taskAssignedTo": "a@b.c", "isCompleted": False, "isOverDue": False})
VERIFY_CALLS: dict[str, list[tuple[int, str, str, str]]] = {
    "processor": [(3, "POST", "/api/tasksnotifier/tasksaved", _TASK), (4, "POST", "/api/tasksnotifier/tasksaved", _TASK)],
}
BUILD_ONLY = {"pybind11"}  # compiles the native module in-tree; images ship the built .so
APP_DIR = "/app"
NONROOT = 65532
_STDLIB_SKIP = {"test", "idlelib", "tkinter", "turtledemo", "ensurepip", "lib2to3", "pydoc_data", "__pycache__",
                "unittest", "distutils", "venv"}
_DATA_SUFFIXES = {".json", ".html", ".css", ".js", ".ico", ".svg", ".png", ".txt"}

_BOOT = r"""
import json, os, signal, sys, runpy
dump, mod = sys.argv[1], sys.argv[2]
sys.argv = [mod] + sys.argv[3:]
def _dump(*_):
    mods = sorted({os.path.realpath(f) for f in (getattr(m, "__file__", None) for m in list(sys.modules.values())) if f})
    maps = set()
    with open("/proc/self/maps") as fh:
        for line in fh:
            p = line.split()
            if len(p) >= 6 and p[5].startswith("/"):
                maps.add(p[5])
    with open(dump + ".tmp", "w") as fh:
        json.dump({"modules": mods, "maps": sorted(maps), "exe": sys.executable, "path": sys.path}, fh)
    os.replace(dump + ".tmp", dump)
signal.signal(signal.SIGUSR1, _dump)
runpy.run_module(mod, run_name="__main__", alter_sys=True)
"""


@dataclass
class ImageResult:
    service: str
    variant: str
    path: Path
    files: int
    uncompressed: int
    compressed: int
    packages: list[str] = field(default_factory=list)
    shared_libs: int = 0
    digest: str = ""

    def row(self) -> dict:
        return {"service": self.service, "variant": self.variant, "files": self.files,
                "uncompressed_mb": round(self.uncompressed / 1e6, 1), "compressed_mb": round(self.compressed / 1e6, 1),
                "python_distributions": len(self.packages), "shared_libs": self.shared_libs,
                "digest": self.digest, "archive": str(self.path)}


# --------------------------------------------------------------------------- tracing
def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _http_get(port: int, path: str, timeout: float = 5.0) -> tuple[int, bytes]:
    import http.client
    c = http.client.HTTPConnection("127.0.0.1", port, timeout=timeout)
    try:
        c.request("GET", path)
        r = c.getresponse()
        return r.status, r.read()
    finally:
        c.close()


def _wait_http(port: int, path: str, proc: subprocess.Popen, timeout: float = 60.0) -> tuple[int, bytes]:
    deadline = time.time() + timeout
    while True:
        if proc.poll() is not None:
            raise RuntimeError(f"service exited with {proc.returncode}")
        try:
            return _http_get(port, path)
        except OSError:
            if time.time() > deadline:
                raise TimeoutError(f"service did not answer {path}")
            time.sleep(0.1)


def _service_env(port: int) -> dict[str, str]:
    env = {"ASPNETCORE_URLS": f"http://127.0.0.1:{port}", "ASPNETCORE_ENVIRONMENT": "Production",
           "PYTHONDONTWRITEBYTECODE": "1", "Logging__LogLevel__Default": "Warning",
           # frontend's required backend base URL (reference Frontend Program.cs:15-27)
           "BackendApiConfig__BaseUrlExternalHttp": "http://127.0.0.1:9"}
    return env


def trace_closure(service: str, mode: dict[str, str] | None = None) -> dict:
    """Start the service under the tracer (in configuration ``mode``), probe it, and return the
    files it loaded."""
    port = _free_port()
    with tempfile.TemporaryDirectory(prefix="ttimg-") as d:
        dump = os.path.join(d, "closure.json")
        env = {"PATH": os.environ.get("PATH", ""), "PYTHONPATH": str(PKG_ROOT.parent), **_service_env(port),
               **(mode or {})}
        proc = subprocess.Popen([sys.executable, "-c", _BOOT, dump, f"{PKG}.services.{service}"], env=env,
                                stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
        try:
            _wait_http(port, PROBE[service], proc)
            proc.send_signal(signal.SIGUSR1)
            deadline = time.time() + 10
            while not os.path.exists(dump):
                if time.time() > deadline:
                    raise TimeoutError("closure dump not written")
                time.sleep(0.05)
            with open(dump) as f:
                return json.load(f)
        finally:
            proc.terminate()
            try:
                proc.wait(10)
            except subprocess.TimeoutExpired:
                proc.kill()
                proc.wait()


def _module_file(mod: str) -> Path | None:
    p = PKG_ROOT.joinpath(*mod.split(".")[1:])
    if (p / "__init__.py").exists():
        return p / "__init__.py"
    if p.with_suffix(".py").exists():
        return p.with_suffix(".py")
    return None


def static_closure(service: str) -> tuple[set[Path], set[str]]:
    """The static import graph from the service's entry module through this package: (package
    module files, dotted names of the external modules they import).  Every import statement
    counts -- module level or inside a function -- except the lazy re-exports of a package's
    ``__getattr__`` (PEP 562), which serve other importers, not the package itself."""
    import ast
    files: set[Path] = set()
    external: set[str] = set()
    todo = [f"{PKG}.services.{service}.__main__"]
    seen: set[str] = set()
    while todo:
        mod = todo.pop()
        if mod in seen:
            continue
        seen.add(mod)
        f = _module_file(mod)
        if f is None:
            continue
        files.add(f)
        parts = mod.split(".")
        todo.extend(".".join(parts[:i]) for i in range(2, len(parts)))  # parent packages' __init__
        tree = ast.parse(f.read_text())
        lazy: set[int] = set()
        for fn in ast.walk(tree):
            if isinstance(fn, ast.FunctionDef) and fn.name == "__getattr__":
                lazy.update(id(x) for x in ast.walk(fn))
        is_pkg = f.name == "__init__.py"
        for n in ast.walk(tree):
            if id(n) in lazy:
                continue
            names: list[str] = []
            if isinstance(n, ast.Import):
                names = [a.name for a in n.names]
            elif isinstance(n, ast.ImportFrom):
                if n.level:
                    base = parts if is_pkg else parts[:-1]
                    base = base[:len(base) - (n.level - 1)]
                    head = ".".join(base + ([n.module] if n.module else []))
                else:
                    head = n.module or ""
                names = [head] + [f"{head}.{a.name}" for a in n.names]
            for nm in names:
                if not nm:
                    continue
                if nm.split(".")[0] == PKG:
                    todo.append(nm)
                elif nm.split(".")[0] not in BUILD_ONLY:
                    external.add(nm)
    return files, external


def _external_files(names: set[str]) -> tuple[set[Path], set[Path]]:
    """(python files, shared objects) of the standard-library modules and site-packages
    distributions named in ``names`` -- whole top-level packages (a namespace package such as
    ``google``: its imported subpackage)."""
    import importlib.util
    py: set[Path] = set()
    so: set[Path] = set()
    done: set[str] = set()
    for name in sorted(names):
        parts = name.split(".")
        top = parts[0]
        try:
            spec = importlib.util.find_spec(top)
        except (ImportError, ValueError):
            continue
        if spec is None:
            continue
        if spec.origin is None and spec.submodule_search_locations and len(parts) > 1:  # namespace package
            top = ".".join(parts[:2])
            try:
                spec = importlib.util.find_spec(top)
            except (ImportError, ValueError):
                continue
            if spec is None:
                continue
        if top in done:
            continue
        done.add(top)
        if spec.origin in (None, "built-in", "frozen"):
            continue
        origin = Path(spec.origin)
        if spec.submodule_search_locations:  # package: ship it whole
            for loc in spec.submodule_search_locations:
                for f in Path(loc).rglob("*"):
                    if not f.is_file() or "__pycache__" in f.parts or {"tests", "test"} & set(f.parts):
                        continue
                    if f.suffix == ".py":
                        py.add(f)
                    elif ".so" in f.name:
                        so.add(f)
        elif origin.suffix == ".py":
            py.add(origin)
        elif ".so" in origin.name:
            so.add(origin)
    return py, so


def full_closure(service: str) -> dict:
    """The chiseled closure: traces of every mode of ``MODES`` plus the static import graph."""
    merged: dict[str, Any] = {"modules": set(), "maps": set()}
    for mode in MODES.get(service, [{}]):
        c = trace_closure(service, mode)
        merged["exe"] = c["exe"]
        merged["modules"].update(c["modules"])
        merged["maps"].update(c["maps"])
    files, external = static_closure(service)
    py, so = _external_files(external)
    merged["modules"].update(str(p.resolve()) for p in files | py)
    merged["maps"].update(str(p.resolve()) for p in so)
    merged["static"] = {"package_modules": len(files), "external": sorted(external)}
    merged["modes"] = MODES.get(service, [{}])
    merged["modules"] = sorted(merged["modules"])
    merged["maps"] = sorted(merged["maps"])
    return merged


# --------------------------------------------------------------------------- file sets
def _stdlib_dir() -> Path:
    return Path(sysconfig.get_paths()["stdlib"]).resolve()


def _site_dirs() -> list[Path]:
    import site
    out = [Path(p).resolve() for p in site.getsitepackages() if os.path.isdir(p)]
    user = site.getusersitepackages()
    if user and os.path.isdir(user):
        out.append(Path(user).resolve())
    return out


def _distribution_of(path: Path, sites: list[Path]) -> tuple[Path, str] | None:
    """(site dir, top-level name) of a site-packages file."""
    for s in sites:
        try:
            rel = path.relative_to(s)
        except ValueError:
            continue
        return s, rel.parts[0]
    return None


def _package_data(service: str) -> list[Path]:
    """Non-Python files the service's packages need (appsettings, templates, static assets)."""
    out = []
    roots = [PKG_ROOT / "services" / service]
    for root in roots:
        for p in root.rglob("*"):
            if p.is_file() and p.suffix in _DATA_SUFFIXES and "__pycache__" not in p.parts:
                out.append(p)
    return out


def _elf_closure(paths: set[Path]) -> set[Path]:
    """Shared libraries the given ELF files need (via the loader's ``--list``), for files the
    tracer did not see mapped (``standard`` variant's unused extension modules)."""
    out: set[Path] = set()
    for p in paths:
        try:
            r = subprocess.run(["ldd", str(p)], capture_output=True, text=True, timeout=20)
        except (OSError, subprocess.TimeoutExpired):
            continue
        for line in r.stdout.splitlines():
            parts = line.split("=>")
            cand = (parts[1] if len(parts) == 2 else parts[0]).strip().split(" (")[0].strip()
            if cand.startswith("/") and os.path.exists(cand):
                out.add(Path(cand))
    return out


@dataclass
class _Plan:
    files: dict[str, Path] = field(default_factory=dict)      # image path -> host file
    compile: dict[str, Path] = field(default_factory=dict)    # image path (.pyc) -> host .py
    links: dict[str, str] = field(default_factory=dict)       # image path -> link target
    packages: set[str] = field(default_factory=set)
    libs: int = 0

    def add(self, host: Path, image: str | None = None) -> None:
        self.files[image or str(host)] = host


_TOP_LINKS = {n: os.readlink(f"/{n}") for n in ("bin", "sbin", "lib", "lib32", "lib64", "libx32")
              if os.path.islink(f"/{n}")}  # merged-/usr hosts: /lib -> usr/lib ...


def _canon(path: str) -> str:
    """The path with a top-level merged-/usr symlink expanded (``/lib/x`` -> ``/usr/lib/x``),
    so the image holds those names as symlinks and every file under one real directory."""
    parts = path.lstrip("/").split("/", 1)
    if parts[0] in _TOP_LINKS:
        return "/" + _TOP_LINKS[parts[0]].strip("/") + ("/" + parts[1] if len(parts) > 1 else "")
    return path


def _add_host_path(plan: _Plan, p: Path) -> None:
    """Add a host file, keeping symlinked names (``/lib64/ld-linux...`` -> real file)."""
    real = p.resolve()
    plan.add(real)
    name = _canon(str(p))
    if name != str(real):
        plan.links[name] = str(real)


def plan_image(service: str, variant: str, closure: dict) -> _Plan:
    plan = _Plan()
    stdlib = _stdlib_dir()
    sites = _site_dirs()
    exe = Path(closure["exe"])
    _add_host_path(plan, exe)
    plan.links["/usr/bin/python3"] = str(exe.resolve())
    so_files = {Path(m) for m in closure["maps"] if (".so" in Path(m).name or m == str(exe.resolve()))}
    pkg_parent = PKG_ROOT.parent
    for so in so_files:
        if not so.exists() or so.resolve() == exe.resolve():
            continue
        if PKG_ROOT in so.resolve().parents:  # our own extension modules live with the package
            plan.add(so.resolve(), f"{APP_DIR}/{so.resolve().relative_to(pkg_parent)}")
        else:
            _add_host_path(plan, so)
    # the loader is also reached by its canonical name; sonames (libexpat.so.1 -> .so.1.8.7)
    for ld in ("/lib64/ld-linux-x86-64.so.2",):
        if os.path.exists(ld):
            _add_host_path(plan, Path(ld))
    for lib in _elf_closure({exe.resolve()} | {so for so in so_files if so.exists()}):
        if PKG_ROOT not in lib.resolve().parents:
            _add_host_path(plan, lib)
    loaded = [Path(m) for m in closure["modules"]]
    site_tops: set[tuple[Path, str]] = set()
    for m in loaded:
        if m.suffix == ".so":
            continue  # came through maps
        try:
            rel = m.relative_to(pkg_parent)
            if rel.parts[0] == PKG:
                dst = f"{APP_DIR}/{rel}"
                if variant == "chiseled" and m.suffix == ".py":
                    plan.compile[dst + "c"] = m
                else:
                    plan.add(m, dst)
                continue
        except ValueError:
            pass
        dist = _distribution_of(m, sites)
        if dist is not None:
            site_tops.add(dist)
        if variant == "chiseled" and m.suffix == ".py":
            plan.compile[str(m) + "c"] = m
        else:
            plan.add(m)
    for p in _package_data(service):
        plan.add(p, f"{APP_DIR}/{p.relative_to(pkg_parent)}")
    for site_dir, top in site_tops:
        plan.packages.add(top.split(".")[0])
        if variant == "standard":
            root = site_dir / top
            if root.is_dir():
                for f in root.rglob("*"):
                    if f.is_file() and "__pycache__" not in f.parts:
                        plan.add(f)
            for info in site_dir.glob(f"{top.split('.')[0]}*-info"):
                for f in info.rglob("*"):
                    if f.is_file():
                        plan.add(f)
    if variant == "standard":
        ext: set[Path] = set()
        for f in stdlib.rglob("*"):
            rel = f.relative_to(stdlib)
            if not f.is_file() or (rel.parts and rel.parts[0] in _STDLIB_SKIP) or "__pycache__" in rel.parts \
                    or "test" in rel.parts or "tests" in rel.parts:
                continue
            plan.add(f)
            if f.suffix == ".so":
                ext.add(f)
        dyn = Path(sysconfig.get_config_var("DESTSHARED") or "")
        if dyn.is_dir():
            for f in dyn.glob("*.so"):
                plan.add(f)
                ext.add(f)
        for lib in _elf_closure(ext) - {Path(p) for p in plan.files}:
            _add_host_path(plan, lib)
    else:
        # getpath's landmarks: lib/pythonX.Y/os.py(c) and lib-dynload must exist
        dyn = Path(sysconfig.get_config_var("DESTSHARED") or "")
        if dyn.is_dir():
            plan.links.setdefault(str(dyn / ".keep"), "")
    plan.libs = sum(1 for k in plan.files if ".so" in Path(k).name)
    return plan


# --------------------------------------------------------------------------- OCI writer
def _tar_layer(plan: _Plan, variant: str) -> bytes:
    buf = io.BytesIO()
    dirs: set[str] = set()

    def add_dirs(tf: tarfile.TarFile, path: str) -> None:
        parts = path.strip("/").split("/")[:-1]
        for i in range(1, len(parts) + 1):
            d = "/".join(parts[:i])
            if d not in dirs:
                dirs.add(d)
                ti = tarfile.TarInfo(d)
                ti.type, ti.mode, ti.mtime = tarfile.DIRTYPE, 0o755, 0
                tf.addfile(ti)

    def add_bytes(tf: tarfile.TarFile, path: str, data: bytes, mode: int = 0o644) -> None:
        add_dirs(tf, path)
        ti = tarfile.TarInfo(path.lstrip("/"))
        ti.size, ti.mode, ti.mtime = len(data), mode, 0
        tf.addfile(ti, io.BytesIO(data))

    with tarfile.open(fileobj=buf, mode="w", format=tarfile.PAX_FORMAT) as tf:
        entries: list[tuple[str, str, object]] = []
        for dst, src in plan.files.items():
            entries.append((dst, "file", src))
        for dst, src in plan.compile.items():
            entries.append((dst, "pyc", src))
        for dst, target in plan.links.items():
            entries.append((dst, "link", target))
        entries.append(("/etc/passwd", "bytes", f"root:x:0:0:root:/root:/sbin/nologin\n"
                                                f"nonroot:x:{NONROOT}:{NONROOT}:nonroot:/home/nonroot:/sbin/nologin\n".encode()))
        entries.append(("/etc/group", "bytes", f"root:x:0:\nnonroot:x:{NONROOT}:\n".encode()))
        for name, target in _TOP_LINKS.items():
            entries.append((f"/{name}", "link", target))
        entries.append(("/tmp/.keep", "bytes", b""))
        entries.append(("/home/nonroot/.keep", "bytes", b""))
        for dst, kind, src in sorted(entries, key=lambda e: e[0]):
            if kind == "file":
                p = Path(src)  # type: ignore[arg-type]
                st = p.stat()
                add_bytes(tf, dst, p.read_bytes(), 0o755 if st.st_mode & 0o111 else 0o644)
            elif kind == "pyc":
                with tempfile.NamedTemporaryFile(suffix=".pyc") as tmp:
                    py_compile.compile(str(src), cfile=tmp.name, dfile=dst[:-1], doraise=True,
                                       invalidation_mode=py_compile.PycInvalidationMode.UNCHECKED_HASH)
                    add_bytes(tf, dst, Path(tmp.name).read_bytes())
            elif kind == "link":
                if not src:  # directory placeholder
                    add_dirs(tf, dst)
                    continue
                add_dirs(tf, dst)
                ti = tarfile.TarInfo(dst.lstrip("/"))
                ti.type, ti.linkname, ti.mtime = tarfile.SYMTYPE, str(src), 0
                tf.addfile(ti)
            else:
                add_bytes(tf, dst, src)  # type: ignore[arg-type]
        if variant == "standard":
            # the standard image keeps a shell like language base images do
            for sh in ("/bin/sh", "/usr/bin/dash"):
                if os.path.exists(sh) and f"{sh}" not in plan.files:
                    p = Path(sh).resolve()
                    add_bytes(tf, str(p), p.read_bytes(), 0o755)
                    if str(p) != sh:
                        add_dirs(tf, sh)
                        ti = tarfile.TarInfo(sh.lstrip("/"))
                        ti.type, ti.linkname, ti.mtime = tarfile.SYMTYPE, str(p), 0
                        tf.addfile(ti)
                    break
    return buf.getvalue()


def _sha(b: bytes) -> str:
    return "sha256:" + hashlib.sha256(b).hexdigest()


def write_oci(out: Path, tag: str, layer_tar: bytes, service: str, variant: str) -> tuple[int, str]:
    """Write an OCI image-layout tar (plus docker-archive ``manifest.json``); returns
    (compressed layer size, manifest digest)."""
    layer_gz = gzip.compress(layer_tar, compresslevel=6, mtime=0)
    module = f"{PKG}.services.{service}"
    user = "0:0" if variant == "standard" else f"{NONROOT}:{NONROOT}"
    config = {"architecture": "amd64", "os": "linux",
              "config": {"User": user, "WorkingDir": APP_DIR, "ExposedPorts": {"8080/tcp": {}},
                         "Env": ["PYTHONPATH=/app", "PYTHONDONTWRITEBYTECODE=1", "ASPNETCORE_URLS=http://+:8080",
                                 f"TT_APP_ID={SERVICES[service]}"],
                         "Entrypoint": ["/usr/bin/python3", "-m", module]},
              "rootfs": {"type": "layers", "diff_ids": [_sha(layer_tar)]},
              "history": [{"created_by": f"tt image build --service {service} --variant {variant}"}]}
    cfg = json.dumps(config, sort_keys=True).encode()
    manifest = {"schemaVersion": 2, "mediaType": "application/vnd.oci.image.manifest.v1+json",
                "config": {"mediaType": "application/vnd.oci.image.config.v1+json", "digest": _sha(cfg), "size": len(cfg)},
                "layers": [{"mediaType": "application/vnd.oci.image.layer.v1.tar+gzip", "digest": _sha(layer_gz),
                            "size": len(layer_gz)}]}
    man = json.dumps(manifest, sort_keys=True).encode()
    index = {"schemaVersion": 2, "mediaType": "application/vnd.oci.image.index.v1+json",
             "manifests": [{"mediaType": "application/vnd.oci.image.manifest.v1+json", "digest": _sha(man),
                            "size": len(man), "annotations": {"org.opencontainers.image.ref.name": tag}}]}
    blob = lambda d: f"blobs/sha256/{d.split(':', 1)[1]}"  # noqa: E731
    docker = [{"Config": blob(_sha(cfg)), "RepoTags": [tag], "Layers": [blob(_sha(layer_gz))]}]
    out.parent.mkdir(parents=True, exist_ok=True)
    with tarfile.open(out, "w") as tf:
        for name, data in (("oci-layout", b'{"imageLayoutVersion":"1.0.0"}'), ("index.json", json.dumps(index).encode()),
                           ("manifest.json", json.dumps(docker).encode()), (blob(_sha(cfg)), cfg),
                           (blob(_sha(man)), man), (blob(_sha(layer_gz)), layer_gz)):
            ti = tarfile.TarInfo(name)
            ti.size, ti.mtime = len(data), 0
            tf.addfile(ti, io.BytesIO(data))
    return len(layer_gz), _sha(man)


def build_image(service: str, variant: str, out_dir: str | Path, closure: dict | None = None) -> ImageResult:
    if service not in SERVICES:
        raise ValueError(f"unknown service {service!r} (one of {sorted(SERVICES)})")
    if variant not in ("standard", "chiseled"):
        raise ValueError("variant must be 'standard' or 'chiseled'")
    closure = closure or full_closure(service)
    plan = plan_image(service, variant, closure)
    layer = _tar_layer(plan, variant)
    tag = f"tasksmanager/{SERVICES[service]}:{variant}"
    path = Path(out_dir) / f"{SERVICES[service]}-{variant}.oci.tar"
    comp, digest = write_oci(path, tag, layer, service, variant)
    with tarfile.open(fileobj=io.BytesIO(layer)) as tf:
        members = tf.getmembers()
    nfiles = sum(1 for m in members if m.isfile())
    size = sum(m.size for m in members if m.isfile())
    return ImageResult(service, variant, path, nfiles, size, comp, sorted(plan.packages), plan.libs, digest)


# --------------------------------------------------------------------------- verification
def unpack_rootfs(archive: Path, dest: Path) -> dict:
    with tarfile.open(archive) as tf:
        index = json.load(tf.extractfile("index.json"))
        man = json.load(tf.extractfile("blobs/sha256/" + index["manifests"][0]["digest"].split(":")[1]))
        cfg = json.load(tf.extractfile("blobs/sha256/" + man["config"]["digest"].split(":")[1]))
        layer = tf.extractfile("blobs/sha256/" + man["layers"][0]["digest"].split(":")[1]).read()
    with tarfile.open(fileobj=io.BytesIO(gzip.decompress(layer))) as lt:
        lt.extractall(dest)
    return cfg


# The character devices every OCI runtime creates in a container's /dev (runc's default device
# list); grpcio's abseil, for one, reads /dev/urandom for its seed material.
_DEVICES = {"null": (1, 3), "zero": (1, 5), "full": (1, 7), "random": (1, 8), "urandom": (1, 9), "tty": (5, 0)}


# What a closure gap looks like in a service's log.  Other tracebacks are expected: a mode whose
# sidecar is absent fails its requests, but only after importing everything that path needs.
_MISSING_CODE = ("ModuleNotFoundError", "ImportError", "parser unavailable", "cannot open shared object")


def populate_dev(root: Path) -> None:
    """Give an unpacked root filesystem the runtime's default ``/dev`` nodes (needs root)."""
    dev = Path(root) / "dev"
    dev.mkdir(mode=0o755, exist_ok=True)
    for name, (major, minor) in _DEVICES.items():
        node = dev / name
        if not node.exists():
            os.mknod(node, 0o666 | stat.S_IFCHR, os.makedev(major, minor))
            node.chmod(0o666)


def _http(port: int, method: str, path: str, body: str, timeout: float = 10.0) -> int:
    import http.client
    c = http.client.HTTPConnection("127.0.0.1", port, timeout=timeout)
    try:
        c.request(method, path, body.encode(), {"content-type": "application/json"})
        r = c.getresponse()
        r.read()
        return r.status
    finally:
        c.close()


def verify_image(archive: Path, service: str, timeout: float = 60.0, modes: list[dict[str, str]] | None = None) -> dict:
    """Run the image's entrypoint inside its own root filesystem (``chroot``, needs root) in every
    mode (default ``MODES[service]``): GET the probe route, issue the mode's ``VERIFY_CALLS``
    (lazily imported code paths), stop it.  Returns ``{"status", "body", "log", "modes"}``
    (``log`` = stderr of all runs, where a missing module or extension would show)."""
    if os.geteuid() != 0:
        raise PermissionError("verify_image needs root (chroot)")
    modes = MODES.get(service, [{}]) if modes is None else modes
    with tempfile.TemporaryDirectory(prefix="ttroot-") as d:
        root = Path(d)
        root.chmod(0o755)  # mkdtemp is 0700: the non-root user must traverse "/"
        cfg = unpack_rootfs(archive, root)["config"]
        populate_dev(root)
        user = cfg.get("User", "0:0")
        cmd = [shutil.which("chroot") or "/usr/sbin/chroot", f"--userspec={user}", str(root)] + cfg["Entrypoint"]
        logs, first, results = [], None, []
        for i, mode in enumerate(modes):
            port = _free_port()
            env = {e.split("=", 1)[0]: e.split("=", 1)[1] for e in cfg["Env"]}
            env.update(_service_env(port))
            env.update(mode)
            env["Logging__LogLevel__Default"] = "Information"
            with tempfile.TemporaryFile() as errf:
                proc = subprocess.Popen(cmd, env=env, cwd=str(root), stdout=subprocess.DEVNULL, stderr=errf)
                try:
                    status, body = _wait_http(port, PROBE[service], proc, timeout)
                    calls = [(m, p, _http(port, m, p, b)) for k, m, p, b in VERIFY_CALLS.get(service, []) if k == i]
                except Exception as e:
                    proc.kill()
                    proc.wait()
                    errf.seek(0)
                    raise RuntimeError(f"image {archive.name} failed in mode {mode}: {e}\n"
                                       f"{errf.read().decode('utf-8', 'replace')[-2000:]}") from None
                proc.terminate()
                try:
                    proc.wait(10)
                except subprocess.TimeoutExpired:
                    proc.kill()
                    proc.wait()
                errf.seek(0)
                log = errf.read().decode("utf-8", "replace")
            logs.append(log)
            results.append({"mode": mode, "status": status, "calls": calls,
                            "clean": not any(m in log for m in _MISSING_CODE)})
            if first is None:
                first = (status, body)
        return {"status": first[0], "body": first[1], "log": "\n".join(logs), "modes": results}


def report(out_dir: str | Path, services: list[str] | None = None, verify: bool = False) -> list[dict]:
    rows = []
    for svc in services or list(SERVICES):
        closure = full_closure(svc)
        for variant in ("standard", "chiseled"):
            r = build_image(svc, variant, out_dir, closure)
            row = r.row()
            row["traced_modes"] = len(closure.get("modes", [])) or 1
            if verify:
                v = verify_image(r.path, svc)
                row["verified_status"] = v["status"]
                row["verified_modes"] = len(v["modes"])
                row["verified_clean_log"] = all(m["clean"] for m in v["modes"])
            rows.append(row)
    return rows


def main(argv: list[str] | None = None) -> int:
    import argparse
    ap = argparse.ArgumentParser(prog="tt image", description="build OCI images of the services (module 12)")
    ap.add_argument("--service", action="append", choices=sorted(SERVICES))
    ap.add_argument("--out", default="dist/images")
    ap.add_argument("--verify", action="store_true", help="run each image under chroot and probe it (root)")
    a = ap.parse_args(argv)
    for row in report(a.out, a.service, a.verify):
        print(json.dumps(row), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
