"""Multi-process local stack: the production process topology on one host.

Every app replica is a pair of OS processes -- the sidecar (``sidecar run``) and the app
(its child) -- talking over Unix sockets; sidecars find each other through the shared
registry directory and reach the backing-services process over HTTP.  This is the
``dapr run`` x N topology of the reference's local dev loop (snippets/dapr-run-*.md,
.vscode/tasks.json:126-165) and the unit the platform layer scales.

Children are started with ``subprocess.Popen`` (fork+exec of a fresh interpreter), never
by ``exec`` in the calling process.
"""
from __future__ import annotations

import json
import os
import shutil
import signal
import subprocess
import sys
import tempfile
import time
import urllib.request
from dataclasses import dataclass, field
from pathlib import Path
from typing import Any

REPO_ROOT = Path(__file__).resolve().parents[2]
SERVICE_MODULES = {
    "tasksmanager-backend-api": "aca_dotnet_workshop_amd.services.backend_api",
    "tasksmanager-backend-processor": "aca_dotnet_workshop_amd.services.processor",
    "tasksmanager-frontend-webapp": "aca_dotnet_workshop_amd.services.frontend",
}


@dataclass
class ReplicaProc:
    app_id: str
    name: str
    proc: subprocess.Popen
    sidecar_uds: str
    http_port: int | None = None
    app_port_file: str | None = None
    started: float = field(default_factory=time.time)
    fixed_app_port: int | None = None  # container replicas: the port the platform mapped for the app
    container: dict[str, Any] | None = None
    app_uds: str | None = None  # module replicas: the app also serves this Unix socket (TT_APP_UDS)

    @property
    def app_port(self) -> int | None:
        if self.fixed_app_port is not None:
            return self.fixed_app_port
        if self.app_port_file and os.path.exists(self.app_port_file):
            try:
                return int(Path(self.app_port_file).read_text())
            except ValueError:
                return None
        return None

    def alive(self) -> bool:
        return self.proc.poll() is None


class LocalStack:
    def __init__(self, root: str | os.PathLike | None = None, components: list[str] | None = None,
                 env: dict[str, str] | None = None, log_dir: str | None = None, quiet: bool = True) -> None:
        self.root = Path(root or tempfile.mkdtemp(prefix="tt-stack-"))
        self.root.mkdir(parents=True, exist_ok=True)
        self.sock_dir = Path(tempfile.mkdtemp(prefix="tts-"))
        self.registry = self.root / "registry"
        self.components = components or [str(REPO_ROOT / "deploy" / "components")]
        self.base_env = dict(os.environ)
        # process-based deployments run the sidecar's native C++ data plane unless told otherwise
        self.base_env.setdefault("TT_SIDECAR_DATAPLANE", "native")
        # ... and the services' HTTP I/O on the native app host (native/src/apphost.hpp)
        self.base_env.setdefault("TT_APP_HOST", "native")
        self.base_env["PYTHONPATH"] = str(REPO_ROOT) + os.pathsep + self.base_env.get("PYTHONPATH", "")
        self.base_env.update(env or {})
        self.log_dir = Path(log_dir) if log_dir else self.root / "logs"
        self.log_dir.mkdir(parents=True, exist_ok=True)
        self.quiet = quiet
        self.backing_proc: subprocess.Popen | None = None
        self.backing_url: str | None = None
        self.extra_backing: dict[str, tuple[subprocess.Popen, str]] = {}
        self.replicas: dict[str, list[ReplicaProc]] = {}
        self._seq = 0

    # -- processes --------------------------------------------------------------
    def _spawn(self, args: list[str], env: dict[str, str], log_name: str, role: str = "replica") -> subprocess.Popen:
        """``role``: ``platform`` (the backing services) or ``replica`` (a sidecar and the app it
        starts): the CPU subset the process is pinned to when the rank's set is split
        (``TT_PLATFORM_CPUS`` / ``TT_REPLICA_CPUS``, parallel.split_platform)."""
        from ..parallel import pin_preexec
        out = open(self.log_dir / f"{log_name}.log", "ab")
        return subprocess.Popen(args, env=env, stdout=out, stderr=subprocess.STDOUT, cwd=str(REPO_ROOT),
                                start_new_session=True, preexec_fn=pin_preexec(role))

    def _backing_env(self) -> dict[str, str]:
        """The backing's environment: its math libraries' thread pools at TT_BACKING_MATH_THREADS
        (default 1).  Its hot work is the native front's loops and the GPU scans; a BLAS or
        OpenMP pool sized for the whole machine (the box exports OMP_NUM_THREADS=16) only spins on
        the platform's few reserved CPUs next to the ingress and the load generator."""
        n = os.environ.get("TT_BACKING_MATH_THREADS", "1")
        return {**self.base_env, "OMP_NUM_THREADS": n, "OPENBLAS_NUM_THREADS": n, "MKL_NUM_THREADS": n}

    def start_backing(self, data_dir: str | None = None, policy: dict[str, Any] | None = None,
                      timeout: float = 60.0) -> str:
        pf = self.root / "backing.port"
        if pf.exists():
            pf.unlink()
        args = [sys.executable, "-m", "aca_dotnet_workshop_amd.backing.server", "--port", "0", "--port-file", str(pf)]
        args += self._uds_args("")
        if data_dir:
            args += ["--data-dir", data_dir]
        if policy:
            pp = self.root / "policy.json"
            pp.write_text(json.dumps(policy))
            args += ["--policy", str(pp)]
        self.backing_proc = self._spawn(args, self._backing_env(), "backing", role="platform")
        port = _wait_file(pf, timeout, self.backing_proc)
        self.backing_url = f"http://127.0.0.1:{port}"
        self._backing_args = args
        self._backing_port = int(port)
        return self.backing_url

    def backing_alive(self) -> bool:
        return self.backing_proc is not None and self.backing_proc.poll() is None

    def restart_backing(self, timeout: float = 60.0) -> str:
        """Start the backing-services process again on the SAME port (sidecars keep their URL)
        over the same data directory: documents, messages, subscriptions and locks come back from
        the engines' durable logs (replayed on open)."""
        if self.backing_proc is not None and self.backing_proc.poll() is None:
            self.backing_proc.kill()
            self.backing_proc.wait()
        pf = self.root / "backing.port"
        if pf.exists():
            pf.unlink()
        args = list(self._backing_args)
        args[args.index("--port") + 1] = str(self._backing_port)
        deadline = time.time() + timeout
        while True:  # the old listener's port may take a moment to be released
            self.backing_proc = self._spawn(args, self._backing_env(), "backing", role="platform")
            try:
                _wait_file(pf, max(1.0, deadline - time.time()), self.backing_proc)
                return self.backing_url
            except Exception:
                if time.time() > deadline:
                    raise
                time.sleep(0.2)

    def start_backing_family(self, families: list[str], timeout: float = 60.0) -> str:
        """Run a separate backing-services process for some service families (e.g.
        ``["SERVICEBUS", "STORAGE"]``); replicas started afterwards route those families to it."""
        tag = "-".join(f.lower() for f in families)
        pf = self.root / f"backing-{tag}.port"
        if pf.exists():
            pf.unlink()
        args = [sys.executable, "-m", "aca_dotnet_workshop_amd.backing.server", "--port", "0", "--port-file", str(pf)]
        uds = self._uds_args(tag)
        p = self._spawn(args + uds, self._backing_env(), f"backing-{tag}", role="platform")
        url = f"http://127.0.0.1:{_wait_file(pf, timeout, p)}"
        for f in families:
            self.extra_backing[f] = (p, url)
            self.base_env[f"TT_BACKING_URL_{f}"] = url
            if uds:
                self.base_env[f"TT_BACKING_UDS_{f}"] = uds[1]
        return url

    def _uds_args(self, tag: str) -> list[str]:
        """The backing process also serves on a Unix socket in this stack's socket dir; the
        replicas started afterwards reach it there (``TT_BACKING_UDS``, sidecar/base.py) while
        the TCP URL stays the environment's address for everything else.  ``TT_BACKING_TRANSPORT=
        tcp`` keeps every process on TCP."""
        if os.environ.get("TT_BACKING_TRANSPORT", "uds").lower() == "tcp":
            return []
        path = str(self.sock_dir / (f"backing-{tag}.sock" if tag else "backing.sock"))
        if len(path.encode()) >= 104:
            return []
        if not tag:
            self.base_env["TT_BACKING_UDS"] = path
        return ["--uds", path]

    def shared_info(self) -> dict[str, Any]:
        """What another stack needs to join this one's backing services and name registry."""
        return {"backing": self.backing_url, "registry": str(self.registry),
                "families": {f: url for f, (_p, url) in self.extra_backing.items()}}

    def attach(self, info: dict[str, Any]) -> None:
        """Join another stack's backing services (Cosmos/Service Bus/Storage equivalents) and
        name registry instead of starting our own: replicas started afterwards share its state
        store and compete on its subscriptions (one environment spread over several hosts'
        worth of replicas)."""
        self.backing_url = info["backing"]
        self.registry = Path(info["registry"])
        for f, url in info.get("families", {}).items():
            self.base_env[f"TT_BACKING_URL_{f}"] = url

    def backing_url_for(self, family: str) -> str:
        return self.extra_backing[family][1] if family in self.extra_backing else self.backing_url

    def start_replica(self, app_id: str, config: dict[str, str] | None = None, extra_env: dict[str, str] | None = None,
                      http_port: int | None = None, module: str | None = None, log_level: str = "warning",
                      identity: str | None = None, external_port: int | None = None,
                      api_logging: bool = False, grpc: bool = False,
                      container: dict[str, Any] | None = None) -> ReplicaProc:
        """``grpc``: the sidecar also serves its gRPC API and the app's SDK uses it
        (``Dapr:ApiProtocol=grpc``), the transport of the reference's .NET ``DaprClient``.

        ``container`` = ``{"rootfs", "config"}`` of a pulled image (``registry.unpack``): the app
        runs the image's entrypoint inside the image's root filesystem -- ``chroot`` as the image's
        ``User`` when the platform runs as root, otherwise the host interpreter over the image's
        ``/app`` (``isolation: none``) -- with only the image's ``Env`` plus the app settings.  Like
        a container sharing the replica's network namespace with its sidecar, it reaches the sidecar
        on ``DAPR_HTTP_PORT``/``DAPR_GRPC_PORT`` and serves a TCP port the sidecar calls."""
        idx = self._seq
        self._seq += 1
        name = f"{app_id}-{idx}"
        app_uds = str(self.sock_dir / f"{name}.a.sock")
        port_file = str(self.root / f"{name}.app.port")
        env = dict(self.base_env)
        env.update({"TT_BACKING_URL": self.backing_url or "", "TT_REGISTRY_DIR": str(self.registry),
                    "TT_REPLICA_NAME": name, "TT_APP_UDS": app_uds, "TT_PORT_FILE": port_file,
                    "TT_IDENTITY": identity or app_id})
        for k, v in (config or {}).items():
            env[k.replace(":", "__")] = str(v)
        env.update(extra_env or {})
        urls = f"http://127.0.0.1:{external_port if external_port is not None else 0}"
        args = [sys.executable, "-m", "aca_dotnet_workshop_amd.sidecar", "run", "--app-id", app_id,
                "--app-uds", app_uds, "--dapr-http-port", str(http_port if http_port is not None else 0),
                "--unix-socket-dir", str(self.sock_dir), "--replica-name", name, "--log-level", log_level]
        for c in self.components:
            args += ["--resources-path", c]
        if api_logging:
            args.append("--enable-api-logging")
        if grpc:
            args += ["--dapr-grpc-port", "0"]
            env["Dapr__ApiProtocol"] = "grpc"
        if container is None:
            args += ["--", sys.executable, "-m", module or SERVICE_MODULES[app_id], "--urls", urls]
            p = self._spawn(args, env, name)
            rp = ReplicaProc(app_id, name, p, str(self.sock_dir / f"{name}.d.sock"), http_port, port_file,
                             app_uds=app_uds)
        else:
            app_port = free_port()
            cmd, app_env, isolation = container_command(container, f"http://127.0.0.1:{app_port}")
            for k, v in (config or {}).items():
                app_env[k.replace(":", "__")] = str(v)
            for k, v in (extra_env or {}).items():  # the app's settings; platform paths stay outside
                if not k.startswith(("TT_MTLS_", "TT_INTERNAL_URL_")):
                    app_env[k] = v
            for k in ("TT_APP_HOST", "TT_REPLICA_NAME", "Dapr__ApiProtocol"):
                if k in env:
                    app_env[k] = env[k]
            env_file = self.root / f"{name}.app-env.json"
            env_file.write_text(json.dumps(app_env))
            i = args.index("--app-uds")
            args[i:i + 2] = ["--app-port", str(app_port)]
            args += ["--app-env-file", str(env_file), "--"] + cmd
            p = self._spawn(args, env, name)
            rp = ReplicaProc(app_id, name, p, str(self.sock_dir / f"{name}.d.sock"), http_port, None,
                             fixed_app_port=app_port, container={**container, "isolation": isolation})
        self.replicas.setdefault(app_id, []).append(rp)
        return rp

    def wait_ready(self, timeout: float = 90.0, replicas: list[ReplicaProc] | None = None) -> None:
        """Sidecar socket up and the app handshake (subscriptions/bindings) complete."""
        deadline = time.time() + timeout
        pending = list(replicas or [r for rs in self.replicas.values() for r in rs])
        while pending:
            for r in list(pending):
                if not r.alive():
                    raise RuntimeError(f"replica {r.name} exited with {r.proc.returncode}; "
                                       f"see {self.log_dir / (r.name + '.log')}")
                meta = uds_get_json(r.sidecar_uds, "/v1.0/metadata")
                if meta and meta.get("extended", {}).get("appReady"):
                    pending.remove(r)
            if time.time() > deadline:
                raise TimeoutError(f"replicas not ready: {[r.name for r in pending]}")
            time.sleep(0.05)

    def cpu_seconds(self, part: str = "total") -> dict[str, float]:
        """User+system (``part="system"``: kernel-mode only) CPU seconds consumed so far by every
        process of the stack, keyed by role (``backing``, ``backing-<families>``,
        ``<replica>.sidecar``, ``<replica>.app``).  Used by ``bench.py`` to attribute where the
        end-to-end flow spends its cycles."""
        import psutil

        def cpu(pid: int) -> float:
            try:
                t = psutil.Process(pid).cpu_times()
                return t.system if part == "system" else t.user + t.system
            except psutil.Error:
                return 0.0

        out: dict[str, float] = {}
        if self.backing_proc is not None:
            out["backing"] = cpu(self.backing_proc.pid)
        seen = {self.backing_proc.pid} if self.backing_proc is not None else set()
        for fam, (p, _url) in self.extra_backing.items():
            if p.pid not in seen:  # one process may serve several service families
                seen.add(p.pid)
                out[f"backing-{fam.lower()}"] = cpu(p.pid)
        for rs in self.replicas.values():
            for r in rs:
                out[f"{r.name}.sidecar"] = cpu(r.proc.pid)
                try:
                    kids = psutil.Process(r.proc.pid).children(recursive=True)
                except psutil.Error:
                    kids = []
                dp = [k for k in kids if _is_dataplane(k)]
                if dp:
                    out[f"{r.name}.dataplane"] = sum(cpu(k.pid) for k in dp)
                out[f"{r.name}.app"] = sum(cpu(k.pid) for k in kids if k not in dp)
        return out

    def thread_cpu(self, extra: dict[str, int] | None = None) -> dict[tuple[str, str, int], tuple[float, float]]:
        """(user, kernel) CPU seconds so far of every thread of the stack's processes (plus
        ``extra``: role -> pid), keyed by (role, thread name, tid): which single thread saturates
        first under load (an event loop at 100 % caps throughput while the process as a whole
        looks idle), and how much of it is system calls."""
        import psutil
        tick = os.sysconf("SC_CLK_TCK")
        procs: dict[str, list[int]] = {}
        if self.backing_proc is not None:
            procs["backing"] = [self.backing_proc.pid]
        for fam, (p, _url) in self.extra_backing.items():
            procs.setdefault(f"backing-{fam.lower()}", []).append(p.pid)
        for rs in self.replicas.values():
            for r in rs:
                procs[f"{r.name}.sidecar"] = [r.proc.pid]
                try:
                    kids = psutil.Process(r.proc.pid).children(recursive=True)
                except psutil.Error:
                    kids = []
                dp = [k for k in kids if _is_dataplane(k)]
                procs[f"{r.name}.dataplane"] = [k.pid for k in dp]
                procs[f"{r.name}.app"] = [k.pid for k in kids if k not in dp]
        for role, pid in (extra or {}).items():
            procs.setdefault(role, []).append(pid)
        out: dict[tuple[str, str, int], float] = {}
        for role, pids in procs.items():
            for pid in pids:
                try:
                    tids = os.listdir(f"/proc/{pid}/task")
                except OSError:
                    continue
                for t in tids:
                    try:
                        with open(f"/proc/{pid}/task/{t}/stat", "rb") as f:
                            raw = f.read()
                        lp, rp = raw.find(b"("), raw.rfind(b")")
                        fields = raw[rp + 2:].split()
                        # fields[11], [12] = utime, stime (stat fields 14 and 15) in clock ticks
                        out[(role, raw[lp + 1:rp].decode(errors="replace"), int(t))] = \
                            (int(fields[11]) / tick, int(fields[12]) / tick)
                    except (OSError, IndexError, ValueError):  # the thread ended while being read
                        continue
        return out

    def stop_replica(self, r: ReplicaProc, timeout: float = 10.0) -> None:
        _terminate(r.proc, timeout)
        if r in self.replicas.get(r.app_id, []):
            self.replicas[r.app_id].remove(r)

    def stop(self) -> None:
        for rs in list(self.replicas.values()):
            for r in list(rs):
                try:
                    r.proc.send_signal(signal.SIGTERM)
                except ProcessLookupError:
                    pass
        for rs in list(self.replicas.values()):
            for r in list(rs):
                _terminate(r.proc, 10.0)
        self.replicas.clear()
        if self.backing_proc is not None:
            _terminate(self.backing_proc, 10.0)
            self.backing_proc = None
        for p, _ in {id(p): (p, u) for p, u in self.extra_backing.values()}.values():
            _terminate(p, 10.0)
        self.extra_backing.clear()
        import shutil
        shutil.rmtree(self.sock_dir, ignore_errors=True)

    def __enter__(self) -> "LocalStack":
        return self

    def __exit__(self, *exc) -> None:
        self.stop()


def free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def container_command(container: dict[str, Any], urls: str) -> tuple[list[str], dict[str, str], str]:
    """(argv, environment, isolation) that run an unpacked image's entrypoint serving ``urls``."""
    cfg = container["config"]
    rootfs = Path(container["rootfs"])
    env = dict(e.split("=", 1) for e in cfg.get("Env") or [])
    env.update({"ASPNETCORE_URLS": urls, "TT_LOG_CONSOLE": "1", "PATH": "/usr/local/bin:/usr/bin:/bin"})
    entry = list(cfg["Entrypoint"]) + list(cfg.get("Cmd") or [])
    if os.geteuid() == 0:
        from .image import populate_dev
        populate_dev(rootfs)
        chroot = shutil.which("chroot") or "/usr/sbin/chroot"
        return [chroot, f"--userspec={cfg.get('User') or '0:0'}", str(rootfs)] + entry, env, "chroot"
    # no privileges for a root-filesystem switch: the image's code on the host interpreter
    env["PYTHONPATH"] = str(rootfs / cfg.get("WorkingDir", "/app").lstrip("/"))
    return [sys.executable] + entry[1:], env, "none"


def _is_dataplane(p) -> bool:
    try:
        cmd = p.cmdline()
    except Exception:
        return False
    return bool(cmd) and cmd[0].endswith("ttsidecar-dataplane")


def _terminate(p: subprocess.Popen, timeout: float) -> None:
    if p.poll() is not None:
        return
    try:
        p.send_signal(signal.SIGTERM)
        p.wait(timeout)
    except subprocess.TimeoutExpired:
        try:
            os.killpg(p.pid, signal.SIGKILL)
        except ProcessLookupError:
            pass
        p.wait(5)
    except ProcessLookupError:
        pass


def _wait_file(path: Path, timeout: float, proc: subprocess.Popen | None = None) -> int:
    deadline = time.time() + timeout
    while time.time() < deadline:
        if path.exists():
            try:
                return int(path.read_text())
            except ValueError:
                pass
        if proc is not None and proc.poll() is not None:
            raise RuntimeError(f"process exited with {proc.returncode} before writing {path}")
        time.sleep(0.02)
    raise TimeoutError(f"{path} not written in {timeout}s")


def uds_get_json(sock: str, path: str, timeout: float = 2.0) -> Any:
    """Tiny blocking HTTP GET over a Unix socket (readiness probes)."""
    import socket
    if not os.path.exists(sock):
        return None
    try:
        s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        s.settimeout(timeout)
        s.connect(sock)
        s.sendall(f"GET {path} HTTP/1.1\r\nHost: localhost\r\nConnection: close\r\n\r\n".encode())
        data = b""
        while True:
            chunk = s.recv(65536)
            if not chunk:
                break
            data += chunk
        s.close()
        head, _, body = data.partition(b"\r\n\r\n")
        if not head.startswith(b"HTTP/1.1 200"):
            return None
        return json.loads(body) if body else None
    except (OSError, ValueError):
        return None


def http_get_json(url: str, timeout: float = 2.0) -> Any:
    try:
        with urllib.request.urlopen(url, timeout=timeout) as r:
            return json.loads(r.read() or b"null")
    except (OSError, ValueError):
        return None
