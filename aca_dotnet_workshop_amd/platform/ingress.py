"""Environment ingress: the Container Apps ingress (Envoy) equivalent.

* **external** ingress (the frontend, reference webapp-frontend-service.bicep:54-57): a public
  listener load-balancing across the app's ready replicas; with ``transport: auto`` it serves
  HTTPS with a certificate from the environment CA and a plain-HTTP listener next to it
  answers ``301`` to the HTTPS URL (``allowInsecure: false``) or proxies too;
* **internal** ingress (the API, webapi-backend-service.bicep:94-97): reachable from inside
  the environment only; the public listener answers **403 Forbidden**, which is exactly what
  the workshop's module-2 check expects when the internal FQDN is called from outside
  (docs/aca/02-aca-comm/index.md:278);
* revision traffic splitting (``traffic: [{revision, weight}]``);
* in-flight request accounting (the ``http`` scale rule's metric) and access counters.

Two data planes behind one control interface (``make_ingress``):

* ``NativeIngress`` (default) -- ``native/bin/ttingress`` (``native/src/ingress.cpp``): epoll
  event loops sharing the public port, OpenSSL TLS termination, keep-alive upstream pools per
  replica, least-in-flight replica choice inside the weighted revision.  This module is its
  control plane: it writes the listener config, starts the process, pushes the replica set
  (``PUT /backends`` on the control socket) and reads the counters from the shared stats file.
* ``Ingress`` -- the asyncio proxy, kept for environments without the native binary
  (``TT_INGRESS=python``); same routing and replay rules.
"""
from __future__ import annotations

import asyncio
import itertools
import json
import mmap
import os
import random
import socket
import struct
import subprocess
import time
from dataclasses import dataclass, field
from pathlib import Path

from ..web.app import WebApp
from ..web.client import ConnectionClosed, HttpClient
from ..web.http import Request, Response, json_response, problem
from ..web.server import HttpServer

_HOP = {"connection", "keep-alive", "transfer-encoding", "content-length", "upgrade", "te", "trailer", "host"}


@dataclass
class Backend:
    revision: str
    url: str


@dataclass
class IngressRoute:
    app: str
    external: bool
    backends: list[Backend] = field(default_factory=list)
    weights: dict[str, int] = field(default_factory=dict)  # revision -> percent
    inflight: int = 0
    requests: int = 0
    failures: int = 0
    _rr: itertools.count = field(default_factory=itertools.count)

    def pick(self) -> list[Backend]:
        if not self.backends:
            return []
        revs = sorted({b.revision for b in self.backends})
        if self.weights:
            live = [(r, self.weights.get(r, 0)) for r in revs if self.weights.get(r, 0) > 0]
            if live:
                total = sum(w for _, w in live)
                x = random.uniform(0, total)
                acc = 0.0
                for r, w in live:
                    acc += w
                    if x <= acc:
                        revs = [r] + [o for o in revs if o != r]
                        break
        ordered: list[Backend] = []
        for r in revs:
            bs = [b for b in self.backends if b.revision == r]
            n = next(self._rr) % len(bs)
            ordered += bs[n:] + bs[:n]
        return ordered


def _server_context(tls):
    """``tls``: an ``ssl.SSLContext`` or a ``platform.pki.CertPair`` (files)."""
    if tls is None or not hasattr(tls, "server_context"):
        return tls
    return tls.server_context()


class Ingress:
    """The asyncio ingress (``TT_INGRESS=python``)."""

    native = False

    def __init__(self, route: IngressRoute, http: HttpClient | None = None) -> None:
        self.route = route
        self.http = http or HttpClient()
        self.public: HttpServer | None = None
        self.internal: HttpServer | None = None
        self.insecure: HttpServer | None = None
        self.public_port: int | None = None
        self.insecure_port: int | None = None  # plain-HTTP listener next to an HTTPS one
        self.tls = False

    # -- control interface shared with NativeIngress --------------------------------------
    def set_backends(self, backends: list[Backend], weights: dict[str, int]) -> None:
        self.route.backends = backends
        self.route.weights = weights

    @property
    def inflight(self) -> int:
        return self.route.inflight

    @property
    def requests(self) -> int:
        return self.route.requests

    def describe(self) -> dict:
        return {"dataPlane": "python"}

    def _app(self, internal_listener: bool) -> WebApp:
        app = WebApp(f"ingress-{self.route.app}")
        ing = self

        async def proxy(req: Request) -> Response:
            if not internal_listener and not ing.route.external:
                return problem(403, detail=f"{ing.route.app} has internal ingress only")
            return await ing.forward(req)

        async def stats(req: Request) -> Response:
            r = ing.route
            return json_response({"app": r.app, "inflight": r.inflight, "requests": r.requests, "failures": r.failures,
                                  "backends": [b.__dict__ for b in r.backends], "weights": r.weights})

        app.add_route("/.tt/ingress", stats, ("GET",), include_in_schema=False)
        app.add_route("/{*path}", proxy, ("GET", "POST", "PUT", "DELETE", "PATCH", "HEAD", "OPTIONS"))
        app.add_route("/", proxy, ("GET", "POST", "PUT", "DELETE", "PATCH", "HEAD", "OPTIONS"))
        return app

    async def forward(self, req: Request) -> Response:
        r = self.route
        r.inflight += 1
        r.requests += 1
        try:
            headers = [(k, v) for k, v in req.headers.items() if k not in _HOP and not isinstance(v, list)]
            headers.append(("X-Forwarded-For", str(req.client[0]) if isinstance(req.client, tuple) else "local"))
            headers.append(("X-Forwarded-Proto", "https" if req.state.get("tls") is not None else "http"))
            last = None
            for b in r.pick()[:3]:
                try:
                    resp = await self.http.request(req.method, b.url + req.target, headers=headers, body=req.body,
                                                   retry_stale=req.method in _IDEMPOTENT)
                    out = [(k, x) for k, v in resp.headers.items() if k not in _HOP
                           for x in (v if isinstance(v, list) else [v])]
                    return Response(resp.body, resp.status, out)
                except (ConnectionRefusedError, FileNotFoundError) as e:
                    last = e  # nothing was delivered: any method may go to the next replica
                    continue
                except (ConnectionClosed, OSError) as e:
                    # the replica may already have acted on the request: replaying a
                    # non-idempotent one (createTask) on another replica would duplicate it
                    if req.method not in _IDEMPOTENT:
                        r.failures += 1
                        return problem(502, detail=f"{r.app} replica failed mid-request: {e!r}")
                    last = e
                    continue
            r.failures += 1
            return problem(503, detail=f"no healthy replica for {r.app}: {last!r}" if last else f"{r.app} has no replicas")
        finally:
            r.inflight -= 1

    def _redirect_app(self) -> WebApp:
        """``allowInsecure: false``: plain HTTP is answered 301 to the HTTPS endpoint (ACA)."""
        app = WebApp(f"ingress-{self.route.app}-redirect")

        async def redirect(req: Request) -> Response:
            host = (req.headers.get("host") or "127.0.0.1").rpartition(":")[0] or "127.0.0.1"
            return Response(b"", 301, [("Location", f"https://{host}:{self.public_port}{req.target}")])
        for path in ("/{*path}", "/"):
            app.add_route(path, redirect, ("GET", "POST", "PUT", "DELETE", "PATCH", "HEAD", "OPTIONS"))
        return app

    async def start(self, public_port: int | None, internal_uds: str | None, tls=None,
                    allow_insecure: bool = False) -> None:
        """``tls``: an ``ssl.SSLContext`` or a ``CertPair`` -- the public listener serves HTTPS
        (ACA ingress ``transport: auto`` with a managed certificate) and a second, plain-HTTP
        listener either redirects (``allowInsecure: false``, the default) or proxies too."""
        tls = _server_context(tls)
        loop = asyncio.get_running_loop()
        self.public = HttpServer(self._app(False), loop)
        self.public_port = await self.public.listen_tcp("127.0.0.1", public_port or 0, ssl=tls)
        self.tls = tls is not None
        if tls is not None:
            self.insecure = HttpServer(self._app(False) if allow_insecure else self._redirect_app(), loop)
            self.insecure_port = await self.insecure.listen_tcp("127.0.0.1", 0)
        if internal_uds:
            self.internal = HttpServer(self._app(True), loop)
            await self.internal.listen_unix(internal_uds)

    async def stop(self) -> None:
        for s in (self.public, self.internal, self.insecure):
            if s is not None:
                await s.close(1.0)
        await self.http.close()


_IDEMPOTENT = frozenset(("GET", "HEAD", "OPTIONS", "PUT", "DELETE"))

# SharedStats in native/src/ingress.cpp: magic, inflight (signed), requests, failures, forbidden, redirects
_STATS = struct.Struct("<Qq4Q")
_STATS_MAGIC = 0x315352474E495454


class IngressError(RuntimeError):
    pass


def default_threads() -> int:
    """Event loops of a native ingress: ``TT_INGRESS_THREADS``, else one per 8 CPUs (1..4)."""
    raw = os.environ.get("TT_INGRESS_THREADS", "")
    if raw.isdigit() and int(raw) > 0:
        return int(raw)
    return max(1, min(4, (os.cpu_count() or 8) // 8))


class NativeIngress:
    """Control plane of ``native/bin/ttingress`` (see the module docstring)."""

    native = True

    def __init__(self, route: IngressRoute, work_dir: str | os.PathLike, threads: int | None = None) -> None:
        self.route = route
        self.dir = Path(work_dir)
        self.threads = threads or default_threads()
        self.proc: subprocess.Popen | None = None
        self.public_port: int | None = None
        self.insecure_port: int | None = None
        self.tls = False
        self._stats: mmap.mmap | None = None
        base = self.dir / f"{route.app}.ingress"
        self.cfg_file, self.port_file = Path(f"{base}.json"), Path(f"{base}.port")
        self.stats_file, self.control = Path(f"{base}.stats"), f"{base}-ctl.sock"

    # -- control interface ------------------------------------------------------------------
    def set_backends(self, backends: list[Backend], weights: dict[str, int]) -> None:
        self.route.backends = backends
        self.route.weights = weights
        if self.proc is not None:
            self._control("PUT", "/backends", json.dumps(self._routes()).encode())

    def _counters(self) -> tuple[int, int, int, int, int]:
        if self._stats is None:
            return (0, 0, 0, 0, 0)
        magic, *vals = _STATS.unpack_from(self._stats, 0)
        return tuple(vals) if magic == _STATS_MAGIC else (0, 0, 0, 0, 0)  # type: ignore[return-value]

    @property
    def inflight(self) -> int:
        return max(0, self._counters()[0])

    @property
    def requests(self) -> int:
        return self._counters()[1]

    def stats(self) -> dict:
        """The full ``GET /stats`` document (per-replica counters included)."""
        return json.loads(self._control("GET", "/stats"))

    def describe(self) -> dict:
        return {"dataPlane": "native", "threads": self.threads, "pid": self.proc.pid if self.proc else None}

    def _routes(self) -> dict:
        return {"backends": [{"revision": b.revision, "url": b.url} for b in self.route.backends],
                "weights": self.route.weights}

    def _control(self, method: str, path: str, body: bytes = b"") -> bytes:
        """One request on the control socket (local, answered from the ingress's first loop)."""
        s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        try:
            s.settimeout(10.0)
            s.connect(self.control)
            s.sendall(f"{method} {path} HTTP/1.1\r\nhost: ingress\r\ncontent-length: {len(body)}\r\n"
                      "connection: close\r\n\r\n".encode() + body)
            buf = b""
            while True:
                chunk = s.recv(65536)
                if not chunk:
                    break
                buf += chunk
        finally:
            s.close()
        head, _, rest = buf.partition(b"\r\n\r\n")
        status = int(head.split(b" ", 2)[1]) if head else 0
        if status >= 300 or status == 0:
            raise IngressError(f"ingress control {method} {path}: {status} {rest[:200]!r}")
        return rest

    # -- lifecycle --------------------------------------------------------------------------
    async def start(self, public_port: int | None, internal_uds: str | None, tls=None,
                    allow_insecure: bool = False) -> None:
        """``tls``: a ``CertPair`` (certificate and key files the native listener loads)."""
        from ..native.build import build_ingress
        exe = await asyncio.to_thread(build_ingress)
        if tls is not None and not hasattr(tls, "cert"):
            raise IngressError("the native ingress needs certificate files (a CertPair), not an SSLContext")
        self.dir.mkdir(parents=True, exist_ok=True)
        for f in (self.port_file, self.stats_file):
            f.unlink(missing_ok=True)
        cfg = {"app": self.route.app, "external": self.route.external, "public": f"127.0.0.1:{public_port or 0}",
               "tls": {"cert": tls.cert, "key": tls.key} if tls is not None else None,
               "insecure": "127.0.0.1:0" if tls is not None else None, "allowInsecure": bool(allow_insecure),
               "internal": f"unix:{internal_uds}" if internal_uds else None, "control": f"unix:{self.control}",
               "threads": self.threads, "statsFile": str(self.stats_file), "portFile": str(self.port_file),
               **self._routes()}
        self.cfg_file.write_text(json.dumps(cfg))
        from ..parallel import pin_preexec  # the environment's ingress runs on the platform's CPUs
        self.proc = subprocess.Popen([str(exe), str(self.cfg_file)], stdin=subprocess.DEVNULL,
                                     preexec_fn=pin_preexec("platform"))
        deadline = time.monotonic() + 30.0
        while not self.port_file.exists():
            if self.proc.poll() is not None:
                raise IngressError(f"ttingress exited with {self.proc.returncode} (config {self.cfg_file})")
            if time.monotonic() > deadline:
                self.proc.kill()
                raise IngressError("ttingress did not report its ports within 30 s")
            await asyncio.sleep(0.01)
        ports = json.loads(self.port_file.read_text())
        self.public_port = int(ports["public"])
        self.insecure_port = int(ports["insecure"]) or None
        self.tls = bool(ports["tls"])
        with open(self.stats_file, "r+b") as f:
            self._stats = mmap.mmap(f.fileno(), 4096, access=mmap.ACCESS_READ)

    async def stop(self) -> None:
        if self.proc is not None and self.proc.poll() is None:
            self.proc.terminate()
            try:
                await asyncio.to_thread(self.proc.wait, 10)
            except subprocess.TimeoutExpired:
                self.proc.kill()
                await asyncio.to_thread(self.proc.wait, 10)
        if self._stats is not None:
            self._stats.close()
            self._stats = None


def make_ingress(route: IngressRoute, work_dir: str | os.PathLike) -> Ingress | NativeIngress:
    """The native ingress unless ``TT_INGRESS=python`` (or the binary cannot be built here)."""
    if os.environ.get("TT_INGRESS", "native").lower() == "python":
        return Ingress(route)
    try:
        from ..native.build import build_ingress
        build_ingress()
    except Exception:
        if os.environ.get("TT_INGRESS", "").lower() == "native":
            raise
        return Ingress(route)
    return NativeIngress(route, work_dir)


async def make_ingress_async(route: IngressRoute, work_dir: str | os.PathLike) -> Ingress | NativeIngress:
    """``make_ingress`` for an event loop: a first-time native build runs on a worker thread, so
    the controller's loop (health, scaling, the control API) keeps running meanwhile."""
    return await asyncio.to_thread(make_ingress, route, work_dir)


def now_ms() -> int:
    return int(time.time() * 1000)
