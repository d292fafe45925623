"""Environment ingress: the Container Apps ingress (Envoy) equivalent.

* **external** ingress (the frontend, reference webapp-frontend-service.bicep:54-57): a public
  listener load-balancing across the app's ready replicas;
* **internal** ingress (the API, webapi-backend-service.bicep:94-97): reachable from inside
  the environment only; the public listener answers **403 Forbidden**, which is exactly what
  the workshop's module-2 check expects when the internal FQDN is called from outside
  (docs/aca/02-aca-comm/index.md:278);
* revision traffic splitting (``traffic: [{revision, weight}]``) with round-robin across
  replicas of the chosen revision;
* in-flight request accounting (the ``http`` scale rule's metric) and access counters.
"""
from __future__ import annotations

import asyncio
import itertools
import random
import time
from dataclasses import dataclass, field

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


class Ingress:
    def __init__(self, route: IngressRoute, http: HttpClient | None = None) -> None:
        self.route = route
        self.http = http or HttpClient()
        self.public: HttpServer | None = None
        self.internal: HttpServer | None = None
        self.insecure: HttpServer | None = None
        self.public_port: int | None = None
        self.insecure_port: int | None = None  # plain-HTTP listener next to an HTTPS one
        self.tls = False

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
                    resp = await self.http.request(req.method, b.url + req.target, headers=headers, body=req.body)
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
        """``tls``: an ``ssl.SSLContext`` -- the public listener serves HTTPS (ACA ingress
        ``transport: auto`` with a managed certificate) and a second, plain-HTTP listener either
        redirects (``allowInsecure: false``, the default) or proxies too."""
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


def now_ms() -> int:
    return int(time.time() * 1000)
