"""Service host -- the ``WebApplication.CreateBuilder(args)`` / ``app.Run()`` equivalent.

``create_host(role, content_root)`` loads layered configuration, configures structured
logging and the tracer with the service's cloud role name (the reference's
``AppInsightsTelemetryInitializer`` classes), and returns a ``WebApp`` with the standard
pipeline: tracing -> metrics -> (service middlewares) -> routing.  ``/healthz`` and
``/metrics`` are always mapped (used by the platform's probes and scaler).

``run_host(app)`` binds the listener the way ASP.NET does: ``--urls`` /
``ASPNETCORE_URLS`` (``http://+:8080`` in the reference Dockerfiles, e.g.
Backend.Api/Dockerfile:3-5) or ``APP_PORT``; optionally a Unix socket ``TT_APP_UDS``
for the co-located sidecar.  SIGTERM/SIGINT trigger a graceful drain.
"""
from __future__ import annotations

import asyncio
import gc
import logging
import os
import signal
import sys
from pathlib import Path
from typing import Any, Callable

from ..telemetry import REGISTRY, configure, configure_logging
from ..telemetry.metrics import request_telemetry_middleware
from ..telemetry.profiler import maybe_profile
from ..utils import gctrace
from ..utils.config import Configuration, load_configuration
from ..web.app import WebApp
from ..web.http import Response, empty, json_response, text_response
from ..web.server import HttpServer

log = logging.getLogger("hosting")


def create_host(role: str, content_root: str | os.PathLike | None = None, argv: list[str] | None = None,
                config: Configuration | None = None, overrides: dict[str, Any] | None = None) -> WebApp:
    if config is None:
        config = load_configuration(content_root, argv=argv or [], overrides=overrides)
    role = config.get_str("TT_ROLE_NAME") or role
    configure_logging(role, config)
    tr = configure(role)
    app = WebApp(role, config)
    app.services["config"] = config
    app.services["tracer"] = tr
    app.use(request_telemetry_middleware())  # request span + request metrics

    async def healthz(req) -> Response:
        return empty(204)

    async def metrics(req) -> Response:
        return text_response(REGISTRY.expose())

    app.add_route("/healthz", healthz, ("GET",), include_in_schema=False)
    app.add_route("/metrics", metrics, ("GET",), include_in_schema=False)

    async def _flush() -> None:
        tr.flush()
    app.on_shutdown.append(_flush)
    return app


def map_openapi(app: WebApp, path: str = "/openapi/v1.json") -> None:
    """``if (app.Environment.IsDevelopment()) app.MapOpenApi();``"""
    if not app.is_development:
        return

    async def doc(req) -> Response:
        return json_response(app.openapi())
    app.add_route(path, doc, ("GET",), include_in_schema=False)


def parse_urls(urls: str | None) -> list[tuple[str, str, int]]:
    """``http://+:8080;https://localhost:7112`` -> [(scheme, host, port)]."""
    out = []
    for u in (urls or "").split(";"):
        u = u.strip()
        if not u:
            continue
        scheme, sep, rest = u.partition("://")
        if not sep:
            scheme, rest = "http", u
        rest = rest.rstrip("/")
        host, _, port = rest.rpartition(":")
        if host in ("+", "*", "[::]", "0.0.0.0", ""):
            host = "0.0.0.0"
        elif host == "localhost":
            host = "127.0.0.1"
        out.append((scheme.lower(), host, int(port)))
    return out


def listen_addresses(config: Configuration) -> list[tuple[str, str, int]]:
    urls = config.get_str("urls") or config.get_str("ASPNETCORE_URLS")
    addrs = parse_urls(urls)
    if not addrs:
        port = config.get_int("APP_PORT", config.get_int("PORT", 8080))
        addrs = [("http", config.get_str("APP_HOST", "127.0.0.1"), port)]
    return addrs


def https_certificate(config: Configuration) -> tuple[str, str]:
    """Kestrel's default certificate: ``Kestrel:Certificates:Default:Path/KeyPath`` when
    configured, else a development certificate for localhost (``dotnet dev-certs https``
    equivalent), issued once under ``TT_DEV_CERTS_DIR`` (default ``~/.tt-dev-certs``)."""
    cert = config.get_str("Kestrel:Certificates:Default:Path")
    key = config.get_str("Kestrel:Certificates:Default:KeyPath")
    if cert and key:
        return cert, key
    from ..platform.pki import EnvironmentPki
    d = config.get_str("TT_DEV_CERTS_DIR") or os.path.join(os.path.expanduser("~"), ".tt-dev-certs")
    pair = EnvironmentPki(d, trust_domain="localhost-dev").server("aspnetcore-dev")
    return pair.cert, pair.key


def https_redirect_app(https_port: int) -> WebApp:
    """``app.UseHttpsRedirection()`` (reference Backend.Api/Program.cs:26): every request on the
    plain-HTTP endpoint is answered 307 Temporary Redirect to the HTTPS one."""
    app = WebApp("https-redirection")

    async def redirect(req) -> Response:
        host = req.headers.get("host") or "localhost"
        if host.startswith("["):  # [v6]:port
            host = host[:host.find("]") + 1]
        elif ":" in host:
            host = host.rpartition(":")[0]
        return Response(b"", 307, [("Location", f"https://{host}:{https_port}{req.target}")])
    app.add_route("/{*path}", redirect, ("GET", "POST", "PUT", "DELETE", "PATCH", "HEAD", "OPTIONS"))
    app.add_route("/", redirect, ("GET", "POST", "PUT", "DELETE", "PATCH", "HEAD", "OPTIONS"))
    return app


def tune_gc(environ: dict[str, str] | None = None) -> bool:
    """Server-process GC settings (the .NET server-GC analogue): objects alive after startup
    (modules, routes, DI graph) move to the permanent generation, and young collections run
    every ``TT_GC_GEN0`` allocations instead of 700 -- a request allocates a few hundred
    short-lived objects, so the default threshold collects several times per request batch.
    ``TT_GC_GEN0=0`` keeps the interpreter defaults."""
    env = os.environ if environ is None else environ
    gen0 = int(env.get("TT_GC_GEN0", "20000"))
    if gen0 <= 0:
        return False
    gc.collect()
    gc.freeze()
    gc.set_threshold(gen0, 20, 50)
    return True


async def serve_host(app: WebApp, stop: asyncio.Event | None = None,
                     ready: Callable[[list[int]], None] | None = None) -> None:
    config: Configuration = app.services["config"]
    loop = asyncio.get_running_loop()
    from ..web import native_host
    srv = native_host.NativeHttpServer(app, loop) if native_host.enabled(part="server") else HttpServer(app, loop)
    # routes the service hands to the native host's I/O thread (``native_routes`` specs; off
    # with TT_NATIVE_ROUTES=0, or on the asyncio server)
    if isinstance(srv, native_host.NativeHttpServer) and os.environ.get("TT_NATIVE_ROUTES", "1") != "0":
        for spec in app.services.get("native_routes") or []:
            try:
                srv.native_route(spec["kind"], spec["method"], spec["path"], spec["route"], spec["cfg"])
            except ValueError as e:  # the definition holds text the native route cannot reproduce
                log.warning("native route %s %s declined: %s (the Python handler serves it)",
                            spec["method"], spec["path"], e)
    await app.startup()
    ports = []
    addrs = listen_addresses(config)
    extra: list[HttpServer] = []
    https_port = None
    for scheme, host, port in addrs:  # HTTPS endpoints first: the redirect needs their port
        if scheme != "https":
            continue
        cert, key = https_certificate(config)
        if isinstance(srv, HttpServer):
            from ..platform.pki import CertPair
            p = await srv.listen_tcp(host, port, ssl=CertPair(cert, key, "").server_context())
        else:
            p = await srv.listen_tcp(host, port, tls_files=(cert, key))
        https_port = https_port or p
        ports.append(p)
    redirect = https_port is not None and config.get_bool("HttpsRedirection:Enabled", True)
    for scheme, host, port in addrs:
        if scheme == "https":
            continue
        if redirect:  # UseHttpsRedirection: the HTTP endpoint only redirects
            r = HttpServer(https_redirect_app(https_port), loop)
            ports.append(await r.listen_tcp(host, port))
            extra.append(r)
        else:
            ports.append(await srv.listen_tcp(host, port))
    uds = config.get_str("TT_APP_UDS")
    if uds:
        await srv.listen_unix(uds)
    stop = stop or asyncio.Event()
    for sig in (signal.SIGTERM, signal.SIGINT):
        try:
            loop.add_signal_handler(sig, stop.set)
        except (NotImplementedError, RuntimeError):
            pass
    log.info("%s listening on %s%s", app.name, ports, f" + {uds}" if uds else "")
    tune_gc()
    gctrace.install(app.name)
    if ready:
        ready(ports)
    port_file = config.get_str("TT_PORT_FILE")
    if port_file:
        tmp = port_file + ".tmp"
        Path(tmp).write_text(str(ports[0]) if ports else "0")
        os.replace(tmp, port_file)
    await stop.wait()
    for r in extra:
        await r.close()
    await srv.close()
    await app.shutdown()


def run_host(app: WebApp) -> None:
    try:
        with maybe_profile(f"{os.environ.get('TT_REPLICA_NAME') or app.name}.app"):
            asyncio.run(serve_host(app))
    except KeyboardInterrupt:
        pass
    sys.exit(0)
