"""Native I/O host for app processes: HTTP server and client on a C++ epoll thread.

``NativeHttpServer`` and ``NativeHttpClient`` are drop-in equivalents of ``HttpServer`` and
``HttpClient`` whose sockets, HTTP parsing/serialisation, keep-alive pools and timeouts live in
``native/src/apphost.hpp`` (one I/O thread per process and event loop), the way Kestrel runs an
ASP.NET Core app's I/O on native threads while the app code runs elsewhere (reference
SURVEY.md §2.9 X5).  The asyncio thread only runs handlers: it wakes on one eventfd per batch
of completed I/O, turns each event into a ``Request`` (server side) or resolves a future with
a ``ClientResponse`` (client side), and hands responses / new requests back in one call each.

Selected with ``TT_APP_HOST=native`` (``hosting.serve_host`` and the SDK's ``SidecarClient``);
the platform's process launcher (``LocalStack``) sets it for the service processes unless the
environment says otherwise; in-process uses (tests, ``inproc``) keep the asyncio I/O.  Missing extension = hard
error (no silent fallback when the native host was asked for).
"""
from __future__ import annotations

import asyncio
import errno as _errno
import json
import logging
import os
import weakref
from typing import Any, Awaitable, Callable

from .client import ClientResponse, ConnectionClosed, parse_endpoint
from .http import Headers, Request, Response, problem

log = logging.getLogger("web.native")

Handler = Callable[[Request], Awaitable[Response]]


def enabled(environ: dict[str, str] | None = None, part: str = "") -> bool:
    """``TT_APP_HOST=native`` (server and client), or ``native-server`` / ``native-client``."""
    env = os.environ if environ is None else environ
    v = env.get("TT_APP_HOST", "").lower()
    return v == "native" or (bool(part) and v == f"native-{part}")


_native_loggers: dict[str, logging.Logger] = {}


def _native_log(level: int, name: str, message: str, trace_id: str, span_id: str, line: str = "") -> None:
    """A native route's log record, written by this process's logging with the route's trace
    context (what the Python handler's own ``log.info`` inside the request would write).
    ``line``: the record already formatted by the route (the sink's prefix, handed over at
    registration) -- appended as is while that sink still writes these records."""
    if line:
        from ..telemetry.logging import native_line_sink
        sink = native_line_sink(name, level)
        if sink is not None:
            sink._put(line)
            return
    lg = _native_loggers.get(name)
    if lg is None:
        lg = _native_loggers[name] = logging.getLogger(name)
    log_ids = getattr(lg, "log_ids", None)  # telemetry.logging.FastLogger
    if log_ids is not None:
        log_ids(level, message, trace_id, span_id)
        return
    if not lg.isEnabledFor(level):
        return
    from ..telemetry import tracing
    tok = tracing._current.set(tracing.Span(tracing.tracer(), "", "server", trace_id, span_id, None, False, None))
    try:
        lg.log(level, message)
    finally:
        tracing._current.reset(tok)


def _native_lines(level: int, name: str, lines: str) -> None:
    """Native routes' records already formatted as the JSON sink's lines (``_native_log``'s
    ``line``), several at once: appended in one piece while that sink still writes them."""
    from ..telemetry.logging import native_line_sink
    sink = native_line_sink(name, level)
    if sink is not None:
        sink._put(lines)
        return
    for ln in lines.splitlines():  # the sink changed since the route was registered
        try:
            rec = json.loads(ln)
        except ValueError:
            continue
        _native_log(level, name, rec.get("message", ""), rec.get("traceId", ""), rec.get("spanId", ""))


def _client_error(err: int, msg: str) -> BaseException:
    if err == _errno.ECONNREFUSED:
        return ConnectionRefusedError(err, msg)
    if err == _errno.ENOENT:
        return FileNotFoundError(err, msg)
    if err == _errno.ETIMEDOUT:
        return asyncio.TimeoutError("HTTP request timed out")
    return ConnectionClosed(f"{msg} (errno {err})")


class NativeHost:
    """One ``AppHost`` (I/O thread) per event loop."""

    _by_loop: "weakref.WeakKeyDictionary[asyncio.AbstractEventLoop, NativeHost]" = weakref.WeakKeyDictionary()

    @classmethod
    def get(cls, loop: asyncio.AbstractEventLoop | None = None) -> "NativeHost":
        loop = loop or asyncio.get_running_loop()
        h = cls._by_loop.get(loop)
        if h is None or h.closed:
            h = cls._by_loop[loop] = cls(loop)
        return h

    def __init__(self, loop: asyncio.AbstractEventLoop) -> None:
        from ..native import load
        self.loop = loop
        self.h = load().AppHost()
        self.h.start()
        self.fd = self.h.event_fd()
        loop.add_reader(self.fd, self._on_events)
        self.servers: dict[int, NativeHttpServer] = {}
        self.pending: dict[int, asyncio.Future] = {}
        self._next_id = 1
        self._next_server = 1
        self.users = 0
        self.closed = False
        self._ops: list[tuple] = []  # respond/request operations of this loop iteration
        # TT_STALL_LOG=<file>: record every hand-off slower than 20 ms (diagnostics)
        path = os.environ.get("TT_STALL_LOG")
        self._stall = open(path, "a", buffering=1) if path else None
        self._t_submit: dict[int, float] = {}
        self._t_flush: dict[int, tuple[float, str]] = {}
        self._last_wake = 0.0

    def _note(self, what: str, **kw: Any) -> None:
        import time as _t
        kw.update(what=what, pid=os.getpid(), wall=round(_t.time(), 4))
        self._stall.write(json.dumps(kw) + "\n")

    def _on_events_traced(self) -> None:
        import time as _t
        now = _t.monotonic()
        evs = self.h.drain_times()
        if self._last_wake and now - self._last_wake > 0.05:
            self._note("python-idle-gap", gap_ms=round((now - self._last_wake) * 1e3, 2), events=len(evs))
        self._last_wake = now
        if evs:
            lag = now - min(e[-1] for e in evs)
            if lag > 0.02:
                self._note("wake-lag", lag_ms=round(lag * 1e3, 2), batch=len(evs),
                           kinds=sorted({e[0] for e in evs}))
        for ev in evs:
            lag = now - ev[-1]
            kind = ev[0]
            if kind == 3:
                _native_log(*ev[1:7])
                continue
            if kind == 0:
                _, token, sid, method, target, http10, hd, body, _ = ev
                srv = self.servers.get(sid)
                if srv is None:
                    self.respond(token, 503, [], b"")
                    continue
                srv._dispatch(token, method, target, http10, hd, body)
            else:
                rid = ev[1]
                t0 = self._t_submit.pop(rid, None)
                tf = self._t_flush.pop(rid, None)
                if t0 is not None and tf is not None and ev[-1] - tf[0] > 0.02:
                    self._note("client-slow", rid=rid, target=tf[1], queue_ms=round((tf[0] - t0) * 1e3, 2),
                               io_ms=round((ev[-1] - tf[0]) * 1e3, 2), wake_ms=round(lag * 1e3, 2))
                fut = self.pending.pop(rid, None)
                if fut is None or fut.done():
                    continue
                if kind == 1:
                    fut.set_result(ClientResponse(ev[2], Headers(ev[3]), ev[4]))
                else:
                    fut.set_exception(_client_error(ev[2], ev[3]))

    def _queue(self, op: tuple) -> None:
        if not self._ops:
            self.loop.call_soon(self._flush)
        self._ops.append(op)

    def _flush(self) -> None:
        ops, self._ops = self._ops, []
        if self._stall is not None:
            import time as _t
            now = _t.monotonic()
            for op in ops:
                if op[0] == 1:
                    self._t_flush[op[1]] = (now, op[4][:48])
        if ops and not self.closed:
            try:
                self.h.submit(ops)
            except Exception:
                # one malformed operation must not lose the whole batch: retry one by one and
                # fail only the bad ones (500 for a response, an exception for a request)
                for op in ops:
                    try:
                        self.h.submit([op])
                    except Exception as e:
                        log.exception("native host rejected an operation")
                        if op[0] == 0:
                            self.h.submit([(0, op[1], 500, [], b"")])
                        else:
                            fut = self.pending.pop(op[1], None)
                            if fut is not None and not fut.done():
                                fut.set_exception(ValueError(f"invalid request: {e}"))

    def respond(self, token: int, status: int, headers: list, body: bytes) -> None:
        self._queue((0, token, status, headers, body))

    def new_server_id(self, srv: "NativeHttpServer") -> int:
        sid = self._next_server
        self._next_server += 1
        self.servers[sid] = srv
        return sid

    def _on_events(self) -> None:
        if self._stall is not None:
            return self._on_events_traced()
        for ev in self.h.drain():
            try:
                kind = ev[0]
                if kind == 1:  # a client response: resolve the caller's future (headers: lower-cased dict)
                    fut = self.pending.pop(ev[1], None)
                    if fut is not None and not fut.done():
                        fut.set_result(ClientResponse(ev[2], ev[3], ev[4]))
                elif kind == 0:
                    _, token, sid, method, target, http10, hd, body = ev
                    srv = self.servers.get(sid)
                    if srv is None:
                        self.respond(token, 503, [], b"")
                        continue
                    srv._dispatch(token, method, target, http10, hd, body)
                elif kind == 3:  # a native route's log record
                    _native_log(ev[1], ev[2], ev[3], ev[4], ev[5], ev[6])
                elif kind == 4:  # native routes' finished log lines of one logger, batched
                    _native_lines(ev[1], ev[2], ev[3])
                else:
                    fut = self.pending.pop(ev[1], None)
                    if fut is not None and not fut.done():
                        fut.set_exception(_client_error(ev[2], ev[3]))
            except Exception:  # one bad event must not strand the rest of the batch
                log.exception("native host event %r failed", ev[:2])

    def grpc_call(self, endpoint: str, path: str, metadata: list[tuple[str, str]], message: bytes,
                  timeout: float) -> asyncio.Future:
        """A unary gRPC call on the host's HTTP/2 client (h2.hpp GrpcClient).  Resolves to a
        ``ClientResponse`` whose ``status`` is the grpc-status, ``headers`` the response metadata
        (with ``grpc-message``) and ``body`` the serialized response message."""
        rid = self._next_id
        self._next_id += 1
        fut = self.loop.create_future()
        self.pending[rid] = fut
        self._queue((2, rid, endpoint, "", path, metadata, message, timeout))
        return fut

    def request(self, endpoint: str, method: str, target: str, headers: list[tuple[str, str]], body: bytes,
                timeout: float) -> asyncio.Future:
        rid = self._next_id
        self._next_id += 1
        fut = self.loop.create_future()
        self.pending[rid] = fut
        if self._stall is not None:
            import time as _t
            self._t_submit[rid] = _t.monotonic()
        self._queue((1, rid, endpoint, method, target, headers, body, timeout))
        return fut

    def release(self) -> None:
        """Drop one user; the last one stops the I/O thread."""
        self.users -= 1
        if self.users <= 0 and not self.servers and not self.closed:
            self.close()

    def close(self) -> None:
        if self.closed:
            return
        self.closed = True
        try:
            self.loop.remove_reader(self.fd)
        except Exception:
            pass
        self.h.stop()
        try:  # log records the I/O thread held back for its next flush (apphost.hpp emit)
            for ev in self.h.drain():
                if ev[0] == 3:
                    _native_log(ev[1], ev[2], ev[3], ev[4], ev[5], ev[6])
                elif ev[0] == 4:
                    _native_lines(ev[1], ev[2], ev[3])
        except Exception:
            log.exception("native host: flushing log records at close failed")
        for fut in self.pending.values():
            if not fut.done():
                fut.set_exception(ConnectionClosed("native host stopped"))
        self.pending.clear()


class NativeHttpServer:
    """``HttpServer`` on the native host."""

    def __init__(self, handler: Handler, loop: asyncio.AbstractEventLoop | None = None) -> None:
        self.handler = handler
        self.loop = loop or asyncio.get_event_loop()
        self.host = NativeHost.get(self.loop)
        self.host.users += 1
        self.sid = self.host.new_server_id(self)
        self._inflight = 0
        self._closing = False
        self.ports: list[int] = []
        self._routes: dict[int, tuple[str, str]] = {}  # native route id -> (method, route template)
        self._collector = None

    async def listen_tcp(self, host: str = "127.0.0.1", port: int = 0, reuse_port: bool = False,
                         sock=None, tls_files: tuple[str, str] | None = None) -> int:
        """``tls_files``: (certificate, key) PEM paths -- HTTPS, terminated on the I/O thread."""
        if sock is not None:
            raise ValueError("NativeHttpServer binds its own sockets")
        cert, key = tls_files or ("", "")
        p = self.host.h.listen(self.sid, f"tcp:{host}:{port}", cert, key)
        self.ports.append(p)
        return p

    async def listen_unix(self, path: str) -> str:
        self.host.h.listen(self.sid, f"unix:{path}")
        return path

    def native_route(self, kind: str, method: str, path: str, route: str, cfg: dict[str, str]) -> int:
        """Hand ``method path`` to the I/O thread (apphost.hpp NativeRoute ``kind``): it serves
        the requests it can decide end to end and passes the rest to the app as before.  ``route``
        is the route template the request metrics carry; ``cfg`` the route's settings (sidecar
        endpoint, targets, ...).  Its requests are counted into the process's registry."""
        from ..telemetry import REGISTRY, tracing
        from ..telemetry.metrics import _DEFAULT_BUCKETS
        settings = {"method": method, "path": path, "sample_rate": repr(float(tracing.tracer().sample_rate)),
                    **{k: str(v) for k, v in cfg.items()}}
        if cfg.get("log_category"):  # the route formats its lines itself when the fast path would
            from ..telemetry.logging import native_line_prefix
            settings["log_prefix"] = native_line_prefix(cfg["log_category"])
        rid = self.host.h.add_route(self.sid, kind, settings, list(_DEFAULT_BUCKETS))
        self._routes[rid] = (method, route)
        if self._collector is None:
            reqs = REGISTRY.counter("http_requests_total", "HTTP requests served")
            lat = REGISTRY.histogram("http_request_duration_seconds", "HTTP request latency")
            # the share of them the I/O thread served end to end (the rest reached the handlers)
            nat = REGISTRY.counter("native_route_requests_total",
                                   "requests the app host's native routes served end to end")
            keys: dict[tuple, tuple] = {}

            def collect() -> None:
                if self.host.closed:
                    return
                for rid_, status, n, total, buckets in self.host.h.route_stats():
                    m, r = self._routes.get(rid_, ("?", "?"))
                    k = keys.get((rid_, status))
                    if k is None:  # the same label keys as the telemetry middleware's
                        k = keys[(rid_, status)] = (tuple(sorted({"method": m, "route": r, "status": str(status)}.items())),
                                                    (("route", r),))
                    reqs.inc_key(k[0], n)
                    nat.inc_key(k[0], n)
                    lat.merge_key(k[1], buckets, total, n)
            self._collector = collect
            REGISTRY.collectors.append(collect)
        return rid

    @property
    def port(self) -> int:
        if not self.ports:
            raise RuntimeError("no TCP listener")
        return self.ports[0]

    def _dispatch(self, token: int, method: str, target: str, http10: bool, hd: dict, body: bytes) -> None:
        if self.host._stall is not None:
            import time as _t
            note = hd.pop("x-tt-native", None)
            req = Request(method, target, Headers(hd), body, None, "HTTP/1.0" if http10 else "HTTP/1.1")
            if note is not None:
                req.state["tt_native"] = note
            self.loop.create_task(self._serve_traced(token, req, _t.monotonic()))
            self._inflight += 1
            return
        note = hd.pop("x-tt-native", None) if "x-tt-native" in hd else None
        req = Request(method, target, hd, body, None, "HTTP/1.0" if http10 else "HTTP/1.1")
        if note is not None:  # a native route's hand-over (apphost.hpp; clients cannot send it)
            req.state["tt_native"] = note
        self._inflight += 1
        self.loop.create_task(self._serve(token, req))

    async def _serve(self, token: int, req: Request) -> None:
        try:
            try:
                resp = await self.handler(req)
            except Exception:
                log.exception("unhandled error serving %s %s", req.method, req.target)
                resp = problem(500)
            body = resp.body if isinstance(resp.body, bytes) else bytes(resp.body)
            self.host.respond(token, resp.status, resp.headers, body)
        finally:
            self._inflight -= 1

    async def _serve_traced(self, token: int, req: Request, t0: float) -> None:
        import time as _t
        t1 = _t.monotonic()
        await self._serve(token, req)
        t2 = _t.monotonic()
        if t2 - t0 > 0.05:
            self.host._note("handler-slow", target=req.target[:60], start_ms=round((t1 - t0) * 1e3, 2),
                            run_ms=round((t2 - t1) * 1e3, 2))

    async def close(self, grace: float = 5.0) -> None:
        if self._closing:
            return
        self._closing = True
        self.host.h.close_server(self.sid)
        deadline = self.loop.time() + grace
        # Python's requests and the native routes' exchanges still in flight
        while (self._inflight or (self._routes and self.host.h.pending_replies())) and self.loop.time() < deadline:
            await asyncio.sleep(0.01)
        self.host._flush()  # responses queued this iteration go out before the connections close
        self.host.h.close_connections(self.sid)
        self.host.servers.pop(self.sid, None)
        if self._collector is not None:
            from ..telemetry import REGISTRY
            self._collector()  # the last counts
            REGISTRY.collectors.remove(self._collector)
            self._collector = None
        self.host.release()


class NativeHttpClient:
    """``HttpClient`` on the native host (keep-alive pools and timeouts in C++)."""

    def __init__(self, max_idle_per_host: int = 256, timeout: float = 60.0) -> None:
        self.timeout = timeout
        self._host: NativeHost | None = None
        self._endpoints: dict[Any, str] = {}

    def _native(self) -> NativeHost:
        h = self._host
        if h is None or h.closed or h.loop is not asyncio.get_running_loop():
            h = self._host = NativeHost.get()
            h.users += 1
        return h

    async def request(self, method: str, url: str, *, headers: dict[str, str] | list[tuple[str, str]] | None = None,
                      body: bytes | str | None = None, json_body: Any = None,
                      timeout: float | None = None) -> ClientResponse:
        key, target = parse_endpoint(url)
        hdrs = list(headers.items()) if isinstance(headers, dict) else list(headers or [])
        if json_body is not None:
            body = json.dumps(json_body, separators=(",", ":")).encode()
            if not any(k.lower() == "content-type" for k, _ in hdrs):
                hdrs.append(("Content-Type", "application/json"))
        if isinstance(body, str):
            body = body.encode()
        ep = self._endpoints.get(key)
        if ep is None:
            ep = self._endpoints[key] = f"unix:{key[1]}" if key[0] == "unix" else f"tcp:{key[1]}:{key[2]}"
        to = self.timeout if timeout is None else timeout
        return await self._native().request(ep, method, target, hdrs, body or b"", to)

    def request_at(self, key: Any, method: str, target: str, headers: list[tuple[str, str]], body: bytes,
                   timeout: float | None = None) -> "asyncio.Future[ClientResponse]":
        """``request`` to an endpoint already split off by ``parse_endpoint`` (the SDK's sidecar
        endpoint): no URL parsing per call; returns the future of the response."""
        ep = self._endpoints.get(key)
        if ep is None:
            ep = self._endpoints[key] = f"unix:{key[1]}" if key[0] == "unix" else f"tcp:{key[1]}:{key[2]}"
        return self._native().request(ep, method, target, headers, body, self.timeout if timeout is None else timeout)

    async def get(self, url: str, **kw: Any) -> ClientResponse:
        return await self.request("GET", url, **kw)

    async def post(self, url: str, **kw: Any) -> ClientResponse:
        return await self.request("POST", url, **kw)

    async def put(self, url: str, **kw: Any) -> ClientResponse:
        return await self.request("PUT", url, **kw)

    async def delete(self, url: str, **kw: Any) -> ClientResponse:
        return await self.request("DELETE", url, **kw)

    async def close(self) -> None:
        if self._host is not None:
            h, self._host = self._host, None
            h.release()
