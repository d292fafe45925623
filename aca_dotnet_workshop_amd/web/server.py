"""Asyncio HTTP/1.1 server -- the Kestrel equivalent (reference SURVEY.md §2.9 X5).

A ``asyncio.Protocol`` parses requests straight out of the socket buffer (no
per-request stream objects), supports keep-alive, pipelining (responses are written
in request order), ``Expect: 100-continue``, ``Content-Length`` and chunked request
bodies, TCP and Unix-domain-socket listeners, and graceful drain on shutdown.

Handlers are ``async def handler(request) -> Response``.
"""
from __future__ import annotations

import asyncio
import logging
import os
import socket
from collections import deque
from typing import Any, Awaitable, Callable

from .http import Headers, Request, Response, encode_response, problem

log = logging.getLogger("web.server")

Handler = Callable[[Request], Awaitable[Response]]

MAX_HEADER_BYTES = 64 * 1024


def _py_parse_head(head: bytes) -> tuple[str, str, str, dict]:
    lines = head.split(b"\r\n")
    a, b, c = (lines[0].decode("latin-1").split(" ", 2) + ["", ""])[:3]
    headers: dict = {}
    for line in lines[1:]:
        k, sep, v = line.partition(b":")
        if not sep:
            raise ValueError("malformed header line")
        key = k.strip().lower().decode("latin-1")
        val = v.strip().decode("latin-1")
        if key in headers:
            if key == "set-cookie":
                prev = headers[key]
                headers[key] = (prev if isinstance(prev, list) else [prev]) + [val]
            else:
                headers[key] = headers[key] + ", " + val
        else:
            headers[key] = val
    return a, b, c, headers


def _native_parser():
    try:
        from ..native import load
        return load().parse_http_head
    except Exception as e:  # pragma: no cover - build toolchain missing
        log.warning("native HTTP parser unavailable (%s); using the Python parser", e)
        return _py_parse_head


parse_head = _native_parser()
MAX_BODY_BYTES = 256 * 1024 * 1024


class _ChunkedDecoder:
    """Incremental ``Transfer-Encoding: chunked`` decoder: consumes what it can from the front
    of the connection buffer on each call (linear in the body size), enforces
    ``MAX_BODY_BYTES`` on the decoded size and rejects malformed size lines."""

    __slots__ = ("body", "need", "state")

    def __init__(self) -> None:
        self.body = bytearray()
        self.need = 0        # bytes left in the current chunk
        self.state = 0       # 0 size line, 1 data, 2 CRLF after data, 3 trailers

    def feed(self, buf: bytearray) -> bytes | None:
        """Decode from ``buf`` (consumed bytes are deleted); the body when complete, else None."""
        pos = 0
        try:
            while True:
                if self.state == 0:
                    eol = buf.find(b"\r\n", pos)
                    if eol < 0:
                        if len(buf) - pos > 1024:
                            raise ValueError("bad chunk header")
                        return None
                    size_s = bytes(buf[pos:eol]).split(b";")[0].strip()
                    if not size_s or len(size_s) > 16 or any(c not in b"0123456789abcdefABCDEF" for c in size_s):
                        raise ValueError("bad chunk header")
                    size = int(size_s, 16)
                    if size > MAX_BODY_BYTES - len(self.body):
                        raise ValueError("body too large")
                    pos = eol + 2
                    self.need, self.state = size, (1 if size else 3)
                elif self.state == 1:
                    take = min(self.need, len(buf) - pos)
                    self.body += buf[pos:pos + take]
                    pos += take
                    self.need -= take
                    if self.need:
                        return None
                    self.state = 2
                elif self.state == 2:
                    if len(buf) - pos < 2:
                        return None
                    if buf[pos:pos + 2] != b"\r\n":
                        raise ValueError("bad chunk terminator")
                    pos += 2
                    self.state = 0
                else:  # trailers until the empty line
                    eol = buf.find(b"\r\n", pos)
                    if eol < 0:
                        if len(buf) - pos > MAX_HEADER_BYTES:
                            raise ValueError("trailers too large")
                        return None
                    done = eol == pos
                    pos = eol + 2
                    if done:
                        return bytes(self.body)
        finally:
            del buf[:pos]


class HttpServerProtocol(asyncio.Protocol):
    __slots__ = ("server", "transport", "buf", "pending", "queue", "worker", "closed", "peer", "_paused", "tls")

    def __init__(self, server: "HttpServer") -> None:
        self.server = server
        self.transport: asyncio.Transport | None = None
        self.buf = bytearray()
        self.pending = None  # parsed head awaiting body
        self.queue: deque[Request] = deque()
        self.worker: asyncio.Task | None = None
        self.closed = False
        self.peer = None
        self._paused = False
        self.tls = None

    def connection_made(self, transport: asyncio.BaseTransport) -> None:
        self.transport = transport  # type: ignore[assignment]
        self.peer = transport.get_extra_info("peername")
        # TLS connection: {"peer": [names in the client certificate's SAN]} (mutual TLS identity)
        self.tls = None
        if transport.get_extra_info("ssl_object") is not None:
            cert = transport.get_extra_info("peercert") or {}
            self.tls = {"peer": [v for _, v in cert.get("subjectAltName", ())]}
        sock = transport.get_extra_info("socket")
        if sock is not None and sock.family in (socket.AF_INET, socket.AF_INET6):
            try:
                sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            except OSError:
                pass
        elif sock is not None and sock.family == socket.AF_UNIX:
            # a page of query results or a bulk save (200-300 KB) in one write, not split over
            # several loop turns of a busy reader (native/src/evhttp.hpp widen_local_sndbuf)
            try:
                sock.setsockopt(socket.SOL_SOCKET, socket.SO_SNDBUF, 4 << 20)
            except OSError:
                pass
        self.server._conns.add(self)

    def connection_lost(self, exc: Exception | None) -> None:
        self.closed = True
        self.server._conns.discard(self)
        if self.worker is not None and not self.worker.done() and not self.queue:
            pass  # in-flight request completes; its write is skipped

    def data_received(self, data: bytes) -> None:
        self.buf += data
        try:
            self._parse()
        except Exception as e:  # malformed request
            log.debug("bad request from %s: %r", self.peer, e)
            if self.transport is not None and not self.closed:
                self.transport.write(encode_response(problem(400, detail="malformed request"), False))
                self.transport.close()
            self.closed = True

    def _parse(self) -> None:
        buf = self.buf
        while True:
            if self.pending is None:
                idx = buf.find(b"\r\n\r\n")
                if idx < 0:
                    if len(buf) > MAX_HEADER_BYTES:
                        raise ValueError("headers too large")
                    return
                head = bytes(buf[:idx])
                del buf[:idx + 4]
                if not head:
                    continue  # stray CRLF between pipelined requests
                method, target, version, hd = parse_head(head)
                headers = Headers(hd)
                chunked = _ChunkedDecoder() if "chunked" in headers.get("transfer-encoding", "").lower() else None
                length = 0 if chunked else int(headers.get("content-length", "0") or 0)
                if length < 0 or length > MAX_BODY_BYTES:
                    raise ValueError("body too large")
                if headers.get("expect", "").lower() == "100-continue" and self.transport is not None:
                    self.transport.write(b"HTTP/1.1 100 Continue\r\n\r\n")
                self.pending = (method, target, version, headers, length, chunked)
            method, target, version, headers, length, chunked = self.pending
            if chunked:
                body = chunked.feed(buf)
                if body is None:
                    return
            else:
                if len(buf) < length:
                    return
                body = bytes(buf[:length])
                del buf[:length]
            self.pending = None
            req = Request(method, target, headers, body, self.peer, version)
            req.state["conn"] = self  # long polls check conn.closed (the client went away)
            if self.tls is not None:
                req.state["tls"] = self.tls
            self.queue.append(req)
            if self.worker is None or self.worker.done():
                self.worker = self.server.loop.create_task(self._drain())
            if len(self.queue) > 64 and not self._paused and self.transport is not None:
                self.transport.pause_reading()
                self._paused = True

    async def _drain(self) -> None:
        server = self.server
        while self.queue:
            req = self.queue.popleft()
            if self._paused and len(self.queue) < 16 and self.transport is not None:
                self.transport.resume_reading()
                self._paused = False
            server._inflight += 1
            try:
                try:
                    resp = await server.handler(req)
                except Exception:
                    log.exception("unhandled error serving %s %s", req.method, req.target)
                    resp = problem(500)
            finally:
                server._inflight -= 1
            if self.closed or self.transport is None:
                return
            conn = req.headers.get("connection", "").lower()
            keep = (req.version == "HTTP/1.1" and conn != "close") or conn == "keep-alive"
            if server._closing:
                keep = False
            self.transport.write(encode_response(resp, keep, head=req.method == "HEAD"))
            if not keep:
                self.transport.close()
                self.closed = True
                return


class HttpServer:
    def __init__(self, handler: Handler, loop: asyncio.AbstractEventLoop | None = None) -> None:
        self.handler = handler
        self.loop = loop or asyncio.get_event_loop()
        self._servers: list[asyncio.AbstractServer] = []
        self._conns: set[HttpServerProtocol] = set()
        self._inflight = 0
        self._closing = False
        self.sockets: list[socket.socket] = []

    async def listen_tcp(self, host: str = "127.0.0.1", port: int = 0, reuse_port: bool = False,
                         sock: socket.socket | None = None, ssl: Any = None) -> int:
        """``ssl``: an ``ssl.SSLContext`` serves HTTPS (Kestrel's https endpoint); with
        ``verify_mode = CERT_REQUIRED`` clients must present a certificate (mutual TLS)."""
        if sock is not None:
            srv = await self.loop.create_server(lambda: HttpServerProtocol(self), sock=sock, backlog=1024, ssl=ssl)
        else:
            srv = await self.loop.create_server(lambda: HttpServerProtocol(self), host, port,
                                                reuse_address=True, reuse_port=reuse_port or None,
                                                backlog=1024, ssl=ssl)
        self._servers.append(srv)
        s = srv.sockets[0]
        self.sockets.append(s)
        return s.getsockname()[1]

    async def listen_unix(self, path: str, ssl: Any = None) -> str:
        if os.path.exists(path):
            os.unlink(path)
        srv = await self.loop.create_unix_server(lambda: HttpServerProtocol(self), path, backlog=1024, ssl=ssl)
        self._servers.append(srv)
        return path

    @property
    def port(self) -> int:
        for s in self.sockets:
            if s.family in (socket.AF_INET, socket.AF_INET6):
                return s.getsockname()[1]
        raise RuntimeError("no TCP listener")

    async def close(self, grace: float = 5.0) -> None:
        self._closing = True
        for s in self._servers:
            s.close()
        deadline = self.loop.time() + grace
        while self._inflight and self.loop.time() < deadline:
            await asyncio.sleep(0.01)
        for c in list(self._conns):
            if c.transport is not None:
                c.transport.close()
        for s in self._servers:
            try:
                await asyncio.wait_for(s.wait_closed(), 1.0)
            except (asyncio.TimeoutError, Exception):
                pass
        self._servers.clear()


async def serve(handler: Handler, host: str = "127.0.0.1", port: int = 0,
                uds: str | None = None) -> HttpServer:
    srv = HttpServer(handler, asyncio.get_running_loop())
    if port is not None and port >= 0:
        await srv.listen_tcp(host, port)
    if uds:
        await srv.listen_unix(uds)
    return srv
