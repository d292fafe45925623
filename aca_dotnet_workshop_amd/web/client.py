"""Pooled asyncio HTTP/1.1 client.

Used by the SDK (app -> sidecar), by the sidecar (sidecar -> sidecar, sidecar -> app,
sidecar -> backing services) and by tests.  Keep-alive connections are pooled per
endpoint; endpoints are ``(host, port)`` TCP addresses or Unix-domain-socket paths
(``unix:/path/to.sock``) -- the sidecar/app hop defaults to UDS when both sides run on
one host, which removes the TCP loopback stack from every call.
"""
from __future__ import annotations

import asyncio
import json
import socket
from collections import deque
from typing import Any
from urllib.parse import urlsplit

from .http import Headers
from .server import parse_head

DEFAULT_TIMEOUT = 60.0


class ClientResponse:
    __slots__ = ("status", "headers", "body")

    def __init__(self, status: int, headers: Headers, body: bytes) -> None:
        self.status = status
        self.headers = headers
        self.body = body

    def json(self) -> Any:
        return json.loads(self.body) if self.body else None

    @property
    def text(self) -> str:
        return self.body.decode("utf-8", "replace")

    @property
    def ok(self) -> bool:
        return 200 <= self.status < 300

    def __repr__(self) -> str:
        return f"<ClientResponse {self.status} {len(self.body)}B>"


class ConnectionClosed(ConnectionError):
    pass


class _Conn(asyncio.Protocol):
    __slots__ = ("transport", "buf", "fut", "closed", "head", "got_bytes", "reused", "is_head", "key")

    def __init__(self, key: Any) -> None:
        self.key = key
        self.transport: asyncio.Transport | None = None
        self.buf = bytearray()
        self.fut: asyncio.Future | None = None
        self.closed = False
        self.head = None
        self.got_bytes = False
        self.reused = False
        self.is_head = False

    def connection_made(self, transport: asyncio.BaseTransport) -> None:
        self.transport = transport  # type: ignore[assignment]
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

    def connection_lost(self, exc: Exception | None) -> None:
        self.closed = True
        fut = self.fut
        if fut is not None and not fut.done():
            # close-delimited body?
            if self.head is not None and self.head[2] is None:
                status, headers, _ = self.head
                fut.set_result((ClientResponse(status, headers, bytes(self.buf)), False))
            else:
                fut.set_exception(ConnectionClosed(str(exc) if exc else "connection closed"))

    def data_received(self, data: bytes) -> None:
        self.got_bytes = True
        self.buf += data
        if self.fut is None or self.fut.done():
            return
        try:
            self._parse()
        except Exception as e:
            if not self.fut.done():
                self.fut.set_exception(e)
            if self.transport:
                self.transport.close()

    def _parse(self) -> None:
        buf = self.buf
        while self.head is None:
            idx = buf.find(b"\r\n\r\n")
            if idx < 0:
                return
            head = bytes(buf[:idx])
            del buf[:idx + 4]
            _, status_s, _, hd = parse_head(head)
            status = int(status_s)
            if 100 <= status < 200:
                continue  # 100 Continue
            headers = Headers(hd)
            if self.is_head or status in (204, 304):
                length: Any = 0
            elif "chunked" in headers.get("transfer-encoding", "").lower():
                from .server import _ChunkedDecoder
                length = _ChunkedDecoder()
            elif "content-length" in headers:
                length = int(headers["content-length"])
            else:
                length = None  # read until close
            self.head = (status, headers, length)
        status, headers, length = self.head
        keep = headers.get("connection", "").lower() != "close"
        if length is None:
            return
        if not isinstance(length, int):  # chunked
            body = length.feed(buf)
            if body is None:
                return
        else:
            if len(buf) < length:
                return
            body = bytes(buf[:length])
            del buf[:length]
        self.head = None
        self.fut.set_result((ClientResponse(status, headers, body), keep))


def _expire(fut: asyncio.Future) -> None:
    if not fut.done():
        fut.set_exception(asyncio.TimeoutError("HTTP request timed out"))


_SWEEP_S = 0.1  # timeout resolution (per-request TimerHandles cost ~5 us each on the hot path)


def parse_endpoint(url: str) -> tuple[Any, str]:
    """Split ``url`` into (endpoint key, request target).

    ``unix:/path.sock:/target`` | ``http://host:port/target`` | ``https://host:port/target`` |
    ``mtls:<peer-name>@<one of the above>`` -- mutual TLS to a peer whose certificate must carry
    ``<peer-name>`` (the app-id of a sidecar: environment PKI, platform/pki.py)."""
    if url.startswith("mtls:"):
        name, _, rest = url[5:].partition("@")
        inner, target = parse_endpoint(rest)
        if inner[0] == "tls":
            inner = inner[2]
        return ("tls", name, inner), target
    if url.startswith("https://"):
        inner, target = parse_endpoint("http://" + url[8:])
        return ("tls", inner[1], inner), target
    if url.startswith("unix:"):
        # unix:/path/to.sock:/request/target
        rest = url[5:]
        sock, sep, target = rest.partition(".sock")
        sock = sock + ".sock" if sep else sock
        target = target.lstrip(":") or "/"
        return ("unix", sock), target
    sp = urlsplit(url)
    port = sp.port or (443 if sp.scheme == "https" else 80)
    target = sp.path or "/"
    if sp.query:
        target += "?" + sp.query
    return ("tcp", sp.hostname or "127.0.0.1", port), target


class HttpClient:
    def __init__(self, max_idle_per_host: int = 256, timeout: float = DEFAULT_TIMEOUT,
                 tls: "ssl.SSLContext | None" = None) -> None:
        """``tls``: context for ``https://`` / ``mtls:`` endpoints (client certificate for mutual
        TLS, trusted CA); default: the system trust store."""
        self.tls = tls
        self._idle: dict[Any, deque[_Conn]] = {}
        self.max_idle = max_idle_per_host
        self.timeout = timeout
        self._closed = False
        self._deadlines: dict[asyncio.Future, float] = {}
        self._sweeper: asyncio.TimerHandle | None = None
        self._sweep_loop: asyncio.AbstractEventLoop | None = None

    def _sweep(self) -> None:
        """One coarse timer for every in-flight request of this client."""
        self._sweeper = None
        if not self._deadlines:
            return
        loop = asyncio.get_running_loop()
        now = loop.time()
        for fut, dl in list(self._deadlines.items()):
            if fut.done():
                self._deadlines.pop(fut, None)
            elif now >= dl:
                self._deadlines.pop(fut, None)
                _expire(fut)
        if self._deadlines:
            self._sweeper = loop.call_at(now + _SWEEP_S, self._sweep)

    async def _connect(self, key: Any) -> _Conn:
        loop = asyncio.get_running_loop()
        if key[0] == "tls":
            if self.tls is None:
                import ssl
                self.tls = ssl.create_default_context()
            inner = key[2]
            if inner[0] == "unix":
                _, conn = await loop.create_unix_connection(lambda: _Conn(key), inner[1], ssl=self.tls,
                                                            server_hostname=key[1])
            else:
                _, conn = await loop.create_connection(lambda: _Conn(key), inner[1], inner[2], ssl=self.tls,
                                                       server_hostname=key[1])
            return conn
        if key[0] == "unix":
            _, conn = await loop.create_unix_connection(lambda: _Conn(key), key[1])
        else:
            _, conn = await loop.create_connection(lambda: _Conn(key), key[1], key[2])
        return conn

    def _get_idle(self, key: Any) -> _Conn | None:
        dq = self._idle.get(key)
        while dq:
            c = dq.pop()
            if not c.closed:
                return c
        return None

    def _release(self, c: _Conn) -> None:
        if c.closed or self._closed:
            if c.transport:
                c.transport.close()
            return
        dq = self._idle.setdefault(c.key, deque())
        if len(dq) >= self.max_idle:
            c.transport.close()
            return
        dq.append(c)

    async def request(self, method: str, url: str, *, headers: dict[str, str] | list[tuple[str, str]] | None = None,
                      body: bytes | str | None = None, json_body: Any = None,
                      timeout: float | None = None, retry_stale: bool = True) -> ClientResponse:
        """``retry_stale``: a reused keep-alive connection closed before any response byte is
        retried once on a fresh one -- pass False for a non-idempotent request the peer may
        have read (and acted on) before closing."""
        key, target = parse_endpoint(url)
        if json_body is not None:
            body = json.dumps(json_body, separators=(",", ":")).encode()
            hdrs = list(headers.items()) if isinstance(headers, dict) else list(headers or [])
            if not any(k.lower() == "content-type" for k, _ in hdrs):
                hdrs.append(("Content-Type", "application/json"))
        else:
            hdrs = list(headers.items()) if isinstance(headers, dict) else list(headers or [])
        if isinstance(body, str):
            body = body.encode()
        body = body or b""
        inner = key[2] if key[0] == "tls" else key
        host = f"{inner[1]}:{inner[2]}" if inner[0] == "tcp" else "localhost"
        lines = [f"{method} {target} HTTP/1.1", f"Host: {host}"]
        for k, v in hdrs:
            lk = k.lower()
            if lk in ("host", "content-length", "connection", "transfer-encoding"):
                continue
            lines.append(f"{k}: {v}")
        if body or method in ("POST", "PUT", "PATCH"):
            lines.append(f"Content-Length: {len(body)}")
        payload = ("\r\n".join(lines) + "\r\n\r\n").encode("latin-1") + body
        to = self.timeout if timeout is None else timeout
        for attempt in (0, 1):
            conn = self._get_idle(key)
            if conn is None:
                conn = await asyncio.wait_for(self._connect(key), to)
            else:
                conn.reused = True
            loop = asyncio.get_running_loop()
            conn.fut = loop.create_future()
            conn.got_bytes = False
            conn.is_head = method == "HEAD"
            conn.transport.write(payload)
            fut = conn.fut
            self._deadlines[fut] = loop.time() + to
            if self._sweeper is None or self._sweep_loop is not loop:
                self._sweep_loop = loop
                self._sweeper = loop.call_at(loop.time() + min(_SWEEP_S, to), self._sweep)
            try:
                resp, keep = await fut
            except ConnectionClosed:
                # stale keep-alive connection closed by the server: retry once on a fresh one
                if retry_stale and conn.reused and not conn.got_bytes and attempt == 0:
                    continue
                raise
            except BaseException:
                if conn.transport:
                    conn.transport.close()
                conn.closed = True
                raise
            finally:
                self._deadlines.pop(fut, None)
            conn.fut = None
            if keep:
                self._release(conn)
            else:
                conn.transport.close()
            return resp
        raise ConnectionClosed("unreachable")

    async def get(self, url: str, **kw: Any) -> ClientResponse:
        return await self.request("GET", url, **kw)

    async def post(self, url: str, **kw: Any) -> ClientResponse:
        return await self.request("POST", url, **kw)

    async def put(self, url: str, **kw: Any) -> ClientResponse:
        return await self.request("PUT", url, **kw)

    async def delete(self, url: str, **kw: Any) -> ClientResponse:
        return await self.request("DELETE", url, **kw)

    async def close(self) -> None:
        self._closed = True
        if self._sweeper is not None:
            self._sweeper.cancel()
            self._sweeper = None
        for dq in self._idle.values():
            for c in dq:
                if c.transport:
                    c.transport.close()
        self._idle.clear()
