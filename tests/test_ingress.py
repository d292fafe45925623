"""Environment ingress (the Container Apps / Envoy edge): the native data plane
(``native/bin/ttingress``, ``native/src/ingress.cpp``) and the asyncio one, driven through the
same control interface (``platform/ingress.py``).

Reference behaviour: external HTTPS ingress with a plain-HTTP 301 (webapp-frontend-service.bicep
:54-57, ACA ``allowInsecure: false``), internal ingress answering 403 from outside
(webapi-backend-service.bicep:94-97; docs/aca/02-aca-comm/index.md:278), revision traffic
weights, and no replay of a non-idempotent request after a replica may have acted on it.
"""
import asyncio
import collections
import http.client
import json
import socket
import ssl

import pytest

from aca_dotnet_workshop_amd.platform.ingress import Backend, Ingress, IngressRoute, NativeIngress
from aca_dotnet_workshop_amd.platform.pki import EnvironmentPki

PLANES = ["native", "python"]


def _make(plane, route, tmp_path):
    return NativeIngress(route, tmp_path, threads=2) if plane == "native" else Ingress(route)


async def _backend(name, hits, *, status=200, drop=False, extra=b""):
    """A tiny HTTP/1.1 replica that echoes what it saw (headers as JSON) and counts requests."""
    async def handle(reader, writer):
        while True:
            try:
                head = await reader.readuntil(b"\r\n\r\n")
            except (asyncio.IncompleteReadError, ConnectionError):
                break
            lines = head.decode().split("\r\n")
            method, target, _ = lines[0].split(" ", 2)
            hdrs = {}
            for ln in lines[1:]:
                if ":" in ln:
                    k, v = ln.split(":", 1)
                    hdrs[k.strip().lower()] = v.strip()
            n = int(hdrs.get("content-length", "0") or 0)
            body = await reader.readexactly(n) if n else b""
            hits[name] += 1
            if drop:
                writer.close()
                return
            out = json.dumps({"replica": name, "method": method, "target": target, "headers": hdrs,
                              "body": body.decode()}).encode()
            if method == "HEAD":
                out = b""
            writer.write(f"HTTP/1.1 {status} X\r\ncontent-type: application/json\r\nset-cookie: a=1\r\n"
                         f"set-cookie: b=2\r\n".encode() + extra + f"content-length: {len(out)}\r\n\r\n".encode() + out)
            await writer.drain()
        writer.close()
    srv = await asyncio.start_server(handle, "127.0.0.1", 0)
    return srv, f"http://127.0.0.1:{srv.sockets[0].getsockname()[1]}"


def _request(port, method, path, body=None, headers=None, context=None, unix=None):
    if unix:
        class UConn(http.client.HTTPConnection):
            def connect(self):
                self.sock = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
                self.sock.connect(unix)
        c = UConn("localhost", timeout=10)
    elif context is not None:
        c = http.client.HTTPSConnection("127.0.0.1", port, context=context, timeout=10)
    else:
        c = http.client.HTTPConnection("127.0.0.1", port, timeout=10)
    try:
        c.request(method, path, body=body, headers=headers or {})
        r = c.getresponse()
        return r.status, r.getheaders(), r.read()
    finally:
        c.close()


@pytest.mark.parametrize("plane", PLANES)
def test_external_https_ingress_balances_redirects_and_counts(plane, tmp_path):
    pki = EnvironmentPki(tmp_path / "pki")
    cert = pki.server("ingress-web", ["web"])
    ctx = ssl.create_default_context(cafile=str(pki.ca_crt))

    async def main():
        hits = collections.Counter()
        s1, u1 = await _backend("r1", hits)
        s2, u2 = await _backend("r2", hits)
        route = IngressRoute("web", True)
        ing = _make(plane, route, tmp_path)
        await ing.start(None, str(tmp_path / "web.ingress.sock"), tls=cert)
        ing.set_backends([Backend("web--a", u1), Backend("web--a", u2)], {})
        try:
            assert ing.tls and ing.public_port and ing.insecure_port
            # HTTPS, verified against the environment CA
            st, hdrs, body = await asyncio.to_thread(_request, ing.public_port, "POST", "/Tasks/Create?x=1",
                                                     b"a=b", {"Content-Type": "application/x-www-form-urlencoded"},
                                                     ctx)
            assert st == 200
            seen = json.loads(body)
            assert seen["method"] == "POST" and seen["target"] == "/Tasks/Create?x=1" and seen["body"] == "a=b"
            assert seen["headers"]["x-forwarded-proto"] == "https"
            assert seen["headers"]["x-forwarded-for"] == "127.0.0.1"
            assert [v for k, v in hdrs if k.lower() == "set-cookie"] == ["a=1", "b=2"]  # both kept
            # plain HTTP: 301 to the HTTPS endpoint, nothing reaches a replica
            before = sum(hits.values())
            st, hdrs, _ = await asyncio.to_thread(_request, ing.insecure_port, "GET", "/Tasks/Index")
            assert st == 301 and dict(hdrs)["Location" if plane == "python" else "location"] == \
                f"https://127.0.0.1:{ing.public_port}/Tasks/Index"
            assert sum(hits.values()) == before
            # spread over both replicas
            for _ in range(40):
                st, _, _ = await asyncio.to_thread(_request, ing.public_port, "GET", "/", None, None, ctx)
                assert st == 200
            assert hits["r1"] >= 10 and hits["r2"] >= 10, hits
            assert ing.requests >= 41 and ing.inflight == 0
            # the environment-internal listener proxies too
            st, _, body = await asyncio.to_thread(_request, 0, "GET", "/x", None, None, None,
                                                  str(tmp_path / "web.ingress.sock"))
            assert st == 200 and json.loads(body)["target"] == "/x"
        finally:
            await ing.stop()
            s1.close()
            s2.close()
    asyncio.run(main())


@pytest.mark.parametrize("plane", PLANES)
def test_internal_ingress_is_403_from_outside(plane, tmp_path):
    async def main():
        hits = collections.Counter()
        s1, u1 = await _backend("api", hits)
        ing = _make(plane, IngressRoute("api", False), tmp_path)
        await ing.start(None, str(tmp_path / "api.ingress.sock"))
        ing.set_backends([Backend("api--a", u1)], {})
        try:
            st, hdrs, body = await asyncio.to_thread(_request, ing.public_port, "GET", "/api/tasks?createdBy=x")
            assert st == 403 and b"internal ingress only" in body and hits["api"] == 0
            st, _, body = await asyncio.to_thread(_request, 0, "GET", "/api/tasks", None, None, None,
                                                  str(tmp_path / "api.ingress.sock"))
            assert st == 200 and hits["api"] == 1
        finally:
            await ing.stop()
            s1.close()
    asyncio.run(main())


@pytest.mark.parametrize("plane", PLANES)
def test_ingress_never_replays_a_post_after_a_mid_request_failure(plane, tmp_path):
    """A replica that drops the connection after reading a POST may already have created the
    task: the ingress answers 502 instead of replaying it on another replica; idempotent
    methods and connect-time failures still fail over."""
    async def main():
        hits = collections.Counter()
        s1, u1 = await _backend("dropper", hits, drop=True)
        s2, u2 = await _backend("good", hits, status=201)
        route = IngressRoute("api", True)
        ing = _make(plane, route, tmp_path)
        await ing.start(None, None)
        # two revisions, all traffic to the dropper's: it is always tried first
        ing.set_backends([Backend("r1", u1), Backend("r2", u2)], {"r1": 100, "r2": 0})
        try:
            st, _, _ = await asyncio.to_thread(_request, ing.public_port, "POST", "/api/tasks", b"{}")
            assert st == 502 and hits == {"dropper": 1}
            st, _, _ = await asyncio.to_thread(_request, ing.public_port, "GET", "/api/tasks")
            assert st == 201 and hits == {"dropper": 2, "good": 1}
            s1.close()
            await s1.wait_closed()  # refused at connect: nothing delivered, POST may fail over
            st, _, _ = await asyncio.to_thread(_request, ing.public_port, "POST", "/api/tasks", b"{}")
            assert st == 201 and hits["good"] == 2
        finally:
            await ing.stop()
            s2.close()
    asyncio.run(main())


@pytest.mark.parametrize("plane", PLANES)
def test_revision_weights_split_traffic(plane, tmp_path):
    async def main():
        hits = collections.Counter()
        s1, u1 = await _backend("old", hits)
        s2, u2 = await _backend("new", hits)
        ing = _make(plane, IngressRoute("web", True), tmp_path)
        await ing.start(None, None)
        ing.set_backends([Backend("web--old", u1), Backend("web--new", u2)], {"web--old": 80, "web--new": 20})
        try:
            for _ in range(400):
                st, _, _ = await asyncio.to_thread(_request, ing.public_port, "GET", "/")
                assert st == 200
            assert 0.70 <= hits["old"] / 400 <= 0.90, hits
            ing.set_backends([Backend("web--old", u1), Backend("web--new", u2)], {"web--old": 0, "web--new": 100})
            hits.clear()
            for _ in range(50):
                await asyncio.to_thread(_request, ing.public_port, "GET", "/")
            assert hits == {"new": 50}
            ing.set_backends([], {})
            st, _, body = await asyncio.to_thread(_request, ing.public_port, "GET", "/")
            assert st == 503 and b"no replicas" in body
        finally:
            await ing.stop()
            s1.close()
            s2.close()
    asyncio.run(main())


def test_native_ingress_least_in_flight_and_stats(tmp_path):
    """The native plane sends a new request to the replica with the fewest in flight: a replica
    stuck on slow requests stops getting new ones while the other drains them."""
    async def main():
        hits = collections.Counter()
        release = asyncio.Event()

        async def slow(reader, writer):
            while True:
                try:
                    await reader.readuntil(b"\r\n\r\n")
                except (asyncio.IncompleteReadError, ConnectionError):
                    break
                hits["slow"] += 1
                await release.wait()
                writer.write(b"HTTP/1.1 200 OK\r\ncontent-length: 0\r\n\r\n")
                await writer.drain()
        s1 = await asyncio.start_server(slow, "127.0.0.1", 0)
        s2, u2 = await _backend("fast", hits)
        ing = NativeIngress(IngressRoute("web", True), tmp_path, threads=1)
        await ing.start(None, None)
        ing.set_backends([Backend("web--a", f"http://127.0.0.1:{s1.sockets[0].getsockname()[1]}"),
                          Backend("web--a", u2)], {})
        try:
            stuck = [asyncio.create_task(asyncio.to_thread(_request, ing.public_port, "GET", "/s")) for _ in range(2)]
            for _ in range(100):
                if ing.inflight >= 1 and hits["slow"] >= 1:
                    break
                await asyncio.sleep(0.02)
            for _ in range(30):
                st, _, _ = await asyncio.to_thread(_request, ing.public_port, "GET", "/f")
                assert st == 200
            assert hits["slow"] == 1 and hits["fast"] >= 30, hits  # the busy replica got nothing new
            release.set()
            await asyncio.gather(*stuck)
            st = ing.stats()
            assert st["native"] and st["requests"] == 32 and st["inflight"] == 0
            assert sum(b["requests"] for b in st["backends"]) == 32
        finally:
            release.set()
            await ing.stop()
            s1.close()
            s2.close()
    asyncio.run(main())


@pytest.mark.parametrize("plane", PLANES)
def test_ingress_never_resends_a_post_reset_on_a_reused_connection(plane, tmp_path):
    """A replica reads a POST that arrived on a reused keep-alive connection, acts on it, and
    dies with a reset (RST).  The ingress must not take that for a stale idle connection and
    re-send the POST (the client's stale-connection retry): the replica sees the POST
    once and the caller gets 502.  A GET reset the same way is still retried."""
    async def main():
        hits = collections.Counter()

        async def handle(reader, writer):
            while True:
                try:
                    head = await reader.readuntil(b"\r\n\r\n")
                except (asyncio.IncompleteReadError, ConnectionError):
                    break
                method, target = head.split(b" ", 2)[:2]
                method = method.decode()
                n = int((re_len.search(head) or [0, b"0"])[1])
                if n:
                    await reader.readexactly(n)
                hits[method] += 1
                if target.startswith(b"/api/") and hits[method + "-reset"] == 0:  # first of each method: reset
                    hits[method + "-reset"] += 1
                    sock = writer.get_extra_info("socket")
                    sock.setsockopt(socket.SOL_SOCKET, socket.SO_LINGER, b"\x01\x00\x00\x00\x00\x00\x00\x00")
                    writer.transport.abort()
                    return
                hits["served"] += 1
                writer.write(b"HTTP/1.1 200 OK\r\ncontent-length: 2\r\n\r\nok")
                await writer.drain()
            writer.close()
        import re
        re_len = re.compile(rb"(?i)content-length:\s*(\d+)")
        srv = await asyncio.start_server(handle, "127.0.0.1", 0)
        url = f"http://127.0.0.1:{srv.sockets[0].getsockname()[1]}"
        ing = NativeIngress(IngressRoute("api", True), tmp_path, threads=1) if plane == "native" else Ingress(
            IngressRoute("api", True))
        await ing.start(None, None)
        ing.set_backends([Backend("r1", url)], {})
        try:
            st, _, _ = await asyncio.to_thread(_request, ing.public_port, "GET", "/warm")  # opens the keep-alive
            assert st == 200
            st, _, _ = await asyncio.to_thread(_request, ing.public_port, "POST", "/api/tasks", b"{}")
            assert st == 502 and hits["POST"] == 1, (st, hits)  # read once, never re-sent
            st, _, _ = await asyncio.to_thread(_request, ing.public_port, "GET", "/warm")  # a new keep-alive
            assert st == 200
            st, _, body = await asyncio.to_thread(_request, ing.public_port, "GET", "/api/tasks")
            assert st == 200 and body == b"ok" and hits["GET"] == 4, (st, hits)  # idempotent: retried
        finally:
            await ing.stop()
            srv.close()
    asyncio.run(main())
