"""The app-process native host (``web/native_host.py`` over ``native/src/apphost.hpp``):
drop-in ``HttpServer`` / ``HttpClient`` replacements whose I/O runs on a C++ epoll thread.

Checked against the pure-Python server/client: request/response fidelity (methods, query,
headers, bodies, HEAD, status codes), concurrency without cross-talk, pipelined and chunked
requests on one connection, error mapping (refused, missing socket, timeout), server close,
and interop in both directions."""
import asyncio
import json
import random
import socket

import pytest

from aca_dotnet_workshop_amd.web import WebApp, json_response
from aca_dotnet_workshop_amd.web.client import ConnectionClosed, HttpClient
from aca_dotnet_workshop_amd.web.http import Response
from aca_dotnet_workshop_amd.web.native_host import NativeHttpClient, NativeHttpServer, enabled
from aca_dotnet_workshop_amd.web.server import HttpServer

from helpers import run


def _app():
    app = WebApp("nh")

    @app.route("/echo/{x}", ("GET", "POST", "PUT", "DELETE", "HEAD"))
    async def echo(req):
        return json_response({"m": req.method, "x": req.path_params["x"], "q": req.query_get("a"),
                              "h": req.headers.get("x-multi"), "n": len(req.body),
                              "sum": sum(req.body) % 65521})

    @app.route("/sleep/{ms}", ("GET",))
    async def sleep(req):
        ms = int(req.path_params["ms"])
        await asyncio.sleep(ms / 1000)
        return json_response({"ms": ms})

    @app.route("/status/{code}", ("GET",))
    async def status(req):
        return Response(b"custom", int(req.path_params["code"]), [("X-Reply", "yes"), ("Location", "/there")])

    @app.route("/boom", ("GET",))
    async def boom(req):
        raise RuntimeError("handler failure")
    return app


def test_roundtrip_and_interop(tmp_path):
    async def main():
        loop = asyncio.get_running_loop()
        nsrv = NativeHttpServer(_app(), loop)
        nport = await nsrv.listen_tcp("127.0.0.1", 0)
        sock = str(tmp_path / "n.sock")
        await nsrv.listen_unix(sock)
        psrv = HttpServer(_app(), loop)
        pport = await psrv.listen_tcp("127.0.0.1", 0)
        nc, pc = NativeHttpClient(), HttpClient()
        big = random.Random(1).randbytes(1 << 20)
        for client, base in ((nc, f"http://127.0.0.1:{nport}"), (nc, f"unix:{sock}:"), (pc, f"http://127.0.0.1:{nport}"),
                             (nc, f"http://127.0.0.1:{pport}")):
            r = await client.post(f"{base}/echo/1?a=2", body=big, headers=[("X-Multi", "a")])
            assert r.status == 200 and r.json() == {"m": "POST", "x": "1", "q": "2", "h": "a", "n": len(big),
                                                    "sum": sum(big) % 65521}
            r = await client.request("HEAD", f"{base}/echo/2")
            assert r.status == 200 and r.body == b""
            r = await client.get(f"{base}/status/201")
            assert (r.status, r.body, r.headers["x-reply"], r.headers["location"]) == (201, b"custom", "yes", "/there")
            r = await client.get(f"{base}/nope")
            assert r.status == 404
            r = await client.get(f"{base}/boom")
            assert r.status == 500
            r = await client.delete(f"{base}/echo/%2Fenc")
            assert r.json()["x"] == "/enc"
        await nc.close()
        await pc.close()
        await nsrv.close(1)
        await psrv.close(1)
    run(main())


def test_concurrency_no_crosstalk():
    async def main():
        srv = NativeHttpServer(_app(), asyncio.get_running_loop())
        port = await srv.listen_tcp("127.0.0.1", 0)
        c = NativeHttpClient()
        rnd = random.Random(7)

        async def one(i):
            if i % 5 == 0:
                r = await c.get(f"http://127.0.0.1:{port}/sleep/{rnd.randrange(20)}")
                return r.status == 200
            body = str(i).encode() * (i % 50)
            r = await c.put(f"http://127.0.0.1:{port}/echo/{i}", body=body)
            return r.json()["x"] == str(i) and r.json()["n"] == len(body)
        assert all(await asyncio.gather(*(one(i) for i in range(600))))
        await c.close()
        await srv.close(1)
    run(main())


def test_pipelined_and_chunked_requests_on_one_connection():
    async def main():
        srv = NativeHttpServer(_app(), asyncio.get_running_loop())
        port = await srv.listen_tcp("127.0.0.1", 0)

        def raw():
            s = socket.create_connection(("127.0.0.1", port), timeout=5)
            s.sendall(b"GET /sleep/30 HTTP/1.1\r\nHost: x\r\n\r\n"
                      b"POST /echo/c HTTP/1.1\r\nHost: x\r\nTransfer-Encoding: chunked\r\n\r\n3\r\nabc\r\n2\r\nde\r\n0\r\n\r\n"
                      b"GET /echo/last HTTP/1.1\r\nHost: x\r\nConnection: close\r\n\r\n")
            data = b""
            while True:
                d = s.recv(65536)
                if not d:
                    break
                data += d
            s.close()
            return data
        data = await asyncio.get_running_loop().run_in_executor(None, raw)
        bodies = [json.loads(p.split(b"\r\n\r\n", 1)[1][:p.split(b"\r\n\r\n", 1)[1].index(b"}") + 1])
                  for p in data.split(b"HTTP/1.1 ")[1:]]
        # responses in request order although the first handler is the slowest
        assert bodies[0] == {"ms": 30} and bodies[1]["n"] == 5 and bodies[2]["x"] == "last"
        await srv.close(1)
    run(main())


def test_client_errors_and_server_close(tmp_path):
    async def main():
        srv = NativeHttpServer(_app(), asyncio.get_running_loop())
        port = await srv.listen_tcp("127.0.0.1", 0)
        c = NativeHttpClient()
        with pytest.raises(ConnectionRefusedError):
            await c.get("http://127.0.0.1:1/x")
        with pytest.raises(FileNotFoundError):
            await c.get(f"unix:{tmp_path / 'missing.sock'}:/x")
        with pytest.raises(asyncio.TimeoutError):
            await c.get(f"http://127.0.0.1:{port}/sleep/1500", timeout=0.3)
        slow = asyncio.ensure_future(c.get(f"http://127.0.0.1:{port}/sleep/200"))
        await asyncio.sleep(0.05)
        await srv.close(2.0)  # in-flight request completes; new connections are refused
        assert (await slow).status == 200
        fresh = NativeHttpClient()
        with pytest.raises((ConnectionRefusedError, ConnectionClosed)):
            await fresh.get(f"http://127.0.0.1:{port}/echo/1")
        await c.close()
        await fresh.close()
    run(main())


def test_enabled_switch():
    assert enabled({"TT_APP_HOST": "native"}) and not enabled({}) and not enabled({"TT_APP_HOST": "python"})


def test_odd_header_values_and_bad_operations():
    """Non-string header values are stringified (like the asyncio server's f"{k}: {v}"); a
    request with an unusable body fails on its own without losing the rest of the batch."""
    app = WebApp("odd")

    @app.route("/odd", ("GET",))
    async def odd(req):
        return Response(b"ok", 200, [("X-Count", 5), ("X-Ratio", 0.5)])

    async def main():
        srv = NativeHttpServer(app, asyncio.get_running_loop())
        port = await srv.listen_tcp("127.0.0.1", 0)
        c = NativeHttpClient()
        r = await c.get(f"http://127.0.0.1:{port}/odd")
        assert r.status == 200 and r.headers["x-count"] == "5" and r.headers["x-ratio"] == "0.5"
        host = c._native()
        bad = host.request(f"tcp:127.0.0.1:{port}", "POST", "/odd", [], 12345, 5.0)  # body is not bytes
        good = c.get(f"http://127.0.0.1:{port}/odd")
        with pytest.raises(ValueError):
            await bad
        assert (await good).status == 200
        await c.close()
        await srv.close(1)
    run(main())


def test_fd_table_reserved_before_io_thread():
    """The host sizes the process's fd table up front (kernel fd-table growth in a multi-threaded
    process waits for an RCU grace period: 100+ ms event-loop stalls, profiles/r1_native_app_host_ab.md)."""
    import resource

    from aca_dotnet_workshop_amd import native
    h = native.load().AppHost()
    try:
        fdsize = int(open("/proc/self/status").read().split("FDSize:")[1].split()[0])
        soft = resource.getrlimit(resource.RLIMIT_NOFILE)[0]
        assert fdsize >= min(soft, 1 << 16) - 1
    finally:
        h.stop()
