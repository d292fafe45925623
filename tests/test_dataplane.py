"""Sidecar API parity: the same assertions run against the Python plane and the native C++
data plane (native/src/dataplane.cpp) -- state save/get/delete with ETags and concurrency
modes, publish envelopes, self and peer service invocation, API token, error codes,
tracing propagation, HTTP framing (keep-alive, pipelining, Connection: close)."""
import asyncio
import json
import re
import socket

import pytest

from aca_dotnet_workshop_amd.backing import BackingServices
from aca_dotnet_workshop_amd.sdk import cloud_events_middleware, map_subscribe_handler, topic
from aca_dotnet_workshop_amd.sidecar import NameResolver, Sidecar, from_dict
from aca_dotnet_workshop_amd.web import HttpClient, HttpServer, Response, WebApp, empty, json_response

from helpers import run

PLANES = ["python", "native"]


def _comp(name, type_, meta, **extra):
    d = {"apiVersion": "dapr.io/v1alpha1", "kind": "Component", "metadata": {"name": name},
         "spec": {"type": type_, "version": "v1", "metadata": [{"name": k, "value": v} for k, v in meta.items()]}}
    d.update(extra)
    return from_dict(d)


STORE = _comp("statestore", "state.azure.cosmosdb", {"url": "https://acct1.documents.azure.com:443/",
                                                     "database": "db", "collection": "tasks"})
BUS = _comp("bus", "pubsub.azure.servicebus", {"connectionString": "Endpoint=sb://ns1.servicebus.windows.net/"})
MEM = _comp("mem", "state.in-memory", {})


def _app(name, seen):
    app = WebApp(name)
    app.use(cloud_events_middleware())

    async def echo(req):
        seen.append(("echo", req.method, req.path, req.query_string, dict(req.headers.items()), req.body))
        return Response(json.dumps({"app": name, "method": req.method, "q": req.query_string,
                                    "body": req.body.decode()}).encode(), 201,
                        [("X-Echo", "1"), ("Content-Type", "application/json")])

    async def boom(req):
        return json_response({"error": "boom"}, 500)

    async def events(req):
        seen.append(("event", req.headers.get("traceparent"), req.json()))
        return empty(200)

    async def raw_events(req):
        seen.append(("raw", req.content_type, req.body))
        return empty(200)

    app.add_route("/api/echo/{*rest}", echo, ("GET", "POST", "PUT", "DELETE", "HEAD"))
    app.add_route("/api/boom", boom, ("GET",))
    topic("bus", "events")(events)
    app.add_route("/events", events, ("POST",))
    topic("bus", "rawtopic", metadata={"rawPayload": "true"})(raw_events)
    app.add_route("/raw", raw_events, ("POST",))
    map_subscribe_handler(app)
    return app


class Env:
    """Backing services + N (app, sidecar) pairs sharing a registry directory."""

    def __init__(self, plane, tmp_path, apps=("app-a",), pki=None, **sc_kw):
        self.plane, self.tmp, self.names, self.sc_kw = plane, tmp_path, apps, sc_kw
        self.pki = pki  # platform.pki.EnvironmentPki: mutual TLS between the sidecars
        self.seen = {n: [] for n in apps}

    async def __aenter__(self):
        loop = asyncio.get_running_loop()
        self.backing = BackingServices()
        self.bsrv = HttpServer(self.backing.build_app(), loop)
        self.burl = f"http://127.0.0.1:{await self.bsrv.listen_tcp('127.0.0.1', 0)}"
        self.servers, self.sidecars, self.base = [], {}, {}
        for n in self.names:
            app = _app(n, self.seen[n])
            srv = HttpServer(app, loop)
            await app.startup()
            port = await srv.listen_tcp("127.0.0.1", 0)
            self.servers.append(srv)
            sc = Sidecar(n, app_port=port, http_port=0, components=[STORE, BUS, MEM],
                         resolver=NameResolver(str(self.tmp / "registry")), backing_url=self.burl,
                         internal_uds=str(self.tmp / f"{n}.i.sock"), data_plane=self.plane,
                         mtls=self.pki.workload(n).as_config() if self.pki else None, **self.sc_kw)
            await sc.start()
            await asyncio.wait_for(sc.app_ready.wait(), 10)
            assert sc.active_data_plane == self.plane
            self.sidecars[n] = sc
            self.base[n] = f"http://127.0.0.1:{sc.bound_http_port}"
        self.http = HttpClient()
        return self

    async def __aexit__(self, *exc):
        for sc in self.sidecars.values():
            await sc.stop(1.0)
        for s in self.servers:
            await s.close(1.0)
        await self.bsrv.close(1.0)
        await self.http.close()


async def _until(pred, timeout=5.0):
    end = asyncio.get_running_loop().time() + timeout
    while asyncio.get_running_loop().time() < end:
        if pred():
            return True
        await asyncio.sleep(0.02)
    raise AssertionError("timeout")


@pytest.mark.parametrize("plane", PLANES)
def test_state_api(plane, tmp_path):
    async def main():
        async with Env(plane, tmp_path) as e:
            b, h = e.base["app-a"], e.http
            st = f"{b}/v1.0/state/statestore"
            assert (await h.post(st, json_body=[{"key": "k1", "value": {"a": 1, "s": "x y"}}])).status == 204
            r = await h.get(f"{st}/k1")
            assert r.status == 200 and r.json() == {"a": 1, "s": "x y"}
            etag = r.headers.get("etag")
            assert etag
            # key prefix <app-id>|| in the backing store
            coll = e.backing.store("acct1", "db", "tasks")
            assert coll.get("app-a||k1") is not None
            # stale etag -> 409, fresh etag -> 204
            bad = await h.post(st, json_body=[{"key": "k1", "value": 2, "etag": "999"}])
            assert bad.status == 409 and bad.json()["errorCode"] == "ERR_STATE_SAVE"
            assert (await h.post(st, json_body=[{"key": "k1", "value": 2, "etag": etag}])).status == 204
            # first-write concurrency on an existing key -> 409
            fw = await h.post(st, json_body=[{"key": "k1", "value": 3, "options": {"concurrency": "first-write"}}])
            assert fw.status == 409
            # bulk save + special characters in keys
            items = [{"key": f"bulk/{i} é", "value": {"i": i}} for i in range(3)]
            assert (await h.post(st, json_body=items)).status == 204
            from urllib.parse import quote
            for i in range(3):
                r = await h.get(f"{st}/{quote(f'bulk/{i} é', safe='')}")
                assert r.status == 200 and r.json() == {"i": i}
            # bulk get: request order, raw values with their etags, a missing key without data
            r = await h.post(f"{st}/bulk", json_body={"keys": ["bulk/2 é", "nope", "k1"], "parallelism": 2})
            assert r.status == 200
            got = r.json()
            assert [x["key"] for x in got] == ["bulk/2 é", "nope", "k1"]
            assert got[0]["data"] == {"i": 2} and got[0]["etag"] and "data" not in got[1]
            assert got[2]["data"] == 2 and got[2]["etag"] == (await h.get(f"{st}/k1")).headers.get("etag")
            # missing -> 204, delete with bad etag -> 409, delete -> 204 then missing
            assert (await h.get(f"{st}/nope")).status == 204
            r = await h.delete(f"{st}/k1", headers={"If-Match": "123"})
            assert r.status == 409 and r.json()["errorCode"] == "ERR_STATE_DELETE"
            assert (await h.delete(f"{st}/k1")).status == 204
            assert (await h.get(f"{st}/k1")).status == 204
            # malformed bodies
            for body in (b"{not json", b'{"key": "x"}', b'[{"value": 1}]'):
                r = await h.post(st, body=body, headers={"Content-Type": "application/json"})
                assert r.status == 400 and r.json()["errorCode"] == "ERR_MALFORMED_REQUEST", body
            # unknown store / in-memory store (served by the control plane in native mode)
            r = await h.post(f"{b}/v1.0/state/nostore", json_body=[{"key": "a", "value": 1}])
            assert r.status == 400 and r.json()["errorCode"] == "ERR_STATE_STORE_NOT_FOUND"
            assert (await h.post(f"{b}/v1.0/state/mem", json_body=[{"key": "a", "value": 1}])).status == 204
            assert (await h.get(f"{b}/v1.0/state/mem/a")).json() == 1
            # ttl metadata is accepted
            r = await h.post(st, json_body=[{"key": "t", "value": 1, "metadata": {"ttlInSeconds": "60"}}])
            assert r.status == 204
            # state query (native plane: forwarded to the backing planner; Python: control plane)
            r = await h.post(f"{b}/v1.0-alpha1/state/statestore/query", json_body={"filter": {"EQ": {"i": 1}}})
            assert r.status == 200 and [x["key"] for x in r.json()["results"]] == ["bulk/1 é"]
            r = await h.post(f"{b}/v1.0-beta1/state/statestore/query",
                             json_body={"filter": {"OR": [{"EQ": {"i": 0}}, {"EQ": {"i": 2}}]},
                                        "sort": [{"key": "i", "order": "DESC"}], "page": {"limit": 1}})
            js = r.json()
            assert r.status == 200 and [x["key"] for x in js["results"]] == ["bulk/2 é"] and js["token"]
            r = await h.post(f"{b}/v1.0-alpha1/state/statestore/query", json_body={"filter": {"BOGUS": {"i": 1}}})
            assert r.status == 400 and r.json()["errorCode"] == "ERR_STATE_QUERY"
    run(main())


@pytest.mark.parametrize("plane", PLANES)
def test_publish_api(plane, tmp_path):
    async def main():
        async with Env(plane, tmp_path) as e:
            b, h, seen = e.base["app-a"], e.http, e.seen["app-a"]
            tp = "00-" + "ab" * 16 + "-" + "cd" * 8 + "-01"
            r = await h.post(f"{b}/v1.0/publish/bus/events", json_body={"n": 1, "s": "é"}, headers={"traceparent": tp})
            assert r.status == 204
            await _until(lambda: any(x[0] == "event" for x in seen))
            ev = [x for x in seen if x[0] == "event"][0]
            assert ev[2] == {"n": 1, "s": "é"}
            assert ev[1].split("-")[1] == "ab" * 16  # same trace continues into the subscriber
            # the envelope as stored in the broker
            msgs = e.backing.broker("ns1")
            # text payload + raw payload
            r = await h.post(f"{b}/v1.0/publish/bus/rawtopic?metadata.rawPayload=true", body=b"plain bytes",
                             headers={"Content-Type": "text/plain"})
            assert r.status == 204
            await _until(lambda: any(x[0] == "raw" for x in seen))
            raw = [x for x in seen if x[0] == "raw"][0]
            assert raw[2] == b"plain bytes"
            # unknown pubsub -> 404, empty topic -> 404
            r = await h.post(f"{b}/v1.0/publish/nope/x", json_body={})
            assert r.status == 404 and r.json()["errorCode"] == "ERR_PUBSUB_NOT_FOUND"
            # cloudevents passthrough
            ce = {"specversion": "1.0", "id": "my-id", "source": "me", "type": "t", "data": {"x": 1}}
            r = await h.post(f"{b}/v1.0/publish/bus/events", body=json.dumps(ce).encode(),
                             headers={"Content-Type": "application/cloudevents+json"})
            assert r.status == 204
            await _until(lambda: sum(x[0] == "event" for x in seen) == 2)
            assert [x for x in seen if x[0] == "event"][1][2] == {"x": 1}
            # an envelope's own traceparent (after other keys, spaced, one escaped key) is continued
            tp2 = "00-" + "ef" * 16 + "-" + "12" * 8 + "-01"
            text = ('{ "specversion" : "1.0", "id":"id2", "sou\\u0072ce": "me", "type": "t", '
                    '"data": {"traceparent": "nested"}, "traceparent" : "%s" }' % tp2)
            r = await h.post(f"{b}/v1.0/publish/bus/events", body=text.encode(),
                             headers={"Content-Type": "application/cloudevents+json"})
            assert r.status == 204
            await _until(lambda: sum(x[0] == "event" for x in seen) == 3)
            third = [x for x in seen if x[0] == "event"][2]
            assert third[2] == {"traceparent": "nested"} and third[1].split("-")[1] == "ef" * 16
            assert msgs.counts("events/subscriptions/app-a")["completed"] >= 1
    run(main())


@pytest.mark.parametrize("plane", PLANES)
def test_invoke_api(plane, tmp_path):
    async def main():
        async with Env(plane, tmp_path, apps=("app-a", "app-b")) as e:
            h = e.http
            a = e.base["app-a"]
            # self invocation with query string, custom headers and status/header relay
            r = await h.post(f"{a}/v1.0/invoke/app-a/method/api/echo/x/y?p=1&q=a%20b", body=b"hello",
                             headers={"X-Custom": "v", "Content-Type": "text/plain"})
            assert r.status == 201 and r.headers.get("x-echo") == "1"
            assert r.json() == {"app": "app-a", "method": "POST", "q": "p=1&q=a%20b", "body": "hello"}
            call = e.seen["app-a"][-1]
            assert call[2] == "/api/echo/x/y" and call[4]["x-custom"] == "v"
            assert call[4]["dapr-caller-app-id"] == "app-a" and call[4].get("traceparent")
            # peer invocation through the registry + internal endpoint
            r = await h.get(f"{a}/v1.0/invoke/app-b/method/api/echo/z")
            assert r.status == 201 and r.json()["app"] == "app-b"
            assert e.seen["app-b"][-1][4]["dapr-caller-app-id"] == "app-a"
            # namespace suffix is ignored
            assert (await h.get(f"{a}/v1.0/invoke/app-b.default/method/api/echo/z")).status == 201
            # app errors are relayed, unknown apps are ERR_DIRECT_INVOKE
            r = await h.get(f"{a}/v1.0/invoke/app-b/method/api/boom")
            assert r.status == 500 and r.json() == {"error": "boom"}
            r = await h.get(f"{a}/v1.0/invoke/ghost/method/x")
            assert r.status == 500 and r.json()["errorCode"] == "ERR_DIRECT_INVOKE"
            assert "ghost" in r.json()["message"]
            # HEAD and DELETE pass through
            assert (await h.request("HEAD", f"{a}/v1.0/invoke/app-a/method/api/echo/h")).status == 201
            assert (await h.delete(f"{a}/v1.0/invoke/app-b/method/api/echo/d")).json()["method"] == "DELETE"
            # metadata reports the plane
            meta = (await h.get(f"{a}/v1.0/metadata")).json()
            assert meta["extended"]["dataPlane"] == plane
    run(main())


@pytest.mark.parametrize("plane", PLANES)
def test_api_token(plane, tmp_path):
    async def main():
        async with Env(plane, tmp_path, api_token="tok") as e:
            b, h = e.base["app-a"], e.http
            r = await h.get(f"{b}/v1.0/state/statestore/a")
            assert r.status == 401 and r.json()["errorCode"] == "ERR_API_TOKEN"
            assert (await h.get(f"{b}/v1.0/invoke/app-a/method/api/echo/x")).status == 401
            assert (await h.get(f"{b}/v1.0/healthz")).status == 204
            hdr = {"dapr-api-token": "tok"}
            assert (await h.get(f"{b}/v1.0/state/statestore/a", headers=hdr)).status == 204
            r = await h.get(f"{b}/v1.0/invoke/app-a/method/api/echo/x", headers=hdr)
            assert r.status == 201
            assert "dapr-api-token" not in e.seen["app-a"][-1][4]  # the API token is not leaked to the app
    run(main())


def _raw_exchange(port, payload: bytes, expect_responses: int, timeout=5.0) -> bytes:
    s = socket.create_connection(("127.0.0.1", port), timeout=timeout)
    s.sendall(payload)
    data = b""
    while data.count(b"HTTP/1.1 ") < expect_responses or not data.endswith((b"}", b"\r\n\r\n")):
        chunk = s.recv(65536)
        if not chunk:
            break
        data += chunk
    s.close()
    return data


def test_native_http_framing(tmp_path):
    """Pipelined requests answered in order; chunked request bodies; Connection: close."""
    async def main():
        async with Env("native", tmp_path) as e:
            port = e.sidecars["app-a"].bound_http_port
            loop = asyncio.get_running_loop()
            req = (b"POST /v1.0/state/statestore HTTP/1.1\r\nHost: x\r\nContent-Length: 29\r\n\r\n"
                   b'[{"key":"p","value":{"v":1}}]'
                   b"GET /v1.0/state/statestore/p HTTP/1.1\r\nHost: x\r\n\r\n"
                   b"GET /v1.0/state/statestore/nope HTTP/1.1\r\nHost: x\r\n\r\n")
            data = await loop.run_in_executor(None, _raw_exchange, port, req, 3)
            statuses = re.findall(rb"HTTP/1\.1 (\d{3})", data)
            assert statuses == [b"204", b"200", b"204"], data
            parts = [b'[{"key":"c","va', b'lue":"chunk"}]']
            chunked = (b"POST /v1.0/state/statestore HTTP/1.1\r\nHost: x\r\nTransfer-Encoding: chunked\r\n"
                       b"Connection: close\r\n\r\n" + b"".join(b"%x\r\n%s\r\n" % (len(p), p) for p in parts)
                       + b"0\r\n\r\n")
            data = await loop.run_in_executor(None, _raw_exchange, port, chunked, 1)
            assert data.startswith(b"HTTP/1.1 204") and b"connection: close" in data.lower()
            r = await e.http.get(f"{e.base['app-a']}/v1.0/state/statestore/c")
            assert r.json() == "chunk"
            m = await e.http.get(f"{e.base['app-a']}/metrics")
            assert b"sidecar_native_requests_total" in m.body
            # Expect: 100-continue -> interim response before the body is sent
            body = b'[{"key":"x","value":2}]'

            def expect_continue():
                s = socket.create_connection(("127.0.0.1", port), timeout=5)
                s.sendall(b"POST /v1.0/state/statestore HTTP/1.1\r\nHost: x\r\nExpect: 100-continue\r\n"
                          b"Content-Length: %d\r\n\r\n" % len(body))
                first = s.recv(4096)
                s.sendall(body)
                rest = b""
                while b"\r\n\r\n" not in rest:
                    rest += s.recv(4096)
                s.close()
                return first, rest
            first, rest = await loop.run_in_executor(None, expect_continue)
            assert first.startswith(b"HTTP/1.1 100 Continue") and rest.startswith(b"HTTP/1.1 204")
    run(main())


@pytest.mark.parametrize("plane", PLANES)
def test_delivery_outcomes(plane, tmp_path):
    """SUCCESS / RETRY (-> DLQ after maxDeliveryCount) / DROP with deadLetterTopic / 404 /
    non-2xx retried until success -- identical on both planes."""
    app = WebApp("sub")
    app.use(cloud_events_middleware())
    seen = {k: [] for k in ("ok", "retry", "drop", "flaky", "gone", "poison")}
    attempts = {"flaky": 0}

    def handler(kind, resp):
        async def h(req):
            seen[kind].append(req.json())
            return resp() if callable(resp) else resp
        return h

    def flaky():
        attempts["flaky"] += 1
        return Response(b"", 503) if attempts["flaky"] <= 2 else empty(200)

    for kind, resp, extra in (("ok", json_response({"status": "SUCCESS"}), {}),
                              ("retry", json_response({"status": "RETRY"}), {}),
                              ("drop", json_response({"status": "DROP"}), {"dead_letter_topic": "poison"}),
                              ("flaky", flaky, {}), ("gone", empty(404), {}), ("poison", empty(200), {})):
        fn = handler(kind, resp)
        topic("bus3", kind, **extra)(fn)
        app.add_route(f"/{kind}", fn, ("POST",))
    map_subscribe_handler(app)
    bus = _comp("bus3", "pubsub.azure.servicebus", {"connectionString": "Endpoint=sb://ns3.servicebus.windows.net/",
                                                     "maxDeliveryCount": "3"})

    async def main():
        loop = asyncio.get_running_loop()
        backing = BackingServices()
        bsrv = HttpServer(backing.build_app(), loop)
        burl = f"http://127.0.0.1:{await bsrv.listen_tcp('127.0.0.1', 0)}"
        asrv = HttpServer(app, loop)
        port = await asrv.listen_tcp("127.0.0.1", 0)
        sc = Sidecar("subapp", app_port=port, http_port=0, components=[bus], backing_url=burl,
                     resolver=NameResolver(str(tmp_path / "reg")), data_plane=plane)
        await sc.start()
        http = HttpClient()
        try:
            await asyncio.wait_for(sc.app_ready.wait(), 10)
            base = f"http://127.0.0.1:{sc.bound_http_port}"
            for t in ("ok", "retry", "drop", "flaky", "gone"):
                assert (await http.post(f"{base}/v1.0/publish/bus3/{t}", json_body={"t": t})).status == 204
            b = backing.broker("ns3")

            def counts(t):
                return b.counts(f"{t}/subscriptions/subapp")
            await _until(lambda: counts("ok")["completed"] == 1)
            assert seen["ok"] == [{"t": "ok"}]
            await _until(lambda: counts("retry")["dead_letter"] == 1)
            assert len(seen["retry"]) == 3
            await _until(lambda: len(seen["poison"]) == 1)
            await _until(lambda: counts("drop")["completed"] == 1)
            assert counts("drop")["dead_letter"] == 0 and seen["poison"] == [{"t": "drop"}]
            await _until(lambda: counts("flaky")["completed"] == 1)
            assert attempts["flaky"] == 3
            await _until(lambda: counts("gone")["dead_letter"] == 1)
            assert len(seen["gone"]) == 1
            meta = (await http.get(f"{base}/v1.0/metadata")).json()
            st = meta["extended"]["consumers"]["bus3/ok"]
            assert st["succeeded"] == 1 and st["delivered"] == 1
            assert meta["extended"]["consumers"]["bus3/retry"]["retried"] == 3
        finally:
            await http.close()
            await sc.stop(1.0)
            await asrv.close(1.0)
            await bsrv.close(1.0)
    run(main())


@pytest.mark.parametrize("plane", PLANES)
def test_api_logging(plane, tmp_path, capfd, caplog):
    """enableApiLogging: every sidecar API call is logged (method, path, status, duration)."""
    import logging
    caplog.set_level(logging.INFO, logger="sidecar.http-info")

    async def main():
        async with Env(plane, tmp_path, api_logging=True) as e:
            b = e.base["app-a"]
            assert (await e.http.post(f"{b}/v1.0/state/statestore", json_body=[{"key": "L", "value": 1}])).status == 204
            assert (await e.http.get(f"{b}/v1.0/invoke/app-a/method/api/echo/log")).status == 201
    run(main())
    text = capfd.readouterr().err + "\n".join(r.getMessage() for r in caplog.records)
    assert "HTTP API Called method=POST path=/v1.0/state/statestore status=204" in text
    assert "HTTP API Called method=GET path=/v1.0/invoke/app-a/method/api/echo/log status=201" in text


def test_native_http_parser_survives_garbage(tmp_path):
    """Malformed / hostile requests get a 400 (or a closed connection), never a crash: a valid
    request still works afterwards (run under ASan by test_native_sanitizers)."""
    import random
    rnd = random.Random(5)
    samples = [b"GARBAGE\r\n\r\n", b"GET\r\n\r\n", b"POST /x HTTP/1.1\r\nContent-Length: -5\r\n\r\n",
               b"POST /x HTTP/1.1\r\nContent-Length: 99999999999\r\n\r\n",
               b"POST /v1.0/state/statestore HTTP/1.1\r\nTransfer-Encoding: chunked\r\n\r\nzz\r\nabc\r\n0\r\n\r\n",
               b"GET /" + b"a" * 70000 + b" HTTP/1.1\r\n\r\n", b"GET / HTTP/1.1\r\nNoColonHeader\r\n\r\n",
               b"POST /v1.0/state/statestore HTTP/1.1\r\nContent-Length: 3\r\n\r\n[{]",
               b"POST /v1.0/publish/bus/t HTTP/1.1\r\nContent-Type: application/json\r\nContent-Length: 4\r\n\r\n\xff\xfe{]",
               # 1-byte chunk, then a size that would saturate strtoull (and wrap the body cap)
               b"POST /v1.0/state/statestore HTTP/1.1\r\nTransfer-Encoding: chunked\r\n\r\n1\r\n[\r\n"
               b"FFFFFFFFFFFFFFFFF\r\n" + b"x" * 4096,
               # a size line without digits is not the last chunk
               b"POST /v1.0/state/statestore HTTP/1.1\r\nTransfer-Encoding: chunked\r\n\r\n;ext\r\n\r\n",
               b"POST /v1.0/state/statestore HTTP/1.1\r\nTransfer-Encoding: chunked\r\n\r\n3\r\nabcXY0\r\n\r\n"]
    for _ in range(40):
        samples.append(bytes(rnd.randrange(256) for _ in range(rnd.randrange(1, 300))) + b"\r\n\r\n")

    async def main():
        async with Env("native", tmp_path) as e:
            port = e.sidecars["app-a"].bound_http_port
            loop = asyncio.get_running_loop()

            def blast():
                for payload in samples:
                    s = socket.create_connection(("127.0.0.1", port), timeout=5)
                    try:
                        s.sendall(payload)
                        s.shutdown(socket.SHUT_WR)
                        while s.recv(65536):
                            pass
                    except OSError:
                        pass
                    finally:
                        s.close()
            await loop.run_in_executor(None, blast)
            assert e.sidecars["app-a"]._dp_proc.returncode is None  # still running
            r = await e.http.post(f"{e.base['app-a']}/v1.0/state/statestore", json_body=[{"key": "ok", "value": 1}])
            assert r.status == 204
    run(main())


@pytest.mark.parametrize("plane", PLANES)
def test_state_throttling_is_retried(plane, tmp_path):
    """Provisioned RU/s (Cosmos 4000 RU/s in the reference's Bicep, scaled down here): the store
    answers 429 + x-ms-retry-after-ms once the budget is spent, and both sidecar planes retry after
    the hint, so the application sees success -- just later."""
    import time

    async def main():
        async with Env(plane, tmp_path) as e:
            st = e.backing.store("acct1", "db", "tasks")
            st.set_throughput(50.0)  # 10 writes of <= 1 KiB per second, the bucket starting empty
            b = e.base["app-a"]
            t0 = time.perf_counter()
            for i in range(20):
                r = await e.http.post(f"{b}/v1.0/state/statestore", json_body=[{"key": f"k{i}", "value": {"i": i}}])
                assert r.status == 204, r.body
            dt = time.perf_counter() - t0
            assert dt > 1.8  # 20 writes x 5 RU = 100 RU at 50 RU/s from an empty bucket
            ts = st.throughput_stats()
            assert ts["throttled"] >= 1 and ts["ru_consumed"] >= 100
            r = await e.http.get(f"{b}/v1.0/state/statestore/k19")
            assert r.status == 200 and r.json() == {"i": 19}
    run(main())


@pytest.mark.parametrize("plane", PLANES)
def test_throttled_writers_get_slots_not_failures(plane, tmp_path):
    """16 concurrent writers against 500 RU/s (5 RU per write: 100 writes/s, the bucket starting
    empty).  A throttled write is given a reserved slot (the 429's hint + ticket), so waiters
    are spread instead of waking together: every write succeeds, the store answers at most
    about one 429 per write, and the writes come through at the budget's rate."""
    import time

    async def main():
        async with Env(plane, tmp_path) as e:
            st = e.backing.store("acct1", "db", "tasks")
            st.set_throughput(500.0)
            b = e.base["app-a"]
            n, statuses = 400, []
            it = iter(range(n))

            async def writer():
                for i in it:
                    r = await e.http.post(f"{b}/v1.0/state/statestore", json_body=[{"key": f"w{i}", "value": {"i": i}}])
                    statuses.append(r.status)
            t0 = time.perf_counter()
            await asyncio.gather(*(writer() for _ in range(16)))
            dt = time.perf_counter() - t0
            assert statuses.count(204) == n, {s: statuses.count(s) for s in set(statuses)}
            ts = st.throughput_stats()
            assert ts["throttled"] <= n, ts                  # ~1 per throttled write, not 7.8 per task
            assert ts["reserved_admits"] >= 0.5 * (n - 100), ts  # the retries came back on their tickets
            # 400 writes at 100/s from an empty bucket: ~4 s at the budget's rate
            assert 0.95 * 4.0 <= dt <= 4.0 / 0.9, dt
    run(main())


def test_native_store_calls_pipelined_over_the_backing_socket(tmp_path, monkeypatch):
    """With the backing on a Unix socket the native plane sends store and broker calls over
    pipelined connections (ev::PipeConn): the calls of one loop iteration leave in one write and
    their answers come back in order.  Concurrent saves, reads and publishes all land, each answer
    reaches its own caller, and a query (never pipelined) still works alongside."""
    async def main():
        loop = asyncio.get_running_loop()
        backing = BackingServices()
        bsrv = HttpServer(backing.build_app(), loop)
        burl = f"http://127.0.0.1:{await bsrv.listen_tcp('127.0.0.1', 0)}"
        uds = str(tmp_path / "backing.sock")
        await bsrv.listen_unix(uds)
        monkeypatch.setenv("TT_BACKING_URL", burl)
        monkeypatch.setenv("TT_BACKING_UDS", uds)
        seen = []
        app = _app("app-a", seen)
        srv = HttpServer(app, loop)
        await app.startup()
        port = await srv.listen_tcp("127.0.0.1", 0)
        sc = Sidecar("app-a", app_port=port, http_port=0, components=[STORE, BUS, MEM],
                     resolver=NameResolver(str(tmp_path / "registry")), backing_url=burl,
                     internal_uds=str(tmp_path / "a.i.sock"), data_plane="native")
        await sc.start()
        http = HttpClient()
        try:
            await asyncio.wait_for(sc.app_ready.wait(), 10)
            assert sc.active_data_plane == "native"
            b = f"http://127.0.0.1:{sc.bound_http_port}"

            async def one(i):
                r = await http.post(f"{b}/v1.0/state/statestore", json_body=[{"key": f"p{i}", "value": {"i": i}}])
                assert r.status == 204, r.body
                r = await http.get(f"{b}/v1.0/state/statestore/p{i}")
                assert r.status == 200 and r.json() == {"i": i}, (i, r.body)
                r = await http.post(f"{b}/v1.0/publish/bus/events", json_body={"n": i})
                assert r.status == 204, r.body
            await asyncio.gather(*(one(i) for i in range(200)))
            r = await http.post(f"{b}/v1.0-alpha1/state/statestore/query",
                                json_body={"filter": {"EQ": {"i": 7}}})
            assert r.status == 200 and [x["key"] for x in r.json()["results"]] == ["p7"], r.body
            m = (await http.get(f"{b}/metrics")).body.decode()
            got = re.search(r'sidecar_pipelined_requests_total\{app="app-a"\} (\d+)', m)
            assert got and int(got.group(1)) >= 600, m[-800:]  # 200 saves + 200 reads + 200 publishes
            await _until(lambda: len([x for x in seen if x[0] == "event"]) == 200, 10)
            assert sorted(x[2]["n"] for x in seen if x[0] == "event") == list(range(200))
            # the backing goes away: calls fail (500), none hangs; a backing back on the same
            # socket is reached over new connections
            await bsrv.close(0.5)
            r = await asyncio.wait_for(http.post(f"{b}/v1.0/state/statestore", json_body=[{"key": "x", "value": 1}]), 10)
            assert r.status == 500, r.body
            bsrv2 = HttpServer(backing.build_app(), loop)
            await bsrv2.listen_unix(uds)
            try:
                r = await asyncio.wait_for(http.post(f"{b}/v1.0/state/statestore", json_body=[{"key": "x", "value": 1}]), 10)
                assert r.status == 204, r.body
                r = await http.get(f"{b}/v1.0/state/statestore/p3")
                assert r.status == 200 and r.json() == {"i": 3}
            finally:
                await bsrv2.close(1.0)
        finally:
            await sc.stop(1.0)
            await srv.close(1.0)
            await bsrv.close(1.0)
            await http.close()
    run(main())


@pytest.mark.parametrize("plane", PLANES)
def test_sidecar_mutual_tls(plane, tmp_path):
    """Sidecar-to-sidecar calls over mutual TLS with per-app-id workload certificates from the
    environment CA (Dapr Sentry equivalent): invocation works; a peer without a certificate, with
    one from another CA, or claiming another app-id than its certificate names is rejected."""
    import ssl

    from aca_dotnet_workshop_amd.platform.pki import EnvironmentPki

    pki = EnvironmentPki(tmp_path / "pki")
    rogue = EnvironmentPki(tmp_path / "rogue-pki")

    async def main():
        async with Env(plane, tmp_path, apps=("app-a", "app-b"), pki=pki) as e:
            ep = e.sidecars["app-b"].bound_internal
            assert ep.startswith("mtls:app-b@")
            r = await e.http.post(f"{e.base['app-a']}/v1.0/invoke/app-b/method/api/echo/x", body=b"hi")
            assert r.status == 201 and r.json()["app"] == "app-b" and r.json()["body"] == "hi"
            sock = ep.split("@", 1)[1][len("unix:"):].rstrip(":")

            async def raw(ctx, caller="app-a"):
                rd, wr = await asyncio.open_unix_connection(sock, ssl=ctx, server_hostname="app-b")
                wr.write(f"GET /api/echo/y HTTP/1.1\r\nHost: x\r\ndapr-caller-app-id: {caller}\r\n"
                         "Connection: close\r\n\r\n".encode())
                data = await rd.read()
                wr.close()
                return data
            # a legitimate peer identity (app-a's workload certificate) gets through
            ok = await raw(pki.workload("app-a").client_context())
            assert ok.startswith(b"HTTP/1.1 201"), ok[:100]
            # ... but may not claim to be someone else
            spoof = await raw(pki.workload("app-a").client_context(), caller="app-c")
            assert spoof.startswith(b"HTTP/1.1 403") and b"ERR_MESH_AUTH" in spoof
            # no client certificate / a certificate from another CA: the handshake fails
            for ctx in (pki.workload("app-a").client_context(present_cert=False),
                        rogue.workload("app-a").client_context()):
                if ctx is not None and ctx.verify_mode == ssl.CERT_REQUIRED and ctx is not None:
                    ctx.load_verify_locations(pki.ca_crt)  # trust the real server, present whatever
                try:
                    got = await raw(ctx)
                except (ssl.SSLError, ConnectionError, asyncio.IncompleteReadError):
                    got = b""
                assert not got.startswith(b"HTTP/1.1 2"), got[:100]
            # the server side is verified too: a client trusting only another CA refuses app-b
            bad = ssl.SSLContext(ssl.PROTOCOL_TLS_CLIENT)
            bad.load_verify_locations(rogue.ca_crt)
            with pytest.raises(ssl.SSLError):
                await raw(bad)
    run(main())


def test_native_pc_sample_profile(tmp_path, monkeypatch):
    """TT_PC_SAMPLE (native/src/pcsample.hpp): the native data plane samples its own program
    counter and, when it stops, writes a flat profile by module and symbol to <file>.<pid>."""
    prof = tmp_path / "prof"
    monkeypatch.setenv("TT_PC_SAMPLE", str(prof))

    async def main():
        async with Env("native", tmp_path) as e:
            st = f"{e.base['app-a']}/v1.0/state/statestore"
            for i in range(300):
                assert (await e.http.post(st, json_body=[{"key": f"k{i}", "value": {"i": i}}])).status == 204
            return e.sidecars["app-a"]._dp_proc.pid
    pid = run(main())
    text = (tmp_path / f"prof.{pid}").read_text()
    assert text.startswith(f"== dataplane app-a pid {pid}: ")  # the profile names its app
    n = int(re.match(r"== dataplane app-a pid \d+: (\d+) samples", text).group(1))
    assert "-- by module" in text and "-- by symbol" in text
    assert n == 0 or "%" in text.split("-- by module", 1)[1]
