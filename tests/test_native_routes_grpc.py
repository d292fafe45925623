"""The API's native routes over gRPC -- the reference SDK's wire for state and publish.

The reference's ``DaprClient`` saves, queries and publishes over the sidecar's gRPC API
(``TasksStoreManager.cs:35`` SaveStateAsync, ``:61`` QueryStateAsync, ``:155`` PublishEventAsync;
``Dapr.Client`` speaks gRPC for everything but InvokeMethodAsync).  With ``Dapr:ApiProtocol=grpc``
the app host's native routes (apphost.hpp ``api_create`` / ``api_list`` / ``api_overdue``) send
``SaveState`` / ``PublishEvent`` / ``QueryStateAlpha1`` to the sidecar's gRPC port themselves.

Each case runs the real API app on the native host against a recording gRPC sidecar (grpcio on a
Unix socket), once with the native routes and once with them off (``TT_NATIVE_ROUTES=0``: the
Python handlers over ``GrpcSidecarClient``), and compares:
* the answers (status, Location, body, more-results flag);
* every RPC: method, metadata (trace context, token) and the request message, byte for byte
  apart from the new task's id and creation time;
* the log lines and the request metrics;
* a failed RPC: the same error answer as the SDK's (``InvocationError`` from the gRPC status).
"""
import asyncio
import json
import logging
import re

import grpc
import pytest

from aca_dotnet_workshop_amd.sdk import proto as P
from aca_dotnet_workshop_amd.telemetry import REGISTRY
from aca_dotnet_workshop_amd.utils.config import Configuration
from aca_dotnet_workshop_amd.web.client import HttpClient

from helpers import run
from test_native_routes import _LIST, SAMPLED, TID, UNSAMPLED, _api_body, _Lines, _norm_id, _serve

TOKEN = "s3cret"


class GrpcSidecar:
    """Records every unary call (path, metadata, request bytes); answers QueryStateAlpha1 with
    ``query`` and everything else with Empty, unless ``fail[rpc] = (code, details, http)``."""

    def __init__(self, query: bytes = b"", fail: dict | None = None):
        self.calls = []
        self.query = query
        self.fail = fail or {}
        self.server = None

    async def start(self, sock: str) -> None:
        async def handle(path: str, request: bytes, ctx):
            rpc = path.rsplit("/", 1)[-1]
            self.calls.append((path, dict(ctx.invocation_metadata()), request))
            if rpc in self.fail:
                code, details, http = self.fail[rpc]
                ctx.set_trailing_metadata((("dapr-http-status", str(http)),))
                await ctx.abort(code, details)
            return self.query if rpc == "QueryStateAlpha1" else b""

        class Any(grpc.GenericRpcHandler):
            def service(self, details):
                path = details.method

                async def h(request, ctx):
                    return await handle(path, request, ctx)
                return grpc.unary_unary_rpc_method_handler(h)

        self.server = grpc.aio.server()
        self.server.add_generic_rpc_handlers((Any(),))
        self.server.add_insecure_port(f"unix:{sock}")
        await self.server.start()

    async def stop(self) -> None:
        await self.server.stop(0)


def _query_response(tasks, token=""):
    r = P.rt("QueryStateResponse")()
    for t in tasks:
        it = r.results.add()
        it.key = t["taskId"] if t else "gone"
        if t:
            it.data = json.dumps(t).encode()
            it.etag = "1"
    if token:
        r.token = token
    return r.SerializeToString()


def _grpc_scenario(tmp_path, monkeypatch, native, requests, sidecar, route, method="POST", manager_kw=None):
    """``requests`` [(headers, body-or-target)] against the API over gRPC; returns (answers,
    rpcs, log lines, metric delta, python-side sidecar calls)."""
    monkeypatch.setenv("TT_APP_HOST", "native")
    monkeypatch.setenv("TT_NATIVE_ROUTES", "1" if native else "0")
    monkeypatch.setenv("TT_TRACE_SAMPLE_RATE", "0")
    side_sock = str(tmp_path / f"grpc-side-{native}.sock")
    app_sock = str(tmp_path / f"grpc-app-{native}.sock")
    from aca_dotnet_workshop_amd.sdk.grpc_client import GrpcSidecarClient
    from aca_dotnet_workshop_amd.telemetry import tracing
    tracing.configure("native-routes-grpc-test", None, 0.0)
    ok_status = 201 if method == "POST" else 200

    async def main():
        await sidecar.start(side_sock)
        client = GrpcSidecarClient(f"unix:{side_sock}", api_token=TOKEN, timeout=10.0)
        assert client.transport == "native"
        cfg = Configuration([{"APP_PORT": "0", "Environment": "Production", "TT_APP_UDS": app_sock}])
        from aca_dotnet_workshop_amd.services.backend_api import create_app
        from aca_dotnet_workshop_amd.services.backend_api.managers import TasksStoreManager
        app = create_app(config=cfg, manager=TasksStoreManager(client, **(manager_kw or {})))
        python_calls = []
        real = client._call_encoded

        async def counted(*a, **kw):
            python_calls.append(a[0])
            return await real(*a, **kw)
        client._call_encoded = counted
        lines = _Lines()
        logger = logging.getLogger("TasksManager")
        logger.addHandler(lines)
        REGISTRY.collect()
        ctr = REGISTRY.counter("http_requests_total")
        before = ctr.get(method=method, route=route, status=str(ok_status))
        stop, ports = asyncio.Event(), []
        task = asyncio.create_task(_serve(app, app_sock, stop, ports))
        for _ in range(200):
            if ports:
                break
            await asyncio.sleep(0.01)
        c = HttpClient()
        out = []
        try:
            for headers, x in requests:
                if method == "POST":
                    r = await c.post(f"unix:{app_sock}:{route}", body=x, headers=headers)
                else:
                    r = await c.get(f"unix:{app_sock}:{x}", headers=headers)
                out.append((r.status, r.headers.get("location") or r.headers.get("x-tt-more-results"),
                            r.headers.get("content-type"), r.body))
        finally:
            await c.close()
            stop.set()
            await task
            await sidecar.stop()
            await client.close()
            logger.removeHandler(lines)
        REGISTRY.collect()
        return out, sidecar.calls, lines.lines, ctr.get(method=method, route=route, status=str(ok_status)) - before, \
            python_calls
    return run(main())


def _norm_rpc(call):
    """(method, traceparent's trace id and flags, token, the request message as a dict with the
    new task's id / creation time masked)."""
    from google.protobuf.json_format import MessageToDict
    path, md, raw = call
    req_cls, _ = P.rpc_types(path.rsplit("/", 1)[-1])
    msg = req_cls.FromString(raw)
    d = MessageToDict(msg, preserving_proto_field_name=True)
    for k in ("value", "data"):  # bytes fields: the JSON they carry
        for holder in [d] + list(d.get("states", [])):
            if k in holder:
                import base64
                holder[k] = json.loads(base64.b64decode(holder[k]))
    text = _norm_id(json.dumps(d, sort_keys=True))
    text = re.sub(r'"taskCreatedOn": "[^"]+"', '"taskCreatedOn": "<now>"', text)
    tp = md.get("traceparent", "")
    return path, tp[:36], tp[52:], md.get("dapr-api-token"), text, raw.startswith(b"\n")


_FAIL_SAVE = {"SaveState": (grpc.StatusCode.INTERNAL, "failed saving state in state store statestore", 500)}
_FAIL_PUB = {"PublishEvent": (grpc.StatusCode.NOT_FOUND, "pubsub dapr-pubsub-servicebus not found", 404)}


@pytest.mark.parametrize("fail", [{}, _FAIL_SAVE, _FAIL_PUB], ids=["ok", "save-fails", "publish-fails"])
def test_api_create_grpc_native_equals_python(tmp_path, monkeypatch, fail):
    reqs = [([("Content-Type", "application/json"), ("traceparent", UNSAMPLED)], _api_body()),
            ([("traceparent", UNSAMPLED)], _api_body("Ünïcode ✓ 'quoted'"))]
    got = {n: _grpc_scenario(tmp_path, monkeypatch, n, reqs, GrpcSidecar(fail=fail), "/api/tasks") for n in (True, False)}
    (rn, cn, ln, mn, pn), (rp, cp, lp, mp, pp) = got[True], got[False]
    assert pn == [] and len(pp) == (2 if fail == _FAIL_SAVE else 4)  # the host made the RPCs itself
    norm = lambda rs: [(s, _norm_id(loc or ""), ct, b if s >= 400 else b"") for s, loc, ct, b in rs]
    assert norm(rn) == norm(rp)
    assert [_norm_rpc(c) for c in cn] == [_norm_rpc(c) for c in cp]
    for path, md, _ in cn:  # the route's own span: the caller's trace, unsampled, a new span id
        assert md["traceparent"].startswith(f"00-{TID}-") and md["traceparent"] != UNSAMPLED
        assert md["dapr-api-token"] == TOKEN
    assert [_norm_id(x) for x in ln] == [_norm_id(x) for x in lp]
    assert mn == mp
    if not fail:
        assert [s for s, *_ in rn] == [201, 201] and mn == 2
        assert [c[0].rsplit("/", 1)[1] for c in cn] == ["SaveState", "PublishEvent"] * 2
        save = P.rt("SaveStateRequest").FromString(cn[0][2])
        pub = P.rt("PublishEventRequest").FromString(cn[1][2])
        assert save.store_name == "statestore" and (pub.pubsub_name, pub.topic) == ("dapr-pubsub-servicebus", "tasksavedtopic")
        assert rn[0][1] == f"/api/tasks/{save.states[0].key}" and json.loads(pub.data)["taskId"] == save.states[0].key
        assert pub.data == save.states[0].value and pub.data_content_type == "application/json"
        # the request messages are the ones sdk/grpc_client.py writes, byte for byte
        from aca_dotnet_workshop_amd.sdk.grpc_client import encode_publish_event, encode_save_state
        assert cn[0][2] == encode_save_state("statestore", save.states[0].key, save.states[0].value)
        assert cn[1][2] == encode_publish_event("dapr-pubsub-servicebus", "tasksavedtopic", pub.data, "application/json")
    else:
        assert [s for s, *_ in rn] == [500, 500]  # the SDK's InvocationError, answered by the pipeline


def test_api_create_grpc_leaves_sampled_traces_to_python(tmp_path, monkeypatch):
    reqs = [([("traceparent", SAMPLED)], _api_body())]
    rn, cn, _, _, pn = _grpc_scenario(tmp_path, monkeypatch, True, reqs, GrpcSidecar(), "/api/tasks")
    assert rn[0][0] == 201 and pn == ["SaveState", "PublishEvent"] and len(cn) == 2


def test_api_create_grpc_sidecar_unreachable_is_the_sdks_503(tmp_path, monkeypatch):
    """A transport error on the route's RPC: the SDK's ``sidecar unreachable`` InvocationError
    (503), as GrpcSidecarClient raises it, in both modes."""
    class Down(GrpcSidecar):
        async def start(self, sock):
            self.calls = []

        async def stop(self):
            pass
    reqs = [([("traceparent", UNSAMPLED)], _api_body())]
    got = {n: _grpc_scenario(tmp_path, monkeypatch, n, reqs, Down(), "/api/tasks") for n in (True, False)}
    assert got[True][0][0][0] == got[False][0][0][0] == 500
    assert got[True][2] == got[False][2]


@pytest.mark.parametrize("fail", [{}, {"QueryStateAlpha1": (grpc.StatusCode.INTERNAL, "query failed", 500)}],
                         ids=["ok", "query-fails"])
def test_api_list_grpc_native_equals_python(tmp_path, monkeypatch, fail):
    q = _query_response(_LIST + [None])
    reqs = [([("traceparent", UNSAMPLED)], "/api/tasks?createdBy=me%40x.y"),
            ([("traceparent", UNSAMPLED)], "/api/tasks?CreatedBy=a+%22b%22&createdby=ignored"),
            ([("traceparent", UNSAMPLED)], "/api/tasks")]
    got = {n: _grpc_scenario(tmp_path, monkeypatch, n, reqs, GrpcSidecar(q, fail), "/api/tasks", "GET")
           for n in (True, False)}
    (rn, cn, _, mn, pn), (rp, cp, _, mp, pp) = got[True], got[False]
    assert [r[:1] + r[2:] for r in rn] == [r[:1] + r[2:] for r in rp]
    assert [_norm_rpc(c) for c in cn] == [_norm_rpc(c) for c in cp]
    assert mn == mp
    if not fail:
        assert pn == [] and pp == ["QueryStateAlpha1"] * 2
        assert [t["taskId"][-4:] for t in json.loads(rn[0][3])] == ["e0f1", "950e"]  # newest first
        q0 = P.rt("QueryStateRequest").FromString(cn[1][2])
        assert q0.store_name == "statestore" and json.loads(q0.query) == {"filter": {"EQ": {"taskCreatedBy": 'a "b"'}}}


@pytest.mark.parametrize("fail", [{}, {"QueryStateAlpha1": (grpc.StatusCode.RESOURCE_EXHAUSTED, "throttled", 429)}],
                         ids=["ok", "query-fails"])
def test_api_overdue_grpc_native_equals_python(tmp_path, monkeypatch, fail):
    q = _query_response(_LIST, token="2")
    reqs = [([("traceparent", UNSAMPLED)], "/api/overduetasks?limit=512"),
            ([("traceparent", UNSAMPLED)], "/api/overduetasks")]
    kw = {"overdue_query": "range", "overdue_page": 100}
    got = {n: _grpc_scenario(tmp_path, monkeypatch, n, reqs, GrpcSidecar(q, fail), "/api/overduetasks", "GET", kw)
           for n in (True, False)}
    (rn, cn, ln, mn, pn), (rp, cp, lp, mp, pp) = got[True], got[False]
    assert rn == rp and [_norm_rpc(c) for c in cn] == [_norm_rpc(c) for c in cp] and mn == mp and ln == lp
    if not fail:
        assert pn == [] and len(pp) == 2
        assert [r[1] for r in rn] == ["true", "true"]
        assert [t["taskId"][-4:] for t in json.loads(rn[0][3])] == ["950e", "e0f1"]  # oldest first
    else:
        assert [r[0] for r in rn] == [500, 500]


def test_query_response_json_matches_the_http_layout():
    """GrpcSidecarClient.query_state_raw's JSON is the HTTP API's layout, which the task codec's
    one-pass reader takes (same page as from the HTTP answer)."""
    from aca_dotnet_workshop_amd.models import tasks_from_query_wire
    from aca_dotnet_workshop_amd.sdk.grpc_client import query_response_json
    raw = query_response_json(_query_response(_LIST + [None], token="7"))
    doc = json.loads(raw)
    assert doc["token"] == "7" and doc["results"][-1] == {"key": "gone", "data": None, "etag": ""}
    http = json.dumps({"results": [{"key": t["taskId"], "data": t, "etag": "1"} for t in _LIST], "token": "7"}).encode()
    assert tasks_from_query_wire(raw, by_created=True)[1] == tasks_from_query_wire(http, by_created=True)[1]
