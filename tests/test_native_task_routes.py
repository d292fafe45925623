"""The API's single-task routes on the app host's I/O thread (apphost.hpp ``api_task``) --
``GET / PUT / PUT markcomplete / DELETE api/tasks/{id}`` (TasksController.cs:26-75 over
TasksStoreManager.cs:40-99) -- over both Dapr protocols, against the Python handlers
(``TT_NATIVE_ROUTES=0``: the manager's codec paths).

A fake sidecar keeps a small store (id -> (task, etag)) with first-write ETag checks, and can
make the first save of a read-modify-write conflict after a concurrent edit landed, so the route
must re-read and re-apply.  Both modes must send the same calls (bodies, ETags, If-Match), log
the same lines, publish on an assignee change only, leave the same store and answer the same.
"""
import asyncio
import json
import logging

import grpc
import pytest

from aca_dotnet_workshop_amd.sdk import proto as P
from aca_dotnet_workshop_amd.utils.config import Configuration
from aca_dotnet_workshop_amd.web import WebApp
from aca_dotnet_workshop_amd.web.client import HttpClient
from aca_dotnet_workshop_amd.web.http import Response
from aca_dotnet_workshop_amd.web.server import HttpServer

from helpers import run
from test_native_routes import UNSAMPLED, _Lines, _serve

A, B, GONE = "2b0c7a4e-3f51-4a77-9c39-4a1f3d54e0f1", "0f8fad5b-d9cb-469f-a165-70867728950e", \
    "16fd2706-8baf-433b-82eb-8c7fada847da"


def _task(tid, name, who="x@y.z"):
    return {"taskId": tid, "taskName": name, "taskCreatedBy": "a@b.c", "taskCreatedOn": "2030-01-01T10:00:00.1234567Z",
            "taskDueDate": "2029-12-30T00:00:00", "taskAssignedTo": who, "isCompleted": False, "isOverDue": False}


class Store:
    def __init__(self, conflict=False):
        self.docs = {A: (json.dumps(_task(A, "Ünïcode 'q'"), ensure_ascii=False).encode(), "1"),
                     B: (json.dumps(_task(B, "plain", "X@Y.Z")).encode(), "3")}
        self.conflict = conflict
        self.calls = []
        self.published = []

    def get(self, key):
        self.calls.append(("get", key))
        return self.docs.get(key, (None, None))

    def save(self, items):
        self.calls.append(("save", [(i["key"], i.get("etag"), i["options"], json.loads(i["value"])) for i in items]))
        if self.conflict:  # someone else's edit landed between the read and this save
            self.conflict = False
            k = items[0]["key"]
            doc, e = self.docs[k]
            self.docs[k] = (json.dumps(dict(json.loads(doc), taskName="theirs")).encode(), str(int(e) + 1))
            return 409
        for i in items:
            if i["options"].get("concurrency") == "first-write" and self.docs[i["key"]][1] != i.get("etag"):
                return 409
        for i in items:
            self.docs[i["key"]] = (i["value"], str(int(self.docs[i["key"]][1]) + 1))
        return 204

    def delete(self, key, etag):
        self.calls.append(("delete", key, etag))
        if key in self.docs and etag and self.docs[key][1] != etag:
            return 409
        self.docs.pop(key, None)
        return 204


async def _http_sidecar(store, sock, loop):
    app = WebApp("fake-sidecar")

    async def get(req):
        doc, etag = store.get(req.path_params["key"])
        if doc is None:
            return Response(b"", 204)
        return Response(doc, 200, [("ETag", etag)], "application/json")

    async def save(req):
        items = [dict(i, value=json.dumps(i["value"], ensure_ascii=False).encode()) for i in json.loads(req.body)]
        st = store.save(items)
        return Response(b'{"errorCode":"ERR_STATE_SAVE"}' if st == 409 else b"", st, None, "application/json")

    async def delete(req):
        st = store.delete(req.path_params["key"], req.headers.get("if-match"))
        return Response(b'{"errorCode":"ERR_STATE_DELETE"}' if st == 409 else b"", st, None, "application/json")

    async def publish(req):
        store.published.append((req.content_type, json.loads(req.body)))
        return Response(b"", 204)
    app.add_route("/v1.0/state/statestore/{key}", get, ("GET",))
    app.add_route("/v1.0/state/statestore/{key}", delete, ("DELETE",))
    app.add_route("/v1.0/state/statestore", save, ("POST",))
    app.add_route("/v1.0/publish/dapr-pubsub-servicebus/tasksavedtopic", publish, ("POST",))
    srv = HttpServer(app, loop)
    await srv.listen_unix(sock)
    return srv


async def _grpc_sidecar(store, sock):
    async def handle(path, request, ctx):
        rpc = path.rsplit("/", 1)[-1]
        if rpc == "GetState":
            req = P.rt("GetStateRequest").FromString(request)
            doc, etag = store.get(req.key)
            out = P.rt("GetStateResponse")()
            if doc is not None:
                out.data, out.etag = doc, etag
            return out.SerializeToString()
        if rpc == "SaveState":
            req = P.rt("SaveStateRequest").FromString(request)
            st = store.save([{"key": s.key, "value": s.value, "etag": s.etag.value if s.HasField("etag") else None,
                              "options": {"concurrency": "first-write"} if s.options.concurrency == 1 else {}}
                             for s in req.states])
        elif rpc == "DeleteState":
            req = P.rt("DeleteStateRequest").FromString(request)
            st = store.delete(req.key, req.etag.value if req.HasField("etag") else None)
        else:
            req = P.rt("PublishEventRequest").FromString(request)
            store.published.append((req.data_content_type, json.loads(req.data)))
            st = 204
        if st == 409:
            ctx.set_trailing_metadata((("dapr-http-status", "409"),))
            await ctx.abort(grpc.StatusCode.ABORTED, "possible etag mismatch")
        return b""

    class Any(grpc.GenericRpcHandler):
        def service(self, details):
            path = details.method

            async def h(request, ctx):
                return await handle(path, request, ctx)
            return grpc.unary_unary_rpc_method_handler(h)
    server = grpc.aio.server()
    server.add_generic_rpc_handlers((Any(),))
    server.add_insecure_port(f"unix:{sock}")
    await server.start()
    return server


def _scenario(tmp_path, monkeypatch, protocol, native, requests, conflict=False):
    """``requests``: [(method, target, body)]; returns (answers, store calls, published, log
    lines, final store, python-side codec calls)."""
    monkeypatch.setenv("TT_APP_HOST", "native")
    monkeypatch.setenv("TT_NATIVE_ROUTES", "1" if native else "0")
    monkeypatch.setenv("TT_TRACE_SAMPLE_RATE", "0")
    side_sock = str(tmp_path / f"tside-{protocol}-{native}.sock")
    app_sock = str(tmp_path / f"tapp-{protocol}-{native}.sock")
    from aca_dotnet_workshop_amd.telemetry import tracing
    tracing.configure("native-task-routes-test", None, 0.0)
    store = Store(conflict)

    async def main():
        loop = asyncio.get_running_loop()
        if protocol == "grpc":
            from aca_dotnet_workshop_amd.sdk.grpc_client import GrpcSidecarClient
            srv = await _grpc_sidecar(store, side_sock)
            client = GrpcSidecarClient(f"unix:{side_sock}", timeout=10.0)
        else:
            from aca_dotnet_workshop_amd.sdk.client import SidecarClient
            srv = await _http_sidecar(store, side_sock, loop)
            client = SidecarClient(f"unix:{side_sock}:")
        from aca_dotnet_workshop_amd.services.backend_api import create_app
        from aca_dotnet_workshop_amd.services.backend_api.managers import TasksStoreManager
        cfg = Configuration([{"APP_PORT": "0", "Environment": "Production", "TT_APP_UDS": app_sock}])
        manager = TasksStoreManager(client)
        python_calls = []
        real = client.get_state_raw

        async def counted(*a):
            python_calls.append(a[1])
            return await real(*a)
        client.get_state_raw = counted
        app = create_app(config=cfg, manager=manager)
        lines = _Lines()
        logger = logging.getLogger("TasksManager")
        logger.addHandler(lines)
        stop, ports = asyncio.Event(), []
        task = asyncio.create_task(_serve(app, app_sock, stop, ports))
        for _ in range(200):
            if ports:
                break
            await asyncio.sleep(0.01)
        c = HttpClient()
        out = []
        try:
            for method, target, body in requests:
                r = await c.request(method, f"unix:{app_sock}:{target}", body=body,
                                    headers=[("traceparent", UNSAMPLED)] +
                                    ([("Content-Type", "application/json")] if body else []))
                out.append((r.status, r.headers.get("content-type"), r.body))
        finally:
            await c.close()
            stop.set()
            await task
            if protocol == "grpc":
                await srv.stop(0)
            else:
                await srv.close(1)
            await client.close()
            logger.removeHandler(lines)
        return out, store.calls, store.published, lines.lines, store.docs, python_calls
    return run(main())


def _upd(tid, name, who):
    return json.dumps({"taskId": tid, "taskName": name, "taskDueDate": "2030-02-01", "taskAssignedTo": who},
                      ensure_ascii=False).encode()


REQS = [("GET", f"/api/tasks/{A}", b""), ("GET", f"/api/tasks/{GONE}", b""),
        ("PUT", f"/api/tasks/{A}", _upd(A, "renamed ✓", "x@y.z")),          # same assignee: no publish
        ("PUT", f"/api/tasks/{B}", _upd(B, "moved", "someone@else")),       # assignee changed: publish
        ("PUT", f"/api/tasks/{B}", _upd(B, "case only", "SOMEONE@ELSE")),   # case-insensitive: no publish
        ("PUT", f"/api/tasks/{GONE}", _upd(GONE, "n", "w")),                 # missing: 400
        ("PUT", f"/api/tasks/{A}/markcomplete", b""), ("PUT", f"/api/tasks/{GONE}/markcomplete", b""),
        ("DELETE", f"/api/tasks/{B}", b""), ("DELETE", f"/api/tasks/{GONE}", b""),
        ("GET", f"/api/tasks/{A}", b"")]


@pytest.mark.parametrize("protocol", ["http", "grpc"])
def test_task_routes_native_equal_python(tmp_path, monkeypatch, protocol):
    got = {n: _scenario(tmp_path, monkeypatch, protocol, n, REQS) for n in (True, False)}
    (rn, cn, pubn, ln, dn, pn), (rp, cp, pubp, lp, dp, pp) = got[True], got[False]
    assert pn == [] and len(pp) >= 10  # the host read and wrote every task itself
    assert rn == rp
    assert [r[0] for r in rn] == [200, 404, 200, 200, 200, 400, 200, 400, 200, 404, 200]
    assert cn == cp and pubn == pubp and ln == lp and dn == dp
    assert len(pubn) == 1 and pubn[0][0] == "application/json" and pubn[0][1]["taskAssignedTo"] == "someone@else"
    final = json.loads(rn[-1][2])
    assert final["taskName"] == "renamed ✓" and final["isCompleted"] is True and B not in dn
    saves = [c for c in cn if c[0] == "save"]
    assert all(s[1][0][2] == {"concurrency": "first-write"} for s in saves)
    assert ("delete", B, "5") in cn  # guarded by the ETag it read


@pytest.mark.parametrize("protocol", ["http", "grpc"])
def test_task_route_rereads_on_a_conflict(tmp_path, monkeypatch, protocol):
    reqs = [("PUT", f"/api/tasks/{A}/markcomplete", b"")]
    got = {n: _scenario(tmp_path, monkeypatch, protocol, n, reqs, conflict=True) for n in (True, False)}
    (rn, cn, _, ln, dn, pn), (rp, cp, _, lp, dp, pp) = got[True], got[False]
    assert rn == rp and rn[0][0] == 200 and cn == cp and dn == dp and ln == lp
    assert [c[0] for c in cn] == ["get", "save", "get", "save"]
    doc = json.loads(dn[A][0])
    assert doc["taskName"] == "theirs" and doc["isCompleted"] is True  # their edit kept, ours applied on top


@pytest.mark.parametrize("protocol", ["http", "grpc"])
def test_task_routes_leave_other_spellings_to_python(tmp_path, monkeypatch, protocol):
    reqs = [("GET", f"/api/tasks/{A.upper()}", b""), ("GET", f"/api/tasks/{{{A}}}", b""), ("GET", "/api/tasks/nope", b""),
            ("PUT", f"/api/tasks/{A}", b'{"task_name": "snake"}')]
    got = {n: _scenario(tmp_path, monkeypatch, protocol, n, reqs) for n in (True, False)}
    (rn, cn, _, ln, dn, pn), (rp, cp, _, lp, dp, pp) = got[True], got[False]
    assert rn == rp and [r[0] for r in rn] == [200, 200, 400, 200] and cn == cp and dn == dp
    # the host left the upper-case and braced ids to Python's codec path, and the snake_case body
    # to its general binder (which reads through get_state_and_etag)
    assert pn == [A, A] and any(c == ("get", A) for c in cn[2:])
