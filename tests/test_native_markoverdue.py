"""``POST api/overduetasks/markoverdue`` as a native route of the app host (apphost.hpp
``api_markoverdue``), over both Dapr protocols, against the Python handler
(``TasksStoreManager.mark_overdue_from_body``, ``TT_NATIVE_ROUTES=0``).

Reference: ``OverdueTasksController.cs:26-32`` -> ``TasksStoreManager.MarkOverdueTasks``
(``:141-149``).  Here the mark is conditional: the page's tasks are read back
with their ETags, only the ones still open and not yet overdue are written, each guarded by its
ETag (first-write), and a conflict re-reads and re-applies.

A fake sidecar keeps a small store: ``docs`` id -> (task, etag).  Its first save can be made to
conflict after "completing" one of the tasks in between (a concurrent completion), so the second
pass must skip that task.  Both modes must make the same calls with the same bodies, log the
same lines, leave the store in the same state and answer the same.
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

IDS = ["2b0c7a4e-3f51-4a77-9c39-4a1f3d54e0f1", "0f8fad5b-d9cb-469f-a165-70867728950e",
       "7c9e6679-7425-40de-944b-e07fc1f90ae7", "16fd2706-8baf-433b-82eb-8c7fada847da"]


def _task(i, done=False, over=False, name=None):
    return {"taskId": IDS[i], "taskName": name or f"t{i}", "taskCreatedBy": "a@b.c",
            "taskCreatedOn": f"2030-01-01T10:00:0{i}.1234567Z", "taskDueDate": "2029-12-30T00:00:00",
            "taskAssignedTo": "x@y.z", "isCompleted": done, "isOverDue": over}


class Store:
    """id -> (task dict, etag); ``conflict``: the first save fails after task 1 got completed."""

    def __init__(self, conflict=False):
        self.docs = {IDS[0]: (_task(0, name="Ünïcode 'q'"), "1"), IDS[1]: (_task(1), "1"),
                     IDS[2]: (_task(2, done=True), "1")}  # IDS[3]: deleted since the query
        self.conflict = conflict
        self.calls = []

    def bulk(self, keys):
        return [{"key": k, "data": self.docs[k][0], "etag": self.docs[k][1]} if k in self.docs else {"key": k}
                for k in keys]

    def save(self, items):
        """items: [(key, value dict, etag, first_write)] -> status"""
        if self.conflict:
            self.conflict = False
            t, e = self.docs[IDS[1]]
            self.docs[IDS[1]] = (dict(t, isCompleted=True), str(int(e) + 1))  # a completion landed
            return 409
        for key, value, etag, fw in items:
            if fw and self.docs[key][1] != etag:
                return 409
        for key, value, etag, fw in items:
            self.docs[key] = (value, str(int(self.docs[key][1]) + 1))
        return 204


async def _http_sidecar(store, sock, loop):
    app = WebApp("fake-sidecar")

    async def bulk(req):
        keys = json.loads(req.body)["keys"]
        store.calls.append(("bulk", keys, json.loads(req.body)["parallelism"]))
        return Response(json.dumps(store.bulk(keys), separators=(",", ":")).encode(), 200, None, "application/json")

    async def save(req):
        items = json.loads(req.body)
        store.calls.append(("save", items))
        st = store.save([(i["key"], i["value"], i.get("etag"), (i.get("options") or {}).get("concurrency") == "first-write")
                         for i in items])
        return Response(b'{"errorCode":"ERR_STATE_SAVE"}' if st == 409 else b"", st, None, "application/json")
    app.add_route("/v1.0/state/statestore/bulk", bulk, ("POST",))
    app.add_route("/v1.0/state/statestore", save, ("POST",))
    srv = HttpServer(app, loop)
    await srv.listen_unix(sock)
    return srv


async def _grpc_sidecar(store, sock):
    async def handle(path, request, ctx):
        rpc = path.rsplit("/", 1)[-1]
        if rpc == "GetBulkState":
            req = P.rt("GetBulkStateRequest").FromString(request)
            store.calls.append(("bulk", list(req.keys), req.parallelism))
            out = P.rt("GetBulkStateResponse")()
            for it in store.bulk(list(req.keys)):
                x = out.items.add(key=it["key"])
                if "data" in it:
                    x.data = json.dumps(it["data"]).encode()
                    x.etag = it["etag"]
            return out.SerializeToString()
        req = P.rt("SaveStateRequest").FromString(request)
        items = [{"key": s.key, "value": json.loads(s.value), "etag": s.etag.value,
                  "options": {"concurrency": "first-write"} if s.options.concurrency == 1 else {}} for s in req.states]
        store.calls.append(("save", items, request))
        st = store.save([(i["key"], i["value"], i["etag"], bool(i["options"])) for i in items])
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


def _scenario(tmp_path, monkeypatch, protocol, native, conflict, body):
    monkeypatch.setenv("TT_APP_HOST", "native")
    monkeypatch.setenv("TT_NATIVE_ROUTES", "1" if native else "0")
    monkeypatch.setenv("TT_TRACE_SAMPLE_RATE", "0")
    side_sock = str(tmp_path / f"mside-{protocol}-{native}.sock")
    app_sock = str(tmp_path / f"mapp-{protocol}-{native}.sock")
    from aca_dotnet_workshop_amd.telemetry import tracing
    tracing.configure("native-markoverdue-test", None, 0.0)
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
        real = manager._mark_conditionally

        async def counted(ids):
            python_calls.append(ids)
            return await real(ids)
        manager._mark_conditionally = counted
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
        try:
            r = await c.post(f"unix:{app_sock}:/api/overduetasks/markoverdue", body=body,
                             headers=[("Content-Type", "application/json"), ("traceparent", UNSAMPLED)])
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
        return (r.status, r.body), [c[:2] if c[0] == "bulk" else c[:2] for c in store.calls], \
            [c for c in store.calls if c[0] == "save"], lines.lines, store.docs, python_calls
    return run(main())


def _page(*idx):
    return json.dumps([_task(i) for i in idx] + [_task(0)]).encode()  # a duplicate id too


@pytest.mark.parametrize("protocol", ["http", "grpc"])
@pytest.mark.parametrize("conflict", [False, True], ids=["clean", "conflict"])
def test_markoverdue_native_equals_python(tmp_path, monkeypatch, protocol, conflict):
    body = _page(0, 1, 2, 3)
    got = {n: _scenario(tmp_path, monkeypatch, protocol, n, conflict, body) for n in (True, False)}
    (rn, cn, sn, ln, dn, pn), (rp, cp, sp, lp, dp, pp) = got[True], got[False]
    assert pn == [] and len(pp) == 1  # the host ran the whole pass itself
    assert rn == rp and rn[0] == 200
    assert cn == cp  # the same bulk gets (ids deduplicated, in order) and saves, the same bodies
    if protocol == "grpc":  # the SaveStateRequest bytes too
        assert [s[2] for s in sn] == [s[2] for s in sp]
    assert ln == lp and dn == dp
    marked = [IDS[0]] if conflict else [IDS[0], IDS[1]]
    assert ln == [f"Mark task with Id: '{i}' as OverDue task" for i in ([IDS[0], IDS[1]] + marked if conflict else marked)]
    assert [k for k, (t, _) in dn.items() if t["isOverDue"]] == marked
    assert dn[IDS[2]][0]["isOverDue"] is False  # completed: never marked
    assert cn[0] == ("bulk", IDS) and len(sn) == (2 if conflict else 1)
    if conflict:  # the second pass re-read only the tasks the first one tried to write
        assert cn[2] == ("bulk", [IDS[0], IDS[1]])
    first = sn[0][1]
    assert all(it["options"] == {"concurrency": "first-write"} and it["etag"] == "1" for it in first)


@pytest.mark.parametrize("protocol", ["http", "grpc"])
def test_markoverdue_native_leaves_odd_bodies_to_python(tmp_path, monkeypatch, protocol):
    body = b'{"not": "a list"}'  # not a TaskModel array: the binder's 400
    rn = _scenario(tmp_path, monkeypatch, protocol, True, False, body)
    rp = _scenario(tmp_path, monkeypatch, protocol, False, False, body)
    assert rn[0][0] == rp[0][0] == 400 and rn[1] == rp[1] == []
    # snake_case fields: the native binder declines, the general binder takes them (as Python)
    body = json.dumps([{"task_id": IDS[0]}]).encode()
    rn = _scenario(tmp_path, monkeypatch, protocol, True, False, body)
    rp = _scenario(tmp_path, monkeypatch, protocol, False, False, body)
    assert rn[0] == rp[0] and rn[1] == rp[1] and rn[4] == rp[4] and len(rn[5]) == 1


def test_dapr_pb_save_state_bulk_matches_the_sdk_message():
    """daprpb.hpp save_state_bulk writes what protobuf writes for the SDK's SaveStateRequest."""
    from aca_dotnet_workshop_amd.native import load
    N = load()
    body = json.dumps([{"key": "a", "value": {"x": 1, "s": "Ü"}, "etag": "7", "options": {"concurrency": "first-write"}},
                       {"key": "b\"q", "value": "text", "metadata": {"ttlInSeconds": "5"},
                        "options": {"consistency": "strong"}}], ensure_ascii=False).encode()
    got = N.dapr_pb_save_state_bulk("statestore", body)
    req = P.rt("SaveStateRequest")(store_name="statestore")
    a = req.states.add(key="a", value=json.dumps({"x": 1, "s": "Ü"}, separators=(",", ":"), ensure_ascii=False).encode())
    a.etag.value = "7"
    a.options.concurrency = 1
    b = req.states.add(key="b\"q", value=b'"text"')
    b.metadata["ttlInSeconds"] = "5"
    b.options.consistency = 2
    assert P.rt("SaveStateRequest").FromString(got) == req
    assert got == req.SerializeToString(deterministic=True)
    assert N.dapr_pb_save_state_bulk("s", b"[{\"value\": 1}]") is None  # no key
