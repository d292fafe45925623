"""Native routes of the app host (``native/src/apphost.hpp`` NativeRoute, ``web/native_host.py``
``NativeHttpServer.native_route``): the frontend's ``POST /Tasks/Create`` and the API's
``POST /api/tasks`` served end to end on the I/O thread, against the same apps with the routes
off (``TT_NATIVE_ROUTES=0``: the Python handlers).

Each scenario runs the real app under ``serve_host`` on the native host, with a recording
sidecar on a Unix socket. It compares:
* the response (status, Location);
* every sidecar call: method, path, content type, trace context, body;
* the log lines;
* the request metrics.

It also checks what goes to Python instead:
* bodies the codec declines, bad antiforgery tokens, sampled traces;
* failed sidecar calls, answered with the same error as the Python path;
* a client's own ``x-tt-native`` header, which never reaches the app.
"""
import asyncio
import json
import logging
import re

import pytest

from aca_dotnet_workshop_amd.telemetry import REGISTRY
from aca_dotnet_workshop_amd.utils.config import Configuration
from aca_dotnet_workshop_amd.web import WebApp
from aca_dotnet_workshop_amd.web.client import HttpClient
from aca_dotnet_workshop_amd.web.http import Response
from aca_dotnet_workshop_amd.web.server import HttpServer

from helpers import run

TID = "4bf92f3577b34da6a3ce929d0e0e4736"
UNSAMPLED = f"00-{TID}-00f067aa0ba902b7-00"
SAMPLED = f"00-{TID}-00f067aa0ba902b7-01"


class Sidecar:
    """Records every call; answers with ``status[path prefix]`` (default 204 / 200)."""

    def __init__(self):
        self.calls = []
        self.status: dict[str, tuple[int, bytes]] = {}
        app = WebApp("fake-sidecar")

        async def any_route(req):
            self.calls.append((req.method, req.target, dict(req.headers), req.body))
            for prefix, (st, body) in self.status.items():
                if req.target.startswith(prefix):
                    return Response(body, st, None, "application/json")
            return Response(b"", 204)
        app.add_route("/{*path}", any_route, ("GET", "POST", "PUT", "DELETE"))
        self.app = app


async def _serve(app, sock, stop, ports):
    from aca_dotnet_workshop_amd.services.hosting import serve_host
    await serve_host(app, stop, lambda p: ports.append(p))


class _Lines(logging.Handler):
    def __init__(self):
        super().__init__(logging.INFO)
        self.lines = []

    def emit(self, record):
        self.lines.append(record.getMessage())


def _requests_total(route, status):
    REGISTRY.collect()
    return REGISTRY.counter("http_requests_total").get(method="POST", route=route, status=str(status))


def _scenario(tmp_path, monkeypatch, which, native, sidecar_status, requests, attach=True):
    """Run ``requests`` [(headers, body)] against the app ``which`` ('api' | 'frontend'); returns
    (responses, sidecar calls, log lines, metric deltas)."""
    monkeypatch.setenv("TT_APP_HOST", "native")
    monkeypatch.setenv("TT_NATIVE_ROUTES", "1" if native else "0")
    monkeypatch.setenv("TT_TRACE_SAMPLE_RATE", "0")
    side_sock = str(tmp_path / f"side-{which}-{native}.sock")
    app_sock = str(tmp_path / f"app-{which}-{native}.sock")
    from aca_dotnet_workshop_amd.sdk.client import SidecarClient
    from aca_dotnet_workshop_amd.telemetry import tracing
    tracing.configure("native-routes-test", None, 0.0)
    route = {"api": "/api/tasks", "frontend": "/Tasks/Create", "processor": "/api/tasksnotifier/tasksaved"}[which]
    ok_status = {"api": 201, "frontend": 302, "processor": 200}[which]

    async def main():
        loop = asyncio.get_running_loop()
        side = Sidecar()
        side.status.update(sidecar_status)
        srv = HttpServer(side.app, loop)
        await srv.listen_unix(side_sock)
        client = SidecarClient(f"unix:{side_sock}:")
        cfg = Configuration([{"APP_PORT": "0", "Environment": "Production", "TT_APP_UDS": app_sock}])
        if which == "api":
            from aca_dotnet_workshop_amd.services.backend_api import create_app
            from aca_dotnet_workshop_amd.services.backend_api.managers import TasksStoreManager
            app = create_app(config=cfg, manager=TasksStoreManager(client))
            logger = logging.getLogger("TasksManager")
        elif which == "processor":
            from aca_dotnet_workshop_amd.services.processor import create_app
            app = create_app([], client=client, config=cfg)
            logger = logging.getLogger("TasksNotifierController")
        else:
            from aca_dotnet_workshop_amd.services.frontend import create_app
            app = create_app([], client=client, overrides={"Frontend:AntiforgeryKey": "k3y", "APP_PORT": "0",
                                                           "Environment": "Production", "TT_APP_UDS": app_sock})
            logger = logging.getLogger("Frontend")
        python_calls = []  # the Python handler's own work (not reached when the host serves)
        if which == "api":
            real, real_one = client.save_state_body, client.save_state

            async def counted(store, body):
                python_calls.append(1)
                return await real(store, body)

            async def counted_one(*a, **kw):
                python_calls.append(1)
                return await real_one(*a, **kw)
            client.save_state_body, client.save_state = counted, counted_one
        elif which == "processor":
            from aca_dotnet_workshop_amd.services.processor import app as proc
            real_name = proc.task_model_name

            def counted_name(body):
                python_calls.append(1)
                return real_name(body)
            monkeypatch.setattr(proc, "task_model_name", counted_name)
        else:
            gw = app.services["backend"]
            real_call = gw.call

            async def counted_call(*a, **kw):
                python_calls.append(1)
                return await real_call(*a, **kw)
            gw.call = counted_call
        lines = _Lines()
        if attach:
            logger.addHandler(lines)
        before = _requests_total(route, ok_status)
        stop, ports = asyncio.Event(), []
        task = asyncio.create_task(_serve(app, app_sock, stop, ports))
        for _ in range(200):
            if ports:
                break
            await asyncio.sleep(0.01)
        c = HttpClient()
        out = []
        try:
            for headers, body in requests:
                r = await c.post(f"unix:{app_sock}:{route}", body=body, headers=headers)
                out.append((r.status, r.headers.get("location"), r.headers.get("content-type"), r.body))
        finally:
            await c.close()
            stop.set()
            await task
            await srv.close(1)
            if attach:
                logger.removeHandler(lines)
        return out, side.calls, lines.lines, _requests_total(route, ok_status) - before, len(python_calls)
    return run(main())


def _api_body(name="Buy milk"):
    return json.dumps({"taskName": name, "taskCreatedBy": "a@b.c", "taskDueDate": "2030-01-01T00:00:00",
                       "taskAssignedTo": "x@y.z"}).encode()


def _norm_id(s):
    return re.sub(r"[0-9a-f]{8}-[0-9a-f]{4}-[0-9a-f]{4}-[0-9a-f]{4}-[0-9a-f]{12}", "<id>", s)


def _norm_call(call):
    method, target, headers, body = call
    tp = headers.get("traceparent", "")
    try:
        doc = json.loads(body) if body else None
    except ValueError:
        doc = body
    text = _norm_id(json.dumps(doc, sort_keys=True))
    text = re.sub(r'"taskCreatedOn": "[^"]+"', '"taskCreatedOn": "<now>"', text)
    return (method, target, headers.get("content-type"), tp[:36], tp[52:], "dapr-api-token" in headers, text)


@pytest.mark.parametrize("status", [{}, {"/v1.0/state/": (500, b'{"errorCode":"ERR_STATE_SAVE"}')},
                                    {"/v1.0/publish/": (404, b'{"errorCode":"ERR_PUBSUB_NOT_FOUND"}')}],
                         ids=["ok", "save-fails", "publish-fails"])
def test_api_create_native_equals_python(tmp_path, monkeypatch, status):
    reqs = [([("Content-Type", "application/json"), ("traceparent", UNSAMPLED)], _api_body()),
            ([("traceparent", UNSAMPLED)], _api_body("Ünïcode ✓ 'quoted'"))]
    got = {n: _scenario(tmp_path, monkeypatch, "api", n, status, reqs) for n in (True, False)}
    (rn, cn, ln, mn, pn), (rp, cp, lp, mp, pp) = got[True], got[False]
    assert pn == 0 and pp == 2  # the host served both; with the routes off, the handler did
    norm = lambda rs: [(s, _norm_id(loc or ""), ct, json.loads(b).get("status") if b else None) for s, loc, ct, b in rs]
    assert norm(rn) == norm(rp)
    assert [_norm_call(c) for c in cn] == [_norm_call(c) for c in cp]
    # the child span of the caller's context, unsampled, a span id of its own
    for c in cn:
        tp = c[2]["traceparent"]
        assert tp.startswith(f"00-{TID}-") and tp.endswith("-00") and tp != UNSAMPLED
    assert [_norm_id(x) for x in ln] == [_norm_id(x) for x in lp]
    assert mn == mp
    if not status:
        assert [s for s, *_ in rn] == [201, 201] and mn == 2
        save, pub = cn[0], cn[1]
        key = json.loads(save[3])[0]["key"]
        assert rn[0][1] == f"/api/tasks/{key}" and json.loads(pub[3])["taskId"] == key


def test_api_create_goes_to_python_when_native_cannot_decide(tmp_path, monkeypatch):
    reqs = [([("traceparent", SAMPLED)], _api_body()),                      # a sampled trace
            ([("traceparent", UNSAMPLED), ("Content-Type", "text/plain")], _api_body()),  # not JSON
            ([("traceparent", UNSAMPLED)], b'{"task_name": "snake"}'),      # the general binder's
            ([("traceparent", UNSAMPLED), ("x-tt-native", "fail save 500 eA==")], _api_body())]  # spoofed
    got = {n: _scenario(tmp_path, monkeypatch, "api", n, {}, reqs) for n in (True, False)}
    (rn, cn, ln, mn, pn), (rp, cp, lp, mp, pp) = got[True], got[False]
    assert pn == 2 and pp == 3  # the sampled and the snake_case ones were saved by the handler
    assert [(s, _norm_id(loc or "")) for s, loc, *_ in rn] == [(s, _norm_id(loc or "")) for s, loc, *_ in rp]
    assert [s for s, *_ in rn][-1] == 201  # the client's own hand-over header is ignored
    assert [_norm_call(c) for c in cn] == [_norm_call(c) for c in cp]
    assert mn == mp


def _form(token_ok=True, name="Buy+milk"):
    import hmac
    import hashlib
    tok = hmac.new(b"k3y", b"c0ffee", hashlib.sha256).hexdigest() if token_ok else "0" * 64
    return (f"__RequestVerificationToken={tok}&TaskAdd.TaskName={name}&TaskAdd.TaskDueDate=2030-01-01"
            "&TaskAdd.TaskAssignedTo=a%40b.c").encode()


_FE_HEADERS = [("Content-Type", "application/x-www-form-urlencoded"),
               ("Cookie", "TasksCreatedByCookie=me%40x.y; .AspNetCore.Antiforgery=c0ffee")]


@pytest.mark.parametrize("status", [{}, {"/v1.0/invoke/": (500, b'{"errorCode":"ERR_DIRECT_INVOKE"}')}],
                         ids=["ok", "invoke-fails"])
def test_frontend_create_native_equals_python(tmp_path, monkeypatch, status):
    reqs = [(_FE_HEADERS, _form()), (_FE_HEADERS, _form(name="%C3%9Cn%C3%AF+%27q%27")),
            (_FE_HEADERS, _form(token_ok=False)),                      # 400 from the page
            (_FE_HEADERS + [("x-tt-native", "fail invoke 500 eA==")], _form())]  # spoofed
    got = {n: _scenario(tmp_path, monkeypatch, "frontend", n, status, reqs) for n in (True, False)}
    (rn, cn, ln, mn, pn), (rp, cp, lp, mp, pp) = got[True], got[False]
    assert (pn, pp) == (1, 3)  # the codec leaves the non-ASCII name to the page; a bad token never calls the API
    # the error page carries a fresh request id: compare status, location and content type
    assert [r[:3] for r in rn] == [r[:3] for r in rp]
    assert [_norm_call(c)[:3] + _norm_call(c)[4:] for c in cn] == [_norm_call(c)[:3] + _norm_call(c)[4:] for c in cp]
    assert ln == lp and mn == mp
    if not status:
        assert [r[0] for r in rn] == [302, 302, 400, 302] and mn == 3
        assert all(c[2]["traceparent"].endswith("-00") for c in cn)


def _event(data, ctype="application/json"):
    return json.dumps({"specversion": "1.0", "type": "com.dapr.event.sent", "source": "tasksmanager-backend-api",
                       "id": "e1", "datacontenttype": ctype, "topic": "tasksavedtopic", "pubsubname": "dapr-pubsub-servicebus",
                       "traceparent": UNSAMPLED, "data": data}).encode()


def test_processor_notify_native_equals_python(tmp_path, monkeypatch):
    task = {"taskId": "2b0c7a4e-3f51-4a77-9c39-4a1f3d54e0f1", "taskName": "Ünïcode 'q' ✓", "taskCreatedBy": "a@b.c",
            "taskCreatedOn": "2030-01-01T10:00:00.1234567Z", "taskDueDate": "2030-01-02T00:00:00",
            "taskAssignedTo": "x@y.z", "isCompleted": False, "isOverDue": False}
    ce = [("Content-Type", "application/cloudevents+json"), ("traceparent", UNSAMPLED)]
    reqs = [(ce, _event(task)),                                               # the delivery: native
            ([("Content-Type", "application/json"), ("traceparent", UNSAMPLED)], json.dumps(task).encode()),  # raw
            (ce, _event({"task_name": "snake"})),                            # binder decides (400)
            ([("Content-Type", "application/cloudevents+json"), ("traceparent", SAMPLED)], _event(task)),  # sampled
            (ce, _event("plain text", "text/plain"))]                        # not JSON: the page's 400/415
    got = {n: _scenario(tmp_path, monkeypatch, "processor", n, {}, reqs) for n in (True, False)}
    (rn, cn, ln, mn, pn), (rp, cp, lp, mp, pp) = got[True], got[False]
    assert [(s, ct, b if s == 200 else None) for s, _, ct, b in rn] == [(s, ct, b if s == 200 else None) for s, _, ct, b in rp]
    assert [r[0] for r in rn][:2] == [200, 200]
    assert ln == lp and mn == mp and cn == cp == []
    assert pn == pp - 2  # the delivery and the raw body were answered by the host


def test_native_log_lines_equal_the_python_sinks(tmp_path, monkeypatch):
    """With the process's JSON sink on the fast path, the native route writes the finished log
    line itself (the sink's prefix handed over at registration): the records in the telemetry
    directory equal the Python handler's, apart from the timestamp and the span / task ids."""
    import glob

    from aca_dotnet_workshop_amd.telemetry.logging import flush_logs, native_line_prefix
    root = logging.getLogger()
    saved = list(root.handlers)
    for hd in saved:  # pytest's capture handler would take the records off the fast path
        root.removeHandler(hd)
    recs = {}
    try:
        for n in (True, False):
            d = tmp_path / f"logs-{n}"
            monkeypatch.setenv("TT_TELEMETRY_DIR", str(d))
            monkeypatch.setenv("TT_LOG_CONSOLE", "0")
            reqs = [([("traceparent", UNSAMPLED)], _api_body("tab\tquote\" ✓"))]
            _scenario(tmp_path, monkeypatch, "api", n, {}, reqs, attach=False)
            assert native_line_prefix("TasksManager").startswith('{"level":"Information","role":')
            flush_logs()
            lines = [json.loads(x) for f in glob.glob(str(d / "logs-*")) for x in open(f)]
            recs[n] = [{k: (_norm_id(v) if isinstance(v, str) else v) for k, v in r.items() if k not in ("ts", "spanId")}
                       for r in lines if r.get("category") == "TasksManager"]
    finally:
        for hd in list(root.handlers):
            if hd not in saved:
                root.removeHandler(hd)
        for hd in saved:
            root.addHandler(hd)
    assert len(recs[True]) == 2 and recs[True] == recs[False]
    assert recs[True][0]["traceId"] == TID and "tab\tquote\" ✓" in recs[True][0]["message"]


def test_native_routes_follow_the_python_definitions(tmp_path, monkeypatch):
    """The native routes hold no text of their own: a changed log template, status or Location in
    the Python definitions is what the I/O thread logs and answers -- no C++ edit -- and a
    template it cannot reproduce (another directive than %s) makes the route decline, so the
    Python handler serves every request."""
    from aca_dotnet_workshop_amd.services.backend_api import app as api_app
    from aca_dotnet_workshop_amd.services.backend_api import managers
    from aca_dotnet_workshop_amd.services.processor import app as proc_app
    monkeypatch.setattr(managers, "LOG_SAVE_NEW", "Saving '%s' (edited)")
    monkeypatch.setattr(managers, "LOG_PUBLISH", "Published %s / %s -> %s (100%%)")
    monkeypatch.setattr(api_app, "CREATED_STATUS", 202)
    monkeypatch.setattr(api_app, "CREATED_LOCATION", "/v2/tasks/%s")
    reqs = [([("Content-Type", "application/json"), ("traceparent", UNSAMPLED)], _api_body())]
    got = {n: _scenario(tmp_path, monkeypatch, "api", n, {}, reqs) for n in (True, False)}
    (rn, cn, ln, mn, pn), (rp, cp, lp, mp, pp) = got[True], got[False]
    assert pn == 0 and pp == 1  # the host served it, with the edited text
    assert rn[0][0] == rp[0][0] == 202 and _norm_id(rn[0][1]) == _norm_id(rp[0][1]) == "/v2/tasks/<id>"
    assert [_norm_id(x) for x in ln] == [_norm_id(x) for x in lp] == \
        ["Saving 'Buy milk' (edited)", "Published <id> / Buy milk -> x@y.z (100%)"]
    # the notifier's line and answer
    monkeypatch.setattr(proc_app, "NOTIFY_LOG", "Got '%s'")
    task = {"taskId": "2b0c7a4e-3f51-4a77-9c39-4a1f3d54e0f1", "taskName": "n1", "taskCreatedBy": "a@b.c",
            "taskCreatedOn": "2030-01-01T10:00:00Z", "taskDueDate": "2030-01-02T00:00:00", "taskAssignedTo": "x@y.z",
            "isCompleted": False, "isOverDue": False}
    reqs = [([("Content-Type", "application/cloudevents+json"), ("traceparent", UNSAMPLED)], _event(task))]
    (rn, _, ln, _, pn) = _scenario(tmp_path, monkeypatch, "processor", True, {}, reqs)
    assert pn == 0 and rn[0][0] == 200 and rn[0][3] == b"Got 'n1'" and ln == ["Got 'n1'"]
    # a template the native route cannot fill: it declines, Python answers
    monkeypatch.setattr(managers, "LOG_SAVE_NEW", "Save a new task with name: '%r' to state store")
    reqs = [([("Content-Type", "application/json"), ("traceparent", UNSAMPLED)], _api_body())]
    (rn, _, ln, _, pn) = _scenario(tmp_path, monkeypatch, "api", True, {}, reqs)
    assert pn == 1 and rn[0][0] == 202 and ln[0] == "Save a new task with name: ''Buy milk'' to state store"


def _get_scenario(tmp_path, monkeypatch, which, native, sidecar_status, requests, manager_kw=None, route=None):
    """GET ``requests`` [(headers, target)] against the frontend's Tasks/Index ('frontend') or
    the API's api/tasks ('api'); returns (responses, sidecar calls, metric delta, python calls)."""
    monkeypatch.setenv("TT_APP_HOST", "native")
    monkeypatch.setenv("TT_NATIVE_ROUTES", "1" if native else "0")
    monkeypatch.setenv("TT_TRACE_SAMPLE_RATE", "0")
    side_sock = str(tmp_path / f"gside-{which}-{native}.sock")
    app_sock = str(tmp_path / f"gapp-{which}-{native}.sock")
    from aca_dotnet_workshop_amd.sdk.client import SidecarClient
    from aca_dotnet_workshop_amd.telemetry import tracing
    tracing.configure("native-routes-test", None, 0.0)
    route = route or {"api": "/api/tasks", "frontend": "/Tasks/Index"}[which]

    async def main():
        loop = asyncio.get_running_loop()
        side = Sidecar()
        side.status.update(sidecar_status)
        srv = HttpServer(side.app, loop)
        await srv.listen_unix(side_sock)
        client = SidecarClient(f"unix:{side_sock}:")
        cfg = Configuration([{"APP_PORT": "0", "Environment": "Production", "TT_APP_UDS": app_sock}])
        python_calls = []
        if which == "api":
            from aca_dotnet_workshop_amd.services.backend_api import create_app
            from aca_dotnet_workshop_amd.services.backend_api.managers import TasksStoreManager
            app = create_app(config=cfg, manager=TasksStoreManager(client, **(manager_kw or {})))
            real = client.query_state_raw

            async def counted(*a, **kw):
                python_calls.append(1)
                return await real(*a, **kw)
            client.query_state_raw = counted
        else:
            from aca_dotnet_workshop_amd.services.frontend import create_app
            app = create_app([], client=client, overrides={"Frontend:AntiforgeryKey": "k3y", "APP_PORT": "0",
                                                           "Environment": "Production", "TT_APP_UDS": app_sock})
            gw = app.services["backend"]
            real_call = gw.call

            async def counted_call(*a, **kw):
                python_calls.append(1)
                return await real_call(*a, **kw)
            gw.call = counted_call
        REGISTRY.collect()
        ctr = REGISTRY.counter("http_requests_total")
        before = ctr.get(method="GET", route=route, status="200")
        stop, ports = asyncio.Event(), []
        task = asyncio.create_task(_serve(app, app_sock, stop, ports))
        for _ in range(200):
            if ports:
                break
            await asyncio.sleep(0.01)
        c = HttpClient()
        out = []
        try:
            for headers, target in requests:
                r = await c.get(f"unix:{app_sock}:{target}", headers=headers)
                out.append((r.status, r.headers.get("content-type"), r.headers.get("location") or
                            r.headers.get("x-tt-more-results"), r.body))
        finally:
            await c.close()
            stop.set()
            await task
            await srv.close(1)
        REGISTRY.collect()
        return out, side.calls, ctr.get(method="GET", route=route, status="200") - before, len(python_calls)
    return run(main())


_LIST = [{"taskId": "2b0c7a4e-3f51-4a77-9c39-4a1f3d54e0f1", "taskName": "<b>Ünïcode</b> & 'q' \"x\"",
          "taskCreatedBy": "me@x.y", "taskCreatedOn": "2030-01-01T10:00:00.1234567Z",
          "taskDueDate": "2030-01-02T00:00:00", "taskAssignedTo": "x@y.z", "isCompleted": False, "isOverDue": True},
         {"taskId": "0f8fad5b-d9cb-469f-a165-70867728950e", "taskName": "plain", "taskCreatedBy": "me@x.y",
          "taskCreatedOn": "2030-01-01T09:00:00Z", "taskDueDate": "2029-12-31T23:59:59.5Z",
          "taskAssignedTo": "a@b.c", "isCompleted": True, "isOverDue": False}]


@pytest.mark.parametrize("status", [{}, {"/v1.0/invoke/": (500, b'{"errorCode":"ERR_DIRECT_INVOKE"}')}],
                         ids=["ok", "invoke-fails"])
def test_frontend_list_native_equals_python(tmp_path, monkeypatch, status):
    """GET Tasks/Index on the I/O thread: the page compiled from the templates (rows.py) equals
    the Python page byte for byte, the same invoke goes to the sidecar, and the requests the
    route leaves to the page (no identity, no antiforgery cookie yet, a list outside the rows'
    shape, a failed invoke) are answered as the page answers them."""
    ok = {"/v1.0/invoke/": (200, json.dumps(_LIST).encode())}
    ok.update(status)
    ck = "TasksCreatedByCookie=me%40x.y; .AspNetCore.Antiforgery=c0ffee"
    reqs = [([("Cookie", ck), ("traceparent", UNSAMPLED)], "/Tasks/Index"),
            ([("Cookie", "TasksCreatedByCookie=o%27b%3Cr%3E%2Bx%20y@z; .AspNetCore.Antiforgery=c0ffee"),
              ("traceparent", UNSAMPLED)], "/Tasks/Index"),
            ([("Cookie", ".AspNetCore.Antiforgery=c0ffee"), ("traceparent", UNSAMPLED)], "/Tasks/Index"),  # redirect
            ([("Cookie", "TasksCreatedByCookie=me%40x.y"), ("traceparent", UNSAMPLED)], "/Tasks/Index")]  # new af cookie
    got = {n: _get_scenario(tmp_path, monkeypatch, "frontend", n, ok, reqs) for n in (True, False)}
    (rn, cn, mn, pn), (rp, cp, mp, pp) = got[True], got[False]
    assert [r[:3] for r in rn] == [r[:3] for r in rp]
    assert rn[0][3] == rp[0][3] and rn[1][3] == rp[1][3]  # the 4th hands out a new (random) antiforgery cookie
    assert [_norm_call(c) for c in cn] == [_norm_call(c) for c in cp]
    assert mn == mp
    if not status:
        assert [r[0] for r in rn] == [200, 200, 302, 200]
        assert pn == 1 and pp == 3  # the host served the two with both cookies
        assert b"&lt;b&gt;\xc3\x9cn\xc3\xafcode&lt;/b&gt; &amp; &#39;q&#39; &#34;x&#34;" in rn[0][3]
        assert cn[1][1].endswith("api/tasks?createdBy=o%27b%3Cr%3E%2Bx%20y%40z")
    else:
        assert [r[0] for r in rn][:2] == [500, 500]


def test_frontend_list_declines_a_list_outside_the_rows(tmp_path, monkeypatch):
    odd = [dict(_LIST[0], taskDueDate="2030-01-02T00:00:00+02:00"), _LIST[1]]
    ok = {"/v1.0/invoke/": (200, json.dumps(odd).encode())}
    reqs = [([("Cookie", "TasksCreatedByCookie=me%40x.y; .AspNetCore.Antiforgery=c0ffee"), ("traceparent", UNSAMPLED)],
             "/Tasks/Index")]
    got = {n: _get_scenario(tmp_path, monkeypatch, "frontend", n, ok, reqs) for n in (True, False)}
    (rn, cn, mn, pn), (rp, cp, mp, pp) = got[True], got[False]
    assert rn == rp and pn == 1 and len(cn) == 2 and len(cp) == 1  # asked twice: once native, once by the page


@pytest.mark.parametrize("status", [{}, {"/v1.0-alpha1/state/": (500, b'{"errorCode":"ERR_STATE_QUERY"}')}],
                         ids=["ok", "query-fails"])
def test_api_list_native_equals_python(tmp_path, monkeypatch, status):
    results = {"results": [{"key": t["taskId"], "data": t, "etag": "1"} for t in _LIST] + [{"key": "gone", "data": None}]}
    ok = {"/v1.0-alpha1/state/": (200, json.dumps(results).encode())}
    ok.update(status)
    reqs = [([("traceparent", UNSAMPLED)], "/api/tasks?createdBy=me%40x.y"),
            ([("traceparent", UNSAMPLED)], "/api/tasks?CreatedBy=a+%22b%22&createdby=ignored"),
            ([("traceparent", UNSAMPLED)], "/api/tasks")]  # no creator: the controller's []
    got = {n: _get_scenario(tmp_path, monkeypatch, "api", n, ok, reqs) for n in (True, False)}
    (rn, cn, mn, pn), (rp, cp, mp, pp) = got[True], got[False]
    assert [r[:2] + (r[3],) for r in rn] == [r[:2] + (r[3],) for r in rp]
    assert [_norm_call(c) for c in cn] == [_norm_call(c) for c in cp]
    assert mn == mp
    if not status:
        assert pn == 0 and pp == 2
        assert [t["taskId"][-4:] for t in json.loads(rn[0][3])] == ["e0f1", "950e"]  # newest first
        assert json.loads(cn[1][3]) == {"filter": {"EQ": {"taskCreatedBy": 'a "b"'}}}


@pytest.mark.parametrize("status", [{}, {"/v1.0-alpha1/state/": (500, b'{"errorCode":"ERR_STATE_QUERY"}')}],
                         ids=["ok", "query-fails"])
def test_api_overdue_native_equals_python(tmp_path, monkeypatch, status):
    """GET api/overduetasks (range mode) on the I/O thread: the manager's range query -- today's
    midnight and the page size filled into its own text -- the same page (oldest first) and
    more-results flag, the same log line; a failed query is the SDK's error."""
    results = {"results": [{"key": t["taskId"], "data": t, "etag": "1"} for t in _LIST], "token": "2"}
    ok = {"/v1.0-alpha1/state/": (200, json.dumps(results).encode())}
    ok.update(status)
    reqs = [([("traceparent", UNSAMPLED)], "/api/overduetasks?limit=512"),
            ([("traceparent", UNSAMPLED)], "/api/overduetasks"),
            ([("traceparent", UNSAMPLED)], "/api/overduetasks?limit=007"),
            ([("traceparent", UNSAMPLED)], "/api/overduetasks?limit=x")]
    kw = {"overdue_query": "range", "overdue_page": 100}
    lines = _Lines()
    got = {}
    logger = logging.getLogger("TasksManager")
    for n in (True, False):
        logger.addHandler(lines)
        try:
            got[n] = _get_scenario(tmp_path, monkeypatch, "api", n, ok, reqs, kw, "/api/overduetasks") + (list(lines.lines),)
        finally:
            logger.removeHandler(lines)
            lines.lines.clear()
    (rn, cn, mn, pn, ln), (rp, cp, mp, pp, lp) = got[True], got[False]
    assert rn == rp and [_norm_call(c) for c in cn] == [_norm_call(c) for c in cp] and mn == mp
    assert ln == lp and ln[0].startswith("Getting open tasks due before: '") and ln[0].endswith("(page of 512)")
    if not status:
        assert pn == 0 and pp == 4
        assert [r[2] for r in rn] == ["true"] * 4  # the store's token: more matches
        assert [json.loads(c[3])["page"]["limit"] for c in cn] == [512, 100, 7, 100]
        assert [t["taskId"][-4:] for t in json.loads(rn[0][3])] == ["950e", "e0f1"]  # oldest first
