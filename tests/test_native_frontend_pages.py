"""The frontend's Edit page, Edit post and Index's Complete / Delete posts on the app host's I/O
thread (apphost.hpp ``frontend_page``; Pages/Tasks/Edit.cshtml.cs:38-71, Index.cshtml.cs:57-71),
against the Python pages (``TT_NATIVE_ROUTES=0``).

Same recording sidecar as tests/test_native_routes.py.  Compared per request: status, Location,
content type and the page bytes; every invoke the sidecar saw (method, target, content type,
trace flags, body); and which requests the host left to the page (no identity, no antiforgery
cookie yet, a bad token, a binding error, an unknown handler, an answer outside the page's shape,
a failed invoke -- answered exactly as the page answers them).
"""
import asyncio
import hashlib
import hmac
import json

import pytest

from aca_dotnet_workshop_amd.web.client import HttpClient
from aca_dotnet_workshop_amd.web.server import HttpServer

from helpers import run
from test_native_routes import UNSAMPLED, Sidecar, _norm_call, _serve

TID = "2b0c7a4e-3f51-4a77-9c39-4a1f3d54e0f1"
OTHER = "0f8fad5b-d9cb-469f-a165-70867728950e"
TOKEN = hmac.new(b"k3y", b"c0ffee", hashlib.sha256).hexdigest()
CK = "TasksCreatedByCookie=me%40x.y; .AspNetCore.Antiforgery=c0ffee"
TASK = {"taskId": TID, "taskName": "<b>Ünïcode</b> & 'q' \"x\"", "taskCreatedBy": "me@x.y",
        "taskCreatedOn": "2030-01-01T10:00:00.1234567Z", "taskDueDate": "2030-01-02T00:00:00",
        "taskAssignedTo": "x@y.z", "isCompleted": False, "isOverDue": True}


def _scenario(tmp_path, monkeypatch, native, sidecar_status, requests):
    """``requests``: [(method, target, headers, body)] against the frontend; returns (answers,
    sidecar calls, calls the page made itself)."""
    monkeypatch.setenv("TT_APP_HOST", "native")
    monkeypatch.setenv("TT_NATIVE_ROUTES", "1" if native else "0")
    monkeypatch.setenv("TT_TRACE_SAMPLE_RATE", "0")
    side_sock = str(tmp_path / f"fside-{native}.sock")
    app_sock = str(tmp_path / f"fapp-{native}.sock")
    from aca_dotnet_workshop_amd.sdk.client import SidecarClient
    from aca_dotnet_workshop_amd.telemetry import tracing
    tracing.configure("native-frontend-pages-test", None, 0.0)

    async def main():
        loop = asyncio.get_running_loop()
        side = Sidecar()
        side.status.update(sidecar_status)
        srv = HttpServer(side.app, loop)
        await srv.listen_unix(side_sock)
        client = SidecarClient(f"unix:{side_sock}:")
        from aca_dotnet_workshop_amd.services.frontend import create_app
        app = create_app([], client=client, overrides={"Frontend:AntiforgeryKey": "k3y", "APP_PORT": "0",
                                                       "Environment": "Production", "TT_APP_UDS": app_sock})
        gw = app.services["backend"]
        real_call = gw.call
        python_calls = []

        async def counted_call(*a, **kw):
            python_calls.append(a[:2])
            return await real_call(*a, **kw)
        gw.call = counted_call
        stop, ports = asyncio.Event(), []
        task = asyncio.create_task(_serve(app, app_sock, stop, ports))
        for _ in range(200):
            if ports:
                break
            await asyncio.sleep(0.01)
        c = HttpClient()
        out = []
        try:
            for method, target, headers, body in requests:
                r = await c.request(method, f"unix:{app_sock}:{target}", body=body,
                                    headers=[("traceparent", UNSAMPLED)] + headers)
                page = r.body if r.status in (200, 404) and b"Request ID" not in r.body else None
                out.append((r.status, r.headers.get("location"), r.headers.get("content-type"), page))
        finally:
            await c.close()
            stop.set()
            await task
            await srv.close(1)
        return out, side.calls, python_calls
    return run(main())


_FORM = [("Content-Type", "application/x-www-form-urlencoded"), ("Cookie", CK)]


def _edit(token=TOKEN, tid=None, name="Renamed+task", due="2030-02-01", who="new%40x.y"):
    f = f"__RequestVerificationToken={token}&TaskUpdate.TaskName={name}&TaskUpdate.TaskDueDate={due}" \
        f"&TaskUpdate.TaskAssignedTo={who}"
    return (f + (f"&TaskUpdate.TaskId={tid}" if tid else "")).encode()


@pytest.mark.parametrize("fail", [False, True], ids=["ok", "invoke-fails"])
def test_edit_page_native_equals_python(tmp_path, monkeypatch, fail):
    status = {"/v1.0/invoke/": (500, b'{"errorCode":"ERR_DIRECT_INVOKE"}')} if fail else \
        {"/v1.0/invoke/": (200, json.dumps(TASK).encode())}
    reqs = [("GET", f"/Tasks/Edit/{TID}", [("Cookie", CK)], b""),
            ("GET", f"/Tasks/Edit/{TID}", [("Cookie", ".AspNetCore.Antiforgery=c0ffee")], b""),  # no identity
            ("GET", f"/Tasks/Edit/{TID.upper()}", [("Cookie", CK)], b"")]  # another spelling: the page's
    got = {n: _scenario(tmp_path, monkeypatch, n, status, reqs) for n in (True, False)}
    (rn, cn, pn), (rp, cp, pp) = got[True], got[False]
    assert rn == rp
    assert [_norm_call(c) for c in cn] == [_norm_call(c) for c in cp]
    if not fail:
        assert [r[0] for r in rn] == [200, 302, 200] and len(pn) == 1 and len(pp) == 2
        page = rn[0][3].decode()
        assert "&lt;b&gt;Ünïcode&lt;/b&gt; &amp; &#39;q&#39; &#34;x&#34;" in page and 'value="2030-01-02"' in page
        assert f'value="{TOKEN}"' in page and f'name="TaskUpdate.TaskId" value="{TID}"' in page
    else:
        assert [r[0] for r in rn] == [500, 302, 500]


def test_edit_page_declines_an_answer_outside_the_page(tmp_path, monkeypatch):
    odd = dict(TASK, taskDueDate="2030-01-02T00:00:00+02:00")
    reqs = [("GET", f"/Tasks/Edit/{TID}", [("Cookie", CK)], b"")]
    for body in (json.dumps(odd).encode(), b""):  # an offset date; no such task (the 404 page)
        got = {n: _scenario(tmp_path, monkeypatch, n, {"/v1.0/invoke/": (200, body)}, reqs) for n in (True, False)}
        (rn, cn, pn), (rp, cp, pp) = got[True], got[False]
        assert rn == rp and len(pn) == 1 and len(cn) == 2 and len(cp) == 1  # asked twice: native, then the page


@pytest.mark.parametrize("fail", [False, True], ids=["ok", "invoke-fails"])
def test_edit_post_native_equals_python(tmp_path, monkeypatch, fail):
    status = {"/v1.0/invoke/": (500, b'{"errorCode":"ERR_DIRECT_INVOKE"}')} if fail else {}
    reqs = [("POST", f"/Tasks/Edit/{TID}", _FORM, _edit()),
            ("POST", f"/Tasks/Edit/{TID}", _FORM, _edit(tid=OTHER)),          # the form's TaskId wins
            ("POST", f"/Tasks/Edit/{TID}", _FORM, _edit(token="0" * 64)),     # bad token: 400
            ("POST", f"/Tasks/Edit/{TID}", _FORM, _edit(name="")),            # [Required]: the page again
            ("POST", f"/Tasks/Edit/{TID}", _FORM, _edit(due="2030-02-30")),   # not a date: the page again
            ("POST", f"/Tasks/Edit/{TID}", _FORM, _edit(name="%C3%9Cn%C3%AF"))]  # non-ASCII: the page binds it
    got = {n: _scenario(tmp_path, monkeypatch, n, status, reqs) for n in (True, False)}
    (rn, cn, pn), (rp, cp, pp) = got[True], got[False]
    assert [r[:3] for r in rn] == [r[:3] for r in rp]
    assert [r[3] for r in rn[2:5]] == [r[3] for r in rp[2:5]]  # the error pages
    assert [_norm_call(c) for c in cn] == [_norm_call(c) for c in cp]
    if not fail:
        assert [r[0] for r in rn] == [302, 302, 400, 200, 200, 302] and len(pn) == 1 and len(pp) == 3
        assert [c[1].rsplit("/", 1)[1] for c in cn] == [TID, OTHER, TID] and all(c[0] == "PUT" for c in cn)
        body = json.loads(cn[0][3])
        assert body == {"taskId": TID, "taskName": "Renamed task", "taskDueDate": "2030-02-01T00:00:00",
                        "taskAssignedTo": "new@x.y"}
        assert json.loads(cn[2][3])["taskName"] == "Ünï"
    else:
        assert [r[0] for r in rn] == [500, 500, 400, 200, 200, 500]


@pytest.mark.parametrize("fail", [False, True], ids=["ok", "invoke-fails"])
def test_index_posts_native_equal_python(tmp_path, monkeypatch, fail):
    status = {"/v1.0/invoke/": (404, b'{"errorCode":"ERR_DIRECT_INVOKE"}')} if fail else {}
    af = f"__RequestVerificationToken={TOKEN}".encode()
    reqs = [("POST", f"/Tasks/Index?handler=complete&id={TID}", _FORM, af),
            ("POST", f"/Tasks/Index?handler=Delete&id={TID}", _FORM, af),
            ("POST", f"/Tasks/Index?handler=archive&id={TID}", _FORM, af),                # unknown handler: 400
            ("POST", "/Tasks/Index?handler=delete&id=nope", _FORM, af),                   # not a GUID: 400
            ("POST", f"/Tasks/Index?handler=delete&id={TID}", _FORM, b"__RequestVerificationToken=bad"),  # 400
            ("POST", "/Tasks/Index", _FORM, af + f"&handler=delete&id={TID}".encode())]   # form fields: the page
    got = {n: _scenario(tmp_path, monkeypatch, n, status, reqs) for n in (True, False)}
    (rn, cn, pn), (rp, cp, pp) = got[True], got[False]
    assert [r[:3] for r in rn] == [r[:3] for r in rp]
    assert [_norm_call(c) for c in cn] == [_norm_call(c) for c in cp]
    if not fail:
        assert [r[0] for r in rn] == [302, 302, 400, 400, 400, 302] and len(pn) == 1 and len(pp) == 3
        assert [(c[0], c[1].split("/method/")[1]) for c in cn] == [
            ("PUT", f"api/tasks/{TID}/markcomplete"), ("DELETE", f"api/tasks/{TID}"), ("DELETE", f"api/tasks/{TID}")]
    else:
        assert [r[0] for r in rn] == [500, 500, 400, 400, 400, 500]
