"""The processor's overdue cron job on the app host's I/O thread (apphost.hpp ``processor_sweep``)
against the Python handler (``TT_NATIVE_ROUTES=0``; services/processor/app.py
check_overdue_tasks_job, ScheduledTasksManagerController.cs:19-46).

A recording sidecar serves the API's overdue pages (with the more-results header) and records
every call.  Compared per scenario: the answer's status and its JSON summary (counts and pages;
the run time and the two hop timings only by form), every call the sidecar saw (method, target,
body), and the job's log lines (the trigger time only by form).  Failed calls give the same
error; a page the native filter does not read goes back to Python with the loop's state and
nothing is done twice.
"""
import asyncio
import json
import logging
import re
import uuid

import pytest

from aca_dotnet_workshop_amd.utils.config import Configuration
from aca_dotnet_workshop_amd.web import WebApp
from aca_dotnet_workshop_amd.web.client import HttpClient
from aca_dotnet_workshop_amd.web.http import Response
from aca_dotnet_workshop_amd.web.server import HttpServer

from helpers import run
from test_native_routes import UNSAMPLED, _Lines, _serve

API = "tasksmanager-backend-api"


def _task(i: int, due: str, done=False) -> dict:
    return {"taskId": str(uuid.UUID(int=i + 1)), "taskName": f"task {i}", "taskCreatedBy": "a@b.c",
            "taskCreatedOn": "2026-10-14T10:00:00", "taskDueDate": due, "taskAssignedTo": "x@y.z",
            "isCompleted": done, "isOverDue": False}


def _page(tasks, spaced=False) -> bytes:
    return json.dumps(tasks, separators=(", ", ": ") if spaced else (",", ":")).encode()


PAST, FUTURE = "2020-01-01T00:00:00", "2099-01-01T00:00:00"


def _scenario(tmp_path, monkeypatch, native, pages, page_size, chunk, mark_status=200):
    """``pages``: [(status, body, more header or None)] the sidecar answers the GETs with, in turn
    (the last one repeats).  Returns (status, summary JSON or body, sidecar calls, log lines)."""
    monkeypatch.setenv("TT_APP_HOST", "native")
    monkeypatch.setenv("TT_NATIVE_ROUTES", "1" if native else "0")
    monkeypatch.setenv("TT_TRACE_SAMPLE_RATE", "0")
    side_sock = str(tmp_path / f"side-{native}.sock")
    app_sock = str(tmp_path / f"app-{native}.sock")

    async def main():
        loop = asyncio.get_running_loop()
        calls, served = [], [0]
        side = WebApp("sweep-sidecar")

        async def any_route(req):
            calls.append((req.method, req.target, req.body))
            if req.method == "GET" and "/method/api/overduetasks" in req.target:
                st, body, more = pages[min(served[0], len(pages) - 1)]
                served[0] += 1
                return Response(body, st, [("x-tt-more-results", more)] if more else None, "application/json")
            if req.method == "POST" and req.target.endswith("/markoverdue"):
                st = mark_status(req.body) if callable(mark_status) else mark_status
                return Response(b"" if st < 300 else b'{"errorCode":"ERR_DIRECT_INVOKE"}', st, None,
                                "application/json")
            return Response(b"", 204)
        side.add_route("/{*path}", any_route, ("GET", "POST", "PUT", "DELETE"))
        srv = HttpServer(side, loop)
        await srv.listen_unix(side_sock)
        from aca_dotnet_workshop_amd.sdk.client import SidecarClient
        from aca_dotnet_workshop_amd.services.processor import create_app
        from aca_dotnet_workshop_amd.telemetry import tracing
        tracing.configure("native-sweep-test", None, 0.0)
        client = SidecarClient(f"unix:{side_sock}:")
        cfg = Configuration([{"APP_PORT": "0", "Environment": "Production", "TT_APP_UDS": app_sock,
                              "OverdueTasks": {"PageSize": str(page_size), "MarkChunk": str(chunk)}}])
        app = create_app([], client=client, config=cfg)
        lines = _Lines()
        logger = logging.getLogger("ScheduledTasksManagerController")
        logger.addHandler(lines)
        stop, ports = asyncio.Event(), []
        task = asyncio.create_task(_serve(app, app_sock, stop, ports))
        for _ in range(200):
            if ports:
                break
            await asyncio.sleep(0.01)
        c = HttpClient()
        try:
            r = await c.post(f"unix:{app_sock}:/ScheduledTasksManager", body=b"{}",
                             headers={"Content-Type": "application/json", "traceparent": UNSAMPLED})
        finally:
            await c.close()
            stop.set()
            await task
            await srv.close(1)
            logger.removeHandler(lines)
        out = r.json() if r.status == 200 else r.body
        return r.status, r.headers.get("content-type"), out, calls, lines.lines
    before = _native_served()
    got = run(main())
    served_natively = _native_served() - before
    # the native run's job is the I/O thread's when it ends there (not handed to Python)
    assert served_natively == (1 if native and got[0] == 200 and len(pages) <= 2 and
                               not any(b"+02:00" in p[1] or b"not a date" in p[1] for p in pages) else 0) \
        or not native
    return got


def _native_served() -> float:
    from aca_dotnet_workshop_amd.telemetry import REGISTRY
    REGISTRY.collect()
    c = REGISTRY.counter("native_route_requests_total")
    return sum(c.get(method="POST", route="/ScheduledTasksManager", status=str(s)) for s in (200, 500))


def _norm_summary(s):
    assert re.fullmatch(r"\d{4}-\d\d-\d\dT\d\d:\d\d:\d\d(\.\d{6})?\+00:00", s["runAt"]), s
    assert isinstance(s["queryMs"], float) and isinstance(s["markMs"], float)
    assert list(s) == ["runAt", "retrieved", "markedOverdue", "pages", "emptyMorePages", "queryMs", "markMs"]
    return {k: v for k, v in s.items() if k not in ("runAt", "queryMs", "markMs")}


def _norm_lines(lines):
    out = []
    for ln in lines:
        if ln.startswith("ScheduledTasksManager::Timer Services triggered at: "):
            stamp = ln.rsplit(": ", 1)[1]
            assert re.fullmatch(r"\d{4}-\d\d-\d\d \d\d:\d\d:\d\d(\.\d{6})?\+00:00", stamp), ln
            ln = "TRIGGERED"
        out.append(ln)
    return out


def _both(tmp_path, monkeypatch, **kw):
    return {n: _scenario(tmp_path, monkeypatch, n, **kw) for n in (True, False)}


@pytest.mark.parametrize("spaced", [False, True], ids=["api-layout", "spaced"])
def test_one_page_chunks_and_summary(tmp_path, monkeypatch, spaced):
    tasks = [_task(0, PAST), _task(1, FUTURE), _task(2, PAST), _task(3, "2020-05-05T10:00:00"), _task(4, PAST)]
    got = _both(tmp_path, monkeypatch, pages=[(200, _page(tasks, spaced), "false")], page_size=4096, chunk=2)
    (sn, cn, jn, calln, ln), (sp, cp, jp, callp, lp) = got[True], got[False]
    assert sn == sp == 200 and cn == cp
    assert _norm_summary(jn) == _norm_summary(jp) == {"retrieved": 5, "markedOverdue": 4, "pages": 1,
                                                     "emptyMorePages": 0}
    assert calln == callp and [c[0] for c in calln] == ["GET", "POST", "POST"]
    assert calln[0][1] == f"/v1.0/invoke/{API}/method/api/overduetasks?limit=4096"
    assert [len(json.loads(c[2])) for c in calln[1:]] == [2, 2]
    assert _norm_lines(ln) == _norm_lines(lp) == [
        "TRIGGERED", "ScheduledTasksManager::completed query state store for tasks, retrieved tasks count: 5",
        "ScheduledTasksManager::marking 4 as overdue tasks"]


def test_pages_while_the_api_reports_more(tmp_path, monkeypatch):
    p1 = _page([_task(i, PAST) for i in range(4)])
    p2 = _page([_task(10 + i, PAST) for i in range(2)])
    got = _both(tmp_path, monkeypatch, pages=[(200, p1, "true"), (200, p2, "false")], page_size=4, chunk=3)
    (sn, _, jn, calln, ln), (sp, _, jp, callp, lp) = got[True], got[False]
    assert sn == sp == 200 and calln == callp and _norm_lines(ln) == _norm_lines(lp)
    assert _norm_summary(jn) == _norm_summary(jp) == {"retrieved": 6, "markedOverdue": 6, "pages": 2,
                                                     "emptyMorePages": 0}
    assert [c[0] for c in calln] == ["GET", "POST", "POST", "GET", "POST"]


def test_empty_pages_with_more_stop_at_the_limit(tmp_path, monkeypatch):
    got = _both(tmp_path, monkeypatch, pages=[(200, b"[]", "true")], page_size=8, chunk=4)
    (sn, _, jn, calln, ln), (sp, _, jp, callp, lp) = got[True], got[False]
    assert sn == sp == 200 and calln == callp and _norm_lines(ln) == _norm_lines(lp)
    assert _norm_summary(jn) == _norm_summary(jp) == {"retrieved": 0, "markedOverdue": 0, "pages": 3,
                                                     "emptyMorePages": 3}


def test_without_the_header_a_short_page_ends_the_job(tmp_path, monkeypatch):
    p1 = _page([_task(i, PAST) for i in range(3)])
    p2 = _page([_task(9, PAST)])
    got = _both(tmp_path, monkeypatch, pages=[(200, p1, None), (200, p2, None)], page_size=3, chunk=8)
    (sn, _, jn, calln, _), (sp, _, jp, callp, _) = got[True], got[False]
    # a full page without the header asks for the next one; a short one ends the job
    assert sn == sp == 200 and calln == callp and _norm_summary(jn) == _norm_summary(jp)
    assert _norm_summary(jn) == {"retrieved": 4, "markedOverdue": 4, "pages": 2, "emptyMorePages": 0}


@pytest.mark.parametrize("where", ["get", "mark"])
def test_failed_calls_give_the_same_error(tmp_path, monkeypatch, where):
    tasks = _page([_task(i, PAST) for i in range(5)])
    if where == "get":
        kw = dict(pages=[(500, b'{"errorCode":"ERR_DIRECT_INVOKE"}', None)])
    else:  # the second chunk fails: every chunk is sent, then the job fails
        kw = dict(pages=[(200, tasks, "false")], mark_status=lambda body: 500 if b"task 2" in body else 200)
    got = _both(tmp_path, monkeypatch, page_size=4096, chunk=2, **kw)
    (sn, cn, bn, calln, ln), (sp, cp, bp, callp, lp) = got[True], got[False]
    assert sn == sp and sn >= 500 and bn == bp and cn == cp
    assert calln == callp and _norm_lines(ln) == _norm_lines(lp)


def test_a_page_the_native_filter_declines_goes_on_in_python(tmp_path, monkeypatch):
    """Page 2 holds a task the binder rejects: the native route hands the job's state to Python,
    which asks for that page again -- so the native run makes one extra GET -- and fails there
    exactly as the Python run does."""
    p1 = _page([_task(i, PAST) for i in range(2)])
    bad = json.dumps([_task(5, "not a date")]).encode()
    got = _both(tmp_path, monkeypatch, pages=[(200, p1, "true"), (200, bad, "false")], page_size=2, chunk=4)
    (sn, _, bn, calln, ln), (sp, _, bp, callp, lp) = got[True], got[False]
    assert sn == sp and bn == bp
    assert _norm_lines(ln) == _norm_lines(lp)
    assert [c[0] for c in callp] == ["GET", "POST", "GET"] and len(calln) == 4
    assert calln[:2] == callp[:2] and calln[2] == calln[3] == callp[2]


def test_resumed_job_keeps_its_counts(tmp_path, monkeypatch):
    """Python finishes a job the native route handed over mid-way with the native pages counted."""
    p1 = _page([_task(i, PAST) for i in range(2)])
    odd = _page([_task(7, PAST)]).replace(b'"taskCreatedOn":"2026-10-14T10:00:00"',
                                          b'"taskCreatedOn":"2026-10-14T10:00:00+02:00"')
    got = _both(tmp_path, monkeypatch, pages=[(200, p1, "true"), (200, odd, "false")], page_size=2, chunk=4)
    (sn, _, jn, calln, ln), (sp, _, jp, callp, lp) = got[True], got[False]
    assert sn == sp == 200
    assert _norm_summary(jn) == _norm_summary(jp) == {"retrieved": 3, "markedOverdue": 3, "pages": 2,
                                                     "emptyMorePages": 0}
    assert _norm_lines(ln) == _norm_lines(lp)
    assert [c[0] for c in calln] == ["GET", "POST", "GET", "GET", "POST"]  # page 2 asked twice
