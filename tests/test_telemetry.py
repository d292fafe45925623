"""Telemetry: application map / failures / performance views over spans, traceparent
parsing, JSON log records with trace ids, Prometheus exposition."""
import json
import logging

from aca_dotnet_workshop_amd.telemetry import appmap, tracing
from aca_dotnet_workshop_amd.telemetry.logging import JsonFormatter, _Ctx
from aca_dotnet_workshop_amd.telemetry.metrics import Registry


def _spans():
    web = tracing.Tracer("tasksmanager-frontend-webapp")
    web_sc = tracing.Tracer("tasksmanager-frontend-webapp.sidecar")
    api_sc = tracing.Tracer("tasksmanager-backend-api.sidecar")
    api = tracing.Tracer("tasksmanager-backend-api")
    with web.start_span("GET /Tasks/Index", "server") as s1:
        with web.start_span("invoke api", "client") as c1:
            with web_sc.start_span("POST /v1.0/invoke", "server", parent=c1) as s2:
                with api_sc.start_span("GET /api/tasks", "server", parent=s2) as s3:
                    with api.start_span("GET /api/tasks", "server", parent=s3) as s4:
                        s4.fail("boom")
    out = []
    for t in (web, web_sc, api_sc, api):
        out += t.exporter.memory
    return out, s1.trace_id


def test_application_map_edges_and_views():
    spans, tid = _spans()
    m = appmap.application_map(spans)
    assert {"from": "tasksmanager-frontend-webapp", "to": "tasksmanager-backend-api", "calls": 1, "failures": 0} == \
        {k: v for k, v in m["edges"][0].items() if k != "avgMs"}
    assert m["nodes"]["tasksmanager-backend-api"]["failures"] == 1
    f = appmap.failures(spans)
    assert f[0]["role"] == "tasksmanager-backend-api" and f[0]["count"] == 1
    perf = appmap.performance(spans)
    assert {p["role"] for p in perf} >= {"tasksmanager-backend-api", "tasksmanager-frontend-webapp"}
    tx = appmap.transaction(spans, tid)
    assert len(tx) == 5 and all(s["traceId"] == tid for s in tx)


def test_spans_to_directory_and_load(tmp_path):
    t = tracing.Tracer("svc", str(tmp_path))
    with t.start_span("op", "server"):
        pass
    t.flush()
    assert appmap.load_spans(tmp_path)[0]["role"] == "svc"


def test_traceparent_parsing_and_sampling():
    assert tracing.parse_traceparent("00-" + "a" * 32 + "-" + "b" * 16 + "-01") == ("a" * 32, "b" * 16, True)
    assert tracing.parse_traceparent("00-" + "0" * 32 + "-" + "b" * 16 + "-01") is None
    assert tracing.parse_traceparent("garbage") is None
    t = tracing.Tracer("s", sample_rate=0.0)
    with t.start_span("x", "server"):
        pass
    assert t.exporter.memory == []


def test_json_log_record_carries_trace_ids():
    t = tracing.Tracer("svc")
    rec = logging.LogRecord("cat", logging.INFO, __file__, 1, "hello %s", ("w",), None)
    with t.start_span("op", "server") as sp:
        _Ctx("svc").filter(rec)
    d = json.loads(JsonFormatter().format(rec))
    assert d["message"] == "hello w" and d["role"] == "svc" and d["traceId"] == sp.trace_id


def test_prometheus_exposition():
    r = Registry()
    c = r.counter("reqs", "requests")
    c.inc(route="/a")
    c.inc(2, route="/a")
    h = r.histogram("lat", "latency")
    for v in (0.001, 0.002, 0.2):
        h.observe(v, route="/a")
    text = r.expose()
    assert 'reqs{route="/a"} 3.0' in text and 'lat_count{route="/a"} 3' in text
    assert h.quantile(0.5, route="/a") == 0.0025


def test_log_retention_prunes_whole_days(tmp_path):
    """retentionInDays (Log Analytics, 30 in the reference): telemetry is written one file per
    process per UTC day, and pruning deletes the days that fell out of the window."""
    import os
    import time

    from aca_dotnet_workshop_amd.telemetry.retention import DailyFile, prune, utc_day

    now = time.time()
    day = 86400.0
    for age in (0, 1, 29, 30, 31, 45):
        (tmp_path / f"logs-api-1-{utc_day(now - age * day)}.jsonl").write_text("{}\n")
    legacy_old = tmp_path / "spans-old-7.jsonl"
    legacy_old.write_text("{}\n")
    os.utime(legacy_old, (now - 40 * day, now - 40 * day))
    (tmp_path / "spans-new-8.jsonl").write_text("{}\n")
    res = prune(tmp_path, 30, now)
    assert sorted(res["removed"]) == sorted([f"logs-api-1-{utc_day(now - a * day)}.jsonl" for a in (31, 45)]
                                            + ["spans-old-7.jsonl"])
    assert res["kept"] == 5
    f = DailyFile(str(tmp_path), "logs-x-9")
    f.write("a\n")
    f.close()
    assert (tmp_path / f"logs-x-9-{utc_day()}.jsonl").read_text() == "a\n"
    assert prune(tmp_path, 0, now)["removed"] == []  # 0 = keep forever


def test_info_each_writes_the_same_lines_as_a_loop(tmp_path, monkeypatch):
    """telemetry.logging.info_each (the bulk operations' per-task lines, e.g. markoverdue's
    'Mark task with Id ... as OverDue task'): the JSON lines equal those of ``info`` in a loop
    (apart from the timestamp), carry the span's trace ids, and on a logger with a foreign
    handler (the standard path) it is a plain loop."""
    import glob
    from aca_dotnet_workshop_amd.telemetry.logging import configure_logging, flush_logs, info_each

    monkeypatch.setenv("TT_TELEMETRY_DIR", str(tmp_path))
    monkeypatch.setenv("TT_LOG_CONSOLE", "0")
    root = logging.getLogger()
    saved, saved_tracer = list(root.handlers), tracing._tracer
    try:
        configure_logging("api")
        lg = logging.getLogger("BulkCat")
        t = tracing.configure("api", str(tmp_path / "spans"))
        with t.start_span("op", "server") as sp:
            for i in range(3):
                lg.info("Mark task with Id: '%s' as OverDue task", f"t{i}")
            info_each(lg, "Mark task with Id: '%s' as OverDue task", [(f"t{i}",) for i in range(3)])
        flush_logs()
        recs = [json.loads(x) for f in glob.glob(str(tmp_path / "logs-api-*")) for x in open(f)]
        assert len(recs) == 6
        strip = [{k: v for k, v in r.items() if k != "ts"} for r in recs]
        assert strip[:3] == strip[3:]
        assert strip[0]["traceId"] == sp.trace_id and strip[2]["message"] == "Mark task with Id: 't2' as OverDue task"
        # a foreign handler: the standard logging path, one record per tuple
        seen = []

        class H(logging.Handler):
            def emit(self, record):
                seen.append(record.getMessage())
        h = H()
        lg.addHandler(h)
        info_each(lg, "x %s %s", [(1, 2), (3, 4)])
        lg.removeHandler(h)
        assert seen == ["x 1 2", "x 3 4"]
    finally:
        tracing._tracer = saved_tracer
        for h in list(root.handlers):
            if getattr(h, "_tt", False):
                root.removeHandler(h)
                h.close()
        for h in saved:
            if h not in root.handlers:
                root.addHandler(h)


def test_native_route_log_records_equal_the_handlers_own(tmp_path, monkeypatch):
    """A native route's log record (apphost.hpp LOG event -> web/native_host.py _native_log)
    is the JSON line the handler's own ``log.info`` writes inside its request span: same level,
    role, category, message and trace ids; also on the standard logging path."""
    import glob
    from aca_dotnet_workshop_amd.telemetry.logging import configure_logging, flush_logs
    from aca_dotnet_workshop_amd.web.native_host import _native_log

    monkeypatch.setenv("TT_TELEMETRY_DIR", str(tmp_path))
    monkeypatch.setenv("TT_LOG_CONSOLE", "0")
    root = logging.getLogger()
    saved, saved_tracer = list(root.handlers), tracing._tracer
    try:
        configure_logging("api")
        lg = logging.getLogger("TasksManager")
        t = tracing.configure("api", str(tmp_path / "spans"), 0.0)
        msg = "Save a new task with name: '100% ✓' to state store"
        with t.start_span("POST", "server") as sp:
            lg.info("Save a new task with name: '%s' to state store", "100% ✓")
        _native_log(logging.INFO, "TasksManager", msg, sp.trace_id, sp.span_id)
        flush_logs()
        recs = [json.loads(x) for f in glob.glob(str(tmp_path / "logs-api-*")) for x in open(f)]
        strip = [{k: v for k, v in r.items() if k != "ts"} for r in recs]
        assert len(strip) == 2 and strip[0] == strip[1] and strip[0]["message"] == msg
        seen = []

        class H(logging.Handler):
            def emit(self, record):
                seen.append((record.getMessage(), tracing.current_trace_id()))
        h = H()
        lg.addHandler(h)
        try:
            _native_log(logging.INFO, "TasksManager", msg, sp.trace_id, sp.span_id)
        finally:
            lg.removeHandler(h)
        assert seen == [(msg, sp.trace_id)] and tracing.current_span() is None
    finally:
        for hd in list(root.handlers):
            if hd not in saved:
                root.removeHandler(hd)
        tracing._tracer = saved_tracer
