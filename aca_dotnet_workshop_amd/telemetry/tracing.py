"""Distributed tracing -- the Application Insights + Dapr tracing equivalent.

Reference parity (SURVEY.md §5 "Tracing / profiling"):
* every service stamps its spans with a cloud role name (reference
  Backend.Api/AppInsightsTelemetryInitializer.cs:6-16, Processor ...:13, Frontend ...:13);
* W3C ``traceparent`` propagates across app -> sidecar -> sidecar -> app hops and is
  carried inside the CloudEvent envelope for pub/sub (Dapr behaviour);
* the sidecar emits its own spans (env-level ``daprAIInstrumentationKey``, reference
  bicep/modules/container-apps-environment.bicep:59);
* spans are exported as JSON lines to a telemetry directory (the Log Analytics
  workspace equivalent) from which ``appmap`` builds the Application Map.
"""
from __future__ import annotations

import atexit
import contextvars
import json
import os
import random
import threading
import time
from typing import Any

_current: contextvars.ContextVar["Span | None"] = contextvars.ContextVar("current_span", default=None)

_rand = random.Random()


def new_trace_id() -> str:
    return f"{_rand.getrandbits(128):032x}"


def new_span_id() -> str:
    return f"{_rand.getrandbits(64):016x}"


def parse_traceparent(value: str | None) -> tuple[str, str, bool] | None:
    if not value:
        return None
    parts = value.strip().split("-")
    if len(parts) < 4 or len(parts[1]) != 32 or len(parts[2]) != 16:
        return None
    if parts[1] == "0" * 32 or parts[2] == "0" * 16:
        return None
    try:
        flags = int(parts[3][:2], 16)
    except ValueError:
        return None
    return parts[1], parts[2], bool(flags & 1)


class Exporter:
    """Buffered JSON-lines span/log sink (one file per process)."""

    def __init__(self, directory: str | None, role: str) -> None:
        self.directory = directory
        self.role = role
        self._buf: list[str] = []
        self._lock = threading.Lock()
        self._fh = None
        self._memory: list[dict[str, Any]] = []
        self._sources: list[Any] = []  # callables returning span records produced elsewhere
        self._timer: threading.Thread | None = None
        self.keep_in_memory = directory is None
        if directory:
            os.makedirs(directory, exist_ok=True)
            safe = role.replace("/", "_")
            from .retention import DailyFile
            self._fh = DailyFile(directory, f"spans-{safe}-{os.getpid()}")  # one file per UTC day
            atexit.register(self.flush)

    def export(self, rec: dict[str, Any]) -> None:
        if self.keep_in_memory:
            self._memory.append(rec)
            if len(self._memory) > 10000:
                del self._memory[:5000]
            return
        line = json.dumps(rec, separators=(",", ":"))
        with self._lock:
            self._buf.append(line)
            if len(self._buf) >= 256:
                self._flush_locked()
            elif self._timer is None:  # batched, but never held back more than a second
                self._timer = threading.Thread(target=self._flush_every_second, name="tt-span-flush", daemon=True)
                self._timer.start()

    def _flush_every_second(self) -> None:
        while True:
            time.sleep(1.0)
            self.flush()

    @property
    def memory(self) -> list[dict[str, Any]]:
        """In-memory spans (no telemetry directory), including those relayed by attached
        sources such as the native sidecar data plane."""
        for src in self._sources:
            for rec in src():
                self.export(rec)
        return self._memory

    def attach_source(self, fn) -> None:
        self._sources.append(fn)

    def _flush_locked(self) -> None:
        if self._fh is not None and self._buf:
            self._fh.write("\n".join(self._buf) + "\n")
            self._fh.flush()
        self._buf.clear()

    def flush(self) -> None:
        with self._lock:
            self._flush_locked()


class Tracer:
    def __init__(self, role: str, directory: str | None = None, sample_rate: float = 1.0,
                 instance: str | None = None) -> None:
        self.role = role
        self.instance = instance or f"{role}-{os.getpid()}"
        self.sample_rate = sample_rate
        self.exporter = Exporter(directory, role)

    def start_span(self, name: str, kind: str = "internal", parent: "Span | tuple | None" = None,
                   attributes: dict[str, Any] | None = None, activate: bool = True) -> "Span":
        if parent is None:
            parent = _current.get()
        if isinstance(parent, Span):
            trace_id, parent_id, sampled = parent.trace_id, parent.span_id, parent.sampled
        elif isinstance(parent, tuple):
            trace_id, parent_id, sampled = parent
        else:
            trace_id, parent_id = new_trace_id(), None
            sampled = self.sample_rate >= 1.0 or _rand.random() < self.sample_rate
        span = Span(self, name, kind, trace_id, new_span_id(), parent_id, sampled, attributes)
        if activate:
            span._token = _current.set(span)
        return span

    def flush(self) -> None:
        self.exporter.flush()


class Span:
    __slots__ = ("tracer", "name", "kind", "trace_id", "span_id", "parent_id", "sampled", "attributes",
                 "start", "status", "_token", "_t0", "events")

    def __init__(self, tracer: Tracer, name: str, kind: str, trace_id: str, span_id: str, parent_id: str | None,
                 sampled: bool, attributes: dict[str, Any] | None) -> None:
        self.tracer = tracer
        self.name = name
        self.kind = kind
        self.trace_id = trace_id
        self.span_id = span_id
        self.parent_id = parent_id
        self.sampled = sampled
        self.attributes = attributes
        # unsampled spans only carry context (ids for propagation): skip clocks and attributes
        self.start = time.time() if sampled else 0.0
        self._t0 = time.perf_counter() if sampled else 0.0
        self.status = "ok"
        self._token = None
        self.events: list[tuple[float, str]] | None = None

    @property
    def traceparent(self) -> str:
        return f"00-{self.trace_id}-{self.span_id}-{'01' if self.sampled else '00'}"

    def set(self, key: str, value: Any) -> None:
        if not self.sampled:
            return
        if self.attributes is None:
            self.attributes = {}
        self.attributes[key] = value

    def event(self, name: str) -> None:
        if self.events is None:
            self.events = []
        self.events.append((time.time(), name))

    def fail(self, err: Any = None) -> None:
        self.status = "error"
        if err is not None:
            self.set("error", str(err))

    def end(self) -> None:
        if self._token is not None:
            try:
                _current.reset(self._token)
            except ValueError:
                _current.set(None)
            self._token = None
        if not self.sampled:
            return
        dur = (time.perf_counter() - self._t0) * 1000.0
        rec = {"type": "span", "role": self.tracer.role, "instance": self.tracer.instance, "name": self.name,
               "kind": self.kind, "traceId": self.trace_id, "spanId": self.span_id, "parentId": self.parent_id,
               "ts": self.start, "durationMs": round(dur, 3), "status": self.status}
        if self.attributes:
            rec["attributes"] = self.attributes
        if self.events:
            rec["events"] = self.events
        self.tracer.exporter.export(rec)

    def __enter__(self) -> "Span":
        return self

    def __exit__(self, et, ev, tb) -> None:
        if ev is not None:
            self.fail(ev)
        self.end()


_tracer: Tracer | None = None


def configure(role: str, directory: str | None = None, sample_rate: float | None = None) -> Tracer:
    """Telemetry initializer: sets the process-wide cloud role name and sink."""
    global _tracer
    if directory is None:
        directory = os.environ.get("TT_TELEMETRY_DIR") or None
    if sample_rate is None:
        sample_rate = float(os.environ.get("TT_TRACE_SAMPLE_RATE", "1.0"))
    _tracer = Tracer(role, directory, sample_rate, os.environ.get("TT_REPLICA_NAME"))
    return _tracer


def tracer() -> Tracer:
    global _tracer
    if _tracer is None:
        _tracer = Tracer(os.environ.get("TT_ROLE_NAME", "unknown"), os.environ.get("TT_TELEMETRY_DIR") or None)
    return _tracer


def current_span() -> Span | None:
    return _current.get()


def current_traceparent() -> str | None:
    s = _current.get()
    return s.traceparent if s is not None else None


def current_trace_id() -> str | None:
    s = _current.get()
    return s.trace_id if s is not None else None


def server_middleware(role_attr: str = "http"):
    """WebApp middleware creating a server span per request (ASP.NET request telemetry)."""
    from ..web.http import Request, Response

    async def mw(req: Request, nxt) -> Response:
        tr = tracer()
        tp = req.headers.get("traceparent")
        span = tr.start_span(req.method, "server", parse_traceparent(tp) if tp else None)
        req.state["trace_id"] = span.trace_id
        req.state["span"] = span
        try:
            resp = await nxt(req)
        except BaseException as e:
            span.fail(e)
            span.set("http.status", 500)
            span.end()
            raise
        if span.sampled:  # names and attributes only matter for exported spans
            span.set("http.status", resp.status)
            route = getattr(req.route, "template", None)
            span.name = f"{req.method} {route or req.path}"
        if resp.status >= 500:
            span.status = "error"
        span.end()
        return resp
    return mw
