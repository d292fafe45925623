"""Counters / histograms with Prometheus text exposition (``GET /metrics``).

Stands in for App Insights Live Metrics / Performance blades (reference
docs/aca/08-aca-monitoring/index.md:383-408): request rates, failure counts and
latency distributions per route, plus sidecar delivery counters used by the scaler.
"""
from __future__ import annotations

import bisect
import threading
from typing import Iterable

_DEFAULT_BUCKETS = (0.0005, 0.001, 0.0025, 0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1.0, 2.5, 5.0, 10.0)


def _labels(lbl: tuple[tuple[str, str], ...]) -> str:
    if not lbl:
        return ""
    return "{" + ",".join(f'{k}="{v}"' for k, v in lbl) + "}"


class Counter:
    def __init__(self, name: str, help: str = "") -> None:
        self.name, self.help = name, help
        self.values: dict[tuple, float] = {}
        self._lock = threading.Lock()

    def inc(self, amount: float = 1.0, **labels: str) -> None:
        key = tuple(sorted(labels.items()))
        with self._lock:
            self.values[key] = self.values.get(key, 0.0) + amount

    def inc_key(self, key: tuple, amount: float = 1.0) -> None:
        """``inc`` with a precomputed label key (``tuple(sorted(labels.items()))``)."""
        with self._lock:
            self.values[key] = self.values.get(key, 0.0) + amount

    def get(self, **labels: str) -> float:
        return self.values.get(tuple(sorted(labels.items())), 0.0)

    def expose(self) -> Iterable[str]:
        yield f"# HELP {self.name} {self.help}"
        yield f"# TYPE {self.name} counter"
        for k, v in self.values.items():
            yield f"{self.name}{_labels(k)} {v}"


class Gauge(Counter):
    def set(self, value: float, **labels: str) -> None:
        with self._lock:
            self.values[tuple(sorted(labels.items()))] = value

    def expose(self) -> Iterable[str]:
        yield f"# HELP {self.name} {self.help}"
        yield f"# TYPE {self.name} gauge"
        for k, v in self.values.items():
            yield f"{self.name}{_labels(k)} {v}"


class Histogram:
    def __init__(self, name: str, help: str = "", buckets: tuple[float, ...] = _DEFAULT_BUCKETS) -> None:
        self.name, self.help, self.buckets = name, help, buckets
        self.series: dict[tuple, list] = {}
        self._lock = threading.Lock()

    def observe(self, value: float, **labels: str) -> None:
        self.observe_key(value, tuple(sorted(labels.items())))

    def observe_key(self, value: float, key: tuple) -> None:
        with self._lock:
            s = self.series.get(key)
            if s is None:
                s = self.series[key] = [[0] * (len(self.buckets) + 1), 0.0, 0]
            s[0][bisect.bisect_left(self.buckets, value)] += 1
            s[1] += value
            s[2] += 1

    def merge_key(self, key: tuple, buckets: list[int], total: float, n: int) -> None:
        """Add observations counted elsewhere (per-bucket counts on this histogram's buckets)."""
        with self._lock:
            s = self.series.get(key)
            if s is None:
                s = self.series[key] = [[0] * (len(self.buckets) + 1), 0.0, 0]
            for i, c in enumerate(buckets):
                s[0][i] += c
            s[1] += total
            s[2] += n

    def quantile(self, q: float, **labels: str) -> float:
        s = self.series.get(tuple(sorted(labels.items())))
        if not s or not s[2]:
            return 0.0
        target, acc = q * s[2], 0
        for i, c in enumerate(s[0]):
            acc += c
            if acc >= target:
                return self.buckets[i] if i < len(self.buckets) else float("inf")
        return float("inf")

    def expose(self) -> Iterable[str]:
        yield f"# HELP {self.name} {self.help}"
        yield f"# TYPE {self.name} histogram"
        for k, (counts, total, n) in self.series.items():
            acc = 0
            for b, c in zip(self.buckets, counts):
                acc += c
                lk = k + (("le", str(b)),)
                yield f"{self.name}_bucket{_labels(lk)} {acc}"
            yield f"{self.name}_bucket{_labels(k + (('le', '+Inf'),))} {n}"
            yield f"{self.name}_sum{_labels(k)} {total}"
            yield f"{self.name}_count{_labels(k)} {n}"


class Registry:
    def __init__(self) -> None:
        self.metrics: dict[str, object] = {}
        self.collectors: list = []  # callables folding counts kept elsewhere (native routes) in

    def collect(self) -> None:
        for c in list(self.collectors):
            c()

    def counter(self, name: str, help: str = "") -> Counter:
        return self.metrics.setdefault(name, Counter(name, help))  # type: ignore[return-value]

    def gauge(self, name: str, help: str = "") -> Gauge:
        return self.metrics.setdefault(name, Gauge(name, help))  # type: ignore[return-value]

    def histogram(self, name: str, help: str = "") -> Histogram:
        return self.metrics.setdefault(name, Histogram(name, help))  # type: ignore[return-value]

    def expose(self) -> str:
        self.collect()
        lines: list[str] = []
        for m in self.metrics.values():
            lines.extend(m.expose())  # type: ignore[attr-defined]
        return "\n".join(lines) + "\n"


REGISTRY = Registry()


def metrics_middleware(registry: Registry = REGISTRY):
    import time
    reqs = registry.counter("http_requests_total", "HTTP requests served")
    lat = registry.histogram("http_request_duration_seconds", "HTTP request latency")

    keys: dict[tuple, tuple] = {}  # (method, route, status) -> precomputed label keys

    async def mw(req, nxt):
        t0 = time.perf_counter()
        resp = await nxt(req)
        route = getattr(req.route, "template", "unmatched")
        ck = (req.method, route, resp.status)
        k = keys.get(ck)
        if k is None:
            k = keys[ck] = (tuple(sorted({"method": req.method, "route": route, "status": str(resp.status)}.items())),
                            (("route", route),))
        reqs.inc_key(k[0])
        lat.observe_key(time.perf_counter() - t0, k[1])
        return resp
    return mw


def request_telemetry_middleware(registry: Registry = REGISTRY):
    """``server_middleware`` (request span, W3C context) and ``metrics_middleware`` (request
    counter and latency histogram) as ONE middleware: what every service host installs, with one
    frame per request instead of two."""
    import time

    from .tracing import new_trace_id, parse_traceparent, tracer
    reqs = registry.counter("http_requests_total", "HTTP requests served")
    lat = registry.histogram("http_request_duration_seconds", "HTTP request latency")
    keys: dict[tuple, tuple] = {}

    async def mw(req, nxt):
        t0 = time.perf_counter()
        tp = req.headers.get("traceparent")
        if tp:
            parent = parse_traceparent(tp)
        elif req.state.get("tt_native") == "sample":  # a native route's sampler picked it
            parent = (new_trace_id(), None, True)
        else:
            parent = None
        span = tracer().start_span(req.method, "server", parent)
        req.state["trace_id"] = span.trace_id
        req.state["span"] = span
        try:
            resp = await nxt(req)
        except BaseException as e:
            span.fail(e)
            span.set("http.status", 500)
            span.end()
            raise
        route = getattr(req.route, "template", None)
        if span.sampled:
            span.set("http.status", resp.status)
            span.name = f"{req.method} {route or req.path}"
        if resp.status >= 500:
            span.status = "error"
        span.end()
        ck = (req.method, route or "unmatched", resp.status)
        k = keys.get(ck)
        if k is None:
            k = keys[ck] = (tuple(sorted({"method": ck[0], "route": ck[1], "status": str(ck[2])}.items())),
                            (("route", ck[1]),))
        reqs.inc_key(k[0])
        lat.observe_key(time.perf_counter() - t0, k[1])
        return resp
    return mw


def parse_exposition(text: str) -> dict[str, float]:
    """Sum every sample of a Prometheus text exposition by ``name{label=...}`` -> value and by
    bare metric name (``name`` -> total over label sets); histogram ``_count``/``_sum`` kept."""
    out: dict[str, float] = {}
    for line in text.splitlines():
        if not line or line.startswith("#"):
            continue
        try:
            series, value = line.rsplit(" ", 1)
            v = float(value)
        except ValueError:
            continue
        out[series] = out.get(series, 0.0) + v
        name = series.split("{", 1)[0]
        if name != series:
            out[name] = out.get(name, 0.0) + v
    return out
