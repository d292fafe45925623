"""Telemetry views over the exported spans -- the Application Insights blades the
reference's module 8 walks through (docs/aca/08-aca-monitoring/index.md:367-408):

* ``application_map``  -- nodes = cloud role names (apps; sidecars folded into their app),
  edges = calls between roles with count / failure count / mean latency, built by joining
  each span to its parent across processes;
* ``failures``         -- failed server/consumer operations grouped by role + operation;
* ``performance``      -- per role + operation: count, p50 / p95 / p99 duration;
* ``transaction``      -- every span of one trace id ordered in time (Transaction Search).
"""
from __future__ import annotations

import json
from collections import defaultdict
from pathlib import Path
from typing import Any, Iterable


def load_spans(directory: str | Path) -> list[dict[str, Any]]:
    out = []
    d = Path(directory)
    if not d.exists():
        return out
    for f in sorted(d.glob("spans-*.jsonl")):
        with open(f, errors="replace") as fh:
            for line in fh:
                line = line.strip()
                if line:
                    try:
                        out.append(json.loads(line))
                    except ValueError:
                        continue
    return out


def _app_of(role: str) -> str:
    return role[:-len(".sidecar")] if role.endswith(".sidecar") else role


def application_map(spans_or_dir: Iterable[dict[str, Any]] | str | Path, fold_sidecars: bool = True) -> dict[str, Any]:
    spans = load_spans(spans_or_dir) if isinstance(spans_or_dir, (str, Path)) else list(spans_or_dir)
    by_id = {s["spanId"]: s for s in spans}
    nodes: dict[str, dict[str, Any]] = defaultdict(lambda: {"requests": 0, "failures": 0})
    edges: dict[tuple[str, str], dict[str, Any]] = defaultdict(lambda: {"calls": 0, "failures": 0, "totalMs": 0.0})
    for s in spans:
        role = _app_of(s["role"]) if fold_sidecars else s["role"]
        if s["kind"] in ("server", "consumer"):
            nodes[role]["requests"] += 1
            if s.get("status") == "error":
                nodes[role]["failures"] += 1
        p = by_id.get(s.get("parentId") or "")
        if p is None or s["kind"] not in ("server", "consumer"):
            continue
        src = _app_of(p["role"]) if fold_sidecars else p["role"]
        if src == role:
            continue
        e = edges[(src, role)]
        e["calls"] += 1
        e["totalMs"] += float(s.get("durationMs", 0.0))
        if s.get("status") == "error":
            e["failures"] += 1
    return {"nodes": {k: dict(v) for k, v in sorted(nodes.items())},
            "edges": [{"from": a, "to": b, "calls": e["calls"], "failures": e["failures"],
                       "avgMs": round(e["totalMs"] / e["calls"], 3) if e["calls"] else 0.0}
                      for (a, b), e in sorted(edges.items())]}


def failures(spans_or_dir) -> list[dict[str, Any]]:
    spans = load_spans(spans_or_dir) if isinstance(spans_or_dir, (str, Path)) else list(spans_or_dir)
    agg: dict[tuple[str, str], dict[str, Any]] = {}
    for s in spans:
        if s.get("status") != "error" or s["kind"] not in ("server", "consumer"):
            continue
        k = (s["role"], s["name"])
        a = agg.setdefault(k, {"role": k[0], "operation": k[1], "count": 0, "statuses": defaultdict(int), "sampleTraceIds": []})
        a["count"] += 1
        a["statuses"][str((s.get("attributes") or {}).get("http.status", "exception"))] += 1
        if len(a["sampleTraceIds"]) < 3:
            a["sampleTraceIds"].append(s["traceId"])
    out = []
    for a in sorted(agg.values(), key=lambda x: -x["count"]):
        a["statuses"] = dict(a["statuses"])
        out.append(a)
    return out


def _pct(xs: list[float], q: float) -> float:
    if not xs:
        return 0.0
    xs = sorted(xs)
    return round(xs[min(len(xs) - 1, int(q * len(xs)))], 3)


def performance(spans_or_dir) -> list[dict[str, Any]]:
    spans = load_spans(spans_or_dir) if isinstance(spans_or_dir, (str, Path)) else list(spans_or_dir)
    groups: dict[tuple[str, str], list[float]] = defaultdict(list)
    for s in spans:
        if s["kind"] in ("server", "consumer"):
            groups[(s["role"], s["name"])].append(float(s.get("durationMs", 0.0)))
    return [{"role": r, "operation": op, "count": len(xs), "p50Ms": _pct(xs, 0.5), "p95Ms": _pct(xs, 0.95),
             "p99Ms": _pct(xs, 0.99)} for (r, op), xs in sorted(groups.items(), key=lambda kv: -len(kv[1]))]


def transaction(spans_or_dir, trace_id: str) -> list[dict[str, Any]]:
    spans = load_spans(spans_or_dir) if isinstance(spans_or_dir, (str, Path)) else list(spans_or_dir)
    return sorted((s for s in spans if s["traceId"] == trace_id), key=lambda s: s["ts"])
