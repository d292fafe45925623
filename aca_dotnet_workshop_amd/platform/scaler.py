"""Event-driven autoscaler -- the KEDA + HPA behaviour ACA gives the processor.

Reference (BASELINE.md "Configured capacity"): ``azure-servicebus``
rule on the processor's subscription, ``messageCount: 10`` -> one replica per 10 queued
messages, ``minReplicas 1``, ``maxReplicas 5``; KEDA polls every 30 s and scales in only
after a 300 s cooldown (docs/aca/09-aca-autoscale-keda/index.md:51-55, :224-226).

Semantics implemented:
* per rule: ``ceil(metric / target)`` (KEDA's AverageValue metric through the HPA);
* across rules: the maximum (HPA takes the largest recommendation);
* clamp to ``[minReplicas, maxReplicas]``;
* scale **out** immediately; scale **in** to the highest recommendation seen within the
  last ``cooldown`` seconds (HPA scale-down stabilization window) -- so a burst scales
  1 -> 5 at once, and the environment returns to 1 replica one cooldown after the backlog
  drains;
* ``minReplicas: 0`` scale-to-zero: deactivate (0 replicas) when every trigger reports
  0 for a full cooldown, activate on the first non-zero sample.

Metric sources: ``azure-servicebus`` (subscription or queue active count), ``azure-queue``
(storage queue length), ``http`` (ingress in-flight requests per replica), ``cpu`` /
``memory`` (average utilisation of the app's processes, via psutil), ``cron`` (desired
replica count inside a schedule window).
"""
from __future__ import annotations

import math
import time
from dataclasses import dataclass, field
from datetime import datetime, timezone
from typing import Any, Awaitable, Callable

from ..utils.cron import CronSchedule

DEFAULT_TARGETS = {"azure-servicebus": 5.0, "azure-queue": 5.0, "http": 10.0, "cpu": 75.0, "memory": 75.0}


@dataclass
class ScaleRule:
    name: str
    type: str
    metadata: dict[str, Any]

    @classmethod
    def from_manifest(cls, r: dict[str, Any]) -> "ScaleRule":
        custom = r.get("custom") or {}
        if "http" in r:
            return cls(r.get("name", "http"), "http", dict((r["http"] or {}).get("metadata") or {}))
        t = custom.get("type") or r.get("type")
        return cls(r.get("name", t), t, dict(custom.get("metadata") or r.get("metadata") or {}))

    def target(self) -> float:
        m = self.metadata
        key = {"azure-servicebus": "messageCount", "azure-queue": "queueLength", "http": "concurrentRequests",
               "cpu": "value", "memory": "value"}.get(self.type)
        if key and m.get(key) not in (None, ""):
            return float(m[key])
        return DEFAULT_TARGETS.get(self.type, 1.0)

    def recommend(self, metric: float, current: int) -> int:
        if self.type in ("cpu", "memory"):
            # utilisation targets scale the current replica count (HPA formula)
            return max(1, math.ceil(current * metric / self.target())) if metric > 0 else 0
        if self.type == "cron":
            return int(metric)
        return math.ceil(metric / self.target()) if metric > 0 else 0


@dataclass
class Autoscaler:
    min_replicas: int
    max_replicas: int
    rules: list[ScaleRule]
    cooldown: float = 300.0
    history: list[tuple[float, int]] = field(default_factory=list)
    last_active: float = field(default_factory=time.monotonic)
    last_rec: int = 0

    def decide(self, metrics: dict[str, float], current: int, now: float | None = None) -> int:
        now = time.monotonic() if now is None else now
        recs = [r.recommend(metrics.get(r.name, 0.0), max(current, 1)) for r in self.rules]
        raw = max(recs) if recs else self.min_replicas
        active = any(metrics.get(r.name, 0.0) > 0 for r in self.rules)
        if active:
            self.last_active = now
        rec = min(self.max_replicas, max(self.min_replicas, raw))
        if self.min_replicas == 0:
            if active:
                rec = max(rec, 1)
            elif now - self.last_active < self.cooldown:
                rec = max(rec, min(current, 1))
        self.last_rec = rec  # this poll's own recommendation, before the stabilization window
        self.history.append((now, rec))
        self.history = [(t, r) for t, r in self.history if now - t <= self.cooldown]
        if rec >= current:
            return rec
        stabilized = max(r for _, r in self.history)
        return min(current, max(rec, stabilized))


MetricFn = Callable[[ScaleRule], Awaitable[float]]


def cron_metric(rule: ScaleRule, now: datetime | None = None) -> float:
    """KEDA cron scaler: ``desiredReplicas`` between ``start`` and ``end`` schedules."""
    now = now or datetime.now(timezone.utc)
    start = CronSchedule.parse(rule.metadata["start"])
    end = CronSchedule.parse(rule.metadata["end"])
    # inside the window iff the most recent start is after the most recent end
    from datetime import timedelta
    probe = now - timedelta(days=8)
    last_start = last_end = None
    t = probe
    while True:
        t = start.next_after(t)
        if t > now:
            break
        last_start = t
    t = probe
    while True:
        t = end.next_after(t)
        if t > now:
            break
        last_end = t
    inside = last_start is not None and (last_end is None or last_start > last_end)
    return float(rule.metadata.get("desiredReplicas", 1)) if inside else 0.0
