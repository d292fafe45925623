"""Cron schedule parser for the ``bindings.cron`` component (croniter is not available).

Accepts what the Dapr cron binding accepts (reference components/dapr-scheduled-cron.yaml:10-11
uses ``"5 0 * * *"``):
* 5 fields ``minute hour day-of-month month day-of-week``;
* 6 fields with a leading ``second`` field;
* ``*``, ``?``, lists ``a,b``, ranges ``a-b``, steps ``*/n`` / ``a-b/n`` / ``a/n``,
  month names ``JAN..DEC`` and weekday names ``SUN..SAT`` (``7`` = Sunday);
* descriptors ``@yearly @annually @monthly @weekly @daily @midnight @hourly`` and
  ``@every <duration>`` (``10s``, ``1m30s``, ``2h``, ``500ms``), ticking on multiples of the
  interval since the Unix epoch (replicas agree on the ticks).

Day matching follows cron convention: when both day-of-month and day-of-week are
restricted a day matches if *either* matches.
"""
from __future__ import annotations

import re
from dataclasses import dataclass
from datetime import datetime, timedelta, timezone

_MONTHS = {m: i for i, m in enumerate(["JAN", "FEB", "MAR", "APR", "MAY", "JUN", "JUL", "AUG", "SEP", "OCT", "NOV", "DEC"], 1)}
_DAYS = {d: i for i, d in enumerate(["SUN", "MON", "TUE", "WED", "THU", "FRI", "SAT"])}
_DESCRIPTORS = {"@yearly": "0 0 0 1 1 *", "@annually": "0 0 0 1 1 *", "@monthly": "0 0 0 1 * *",
                "@weekly": "0 0 0 * * 0", "@daily": "0 0 0 * * *", "@midnight": "0 0 0 * * *",
                "@hourly": "0 0 * * * *"}
_DUR = re.compile(r"(\d+(?:\.\d+)?)(ms|h|m|s)")


class CronError(ValueError):
    pass


def parse_duration(s: str) -> timedelta:
    s = s.strip()
    pos, total = 0, 0.0
    for m in _DUR.finditer(s):
        if m.start() != pos:
            raise CronError(f"invalid duration {s!r}")
        v, unit = float(m.group(1)), m.group(2)
        total += v * {"ms": 0.001, "s": 1, "m": 60, "h": 3600}[unit]
        pos = m.end()
    if pos != len(s) or total <= 0:
        raise CronError(f"invalid duration {s!r}")
    return timedelta(seconds=total)


def _field(spec: str, lo: int, hi: int, names: dict[str, int] | None = None) -> frozenset[int]:
    out: set[int] = set()
    for part in spec.split(","):
        part = part.strip().upper()
        if not part:
            raise CronError(f"empty cron field element in {spec!r}")
        step = 1
        if "/" in part:
            part, st = part.split("/", 1)
            step = int(st)
            if step <= 0:
                raise CronError("cron step must be positive")
        if part in ("*", "?"):
            a, b = lo, hi
        elif "-" in part:
            x, y = part.split("-", 1)
            a, b = _val(x, names), _val(y, names)
        else:
            a = _val(part, names)
            b = hi if step != 1 else a
        if a < lo or b > hi or a > b:
            raise CronError(f"cron value out of range in {spec!r} (allowed {lo}-{hi})")
        out.update(range(a, b + 1, step))
    return frozenset(out)


def _val(s: str, names: dict[str, int] | None) -> int:
    if names and s in names:
        return names[s]
    try:
        return int(s)
    except ValueError:
        raise CronError(f"invalid cron value {s!r}") from None


@dataclass(frozen=True)
class CronSchedule:
    expr: str
    seconds: frozenset[int]
    minutes: frozenset[int]
    hours: frozenset[int]
    dom: frozenset[int]
    months: frozenset[int]
    dow: frozenset[int]
    dom_star: bool
    dow_star: bool
    every: timedelta | None = None

    @classmethod
    def parse(cls, expr: str) -> "CronSchedule":
        e = expr.strip()
        low = e.lower()
        if low.startswith("@every"):
            return cls(expr, frozenset(), frozenset(), frozenset(), frozenset(), frozenset(), frozenset(), True, True,
                       parse_duration(e[6:]))
        e = _DESCRIPTORS.get(low, e)
        parts = e.split()
        if len(parts) == 5:
            parts = ["0"] + parts
        if len(parts) != 6:
            raise CronError(f"cron expression needs 5 or 6 fields: {expr!r}")
        sec, mi, hr, dom, mon, dow = parts
        dows = _field(dow, 0, 7, _DAYS)
        if 7 in dows:
            dows = frozenset((dows - {7}) | {0})
        return cls(expr, _field(sec, 0, 59), _field(mi, 0, 59), _field(hr, 0, 23), _field(dom, 1, 31),
                   _field(mon, 1, 12, _MONTHS), dows, dom.strip() in ("*", "?"), dow.strip() in ("*", "?"))

    def _day_ok(self, d: datetime) -> bool:
        dom_ok = d.day in self.dom
        dow_ok = (d.isoweekday() % 7) in self.dow
        if self.dom_star and self.dow_star:
            return True
        if self.dom_star:
            return dow_ok
        if self.dow_star:
            return dom_ok
        return dom_ok or dow_ok

    def next_after(self, after: datetime) -> datetime:
        """First fire time strictly after ``after`` (timezone preserved; naive = UTC)."""
        if self.every is not None:
            # aligned to multiples of the interval since the Unix epoch, so every replica of an
            # app computes the same ticks (the singleReplica lease is keyed by the tick)
            naive = after.tzinfo is None
            base = after.replace(tzinfo=timezone.utc) if naive else after
            step = int(round(self.every.total_seconds() * 1e6))
            us = int(round(base.timestamp() * 1e6))
            nxt = datetime.fromtimestamp((us // step + 1) * step / 1e6, tz=timezone.utc).astimezone(base.tzinfo)
            return nxt.replace(tzinfo=None) if naive else nxt
        t = after.replace(microsecond=0) + timedelta(seconds=1)
        limit = after + timedelta(days=366 * 5)
        while t <= limit:
            if t.month not in self.months:
                y, m = (t.year + 1, 1) if t.month == 12 else (t.year, t.month + 1)
                t = t.replace(year=y, month=m, day=1, hour=0, minute=0, second=0)
                continue
            if not self._day_ok(t):
                t = (t + timedelta(days=1)).replace(hour=0, minute=0, second=0)
                continue
            if t.hour not in self.hours:
                t = (t + timedelta(hours=1)).replace(minute=0, second=0)
                continue
            if t.minute not in self.minutes:
                t = (t + timedelta(minutes=1)).replace(second=0)
                continue
            if t.second not in self.seconds:
                t = t + timedelta(seconds=1)
                continue
            return t
        raise CronError(f"cron expression {self.expr!r} never fires")


def next_fire(expr: str, after: datetime | None = None) -> datetime:
    return CronSchedule.parse(expr).next_after(after or datetime.now(timezone.utc))
