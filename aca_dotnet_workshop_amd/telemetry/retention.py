"""Telemetry retention: the Log Analytics workspace's ``retentionInDays`` (30 in the
reference: bicep/modules/container-apps-environment.bicep:33-36).

Every telemetry writer (Python logs and spans, the native data plane's spans) appends to one
file per process per UTC day, ``<kind>-<role>-<pid>-<YYYYMMDD>.jsonl``, so retention is a
matter of deleting whole days: ``prune`` removes the day files older than the retention
window (and undated files whose last write is older).  The environment controller runs it at
start-up and hourly.
"""
from __future__ import annotations

import os
import re
import threading
import time
from pathlib import Path

_DAY = re.compile(r"-(\d{8})\.jsonl$")


def utc_day(ts: float | None = None) -> str:
    return time.strftime("%Y%m%d", time.gmtime(time.time() if ts is None else ts))


class DailyFile:
    """Append-only text sink rotated per UTC day: ``<stem>-<YYYYMMDD>.jsonl``."""

    def __init__(self, directory: str, stem: str) -> None:
        os.makedirs(directory, exist_ok=True)
        self.directory = directory
        self.stem = stem
        self._day = ""
        self._fh = None
        self._mu = threading.Lock()

    @property
    def path(self) -> str:
        return os.path.join(self.directory, f"{self.stem}-{self._day or utc_day()}.jsonl")

    def write(self, text: str) -> None:
        with self._mu:
            day = utc_day()
            if day != self._day or self._fh is None:
                if self._fh is not None:
                    self._fh.close()
                self._day = day
                self._fh = open(self.path, "a", encoding="utf-8")
            self._fh.write(text)
            self._fh.flush()

    def flush(self) -> None:
        pass  # every write is flushed (writes are already batched by the callers)

    def close(self) -> None:
        with self._mu:
            if self._fh is not None:
                self._fh.close()
                self._fh = None


def prune(directory: str | os.PathLike, retention_days: float, now: float | None = None) -> dict:
    """Delete telemetry older than ``retention_days``; returns what was removed."""
    now = time.time() if now is None else now
    d = Path(directory)
    removed, kept = [], 0
    if retention_days <= 0 or not d.is_dir():
        return {"removed": removed, "kept": kept}
    cutoff = now - retention_days * 86400.0
    cutoff_day = utc_day(cutoff)
    for f in d.glob("*.jsonl"):
        m = _DAY.search(f.name)
        try:
            old = m.group(1) < cutoff_day if m else f.stat().st_mtime < cutoff
        except OSError:
            continue
        if old:
            try:
                f.unlink()
                removed.append(f.name)
            except OSError:
                pass
        else:
            kept += 1
    return {"removed": sorted(removed), "kept": kept}
