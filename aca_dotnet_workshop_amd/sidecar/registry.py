"""Name resolution: app-id -> sidecar internal endpoints.

Self-hosted Dapr resolves app-ids with mDNS; on ACA the environment's internal DNS does it
(SURVEY.md §5 "Distributed communication backend").  Here every sidecar registers its
internal endpoint as a small JSON file under a shared registry directory (the
environment's "DNS zone"); lookups list the directory (cached briefly), drop entries whose
process is gone, and round-robin across replicas -- so invoking an app with several
replicas load-balances like ACA's internal ingress.
"""
from __future__ import annotations

import itertools
import json
import os
import time
from pathlib import Path


def _alive(pid: int) -> bool:
    try:
        os.kill(pid, 0)
        return True
    except ProcessLookupError:
        return False
    except PermissionError:
        return True


class NameResolver:
    def __init__(self, registry_dir: str | None = None, static: dict[str, list[str]] | None = None,
                 ttl: float = 0.5) -> None:
        self.dir = Path(registry_dir) if registry_dir else None
        self.static = {k: list(v) for k, v in (static or {}).items()}
        self.ttl = ttl
        self._cache: dict[str, tuple[float, list[str]]] = {}
        self._rr: dict[str, itertools.count] = {}
        self._mine: Path | None = None

    def register(self, app_id: str, instance: str, endpoint: str, extra: dict | None = None) -> None:
        if self.dir is None:
            self.static.setdefault(app_id, []).append(endpoint)
            return
        d = self.dir / app_id
        d.mkdir(parents=True, exist_ok=True)
        rec = {"appId": app_id, "instance": instance, "endpoint": endpoint, "pid": os.getpid(), "ts": time.time()}
        rec.update(extra or {})
        tmp = d / f".{instance}.tmp"
        tmp.write_text(json.dumps(rec))
        os.replace(tmp, d / f"{instance}.json")
        self._mine = d / f"{instance}.json"

    def unregister(self) -> None:
        if self._mine is not None:
            try:
                self._mine.unlink()
            except FileNotFoundError:
                pass
            self._mine = None

    def resolve(self, app_id: str) -> list[str]:
        if app_id in self.static:
            return self.static[app_id]
        if self.dir is None:
            return []
        now = time.monotonic()
        hit = self._cache.get(app_id)
        if hit and now - hit[0] < self.ttl:
            return hit[1]
        eps: list[str] = []
        d = self.dir / app_id
        if d.is_dir():
            for f in sorted(d.glob("*.json")):
                try:
                    rec = json.loads(f.read_text())
                except (OSError, ValueError):
                    continue
                if _alive(int(rec.get("pid", 0))):
                    eps.append(rec["endpoint"])
        self._cache[app_id] = (now, eps)
        return eps

    def invalidate(self, app_id: str) -> None:
        self._cache.pop(app_id, None)

    def candidates(self, app_id: str) -> list[str]:
        """All endpoints, rotated round-robin so successive calls start at different replicas."""
        eps = self.resolve(app_id)
        if len(eps) <= 1:
            return eps
        n = next(self._rr.setdefault(app_id, itertools.count())) % len(eps)
        return eps[n:] + eps[:n]
