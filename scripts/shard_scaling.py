#!/usr/bin/env python3
"""The partitioned environment at 2, 4 and 8 shards (backing/shards.py; bench.py --shared-env):
idle broker traffic and the overdue sweep's data movement.

For each shard count N: N backing processes (the ranks' shards of the store and the broker),
one API replica and N processor replicas (one per rank, competing on the subscription) whose
sidecars run the native data plane over all N shards.  Measured:

* idle receive requests/s -- every processor sidecar long-polls each shard (one consumer per
  shard, 2 s long polls), summed over the shards' ``sb.receive`` counters while nothing is sent;
* the overdue sweep over a collection of ``--tasks`` tasks (one in ``--due-every`` due
  yesterday): pages, tasks marked, wall time, and the rows the cross-partition query moved --
  sort-key entries from the shards (phase 1) and documents fetched for the merged pages
  (phase 2) -- next to what a one-phase merge would move (every shard's whole page).

    python scripts/shard_scaling.py [--shards 2 4 8] [--tasks 20000] [--out profiles/r4_shards.json]
"""
from __future__ import annotations

import argparse
import asyncio
import json
import sys
import tempfile
import time
from datetime import datetime, timedelta
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from aca_dotnet_workshop_amd.backing.client import BackingClient  # noqa: E402
from aca_dotnet_workshop_amd.backing.shards import ShardedBackingClient  # noqa: E402
from aca_dotnet_workshop_amd.platform.processes import LocalStack  # noqa: E402

ACCT, DB, COLL = "taskstracker-state-store", "tasksmanagerdb", "taskscollection"
PREFIX = "tasksmanager-backend-api||"
NS, TOPIC, SUB = "taskstracker", "tasksavedtopic", "tasksmanager-backend-processor"
MIRROR = {"TT_QUERY_ACCEL": "cpu", "TT_QUERY_ACCEL_MIN_DOCS": "0",
          "TT_QUERY_MIRROR_PATHS": "taskDueDate,isCompleted,isOverDue,taskCreatedOn"}


def _front(url: str) -> dict:
    import urllib.request
    req = urllib.request.Request(url + "/admin/front", headers={"x-tt-identity": "platform-admin"})
    with urllib.request.urlopen(req, timeout=10) as r:
        return json.loads(r.read())


def _receives(urls: list[str]) -> int:
    return sum(int((_front(u).get("requests") or {}).get("sb.receive", 0)) for u in urls)


async def _metric(http, sock: str) -> tuple[int, int]:
    m = (await http.request("GET", f"unix:{sock}:/metrics")).body.decode()

    def val(phase: str) -> int:
        tail = m.split(f'phase="{phase}"}} ')
        return int(tail[1].split()[0]) if len(tail) > 1 else 0
    return val("keys"), val("documents")


def run_one(n: int, tasks: int, due_every: int, idle_s: float, root: Path) -> dict:
    shards: list[LocalStack] = []
    app = None
    try:
        for i in range(n):
            s = LocalStack(root=root / f"n{n}-shard{i}", env=MIRROR)
            s.start_backing()
            shards.append(s)
        urls = [s.backing_url for s in shards]

        async def provision():
            sh = ShardedBackingClient(urls, identity="platform-admin")
            try:
                await sh.sb_create_topic(NS, TOPIC)
                await sh.sb_create_subscription(NS, TOPIC, SUB)
                yday = (datetime.utcnow() - timedelta(days=1)).strftime("%Y-%m-%dT00:00:00")
                items = []
                for i in range(tasks):
                    tid = f"00000000-0000-4000-8000-{i:012d}"
                    t = {"taskId": tid, "taskName": f"t{i}", "taskCreatedBy": f"u{i % 97}@x",
                         "taskCreatedOn": (datetime(2026, 1, 1) + timedelta(seconds=i)).strftime("%Y-%m-%dT%H:%M:%S"),
                         "taskDueDate": yday if i % due_every == 0 else "2030-01-01T00:00:00",
                         "taskAssignedTo": "a@x", "isCompleted": False, "isOverDue": False}
                    items.append({"key": PREFIX + tid, "value": json.dumps(t)})
                for lo in range(0, len(items), 2000):
                    await sh.doc_bulk_set(ACCT, DB, COLL, items[lo:lo + 2000])
            finally:
                await sh.close()
        asyncio.run(provision())
        app = LocalStack(root=root / f"n{n}-apps")
        app.start_backing()  # home services (Key Vault, Storage ...)
        for fam in ("COSMOS", "SERVICEBUS"):
            app.base_env[f"TT_BACKING_SHARDS_{fam}"] = ",".join(urls)
        cfg = {"Logging:LogLevel:Default": "Warning", "TasksNotifier:Mode": "log"}
        api = app.start_replica("tasksmanager-backend-api", {**cfg, "OverdueTasks:Query": "range"})
        procs = [app.start_replica("tasksmanager-backend-processor", {**cfg, "OverdueTasks:PageSize": "1000"})
                 for _ in range(n)]
        app.wait_ready()
        time.sleep(2.5)  # every consumer is in its long poll
        r0, t0 = _receives(urls), time.perf_counter()
        time.sleep(idle_s)
        idle_rate = (_receives(urls) - r0) / (time.perf_counter() - t0)

        async def sweep():
            from aca_dotnet_workshop_amd.web.client import HttpClient
            http = HttpClient()
            try:
                k0, d0 = await _metric(http, api.sidecar_uds)
                t = time.perf_counter()
                r = await http.request("POST", f"unix:{procs[0].sidecar_uds}:/v1.0/invoke/{SUB}/method/"
                                       "ScheduledTasksManager", body=b"{}",
                                       headers=[("Content-Type", "application/json")], timeout=300)
                wall = time.perf_counter() - t
                assert r.status == 200, r.body
                k1, d1 = await _metric(http, api.sidecar_uds)
                return json.loads(r.body), wall, k1 - k0, d1 - d0
            finally:
                await http.close()
        res, wall, keys, docs = asyncio.run(sweep())
        want = len(range(0, tasks, due_every))
        assert res["markedOverdue"] == want, (res, want)
        return {"shards": n, "processor_replicas": n, "consumers_per_shard": n,
                "idle_receive_requests_per_s": round(idle_rate, 1),
                "idle_receive_requests_per_s_per_consumer": round(idle_rate / (n * n), 3),
                "sweep": {"tasks": tasks, "due_yesterday": want, "pages": res["pages"],
                          "marked": res["markedOverdue"], "wall_ms": round(wall * 1e3, 1),
                          "sort_key_entries_moved": keys, "documents_moved": docs,
                          "one_phase_documents_moved": keys,
                          "documents_per_marked_task": round(docs / max(1, want), 3)}}
    finally:
        if app is not None:
            app.stop()
        for s in shards:
            s.stop()


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--shards", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--tasks", type=int, default=20000)
    ap.add_argument("--due-every", type=int, default=8)
    ap.add_argument("--idle-s", type=float, default=10.0)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    out = []
    with tempfile.TemporaryDirectory(prefix="tt-shards-") as d:
        for n in a.shards:
            r = run_one(n, a.tasks, a.due_every, a.idle_s, Path(d))
            print(json.dumps(r), flush=True)
            out.append(r)
    if a.out:
        Path(a.out).write_text(json.dumps(out, indent=1) + "\n")


if __name__ == "__main__":
    main()
