"""Latency of one overdue sweep with no other load: the environment of ``deploy/main.yaml``
(native planes, native app-host routes, the API's sidecar calls over gRPC), ``--overdue``
past-due tasks created through the API before each sweep, then the processor's cron job fired
through its sidecar the way the cron binding fires it.

    python scripts/sweep_probe.py [--overdue 1100] [--sweeps 5] [--api 4] [--chunk 256] [--sampled]

Prints one JSON line: per sweep the wall time, the tasks marked and the processor's own split
(``queryMs`` for the GET hop, ``markMs`` for the markoverdue calls).  ``--sampled`` sends a
sampled traceparent (the Python handlers serve it) instead of an unsampled one (the native
routes serve it).
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import sys
import tempfile
import time
from datetime import timedelta
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

API, PROC = "tasksmanager-backend-api", "tasksmanager-backend-processor"


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--overdue", type=int, default=1100)
    ap.add_argument("--sweeps", type=int, default=5)
    ap.add_argument("--api", type=int, default=4)
    ap.add_argument("--chunk", type=int, default=256)
    ap.add_argument("--page", type=int, default=4096)
    ap.add_argument("--sampled", action="store_true")
    ap.add_argument("--hops", action="store_true", help="also time the GET's levels before each sweep")
    ap.add_argument("--accel", default="cpu")
    ap.add_argument("--ru", type=int, default=0, help="the store's RU/s (0: unlimited, as the headline)")
    a = ap.parse_args()
    os.environ.update({"TT_LOG_CONSOLE": "0", "TT_QUERY_ACCEL": a.accel, "TT_QUERY_ACCEL_MIN_DOCS": "1",
                       "TT_QUERY_MIRROR_PATHS": "taskDueDate,isCompleted,isOverDue,taskCreatedOn"})
    from aca_dotnet_workshop_amd.models import format_fixed, today
    from aca_dotnet_workshop_amd.platform.background import BackgroundEnvironment
    from aca_dotnet_workshop_amd.platform.manifest import load_manifest
    from aca_dotnet_workshop_amd.web.client import HttpClient
    m = load_manifest(str(ROOT / "deploy" / "main.yaml"), str(ROOT / "deploy" / "main.parameters.json"),
                      {"backendApiMinReplicas": a.api, "backendApiMaxReplicas": a.api, "frontendMinReplicas": 1,
                       "frontendMaxReplicas": 1, "processorMinReplicas": 1, "processorMaxReplicas": 1,
                       "notifierMode": "log", "overdueQuery": "range", "overduePageSize": a.page,
                       "overdueMarkChunk": a.chunk, "enforceCpuLimits": False,
                       "cosmosAutoscaleMaxThroughput": a.ru,
                       "appInsightsSamplingPercentage": 0, "backendApiDaprApiProtocol": "grpc",
                       "environmentName": "cae-sweep-probe"})
    env = BackgroundEnvironment(m, tempfile.mkdtemp(prefix="tt-sweep-"), log_level="warning")
    yesterday = format_fixed(today() - timedelta(days=1))

    def tp(sampled: bool) -> str:
        return f"00-{os.urandom(16).hex()}-{os.urandom(8).hex()}-{'01' if sampled else '00'}"

    async def run() -> list[dict]:
        c = HttpClient()
        api_sc = [r.sidecar_uds for r in env.replicas(API)]
        proc_sc = env.replicas(PROC)[0].sidecar_uds
        sem = asyncio.Semaphore(64)
        counts = f"{env.backing_url}/servicebus/taskstracker/counts?entity=tasksavedtopic/subscriptions/{PROC}"
        out = []

        async def create(i: int) -> None:
            async with sem:
                r = await c.post(f"unix:{api_sc[i % len(api_sc)]}:/v1.0/invoke/{API}/method/api/tasks",
                                 json_body={"taskName": f"probe {i}", "taskCreatedBy": "probe@x",
                                            "taskDueDate": yesterday, "taskAssignedTo": "a@x"},
                                 headers={"traceparent": tp(False)})
                assert r.status == 201, (r.status, r.body[:200])
        try:
            for s in range(a.sweeps + 1):  # the first sweep warms the mirror and connections
                await asyncio.gather(*(create(s * a.overdue + i) for i in range(a.overdue)))
                for _ in range(3000):  # the processor done with the tasks' events: a quiet sweep
                    if (await c.get(counts)).json().get("completed", 0) >= (s + 1) * a.overdue:
                        break
                    await asyncio.sleep(0.01)
                hops = {}
                if s and a.hops:  # the GET's levels, best of 3 each: store query, API, processor
                    mid = format_fixed(today(), "yyyy-MM-ddTHH:mm:ss")
                    q = {"filter": {"AND": [{"LT": {"taskDueDate": mid}}, {"EQ": {"isCompleted": False}},
                                            {"EQ": {"isOverDue": False}}]},
                         "sort": [{"key": "taskCreatedOn", "order": "ASC"}], "page": {"limit": a.page}}
                    for name, meth, url, kw in (
                            ("sidecar_query", "POST", f"unix:{api_sc[0]}:/v1.0-alpha1/state/statestore/query",
                             {"json_body": q}),
                            ("api_sidecar_invoke", "GET", f"unix:{api_sc[0]}:/v1.0/invoke/{API}/method/api/"
                             f"overduetasks?limit={a.page}", {}),
                            ("proc_sidecar_invoke", "GET", f"unix:{proc_sc}:/v1.0/invoke/{API}/method/api/"
                             f"overduetasks?limit={a.page}", {})):
                        best = 1e9
                        for _ in range(3):
                            t = time.perf_counter()
                            r = await c.request(meth, url, headers={"traceparent": tp(False)}, timeout=60, **kw)
                            best = min(best, (time.perf_counter() - t) * 1e3)
                            assert r.status == 200, (name, r.status, r.body[:200])
                        hops[name] = (round(best, 2), len(r.body))
                    # one markoverdue chunk's store calls through the API sidecar's HTTP API:
                    # bulk get of 256 keys, then the bulk save of those tasks (no ETag: re-runnable)
                    page = json.loads(r.body)[:256]
                    keys = [t["taskId"] for t in page]
                    for name, url, body in (
                            ("sidecar_bulk_get_256", f"unix:{api_sc[0]}:/v1.0/state/statestore/bulk",
                             json.dumps({"keys": keys, "parallelism": 10})),
                            ("sidecar_bulk_save_256", f"unix:{api_sc[0]}:/v1.0/state/statestore",
                             json.dumps([{"key": t["taskId"], "value": t} for t in page], separators=(",", ":")))):
                        best = 1e9
                        for _ in range(3):
                            t = time.perf_counter()
                            r2 = await c.request("POST", url, body=body.encode(), timeout=60,
                                                 headers={"traceparent": tp(False), "content-type": "application/json"})
                            best = min(best, (time.perf_counter() - t) * 1e3)
                            assert r2.status in (200, 204), (name, r2.status, r2.body[:200])
                        hops[name] = (round(best, 2), len(body))
                t = time.perf_counter()
                r = await c.post(f"unix:{proc_sc}:/v1.0/invoke/{PROC}/method/ScheduledTasksManager", body=b"{}",
                                 headers={"Content-Type": "application/json", "traceparent": tp(a.sampled)},
                                 timeout=120)
                ms = (time.perf_counter() - t) * 1e3
                assert r.status == 200, (r.status, r.body[:300])
                j = r.json()
                if s:
                    out.append({"ms": round(ms, 2), "marked": j.get("markedOverdue"), "queryMs": j.get("queryMs"),
                                "markMs": j.get("markMs"), "pages": j.get("pages"), **hops})
            return out
        finally:
            await c.close()
    env.start()
    try:
        sweeps = asyncio.run(run())
    finally:
        env.stop()
    ms = sorted(s["ms"] for s in sweeps)
    print(json.dumps({"overdue_per_sweep": a.overdue, "api_replicas": a.api, "chunk": a.chunk,
                      "sampled": a.sampled, "p50_ms": ms[len(ms) // 2], "sweeps": sweeps}))


if __name__ == "__main__":
    main()
