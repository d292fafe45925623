"""App-side CPU per task, in process: the Backend API's ``POST /api/tasks`` and the processor's
``tasksaved`` subscriber driven through their whole middleware pipelines (tracing, metrics,
CloudEvents, model binding, Information logging to the telemetry dir) with the sidecar stubbed
out, so the number is the Python work per task and nothing else.

    python scripts/app_cost.py [--n 20000] [--profile]

This is the attribution ``profiles/r1_e2e_cpu_attribution.md`` measured from outside (CPU seconds
of the app processes / tasks) isolated from the I/O host; docs/PERFORMANCE.md quotes both.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import sys
import tempfile
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


class _StubHttp:
    """The sidecar: every call answers 204 at once (a completed future, like a batch wake-up)."""

    def __init__(self) -> None:
        from aca_dotnet_workshop_amd.web.client import ClientResponse
        from aca_dotnet_workshop_amd.web.http import Headers
        self.resp = ClientResponse(204, Headers({}), b"")
        self.calls = 0

    async def request(self, method, url, *, headers=None, body=None, json_body=None, timeout=None):
        self.calls += 1
        return self.resp

    async def close(self) -> None:
        pass


def _env(tmp: str) -> None:
    os.environ.update({"TT_TELEMETRY_DIR": tmp, "TT_LOG_CONSOLE": "0", "TT_APP_HOST": "",
                       "Logging__LogLevel__Default": "Information", "DAPR_HTTP_PORT": "3500",
                       "TT_TRACE_SAMPLE_RATE": "0.01"})  # bench.py's settings


async def _drive(app, reqs, concurrency: int = 64) -> float:
    """Run the requests ``concurrency`` at a time (the native host hands batches to the loop)."""
    t0 = time.perf_counter()
    for i in range(0, len(reqs), concurrency):
        rs = await asyncio.gather(*(app(r) for r in reqs[i:i + concurrency]))
        assert all(r.status < 300 or r.status == 302 for r in rs), rs[0].status
    return time.perf_counter() - t0


def api_cost(n: int) -> dict:
    from aca_dotnet_workshop_amd.sdk.client import SidecarClient
    from aca_dotnet_workshop_amd.services.backend_api.app import create_app
    from aca_dotnet_workshop_amd.services.backend_api.managers import TasksStoreManager
    from aca_dotnet_workshop_amd.web.http import Headers, Request
    stub = _StubHttp()
    client = SidecarClient("unix:/nonexistent:", http=stub)
    app = create_app([], manager=TasksStoreManager(client))
    hd = {"content-type": "application/json"}  # the load generator sends no trace context

    def req(i):
        body = json.dumps({"taskName": f"Task {i}", "taskCreatedBy": "bench@example.com",
                           "taskDueDate": "2030-01-01T00:00:00", "taskAssignedTo": "a@example.com"}).encode()
        return Request("POST", "/api/tasks", Headers(hd), body, None, "HTTP/1.1")
    asyncio.run(_drive(app, [req(i) for i in range(2000)]))  # warm-up
    reqs = [req(i) for i in range(n)]
    dt = asyncio.run(_drive(app, reqs))
    return {"app": "backend-api POST /api/tasks", "tasks": n, "us_per_task": round(dt / n * 1e6, 1),
            "sidecar_calls_per_task": round(stub.calls / (n + 2000), 2)}


def processor_cost(n: int) -> dict:
    from aca_dotnet_workshop_amd.sdk.client import SidecarClient
    from aca_dotnet_workshop_amd.services.processor.app import create_app
    from aca_dotnet_workshop_amd.web.http import Headers, Request
    app = create_app([], client=SidecarClient("unix:/nonexistent:", http=_StubHttp()))

    def req(i):
        ev = {"specversion": "1.0", "id": f"e{i}", "source": "tasksmanager-backend-api", "type": "com.dapr.event.sent",
              "topic": "tasksavedtopic", "pubsubname": "dapr-pubsub-servicebus", "datacontenttype": "application/json",
              "traceparent": "00-4bf92f3577b34da6a3ce929d0e0e4736-00f067aa0ba902b7-00",
              "data": {"taskId": f"00000000-0000-4000-8000-{i:012d}", "taskName": f"Task {i}",
                       "taskCreatedBy": "bench@example.com", "taskCreatedOn": "2030-01-01T00:00:00.1234567Z",
                       "taskDueDate": "2030-01-02T00:00:00", "taskAssignedTo": "a@example.com",
                       "isCompleted": False, "isOverDue": False}}
        return Request("POST", "/api/tasksnotifier/tasksaved", Headers({"content-type": "application/cloudevents+json"}),
                       json.dumps(ev).encode(), None, "HTTP/1.1")
    asyncio.run(_drive(app, [req(i) for i in range(2000)]))
    reqs = [req(i) for i in range(n)]
    dt = asyncio.run(_drive(app, reqs))
    return {"app": "processor POST /api/tasksnotifier/tasksaved", "tasks": n, "us_per_task": round(dt / n * 1e6, 1)}


def frontend_cost(n: int) -> dict:
    """The frontend's ``POST /Tasks/Create`` (form binding, antiforgery check, invoke of the API
    through the sidecar, 302) with the sidecar answering 201 at once."""
    from urllib.parse import urlencode

    from aca_dotnet_workshop_amd.sdk.client import SidecarClient
    from aca_dotnet_workshop_amd.services.frontend.app import AF_COOKIE, Antiforgery, create_app
    from aca_dotnet_workshop_amd.web.client import ClientResponse
    from aca_dotnet_workshop_amd.web.http import Headers, Request
    stub = _StubHttp()
    stub.resp = ClientResponse(201, Headers({"location": "/api/tasks/x"}), b"")
    key = "k" * 64
    app = create_app([], client=SidecarClient("unix:/nonexistent:", http=stub),
                     overrides={"Frontend:AntiforgeryKey": key})
    tok = Antiforgery(key.encode()).token_for("c0ffee")
    hd = {"content-type": "application/x-www-form-urlencoded",
          "cookie": f"TasksCreatedByCookie=bench@bench.local; {AF_COOKIE}=c0ffee"}

    def req(i):
        body = urlencode({"__RequestVerificationToken": tok, "TaskAdd.TaskName": f"bench task {i}",
                          "TaskAdd.TaskDueDate": "2030-01-01", "TaskAdd.TaskAssignedTo": "a@bench.local"}).encode()
        return Request("POST", "/Tasks/Create", Headers(hd), body, None, "HTTP/1.1")
    asyncio.run(_drive(app, [req(i) for i in range(2000)]))
    reqs = [req(i) for i in range(n)]
    dt = asyncio.run(_drive(app, reqs))
    return {"app": "frontend POST /Tasks/Create", "tasks": n, "us_per_task": round(dt / n * 1e6, 1),
            "sidecar_calls_per_task": round(stub.calls / (n + 2000), 2)}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=20000)
    ap.add_argument("--only", choices=("api", "processor", "frontend"), default=None)
    ap.add_argument("--profile", action="store_true")
    a = ap.parse_args()
    tmp = tempfile.mkdtemp(prefix="tt-appcost-")  # kept: tracers flush their files at exit
    if True:
        _env(tmp)
        fns = [f for k, f in (("api", api_cost), ("processor", processor_cost), ("frontend", frontend_cost))
               if a.only in (None, k)]
        for fn in fns:
            if a.profile:
                import cProfile
                import pstats
                pr = cProfile.Profile()
                pr.enable()
                r = fn(a.n)
                pr.disable()
                pstats.Stats(pr).sort_stats("tottime").print_stats(30)
            else:
                r = fn(a.n)
            print(json.dumps(r), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
