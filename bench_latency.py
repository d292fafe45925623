#!/usr/bin/env python3
"""Latency benchmarks the reference never published (SURVEY.md §7.5 "Benchmarks"): report them
as new measurements.

* ``crud``    -- p50/p99 of each Tasks API operation through TWO sidecar hops, the way the
  frontend calls the API (reference Frontend Pages/Tasks/*.cshtml.cs -> InvokeMethodAsync):
  client -> frontend's sidecar -> API's sidecar -> API app -> state store (+ publish on create).
  One request at a time (latency, not throughput).
* ``pubsub``  -- publish -> delivered -> acknowledged: one event published through the API's
  sidecar, timed until the processor's subscription counts it completed (back-to-back counter
  reads).
* ``scale``   -- time-to-scale of the KEDA-style rule (reference
  bicep/modules/container-apps/processor-backend-service.bicep:159-183: 1..5 replicas, one per
  10 messages): a burst lands on the topic, time until 5 processor replicas run, and time until
  the environment is back to 1 replica once drained.  The polling interval / cooldown are
  shortened (the reference's platform defaults are 30 s / 300 s) and reported.

    python bench_latency.py [--ops 200] [--events 200] [--burst 800]

Prints one JSON line per benchmark.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

ENTITY = "tasksavedtopic/subscriptions/tasksmanager-backend-processor"


def pct(xs: list[float], p: float) -> float:
    xs = sorted(xs)
    return round(xs[min(len(xs) - 1, int(len(xs) * p))] * 1e3, 3) if xs else 0.0


def summary(xs: list[float]) -> dict[str, float]:
    return {"p50_ms": pct(xs, 0.5), "p99_ms": pct(xs, 0.99), "max_ms": round(max(xs) * 1e3, 3) if xs else 0.0,
            "n": len(xs)}


async def crud_and_pubsub(stack, backing: str, ops: int, events: int) -> tuple[dict, dict]:
    from aca_dotnet_workshop_amd.backing.client import BackingClient
    from aca_dotnet_workshop_amd.web.client import HttpClient
    fe = stack.replicas["tasksmanager-frontend-webapp"][0]
    api = stack.replicas["tasksmanager-backend-api"][0]
    two_hop = f"unix:{fe.sidecar_uds}:/v1.0/invoke/tasksmanager-backend-api/method/api/tasks"
    c = HttpClient()
    b = BackingClient(backing, identity="tasksmanager-backend-api")
    hdr = {"Content-Type": "application/json"}
    lat: dict[str, list[float]] = {"create": [], "get": [], "list": [], "update": [], "complete": [], "delete": []}
    for i in range(ops + 10):
        warm = i < 10
        body = json.dumps({"taskName": f"lat {i}", "taskCreatedBy": "lat@bench", "taskDueDate": "2030-01-01T00:00:00",
                           "taskAssignedTo": "a@bench"}).encode()
        t = time.perf_counter()
        r = await c.post(two_hop, body=body, headers=hdr)
        t1 = time.perf_counter()
        assert r.status == 201, r
        tid = r.headers["location"].rsplit("/", 1)[1]
        r = await c.get(f"{two_hop}/{tid}")
        t2 = time.perf_counter()
        assert r.status == 200
        r = await c.get(f"{two_hop}?createdBy=lat@bench")
        t3 = time.perf_counter()
        upd = json.dumps({"taskId": tid, "taskName": f"lat {i}!", "taskDueDate": "2030-01-02T00:00:00",
                          "taskAssignedTo": "a@bench"}).encode()
        r = await c.put(f"{two_hop}/{tid}", body=upd, headers=hdr)
        t4 = time.perf_counter()
        assert r.status == 200
        r = await c.put(f"{two_hop}/{tid}/markcomplete")
        t5 = time.perf_counter()
        r = await c.delete(f"{two_hop}/{tid}")
        t6 = time.perf_counter()
        assert r.status == 200
        if not warm:
            for k, a, z in (("create", t, t1), ("get", t1, t2), ("list", t2, t3), ("update", t3, t4),
                            ("complete", t4, t5), ("delete", t5, t6)):
                lat[k].append(z - a)
    crud = {"metric": "crud_latency_two_sidecar_hops", "ops": {k: summary(v) for k, v in lat.items()},
            "path": "client -> frontend sidecar -> API sidecar -> API -> state store"}

    # publish -> delivered -> acked, one event at a time
    pub = f"unix:{api.sidecar_uds}:/v1.0/publish/dapr-pubsub-servicebus/tasksavedtopic"
    base = int((await b.sb_counts("taskstracker", ENTITY))["completed"])
    pl: list[float] = []
    for i in range(events + 10):
        t = time.perf_counter()
        r = await c.post(pub, body=json.dumps({"taskName": f"ev {i}", "taskAssignedTo": "a@bench",
                                               "taskDueDate": "2030-01-01T00:00:00"}).encode(), headers=hdr)
        assert r.status == 204
        base += 1
        while int((await b.sb_counts("taskstracker", ENTITY))["completed"]) < base:
            pass  # back-to-back counter reads (~0.1 ms each): no timer granularity in the figure
        if i >= 10:
            pl.append(time.perf_counter() - t)
    pubsub = {"metric": "publish_to_ack_latency", **summary(pl),
              "path": "API sidecar publish -> broker -> processor sidecar -> processor app -> complete",
              "note": "completion observed by back-to-back counter reads (resolution ~0.1 ms)"}
    await c.close()
    await b.http.close()
    return crud, pubsub


async def time_to_scale(burst: int, polling: float, cooldown: float) -> dict:
    from aca_dotnet_workshop_amd.platform.controller import EnvironmentController
    from aca_dotnet_workshop_amd.platform.manifest import load_manifest
    import tempfile
    m = load_manifest(os.path.join(ROOT, "deploy", "main.yaml"), os.path.join(ROOT, "deploy", "main.parameters.json"),
                      {"notifierSimulatedDelayMs": 150})
    ctl = EnvironmentController(m, tempfile.mkdtemp(prefix="tt-scale-"), polling_interval=polling, cooldown=cooldown)
    await ctl.up(serve_control=False)
    try:
        proc = ctl.apps["tasksmanager-backend-processor"]
        b = ctl.backing
        ce = json.dumps({"specversion": "1.0", "id": "x", "source": "bench", "type": "t",
                         "datacontenttype": "application/json",
                         "data": {"taskName": "burst", "taskAssignedTo": "a@x", "taskDueDate": "2030-01-01T00:00:00"}})
        live = lambda: len([r for r in proc.current.replicas if r.alive()])  # noqa: E731
        t0 = time.perf_counter()
        await b.sb_publish_batch("taskstracker", "tasksavedtopic",
                                 [{"body": ce, "contentType": "application/cloudevents+json"} for _ in range(burst)])
        t_first = t_max = t_drained = t_in = None
        peak = 1
        while time.perf_counter() - t0 < 300:
            await asyncio.sleep(0.05)
            n = live()
            now = time.perf_counter() - t0
            if n > 1 and t_first is None:
                t_first = now
            if n > peak:
                peak = n
            if n == 5 and t_max is None:
                t_max = now
            c = await b.sb_counts("taskstracker", ENTITY)
            if t_drained is None and c["completed"] >= burst:
                t_drained = now
            if t_drained is not None and n == 1:
                t_in = now
                break
        return {"metric": "time_to_scale", "burst_messages": burst, "rule": "azure-servicebus, 1..5, messageCount 10",
                "polling_interval_s": polling, "cooldown_s": cooldown, "peak_replicas": peak,
                "first_scale_out_s": round(t_first, 2) if t_first else None,
                "to_max_replicas_s": round(t_max, 2) if t_max else None,
                "drained_s": round(t_drained, 2) if t_drained else None,
                "back_to_min_s": round(t_in, 2) if t_in else None,
                "simulated_work_ms_per_message": 150}
    finally:
        await ctl.down()


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ops", type=int, default=200, help="CRUD rounds (each: create, get, list, update, complete, delete)")
    ap.add_argument("--events", type=int, default=200)
    ap.add_argument("--burst", type=int, default=800)
    ap.add_argument("--polling", type=float, default=0.5)
    ap.add_argument("--cooldown", type=float, default=3.0)
    ap.add_argument("--skip-scale", action="store_true")
    ap.add_argument("--mtls", action="store_true",
                    help="sidecar-to-sidecar mutual TLS (per-app-id certificates from an environment CA)")
    a = ap.parse_args()
    from aca_dotnet_workshop_amd.native.build import build_dataplane, build_native
    from aca_dotnet_workshop_amd.platform.processes import LocalStack
    build_native()
    build_dataplane()
    cfg = {"Logging:LogLevel:Default": "Warning", "TasksNotifier:Mode": "log"}
    stack = LocalStack(env={"TT_TRACE_SAMPLE_RATE": "0.01"})
    try:
        backing = stack.start_backing()

        def tls_env(app_id: str) -> dict[str, str]:
            if not a.mtls:
                return {}
            from aca_dotnet_workshop_amd.platform.pki import EnvironmentPki
            w = EnvironmentPki(stack.root / "pki").workload(app_id)
            return {"TT_MTLS_CERT": w.cert, "TT_MTLS_KEY": w.key, "TT_MTLS_CA": w.ca}
        stack.start_replica("tasksmanager-backend-api", cfg, extra_env=tls_env("tasksmanager-backend-api"))
        stack.start_replica("tasksmanager-backend-processor", cfg, extra_env=tls_env("tasksmanager-backend-processor"))
        stack.start_replica("tasksmanager-frontend-webapp",
                            {**cfg, "BackendApiConfig:BaseUrlExternalHttp": "http://127.0.0.1:9"},
                            extra_env=tls_env("tasksmanager-frontend-webapp"))
        stack.wait_ready()
        crud, pubsub = asyncio.run(crud_and_pubsub(stack, backing, a.ops, a.events))
    finally:
        stack.stop()
    crud["sidecar_mtls"] = a.mtls
    print(json.dumps(crud), flush=True)
    print(json.dumps(pubsub), flush=True)
    if not a.skip_scale:
        print(json.dumps(asyncio.run(time_to_scale(a.burst, a.polling, a.cooldown))), flush=True)


if __name__ == "__main__":
    main()
