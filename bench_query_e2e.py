#!/usr/bin/env python3
"""State-query latency through the whole stack on a large task collection.

Loads ``--docs`` TaskModel documents into the "Cosmos" account of a backing-services process
(native bulk save), starts one Backend API replica (app + sidecar control plane + native data
plane) and times Dapr state-query API calls made through the sidecar:

* ``overdue_page``: the corrected overdue sweep (``taskDueDate < D AND isCompleted == false AND
  isOverDue == false``) ordered by ``taskDueDate DESC``, first page of 100 -- a scan-shaped query
  the hash indexes cannot answer; with ``--accel gpu`` it runs on the gfx950 scan, ordering and
  top-k kernels (backing/accel.py), with ``--accel off`` on the native engine's CPU scan;
* ``creator_page``: ``taskCreatedBy == X`` (hash-index path, same on both).

Prints one JSON line: first-query latency (includes building / uploading the columnar mirror)
and p50 / p90 of ``--queries`` repetitions, per query.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

ACCOUNT, DB, COLL = "taskstracker-state-store", "tasksmanagerdb", "taskscollection"
PREFIX = "tasksmanager-backend-api||"


def _docs(lo: int, hi: int, rng) -> list[dict]:
    out = []
    for i in range(lo, hi):
        due = f"2024-{rng.randrange(1, 13):02d}-{rng.randrange(1, 29):02d}T00:00:00"
        doc = {"taskId": f"{i:08d}-0000-0000-0000-000000000000", "taskName": f"task {i}",
               "taskCreatedBy": f"user{rng.randrange(10000)}@bench", "taskCreatedOn": "2024-01-01T00:00:00",
               "taskDueDate": due, "taskAssignedTo": f"assignee{rng.randrange(500)}@bench",
               "isCompleted": rng.random() < 0.3, "isOverDue": rng.random() < 0.1}
        out.append({"key": PREFIX + doc["taskId"], "value": json.dumps(doc), "etag": None, "firstWrite": False,
                    "ttlMs": 0})
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=2_000_000)
    ap.add_argument("--queries", type=int, default=20)
    ap.add_argument("--accel", default="gpu", choices=("gpu", "cpu", "off", "auto"))
    a = ap.parse_args()

    import random
    import urllib.request

    from aca_dotnet_workshop_amd.native.build import build_dataplane, build_native
    from aca_dotnet_workshop_amd.platform.processes import LocalStack, uds_get_json
    build_native()
    build_dataplane()
    stack = LocalStack(env={"TT_QUERY_ACCEL": a.accel, "TT_QUERY_ACCEL_MIN_DOCS": "10000",
                            "TT_TRACE_SAMPLE_RATE": "0.0"})
    res: dict = {"metric": "state_query_latency_ms", "docs": a.docs, "accel": a.accel}
    try:
        backing = stack.start_backing()
        r = stack.start_replica("tasksmanager-backend-api", {"Logging:LogLevel:Default": "Warning"})
        stack.wait_ready()
        rng = random.Random(0)
        t0 = time.perf_counter()
        url = f"{backing}/cosmos/{ACCOUNT}/{DB}/{COLL}/bulkset"
        for lo in range(0, a.docs, 20000):
            body = json.dumps(_docs(lo, min(a.docs, lo + 20000), rng)).encode()
            req = urllib.request.Request(url, body, {"Content-Type": "application/json", "x-tt-key": "local-dev-master-key"},
                                         method="POST")
            with urllib.request.urlopen(req, timeout=300) as resp:
                assert resp.status == 200
        res["load_s"] = round(time.perf_counter() - t0, 2)
        print(json.dumps({"loaded": a.docs, "load_s": res["load_s"]}), file=sys.stderr, flush=True)

        import socket

        def query(q: dict) -> tuple[float, dict]:
            body = json.dumps(q).encode()
            s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
            s.settimeout(600)
            s.connect(r.sidecar_uds)
            t = time.perf_counter()
            s.sendall(b"POST /v1.0-alpha1/state/statestore/query HTTP/1.1\r\nHost: x\r\nContent-Type: application/json\r\n"
                      b"Connection: close\r\nContent-Length: " + str(len(body)).encode() + b"\r\n\r\n" + body)
            data = b""
            while True:
                chunk = s.recv(1 << 20)
                if not chunk:
                    break
                data += chunk
            dt = (time.perf_counter() - t) * 1e3
            s.close()
            head, _, payload = data.partition(b"\r\n\r\n")
            if not head.startswith(b"HTTP/1.1 200"):
                raise RuntimeError(f"query failed: {head[:200]!r} {payload[:300]!r}")
            return dt, json.loads(payload)

        queries = {
            "overdue_page": {"filter": {"AND": [{"LT": {"taskDueDate": "2024-07-01T00:00:00"}},
                                                {"EQ": {"isCompleted": False}}, {"EQ": {"isOverDue": False}}]},
                             "sort": [{"key": "taskDueDate", "order": "DESC"}], "page": {"limit": 100}},
            "creator_page": {"filter": {"EQ": {"taskCreatedBy": "user42@bench"}}, "page": {"limit": 100}},
        }
        for name, q in queries.items():
            first, out = query(q)
            lat = sorted(query(q)[0] for _ in range(a.queries))
            res[name] = {"first_ms": round(first, 2), "p50_ms": round(lat[len(lat) // 2], 3),
                         "p90_ms": round(lat[int(len(lat) * 0.9)], 3), "results": len(out.get("results", [])),
                         "token": out.get("token")}
        st = urllib.request.urlopen(f"{backing}/cosmos/{ACCOUNT}/{DB}/{COLL}/stats", timeout=60)
        res["backing_stats"] = json.loads(st.read()).get("accelerator")
    finally:
        stack.stop()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
