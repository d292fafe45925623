"""Per-request CPU of a service process on the native app host, measured from outside.

Starts a stub sidecar (answers every call 204), one service process wired to it exactly as the
platform wires replicas (``TT_APP_HOST=native``, Information logging to a telemetry dir, 1% trace
sampling), and drives it with ``ttloadgen``; reports CPU microseconds per request of the service's
asyncio thread and of its native I/O thread (psutil per-thread times).  ``scripts/app_cost.py``
isolates the handler; the difference is the host glue (events, futures, the event loop).

    python scripts/host_cost.py [--service api|processor] [--requests 40000]
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

STUB = r"""
import asyncio, sys
from aca_dotnet_workshop_amd.web.native_host import NativeHttpServer
from aca_dotnet_workshop_amd.web.http import Response
async def main():
    async def h(req):
        return Response(b"", 204)
    srv = NativeHttpServer(h)
    await srv.listen_unix(sys.argv[1])
    print("ready", flush=True)
    await asyncio.Event().wait()
asyncio.run(main())
"""


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _wait_port(port: int, timeout: float = 60) -> None:
    import socket
    deadline = time.time() + timeout
    while time.time() < deadline:
        try:
            socket.create_connection(("127.0.0.1", port), 0.5).close()
            return
        except OSError:
            time.sleep(0.1)
    raise TimeoutError(port)


def _bodies(service: str, path: Path, n: int = 512) -> None:
    with open(path, "w") as f:
        for i in range(n):
            task = {"taskName": f"Task {i}", "taskCreatedBy": "bench@example.com",
                    "taskDueDate": "2030-01-01T00:00:00", "taskAssignedTo": "a@example.com"}
            if service == "processor":
                task = {"specversion": "1.0", "id": f"e{i}", "source": "tasksmanager-backend-api",
                        "type": "com.dapr.event.sent", "topic": "tasksavedtopic", "pubsubname": "dapr-pubsub-servicebus",
                        "datacontenttype": "application/json",
                        "data": {"taskId": f"00000000-0000-4000-8000-{i:012d}", **task,
                                 "taskCreatedOn": "2030-01-01T00:00:00.1234567Z", "isCompleted": False,
                                 "isOverDue": False}}
            f.write(json.dumps(task) + "\n")


def main() -> int:
    import psutil
    from aca_dotnet_workshop_amd.native.build import build_loadgen
    ap = argparse.ArgumentParser()
    ap.add_argument("--service", choices=("api", "processor"), default="api")
    ap.add_argument("--requests", type=int, default=40000)
    ap.add_argument("--concurrency", type=int, default=48)
    a = ap.parse_args()
    tmp = Path(tempfile.mkdtemp(prefix="tt-hostcost-"))
    sock = str(tmp / "sidecar.sock")
    port = _free_port()
    env = dict(os.environ, PYTHONPATH=str(ROOT), TT_APP_HOST="native", TT_SIDECAR_UDS=sock,
               TT_TELEMETRY_DIR=str(tmp / "telemetry"), TT_LOG_CONSOLE="0", TT_TRACE_SAMPLE_RATE="0.01",
               Logging__LogLevel__Default="Information", TasksManager__Backend="store")
    stub = subprocess.Popen([sys.executable, "-c", STUB, sock], env=env, stdout=subprocess.PIPE)
    stub.stdout.readline()
    mod = {"api": "backend_api", "processor": "processor"}[a.service]
    app = subprocess.Popen([sys.executable, "-m", f"aca_dotnet_workshop_amd.services.{mod}", "--urls",
                            f"http://127.0.0.1:{port}"], env=env)
    try:
        _wait_port(port)
        _bodies(a.service, tmp / "bodies.txt")
        path, expect, ctype = (("/api/tasks", 201, "application/json") if a.service == "api" else
                               ("/api/tasksnotifier/tasksaved", 200, "application/cloudevents+json"))
        lg = [str(build_loadgen()), "--target", f"tcp:127.0.0.1:{port}", "--path", path, "--bodies",
              str(tmp / "bodies.txt"), "--content-type", ctype, "--concurrency", str(a.concurrency),
              "--expect", str(expect)]
        subprocess.run(lg + ["--batch", "4000", "--steps", "1"], check=True, capture_output=True)  # warm-up
        proc = psutil.Process(app.pid)

        def threads():
            return {t.id: t.user_time + t.system_time for t in proc.threads()}
        t0 = threads()
        w0 = time.perf_counter()
        out = subprocess.run(lg + ["--batch", str(a.requests), "--steps", "1"], check=True, capture_output=True,
                             text=True).stdout
        wall = time.perf_counter() - w0
        t1 = threads()
        main_t = t1.get(app.pid, 0) - t0.get(app.pid, 0)
        other = sum(v - t0.get(k, 0) for k, v in t1.items() if k != app.pid)
        n = a.requests
        print(json.dumps({"service": a.service, "requests": n, "req_per_s": round(n / wall),
                          "asyncio_thread_us_per_req": round(main_t / n * 1e6, 1),
                          "io_threads_us_per_req": round(other / n * 1e6, 1),
                          "loadgen": json.loads(out.strip().splitlines()[-1])["latency_ms"]}))
    finally:
        for p in (app, stub):
            p.terminate()
            p.wait(10)
    return 0


if __name__ == "__main__":
    sys.exit(main())
