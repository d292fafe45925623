#!/usr/bin/env python3
"""Flagship benchmark: end-to-end task-creation throughput of the Tasks Tracker environment.

The reference publishes no throughput number (BASELINE.md "Not published"),
so this measures the survey's flagship flow (SURVEY.md §3.1 ``createTask``) and reports it as a
*new* measurement (``vs_baseline: null``).  Default (``--entry frontend``): the environment is
deployed from ``deploy/main.yaml`` by the platform controller (the ``az deployment`` + ACA
equivalent: backing services, RBAC, Dapr components, mTLS identities, revisions, replicas,
resource limits) and load enters where a browser's does -- the frontend's Create page:

    POST /Tasks/Create (form + cookies)  -> Frontend app (Pages/Tasks/Create.cshtml.cs:46)
      -> frontend sidecar invoke -> mTLS -> API sidecar -> Backend API (TasksController.Post)
         -> state save -> backing "Cosmos" (RU/s budget) ; publish -> backing "Service Bus"
      <- 201 <- 302 redirect to /Tasks/Index
    processor sidecar (peek-lock) -> Processor /api/tasksnotifier/tasksaved -> complete

One step = ``--batch`` creates with ``--concurrency`` in flight; a step ends only when the
processor's subscription completed every message of the batch (persisted AND delivered AND
acknowledged).  ``config`` states the entry, mTLS, the RU/s budget, the CPU limits and every
replica count; ``config.api_sidecar_direct`` is a second, shorter run in the same environment
with load sent straight to the API sidecars' invoke (round 2's headline topology).
``--entry api-sidecar`` runs round 2's hand-assembled ``LocalStack`` instead.

Each rank runs its own environment (weak scaling, like adding Container Apps environments);
rank 0 prints ONE JSON line with the aggregate tasks/s (time = max over ranks).

    python bench.py --gpus N --steps K --warmup W
"""
from __future__ import annotations

import argparse
import asyncio
import base64
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


from aca_dotnet_workshop_amd.parallel import Dist, cgroup_throttling, cpu_budget, topology  # noqa: E402


def parse() -> argparse.Namespace:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=16384,
                    help="createTask requests per step per rank (the step quantum: 20 steps >= 3 s timed)")
    ap.add_argument("--concurrency", type=int, default=0,
                    help="requests in flight per rank (0 = 48 per API replica, at most 384)")
    ap.add_argument("--api-replicas", type=int, default=0,
                    help="API replicas behind the client's load balancing (0 = size to this rank's CPU share)")
    ap.add_argument("--processor-replicas", type=int, default=0,
                    help="competing consumers on the subscription (0 = size to this rank's CPU share)")
    ap.add_argument("--split-backing", type=int, default=1, help="separate messaging (Service Bus/Storage) process")
    ap.add_argument("--log-level", default="Information",
                    help="service log level (reference default: Information, appsettings.json); records go as "
                         "structured JSON to the environment's telemetry dir (Log Analytics equivalent)")
    ap.add_argument("--overdue-sweep-ms", type=int, default=1000,
                    help="mixed load: trigger the processor's overdue cron job every N ms during the run "
                         "(OverdueTasks:Query=range -> GPU columnar scan in the backing services); 0 = off")
    ap.add_argument("--mark-chunk", type=int, default=128,
                    help="the sweep's markoverdue calls carry at most this many tasks, concurrently "
                         "(OverdueTasks:MarkChunk; 0 = one call per page, as the reference).  ~1,000 "
                         "tasks a sweep: 128 spreads them over the 4 API replicas in 8 calls; the mark "
                         "hop took 6.6 ms vs 8.0 ms at 256 (gpurun_out/r5d)")
    ap.add_argument("--past-due-every", type=int, default=64,
                    help="every Nth createTask body is due yesterday, so the sweeps mark real tasks overdue")
    ap.add_argument("--app-host", default=os.environ.get("TT_APP_HOST", "native"),
                    help="services' HTTP I/O: python (asyncio) | native (apphost.hpp) | api=native,processor=python")
    ap.add_argument("--api-protocol", choices=("http", "grpc"), default="grpc",
                    help="transport of the API's state and publish calls to its sidecar (grpc: the reference "
                         ".NET DaprClient's, TasksStoreManager.cs:35,61,155; http: the sidecar's HTTP API)")
    ap.add_argument("--alt-steps", type=int, default=-1,
                    help="steps of config.api_protocol_alt, the headline's flow in a second environment with "
                         "the other --api-protocol (-1 = half of --steps, 0 = skip)")
    ap.add_argument("--shared-env", action="store_true",
                    help="multi-rank: ONE partitioned environment -- every rank hosts one shard of the state store "
                         "and of the broker (backing/shards.py: documents and messages by partition-key hash, "
                         "cross-partition queries merged), every rank's replicas reach all shards and the "
                         "processors of all ranks compete on the one subscription (the reference's KEDA scale "
                         "axis); default: one environment per rank (weak scaling)")
    ap.add_argument("--client", choices=("native", "python"), default="native",
                    help="load generator: native/bin/ttloadgen (C++) or the in-process asyncio client")
    ap.add_argument("--entry", choices=("frontend", "api-sidecar"), default="frontend",
                    help="frontend: manifest-deployed environment, load at the frontend's POST /Tasks/Create "
                         "(SURVEY §3.1); api-sidecar: round 2's LocalStack with load at the API sidecars")
    ap.add_argument("--frontend-replicas", type=int, default=0, help="frontend replicas (0 = size to the CPU share)")
    ap.add_argument("--ingress", choices=("native", "python", "bypass"), default="native",
                    help="where --entry frontend load enters: the frontend's external HTTPS ingress (native/bin/"
                         "ttingress, or the asyncio proxy), or bypass it and balance over the frontend replicas")
    ap.add_argument("--mtls", type=int, choices=(0, 1), default=1, help="sidecar-to-sidecar mutual TLS (ACA default: on)")
    ap.add_argument("--ru-per-s", type=float, default=0.0,
                    help="Cosmos container throughput budget in RU/s (reference: 4000 autoscale max); 0 = unlimited")
    ap.add_argument("--cpu-limits", type=int, choices=(0, 1), default=1,
                    help="enforce each replica's vCPU share (manifest resourceLimits.cpu)")
    ap.add_argument("--app-cpu", type=float, default=0.0,
                    help="vCPU per replica (reference: 0.25); 0 = this rank's CPUs divided over its replicas")
    ap.add_argument("--trace-sampling", type=float, default=1.0,
                    help="App Insights sampling percentage of request traces (the manifest default is 100)")
    ap.add_argument("--loadgen-threads", type=int, default=1,
                    help="event loops of the native load generator (ttloadgen --threads)")
    ap.add_argument("--cpu-weights", default="",
                    help="frontend:api:processor relative vCPU per replica (default: CPU_WEIGHT)")
    ap.add_argument("--envelope-s", type=float, default=20.0,
                    help="seconds of the secondary reference-envelope run (config.reference_envelope: the "
                         "manifest defaults -- 1/1 frontend/API, processor 1..5 on KEDA, 0.25 vCPU, 4000 RU/s -- "
                         "with the create's 302 followed to /Tasks/Index); 0 = skip")
    ap.add_argument("--keda-messages", type=int, default=10000,
                    help="messages of the envelope's KEDA stage (config.reference_envelope.keda: the module-9 load "
                         "test, 1 s of simulated work each, processor 1..5 replicas); 0 = skip")
    ap.add_argument("--browser-steps", type=int, default=-1,
                    help="steps of the browser_flow read-path run (create + the 302 followed to Tasks/Index, "
                         "per-user cookies; -1 = a quarter of --steps, 0 = skip)")
    ap.add_argument("--platform-split", type=int, choices=(0, 1), default=1,
                    help="pin the platform's processes (backing, ingress, load generator) to PLATFORM_CPUS of the "
                         "rank's CPUs and the replicas to the rest (1), or let them share the set (0)")
    ap.add_argument("--platform-cpus", type=int, default=PLATFORM_CPUS,
                    help="CPUs of the rank's set reserved for the platform's processes (the replicas' caps "
                         "share the rest of the rank's CPU budget)")
    ap.add_argument("--ingest-messages", type=int, default=4096,
                    help="messages of the external_ingest run (storage queue -> processor -> API -> blob; 0 = skip)")
    ap.add_argument("--session-flows", type=int, default=-1,
                    help="flows of the browser_session run (create, list, Edit GET/POST, Complete, Delete, list; "
                         "-1 = --batch, 0 = skip)")
    ap.add_argument("--direct-steps", type=int, default=-1,
                    help="steps of the api_sidecar_direct comparison run (-1 = a quarter of --steps, 0 = skip)")
    return ap.parse_args()


def app_host(app: str, spec: str) -> str:
    """``native`` / ``python`` for every app, or per app: ``api=native,processor=python``."""
    if "=" not in spec:
        return spec
    return dict(p.split("=", 1) for p in spec.split(",")).get(app, "python")


def rank_device_env(environ: dict[str, str] | None = None) -> dict[str, str]:
    """The rank's environment processes see only the rank's own GPU: a document store that
    turns on its GPU query path opens its context there, not on device 0 for every rank."""
    env = os.environ if environ is None else environ
    if int(env.get("WORLD_SIZE", "1")) <= 1 or "HIP_VISIBLE_DEVICES" in env or "LOCAL_RANK" not in env:
        return {}
    return {"HIP_VISIBLE_DEVICES": env["LOCAL_RANK"]}


def device_sync() -> None:
    """Contract: bracket the timed region with a device sync when a GPU is present -- this
    rank's own GPU (LOCAL_RANK), so N ranks do not all open a context on device 0."""
    try:
        import torch

        from aca_dotnet_workshop_amd.parallel import hold_affinity
        with hold_affinity():  # the GPU runtime's first call must not widen this process's CPUs
            if torch.cuda.is_available():
                dev = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
                torch.cuda.synchronize(dev)
    except Exception:
        pass


async def run_steps(socks: list[str], counts_url: str, entity: str, steps: int, batch: int, conc: int,
                    lat: list[float] | None) -> float:
    from aca_dotnet_workshop_amd.web.client import HttpClient
    c = HttpClient()
    urls = [f"unix:{s}:/v1.0/invoke/tasksmanager-backend-api/method/api/tasks" for s in socks]
    hdr = {"Content-Type": "application/json"}
    bodies = _bodies(batch)

    async def completed() -> int:
        r = await c.get(counts_url)
        return int(r.json()["completed"])

    base = await completed()
    t0 = time.perf_counter()
    for _ in range(steps):
        it = iter(range(batch))

        async def worker(w: int) -> None:
            url = urls[w % len(urls)]  # client-side load balancing across API replicas (ACA ingress)
            for i in it:
                t = time.perf_counter()
                r = await c.post(url, body=bodies[i], headers=hdr)
                if r.status != 201:
                    raise RuntimeError(f"createTask failed: {r.status} {r.body[:200]!r}")
                if lat is not None:
                    lat.append(time.perf_counter() - t)
        await asyncio.gather(*(worker(w) for w in range(conc)))
        base += batch
        while await completed() < base:  # end-to-end: wait until the processor acked the batch
            await asyncio.sleep(0.002)
    dt = time.perf_counter() - t0
    await c.close()
    return dt


def _bodies(batch: int, past_due_every: int = 0) -> list[bytes]:
    from datetime import timedelta

    from aca_dotnet_workshop_amd.models import format_fixed, today
    yesterday = format_fixed(today() - timedelta(days=1))
    return [json.dumps({"taskName": f"bench task {i}", "taskCreatedBy": f"user{i % 97}@bench.local",
                        "taskDueDate": yesterday if past_due_every and i % past_due_every == 0 else "2030-01-01T00:00:00",
                        "taskAssignedTo": f"assignee{i % 13}@bench.local"}).encode()
            for i in range(batch)]


class OverdueSweeper:
    """Mixed load: fires the processor's overdue cron job (the reference's ScheduledTasksManager
    binding, normally daily) every ``period_s`` while createTask load runs, through the
    processor's sidecar exactly as the cron binding does -> API ``GET /api/overduetasks?limit=``
    -> range query -> backing planner -> gfx950 columnar scan; then ``markoverdue`` bulk saves."""

    def __init__(self, proc_sidecar_uds: str, period_s: float) -> None:
        import threading
        self.url = (f"unix:{proc_sidecar_uds}:/v1.0/invoke/tasksmanager-backend-processor/method/"
                    "ScheduledTasksManager")
        self.period_s = period_s
        self.stop_ev = threading.Event()
        self.runs: list[tuple[float, dict]] = []
        self.errors: list[str] = []
        self.marked_all = 0  # tasks marked overdue by every sweep since start (reset() keeps it)
        self.trace_ids: list[str] = []  # the sampled sweeps' traces (per-hop spans)
        # warmup sweeps are sampled traces (their spans attribute the job's hops); the timed
        # region's are not, as a production cron run at the manifest's 1 % sampling almost never
        # is -- the native routes serve unsampled requests only, sampled ones take the handlers
        self.sampled = True
        self.sampled_trace_ids: list[str] = []
        self.thread = threading.Thread(target=self._run, name="overdue-sweeper", daemon=True)

    def start(self) -> None:
        self.thread.start()

    def reset(self, sampled: bool = False) -> None:
        """Forget the sweeps so far (the warmup's): the summary covers what follows; the sampled
        warmup traces stay for the span attribution (``sampled_trace_ids``)."""
        self.sampled_trace_ids += self.trace_ids
        self.runs, self.errors, self.trace_ids = [], [], []
        self.sampled = sampled

    def stop(self) -> None:
        self.stop_ev.set()
        self.thread.join(timeout=120)

    def _run(self) -> None:
        asyncio.run(self._loop())

    async def _loop(self) -> None:
        from aca_dotnet_workshop_amd.web.client import HttpClient
        c = HttpClient()
        try:
            while not self.stop_ev.is_set():
                t = time.perf_counter()
                tid = os.urandom(16).hex()
                try:
                    flags = "01" if self.sampled else "00"
                    r = await c.post(self.url, body=b"{}", timeout=60,
                                     headers={"Content-Type": "application/json",
                                              "traceparent": f"00-{tid}-{os.urandom(8).hex()}-{flags}"})
                    if r.status == 200:
                        self.runs.append((time.perf_counter() - t, r.json()))
                        self.marked_all += int(self.runs[-1][1].get("markedOverdue", 0))
                        if self.sampled:
                            self.trace_ids.append(tid)
                    else:
                        self.errors.append(f"{r.status} {r.body[:200]!r}")
                except Exception as e:  # recorded, reported in the bench line
                    self.errors.append(repr(e))
                left = self.period_s - (time.perf_counter() - t)
                if left > 0:
                    await asyncio.get_running_loop().run_in_executor(None, self.stop_ev.wait, left)
        finally:
            await c.close()

    def drain(self, expected: int, tries: int = 30) -> dict:
        """After the load: fire the job until a sweep marks nothing, then compare every task
        marked since the start with the past-due tasks created (``expected``) -- each of them
        must be marked exactly once, as in a single store, however the store is partitioned."""
        from aca_dotnet_workshop_amd.web.client import HttpClient

        async def fire() -> int:
            c = HttpClient()
            try:
                r = await c.post(self.url, body=b"{}", timeout=120, headers={"Content-Type": "application/json"})
                if r.status != 200:
                    raise RuntimeError(f"drain sweep: {r.status} {r.body[:200]!r}")
                return int(r.json().get("markedOverdue", 0))
            finally:
                await c.close()
        extra = runs = 0
        for _ in range(tries):
            got = asyncio.run(fire())
            extra, runs = extra + got, runs + 1
            if got == 0:
                break
        return {"expected_past_due": expected, "marked_total": self.marked_all + extra, "drain_sweeps": runs,
                "marked_by_drain": extra, "exactly_once": self.marked_all + extra == expected}

    def slowest_trace(self) -> str | None:
        if not self.runs:
            return None
        i = max(range(len(self.runs)), key=lambda j: self.runs[j][0])
        return self.trace_ids[i] if i < len(self.trace_ids) else None

    def summary(self) -> dict:
        ms = sorted(d * 1e3 for d, _ in self.runs)
        return {"sweeps": len(self.runs), "errors": len(self.errors),
                "sweep_p50_ms": round(ms[len(ms) // 2], 2) if ms else None,
                "sweep_p99_ms": round(ms[min(len(ms) - 1, int(len(ms) * 0.99))], 2) if ms else None,
                "sweep_max_ms": round(ms[-1], 2) if ms else None,
                "sweep_ms": [round(d * 1e3, 2) for d, _ in self.runs],  # every sweep, in run order
                # per sweep, in run order: [tasks marked, the GET hop's ms, the markoverdue calls' ms]
                "sweep_detail": [[r.get("markedOverdue", 0), r.get("queryMs"), r.get("markMs")] for _, r in self.runs],
                "tasks_marked_overdue": sum(r.get("markedOverdue", 0) for _, r in self.runs),
                "pages": sum(r.get("pages", 0) for _, r in self.runs),
                # the job's two hops (GET api/overduetasks, POST markoverdue), summed over sweeps
                "query_ms_total": round(sum(r.get("queryMs", 0.0) for _, r in self.runs), 1),
                "mark_ms_total": round(sum(r.get("markMs", 0.0) for _, r in self.runs), 1),
                "first_error": self.errors[0] if self.errors else None}


def sweep_trace(telemetry_dir: str, trace_ids: list[str], slowest: str | None = None) -> dict | None:
    """Per-hop time of the sweeps from their spans (every sweep is a sampled trace): for every
    span of the job -- server spans of each sidecar data plane and app, the apps' client calls
    -- the median duration over the sweeps, in the order of the first sweep.  Keys are
    ``role kind name``."""
    from aca_dotnet_workshop_amd.telemetry.appmap import load_spans
    want = set(trace_ids)
    if not want:
        return None
    by_trace: dict[str, list[dict]] = {}
    for sp in load_spans(telemetry_dir):
        if sp.get("traceId") in want:
            by_trace.setdefault(sp["traceId"], []).append(sp)
    if not by_trace:
        return None
    order: list[str] = []
    durs: dict[str, list[float]] = {}
    attrs: dict[str, list[float]] = {}  # numeric span attributes (the store's hop stamps)
    for tid in trace_ids:
        for sp in sorted(by_trace.get(tid, []), key=lambda x: x.get("ts", 0.0)):
            k = f"{sp.get('role')} {sp.get('kind')} {sp.get('name')}"
            if k not in durs:
                order.append(k)
                durs[k] = []
            durs[k].append(float(sp.get("durationMs", 0.0)))
            for ak, av in (sp.get("attributes") or {}).items():
                if ak.endswith("_ms"):  # numbers, or numeric text (the native planes' attributes)
                    try:
                        attrs.setdefault(f"{k} {ak}", []).append(float(av))
                    except (TypeError, ValueError):
                        pass

    def med(xs: list[float]) -> float:
        return round(sorted(xs)[len(xs) // 2], 2)

    def one(tid: str) -> dict:
        """Every span of one sweep (its slowest): where a tail sweep spent its time."""
        out: dict[str, float] = {}
        for sp in sorted(by_trace.get(tid, []), key=lambda x: x.get("ts", 0.0)):
            k = f"{sp.get('role')} {sp.get('kind')} {sp.get('name')}"
            out[k if k not in out else f"{k} #{sum(1 for x in out if x.startswith(k))}"] = \
                round(float(sp.get("durationMs", 0.0)), 2)
        return out
    res = {"sweeps_traced": len(by_trace), "spans_p50_ms": {k: med(durs[k]) for k in order},
           "stamps_p50_ms": {k: med(v) for k, v in attrs.items()}}
    if slowest and slowest in by_trace:
        res["slowest_sweep_spans_ms"] = one(slowest)
    return res


def _counts(url: str | list[str]) -> dict:
    """The subscription's counters; several URLs (a partitioned broker): summed."""
    import urllib.request
    out: dict = {}
    for u in [url] if isinstance(url, str) else url:
        with urllib.request.urlopen(u, timeout=30) as r:
            for k, v in json.loads(r.read()).items():
                out[k] = out.get(k, 0) + v if isinstance(v, (int, float)) else v
    return out


def _counter(url: str | list[str]) -> int:
    return int(_counts(url)["completed"])


def _until(urls: str | list[str]) -> list[str]:
    out = []
    for u in [urls] if isinstance(urls, str) else urls:
        out += ["--until-url", u]
    return out + ["--until-field", "completed"]


def _accel_stats(backings: list[str]) -> dict:
    """The task collection's accelerator stats summed over its shards (one per backing)."""
    out: dict = {}
    for b in backings:
        for k, v in (_collection_stats(b).get("accelerator") or {}).items():
            if isinstance(v, (int, float)) and not isinstance(v, bool):
                out[k] = round(out.get(k, 0) + v, 3)
            else:
                out.setdefault(k, v)
    return out


def _collection_stats(backing: str) -> dict:
    import urllib.request
    url = f"{backing}/cosmos/taskstracker-state-store/tasksmanagerdb/taskscollection/stats"
    req = urllib.request.Request(url, headers={"x-tt-identity": "platform-admin"})  # the environment owner
    try:
        with urllib.request.urlopen(req, timeout=30) as r:
            return json.loads(r.read())
    except Exception as e:
        return {"error": repr(e)}


def run_loadgen(exe: str, socks: list[str], counts_url: str | list[str], steps: int, batch: int, conc: int,
                bodies_file: str, shared: tuple[int, int] | None = None) -> tuple[float, dict]:
    """Closed-loop load from the native generator; returns (wall seconds, its report).
    ``shared = (base, stride)``: the subscription's completed counter is shared with other
    ranks' generators -- start from ``base`` and wait for ``stride`` more per step."""
    import subprocess
    cmd = [exe, "--path", "/v1.0/invoke/tasksmanager-backend-api/method/api/tasks", "--bodies", bodies_file,
           "--concurrency", str(conc), "--batch", str(batch), "--steps", str(steps), "--expect", "201",
           "--until-timeout", "300", *_until(counts_url)]
    if shared is not None:
        cmd += ["--until-base", str(shared[0]), "--until-stride", str(shared[1])]
    for s in socks:
        cmd += ["--target", "unix:" + s]
    t0 = time.perf_counter()
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    dt = time.perf_counter() - t0
    if p.returncode != 0:
        raise RuntimeError(f"load generator failed ({p.returncode}): {p.stdout[-500:]} {p.stderr[-500:]}")
    return dt, json.loads(p.stdout.strip().splitlines()[-1])


def self_launch(gpus: int, argv: list[str]) -> int | None:
    """``--gpus N > 1`` without a launcher: run the N ranks under ``torch.distributed.run`` as a
    CHILD process (never exec: nothing here has touched HIP yet, but a replaced process image
    is not allowed on the GPU pool), relay rank 0's one JSON line, and return the child's exit
    code.  ``None`` when this process is already a rank (``WORLD_SIZE`` set) or N is 1 -- the
    reported ``n_gpus`` is always the number of ranks that actually ran (``Dist.world``)."""
    if gpus <= 1 or "WORLD_SIZE" in os.environ:
        return None
    import signal
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *argv]
    env = dict(os.environ, TT_BENCH_LAUNCHER="self")
    env.setdefault("OMP_NUM_THREADS", "1")
    progress(f"--gpus {gpus} without a launcher: starting {gpus} ranks under torch.distributed.run")
    p = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, text=True, bufsize=1, start_new_session=True)

    def forward(sig, _frame):  # the driver's timeout reaches every rank, not just this parent
        try:
            os.killpg(p.pid, sig)
        except ProcessLookupError:
            pass
    for sig in (signal.SIGTERM, signal.SIGINT):
        signal.signal(sig, forward)
    assert p.stdout is not None
    for line in p.stdout:  # rank 0's result line to stdout; anything else a rank printed: stderr
        if line.startswith("{") and '"metric"' in line:
            sys.stdout.write(line)
            sys.stdout.flush()
        else:
            sys.stderr.write(line)
    return p.wait()


def main() -> None:
    a = parse()
    rc = self_launch(a.gpus, sys.argv[1:])
    if rc is not None:
        raise SystemExit(rc)
    d = Dist()
    if d.world > 1 and a.gpus not in (1, d.world):
        progress(f"--gpus {a.gpus} but {d.world} ranks were launched: reporting {d.world}")
    local = int(os.environ.get("LOCAL_WORLD_SIZE", d.world if d.world > 1 else 1))
    from aca_dotnet_workshop_amd.parallel import pin_rank
    # ranks sharing a host get disjoint NUMA-local core sets (inherited by the whole stack), on
    # the NUMA node of the rank's GPU when sysfs tells; the CPU budget is read after pinning
    share = cpu_budget() / max(1, local)  # a job-wide CPU quota is shared by the host's ranks
    pinned = pin_rank(int(os.environ.get("LOCAL_RANK", "0")), local)
    cores = min(cpu_budget(), share) if pinned else share
    # weak scaling: every rank's environment is sized for the same CPU budget whatever N is --
    # the 1-GPU box's 16-CPU share by default -- so N=1 on a larger node does not get the whole
    # job's quota and N=8 a sixteenth of it (the driver's efficiency compares per-rank numbers)
    cap = float(os.environ.get("TT_BENCH_CORES_PER_RANK", "16"))
    if cap > 0:
        cores = min(cores, cap)
    if a.entry == "frontend":
        return main_frontend(a, d, cores, pinned)
    return main_localstack(a, d, cores, pinned)


def main_localstack(a: argparse.Namespace, d: Dist, cores: float, pinned) -> None:
    n = d.world  # the ranks that actually ran (self_launch starts them for --gpus N)
    auto_api, auto_proc = topology(cores)
    a.api_replicas = a.api_replicas or auto_api
    a.processor_replicas = a.processor_replicas or auto_proc
    a.concurrency = a.concurrency or min(384, 48 * a.api_replicas)
    from aca_dotnet_workshop_amd.native.build import build_dataplane, build_loadgen, build_native
    from aca_dotnet_workshop_amd.platform.processes import LocalStack
    for b in (build_native, build_dataplane, build_loadgen):  # once, before any child needs them
        b()
    cfg = {"Logging:LogLevel:Default": a.log_level, "TasksNotifier:Mode": "log"}
    api_cfg, proc_cfg = dict(cfg), dict(cfg)
    sweep = a.overdue_sweep_ms > 0
    if sweep:
        api_cfg["OverdueTasks:Query"] = "range"
        proc_cfg["OverdueTasks:PageSize"] = str(OVERDUE_PAGE)
    import tempfile
    root = tempfile.mkdtemp(prefix="tt-bench-")
    env = {"TT_TRACE_SAMPLE_RATE": os.environ.get("TT_TRACE_SAMPLE_RATE", "0.01"),
           # logs as structured JSON into the environment's telemetry dir (Log Analytics), not the console
           "TT_TELEMETRY_DIR": os.path.join(root, "telemetry"), "TT_LOG_CONSOLE": "0", **rank_device_env()}
    if sweep:  # the task collection's column mirror is maintained from its first write
        env["TT_QUERY_MIRROR_PATHS"] = "taskDueDate,isCompleted,isOverDue,taskCreatedOn"
    shared = a.shared_env and d.world > 1
    if shared and a.client != "native":
        raise SystemExit("--shared-env needs the native load generator")
    stack = LocalStack(root=root, env=env)
    sweeper = None
    try:
        backing = doc_backing = stack.start_backing()
        if a.split_backing:
            backing = stack.start_backing_family(["SERVICEBUS", "STORAGE"])
        shards, bus_shards = [doc_backing], [backing]
        if shared:  # one shard of the store and of the broker per rank (backing/shards.py)
            shards, bus_shards = d.allgather(doc_backing), d.allgather(backing)
            stack.base_env["TT_BACKING_SHARDS_COSMOS"] = ",".join(shards)
            stack.base_env["TT_BACKING_SHARDS_SERVICEBUS"] = ",".join(bus_shards)
        for _ in range(a.api_replicas):
            stack.start_replica("tasksmanager-backend-api", api_cfg, grpc=a.api_protocol == "grpc",
                                extra_env={"TT_APP_HOST": app_host("api", a.app_host)})
        for _ in range(a.processor_replicas):
            stack.start_replica("tasksmanager-backend-processor", proc_cfg, grpc=a.api_protocol == "grpc",
                                extra_env={"TT_APP_HOST": app_host("processor", a.app_host)})
        stack.wait_ready()
        socks = [r.sidecar_uds for r in stack.replicas["tasksmanager-backend-api"]]
        entity = "tasksavedtopic/subscriptions/tasksmanager-backend-processor"
        counts_url = f"{backing}/servicebus/taskstracker/counts?entity={entity}"
        if shared:
            counts_url = [f"{u}/servicebus/taskstracker/counts?entity={entity}" for u in bus_shards]
        if a.client == "native":
            from aca_dotnet_workshop_amd.native.build import build_loadgen
            exe = str(build_loadgen())
            bodies_file = str(stack.root / "bodies.jsonl")
            with open(bodies_file, "wb") as f:
                f.write(b"\n".join(_bodies(a.batch, a.past_due_every if sweep else 0)) + b"\n")
        gbase = None
        if shared:  # the subscription's completed counter before anyone sends (global step targets)
            d.barrier()
            gbase = d.broadcast(_counter(counts_url) if d.rank == 0 else None)
        stride = a.batch * d.world
        if a.warmup:
            if a.client == "native":
                run_loadgen(exe, socks, counts_url, a.warmup, a.batch, a.concurrency, bodies_file,
                            (gbase, stride) if shared else None)
            else:
                asyncio.run(run_steps(socks, counts_url, entity, a.warmup, a.batch, a.concurrency, None))
        if sweep and (not shared or d.rank == 0):  # one cron trigger per environment
            sweeper = OverdueSweeper(stack.replicas["tasksmanager-backend-processor"][0].sidecar_uds,
                                     a.overdue_sweep_ms / 1000.0)
        lat: list[float] = []
        d.barrier()
        device_sync()
        import psutil
        me = psutil.Process()
        thr0 = cgroup_throttling()
        cpu0 = stack.cpu_seconds()
        sys0 = stack.cpu_seconds("system")
        t = me.cpu_times()
        cpu0["bench-client"] = t.user + t.system + t.children_user + t.children_system
        report = None
        if sweeper is not None:
            sweeper.start()
        if a.client == "native":
            dt, report = run_loadgen(exe, socks, counts_url, a.steps, a.batch, a.concurrency, bodies_file,
                                     (gbase + stride * a.warmup, stride) if shared else None)
        else:
            dt = asyncio.run(run_steps(socks, counts_url, entity, a.steps, a.batch, a.concurrency, lat))
        device_sync()
        d.barrier()
        if sweeper is not None:
            sweeper.stop()
        cpu1 = stack.cpu_seconds()
        sys1 = stack.cpu_seconds("system")
        thr1 = cgroup_throttling()
        t = me.cpu_times()
        cpu1["bench-client"] = t.user + t.system + t.children_user + t.children_system
        dt_max = d.max(dt)
        if d.rank == 0:
            # cores busy per process role during the timed region (where the E2E flow is CPU bound)
            util = {k: round((cpu1.get(k, 0.0) - v) / dt, 2) for k, v in cpu0.items()}
            kern = {k: round((sys1.get(k, 0.0) - v) / dt, 2) for k, v in sys0.items()}  # kernel-mode part
            print(json.dumps({"cpu_cores_busy": util, "total_cores_busy": round(sum(util.values()), 2),
                              "cpu_cores_busy_kernel_mode": kern,
                              "cpu_budget_per_rank": round(cores, 2),
                              "cgroup_throttling": {k: thr1[k] - thr0.get(k, 0) for k in thr1},
                              "loadgen": report}),
                  file=sys.stderr, flush=True)
        lat.sort()
        if report is not None:
            p50, p99 = d.max(report["latency_ms"]["p50"]), d.max(report["latency_ms"]["p99"])
        else:
            p50 = d.max(lat[len(lat) // 2] * 1e3) if lat else 0.0
            p99 = d.max(lat[min(len(lat) - 1, int(len(lat) * 0.99))] * 1e3) if lat else 0.0
        sweep_info = None
        if sweeper is not None:
            acc = _accel_stats(shards if shared else [doc_backing])
            sweep_info = {**sweeper.summary(), "period_ms": a.overdue_sweep_ms, "past_due_every": a.past_due_every,
                          "page_size": OVERDUE_PAGE,
                          "gpu_queries": acc.get("gpu"), "cpu_queries": acc.get("cpu"),
                          "native_queries": acc.get("native"), "mirror_rows": acc.get("rows"),
                          "shards": len(shards)}
            if d.rank == 0:
                print(json.dumps({"overdue_sweeps": sweep_info}), file=sys.stderr, flush=True)
        delivery = None
        if shared:  # exactly-once across the competing consumers of every rank
            c = _counts(counts_url)
            sent = gbase + stride * (a.warmup + a.steps)
            delivery = {"enqueued": c.get("enqueued"), "completed": c.get("completed"), "received": c.get("received"),
                        "dead_lettered": c.get("dead_letter"), "expected": sent,
                        "exactly_once": c.get("completed") == c.get("received") == c.get("enqueued") == sent}
        total = a.batch * a.steps * (d.world if d.world > 1 else 1)
        value = total / dt_max if dt_max > 0 else 0.0
        if d.rank == 0:
            print(json.dumps({
                "metric": "tasks_e2e_per_sec", "value": round(value, 2), "unit": "tasks/s", "n_gpus": n,
                "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(dt_max / a.steps * 1e3, 3),
                "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "n/a (JSON over HTTP)",
                "data": "synthetic createTask payloads",
                "config": {"model": "tasks-tracker createTask flow (API+sidecars+backing+processor)",
                           "global_batch": a.batch * (d.world if d.world > 1 else 1), "seq_len": None,
                           "parallelism": (f"shared-env x{d.world} (store and broker partitioned over {len(shards)} "
                                           f"shards, one per rank; {a.processor_replicas * d.world} competing "
                                           f"processor replicas)"
                                           if shared else f"env-per-rank x{d.world if d.world > 1 else 1}"),
                           "delivery": delivery, "launcher": launcher_label(d),
                           "concurrency_per_rank": a.concurrency, "api_replicas": a.api_replicas,
                           "processor_replicas": a.processor_replicas, "load_generator": a.client,
                           "sidecar_api_protocol": a.api_protocol,
                           "app_host": a.app_host,
                           "cpu_pinning": pin_label(pinned),
                           "entry": "api-sidecar", "mtls": False, "ru_per_s": None, "cpu_limits": None,
                           "create_latency_p50_ms": round(p50, 3),
                           "create_latency_p99_ms": round(p99, 3), "baseline": "reference publishes no throughput",
                           "step_quantum": f"{a.batch} createTask per step per rank (fixed task quantum)",
                           "timed_region_s": round(dt_max, 3), "log_level": a.log_level,
                           "log_sink": "structured JSON lines in the environment telemetry dir",
                           "overdue_sweeps": sweep_info}}),
                flush=True)
    finally:
        if sweeper is not None and sweeper.thread.is_alive():
            sweeper.stop()
        if shared and sys.exc_info()[0] is None:
            d.barrier()  # rank 0 owns the shared backing services: stop them last
        stack.stop()
        d.close()
        if not os.environ.get("TT_BENCH_KEEP"):
            import shutil
            shutil.rmtree(root, ignore_errors=True)


_T0 = time.perf_counter()


def progress(msg: str) -> None:
    """A phase line on stderr (long runs show they are alive; the JSON result stays on stdout)."""
    print(f"[bench {time.perf_counter() - _T0:7.1f}s] {msg}", file=sys.stderr, flush=True)


def launcher_label(d: Dist) -> str:
    if d.world <= 1:
        return "single process"
    how = "self-launched by bench.py" if os.environ.get("TT_BENCH_LAUNCHER") == "self" else "external launcher"
    return f"torch.distributed.run, {d.world} ranks ({how})"


def pin_label(pinned) -> str:
    from aca_dotnet_workshop_amd.parallel import PIN_INFO
    if not pinned:
        return "none"
    return f"{len(pinned)} CPUs per rank ({PIN_INFO.get('mode', 'pinned')})"


FRONTEND, API, PROC = "tasksmanager-frontend-webapp", "tasksmanager-backend-api", "tasksmanager-backend-processor"


def frontend_topology(cores: float) -> tuple[int, int, int]:
    """(frontend, API, processor) replicas for one rank's CPU share: the two Python web apps on
    the request path get one replica per ~4 CPUs each, the processor (its app only acks) half."""
    fe = max(1, min(12, int(cores / 4)))
    return fe, fe, max(1, min(8, int(cores / 8)))


def _form_session(base_url: str, created_by: str, ca_file: str | None = None) -> tuple[str, str]:
    """What a browser holds after opening Tasks/Create: (Cookie header, antiforgery token)."""
    import re
    import ssl
    import urllib.request
    req = urllib.request.Request(f"{base_url}/Tasks/Create",
                                 headers={"Cookie": f"TasksCreatedByCookie={created_by}"})
    ctx = ssl.create_default_context(cafile=ca_file) if base_url.startswith("https") else None
    with urllib.request.urlopen(req, timeout=30, context=ctx) as r:
        html = r.read().decode()
        cookies = [c.split(";", 1)[0] for c in r.headers.get_all("Set-Cookie") or []]
    m = re.search(r'name="__RequestVerificationToken" value="([^"]+)"', html)
    if not m or not cookies:
        raise RuntimeError("Tasks/Create did not hand out an antiforgery cookie and token")
    return "; ".join([f"TasksCreatedByCookie={created_by}"] + cookies), m.group(1)


def _form_bodies(batch: int, token: str, past_due_every: int) -> list[bytes]:
    """The Create page's form posts (Pages/Tasks/Create.cshtml: TaskAdd.* fields, type=date)."""
    from datetime import timedelta
    from urllib.parse import urlencode

    from aca_dotnet_workshop_amd.models import today
    yesterday = (today() - timedelta(days=1)).strftime("%Y-%m-%d")
    return [urlencode({"__RequestVerificationToken": token, "TaskAdd.TaskName": f"bench task {i}",
                       "TaskAdd.TaskDueDate": yesterday if past_due_every and i % past_due_every == 0 else "2030-01-01",
                       "TaskAdd.TaskAssignedTo": f"assignee{i % 13}@bench.local"}).encode()
            for i in range(batch)]


def _form_loadgen_cmd(exe: str, targets: list[str], cookie: str, counts_url: str | list[str], steps: int,
                      batch: int, conc: int, bodies_file: str, shared: tuple[int, int] | None = None,
                      ca_file: str | None = None, threads: int = 1, extra: list[str] | None = None) -> list[str]:
    cmd = [exe, "--path", "/Tasks/Create", "--bodies", bodies_file, "--content-type",
           "application/x-www-form-urlencoded", "--header", f"Cookie: {cookie}", "--concurrency", str(conc),
           "--batch", str(batch), "--steps", str(steps), "--expect", "302", "--until-timeout", "300",
           *_until(counts_url)]
    if shared is not None:
        cmd += ["--until-base", str(shared[0]), "--until-stride", str(shared[1])]
    if ca_file:
        cmd += ["--tls-ca", ca_file]
    if threads > 1:
        cmd += ["--threads", str(threads)]
    cmd += extra or []
    for t in targets:
        cmd += ["--target", t]
    return cmd


class WarmLoadgen:
    """One ``ttloadgen --pause-after W`` process for the warmup and the timed steps: it runs the
    W warmup steps, prints their line and waits; ``timed()`` sends the go line and waits for the
    timed steps' line.  The timed steps reuse the warmup's connections (TLS handshakes done), as a
    browser keeps its connections; the timed region holds no process start and no handshake."""

    def __init__(self, cmd: list[str], warmup: int, root: str) -> None:
        import subprocess
        self._err = open(os.path.join(root, "loadgen.err"), "w+")
        self.p = subprocess.Popen(cmd + ["--pause-after", str(warmup)], stdin=subprocess.PIPE,
                                  stdout=subprocess.PIPE, stderr=self._err, text=True)

    def _fail(self, what: str) -> None:
        self.p.kill()
        self.p.wait()
        self._err.seek(0)
        raise RuntimeError(f"load generator failed ({what}, rc {self.p.returncode}): {self._err.read()[-500:]}")

    def warmup(self) -> dict:
        line = self.p.stdout.readline()
        if not line:
            self._fail("no warmup line")
        rep = json.loads(line)
        if rep.get("errors"):
            self._fail(f"warmup errors: {rep.get('first_error')}")
        return rep

    def timed(self) -> tuple[float, dict]:
        t0 = time.perf_counter()
        self.p.stdin.write("go\n")
        self.p.stdin.flush()
        out = self.p.stdout.read()
        rc = self.p.wait(timeout=900)
        dt = time.perf_counter() - t0
        lines = out.strip().splitlines()
        if rc != 0 or not lines:
            self._err.seek(0)
            raise RuntimeError(f"load generator failed ({rc}): {out[-500:]} {self._err.read()[-500:]}")
        self._err.close()
        return dt, json.loads(lines[-1])


def run_form_loadgen(exe: str, targets: list[str], cookie: str, counts_url: str | list[str], steps: int, batch: int,
                     conc: int, bodies_file: str, shared: tuple[int, int] | None = None,
                     ca_file: str | None = None, threads: int = 1, extra: list[str] | None = None) -> tuple[float, dict]:
    """``targets``: ``host:port`` (a frontend replica) or ``https://host:port`` (the external
    ingress; ``ca_file`` -- the environment CA -- verifies its certificate like a browser)."""
    import subprocess
    cmd = _form_loadgen_cmd(exe, targets, cookie, counts_url, steps, batch, conc, bodies_file, shared, ca_file,
                            threads, extra)
    t0 = time.perf_counter()
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=900)
    dt = time.perf_counter() - t0
    if p.returncode != 0:
        raise RuntimeError(f"load generator failed ({p.returncode}): {p.stdout[-500:]} {p.stderr[-500:]}")
    return dt, json.loads(p.stdout.strip().splitlines()[-1])


def run_session(exe: str, targets: list[str], cookie: str, token: str, flows: int, conc: int, root: str,
                ca_file: str | None, batch: int) -> dict:
    """``ttloadgen --session``: ``flows`` browser sessions, one per in-flight user at a time
    (create -> list -> Edit GET -> Edit POST -> Complete -> Delete -> list), every page's
    latency; the flow rate and the per-page p50 / p99 (Pages/Tasks/*.cshtml.cs)."""
    import subprocess
    af = "; ".join(c for c in cookie.split("; ") if not c.startswith("TasksCreatedByCookie="))
    bodies = os.path.join(root, "session-bodies.txt")
    with open(bodies, "wb") as f:
        f.write(b"\n".join(_form_bodies(min(batch, 4096), token, 0)) + b"\n")
    cmd = [exe, "--session", token, "--bodies", bodies, "--header", f"Cookie: TasksCreatedByCookie={{user}}; {af}",
           "--concurrency", str(conc), "--batch", str(flows), "--steps", "1"]
    if ca_file:
        cmd += ["--tls-ca", ca_file]
    for t in targets:
        cmd += ["--target", t]
    t0 = time.perf_counter()
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=900)
    dt = time.perf_counter() - t0
    try:
        rep = json.loads(p.stdout.strip().splitlines()[-1])
    except (ValueError, IndexError):
        return {"error": f"load generator exit {p.returncode}: {p.stderr[-300:]}"}
    el = float(rep.get("elapsed_s") or dt)
    pages = rep.get("pages") or {}
    create_p99 = (pages.get("create") or {}).get("p99") or 0.0
    return {"flows_per_s": round(rep.get("flows", 0) / el, 1) if el else None,
            "pages_per_s": round(7 * rep.get("flows", 0) / el, 1) if el else None,
            "flows": rep.get("flows"), "errors": rep.get("errors"), "first_error": rep.get("first_error") or None,
            "concurrency": conc, "latency_ms": {k: [v.get("p50"), v.get("p99")] for k, v in pages.items()},
            "max_page_p99_over_create_p99": round(max((v.get("p99") or 0.0) for v in pages.values()) / create_p99, 2)
            if create_p99 else None,
            "status_counts": rep.get("status_counts"), "loadgen_exit": p.returncode,
            "flow": "Create, Index, Edit GET/POST (assignee change), Complete, Delete, Index; [p50, p99] ms per page"}


def external_ingest(env, n: int, timeout_s: float = 120.0) -> dict:
    """SURVEY §3.4 measured: ``n`` base64 task messages put on the storage queue the processor's
    input binding reads (``externaltasksmanager``, decodeBase64), each taken through
    ExternalTasksProcessorController (invoke POST api/tasks, then the blob output binding
    ``externaltasksblobstore``), until the container holds a blob per message and the queue
    completed them all (ExternalTasksProcessorController.cs:22-53; docs/aca/06-aca-dapr-
    bindingsapi/index.md:267-280).  Messages / s from the first put to the last blob, the
    deliveries per message (a redelivery after a failure or an expired visibility timeout counts)."""
    import urllib.request

    from aca_dotnet_workshop_amd.web.client import HttpClient

    def get(path: str):
        req = urllib.request.Request(base + path, headers={"x-tt-key": key})
        with urllib.request.urlopen(req, timeout=30) as r:
            return json.loads(r.read())
    try:
        st = env.manifest.resources.get("storage") or {}
        acct, queue = st.get("account"), (st.get("queues") or [None])[0]
        container = (st.get("containers") or [None])[0]
        key = env.ctl.storage_keys.get(acct, "")
        base = f"{env.stack.backing_url_for('STORAGE')}/storage/{acct}"
        blobs0 = get(f"/blobs/{container}?count=true")["count"]
        q0 = get(f"/queues/{queue}/count")
        bodies = [base64.b64encode(json.dumps({"taskName": f"external task {i}", "taskAssignedTo": f"ext{i % 7}@bench.local",
                                               "taskCreatedBy": "ext@bench.local",
                                               "taskDueDate": "2030-05-01T00:00:00"}).encode()) for i in range(n)]

        async def put_all() -> None:
            c = HttpClient()
            sem = asyncio.Semaphore(64)

            async def one(b: bytes) -> None:
                async with sem:
                    r = await c.post(f"{base}/queues/{queue}/messages", body=b,
                                     headers={"x-tt-key": key, "Content-Type": "text/plain"})
                    if r.status != 201:
                        raise RuntimeError(f"queue put: {r.status} {r.body[:200]!r}")
            try:
                await asyncio.gather(*(one(b) for b in bodies))
            finally:
                await c.close()
        th0 = env.stack.thread_cpu(_ingress_pid(env))
        t0 = time.perf_counter()
        asyncio.run(put_all())
        t_put = time.perf_counter() - t0
        blobs = blobs0
        while time.perf_counter() - t0 < timeout_s:
            blobs = get(f"/blobs/{container}?count=true")["count"]
            if blobs - blobs0 >= n:
                break
            time.sleep(0.05)
        dt = time.perf_counter() - t0
        for _ in range(40):  # the last deletes follow the last blob
            q1 = get(f"/queues/{queue}/count")
            if int(q1.get("completed", 0)) - int(q0.get("completed", 0)) >= n:
                break
            time.sleep(0.05)
        d = {k: int(q1.get(k, 0)) - int(q0.get(k, 0)) for k in ("enqueued", "received", "completed")}
        made = blobs - blobs0
        # the busiest threads of the ingest window (the stderr diagnostics line, not the record)
        hot = hot_threads(th0, env.stack.thread_cpu(_ingress_pid(env)), dt, top=8)
        return {"messages": n, "msgs_per_s": round(made / dt, 1) if dt else None, "seconds": round(dt, 3),
                "enqueue_s": round(t_put, 3), "blobs_written": made, "queue": d,
                "deliveries_per_message": round(d["received"] / n, 3) if n else None,
                "left_on_queue": int(q1.get("active", 0)) + int(q1.get("locked", 0)),
                "dead": int(q1.get("dead_letter", 0)) - int(q0.get("dead_letter", 0)),
                "all_processed": made == n and d["completed"] == n, "hot_threads": hot}
    except Exception as e:  # reported, not fatal to the headline
        return {"error": repr(e)[:300]}


def _cpu_by_role(stack) -> dict[str, float]:
    """CPU seconds so far per process role (replicas summed per app)."""
    raw = stack.cpu_seconds()
    out: dict[str, float] = {}
    for k, v in raw.items():
        role = k
        for app in (FRONTEND, API, PROC):
            if k.startswith(app + "-"):
                role = app + "." + k.rsplit(".", 1)[1]
        out[role] = out.get(role, 0.0) + v
    return out


# the sweep's page (OverdueTasks:PageSize): the reference reads every match in one query
# (ScheduledTasksManagerController.cs:28); a page covers a second's ~1,000 overdue tasks at the
# headline's create rate with room to spare, and stays within the device top-k (kPageCap 8192).
# At 1000 a faster box crossed into two pages per sweep and doubled it (profiles/r4_sweep_tail.md)
OVERDUE_PAGE = 4096

# identities of the browser_flow run: each user's task list stays small (the reference lists a
# user's whole history on every page view)
BROWSER_USERS = 4096

# cores held back for the external ingress when load enters through it (uncapped, like Envoy)
INGRESS_RESERVE = 1.0
# the platform's own processes -- backing services, external ingress, load generator, the
# controller -- get this many CPUs of the rank's set, pinned, and the replicas the rest:
# measured at the headline's rate they need ~3.8 cores (backing 26.8 + ingress 15.4 + load
# generator 9.4 us/task x 73 k/s); the replicas' caps come out of the rest
PLATFORM_CPUS = 4


def _ingress_cpu(env) -> dict[str, float]:
    """CPU seconds so far of the frontend's native ingress process (empty for the asyncio
    ingress, which runs inside the controller, or without an ingress)."""
    import psutil
    rt = env.ctl.apps.get(FRONTEND)
    proc = getattr(getattr(rt, "ingress", None), "proc", None)
    if proc is None:
        return {}
    try:
        t = psutil.Process(proc.pid).cpu_times()
        return {"ingress": t.user + t.system}
    except psutil.Error:
        return {}


def _ingress_pid(env) -> dict[str, int]:
    rt = env.ctl.apps.get(FRONTEND)
    proc = getattr(getattr(rt, "ingress", None), "proc", None)
    return {"ingress": proc.pid} if proc is not None else {}


def hot_threads(before: dict, after: dict, dt: float, top: int = 12) -> list:
    """The busiest threads of the timed region, [role, thread name, cores busy, kernel-mode
    share]: the single thread that saturates first bounds the throughput of a latency-bound
    closed loop; the kernel share says whether it is system calls or its own code."""
    if dt <= 0:
        return []
    rows = []
    for k, (u, s) in after.items():
        u0, s0 = before.get(k, (0.0, 0.0))
        du, ds = u - u0, s - s0
        rows.append(((du + ds) / dt, ds / (du + ds) if du + ds > 0 else 0.0, k))
    rows.sort(key=lambda r: r[0])
    return [[k[0], k[1], round(c, 3), round(ks, 2)] for c, ks, k in reversed(rows[-top:])]


def _throttling(before: dict, after: dict, dt: float) -> dict | None:
    """Per app, over the timed region: periods in which a replica was stopped by the duty cycle
    and the share of wall time its replicas spent stopped (native duty cycle only)."""
    if not after or dt <= 0:
        return None
    out: dict[str, dict] = {}
    for name, st in after.items():
        app = next((x for x in (FRONTEND, API, PROC) if name.startswith(x + "-")), name)
        b = before.get(name) or {}
        o = out.setdefault(app, {"throttled_periods": 0, "stopped_s": 0.0, "replicas": 0})
        o["throttled_periods"] += int(st["throttled_periods"]) - int(b.get("throttled_periods", 0))
        o["stopped_s"] += float(st["stopped_seconds"]) - float(b.get("stopped_seconds", 0.0))
        o["replicas"] += 1
    for o in out.values():
        o["stopped_share"] = round(o.pop("stopped_s") / (dt * max(1, o["replicas"])), 3)
    return out


def cpu_per_task(util: dict[str, float], tasks_per_s: float) -> dict:
    """Microseconds of CPU per created task: in total and per role, from the timed region's
    cores-busy figures (a box-independent view of the headline: throughput = cores / cost)."""
    if tasks_per_s <= 0:
        return {}
    roles = {k: round(v / tasks_per_s * 1e6, 1) for k, v in sorted(util.items())}
    return {"total": round(sum(util.values()) / tasks_per_s * 1e6, 1),
            "apps_frontend_plus_api": round((util.get(f"{FRONTEND}.app", 0.0) + util.get(f"{API}.app", 0.0))
                                            / tasks_per_s * 1e6, 1),
            "by_role": roles}


# relative vCPU per replica of each app (app process + its data plane) at the default 4 / 4 / 2
# replicas: the round-4 per-role attribution (config.cpu_us_per_task: frontend 58 + 27, API
# 67 + 52, processor 20 + 8 us per task; profiles/r4_ingress_cost.md) gives 1 : 1.42 : 0.67, but
# at 0.67 the duty cycle stopped the processors 8-14 % of the timed region (they also run the
# cron sweep) and their acks gated the steps: 0.85 measured +7 % (profiles/r4_cpu_weights.md).
# At ~61 k tasks/s (4 backing-front loops) 0.85 stopped them 9-13 % again, and a sweep that runs
# into a stop waits it out through the processor's sidecar (a 42.8 ms sweep max); 1.1 stops them
# < 1 % at the same throughput (profiles/r4_hot_threads.md)
CPU_WEIGHT = {"frontend": 1.0, "api": 1.42, "processor": 1.1}


def _sidecar_counter(uds: str, op: str) -> int:
    """A native data plane's ``sidecar_native_requests_total`` for one operation (all statuses)."""
    import socket as _socket
    s = _socket.socket(_socket.AF_UNIX, _socket.SOCK_STREAM)
    try:
        s.settimeout(10)
        s.connect(uds)
        s.sendall(b"GET /metrics HTTP/1.1\r\nhost: x\r\nconnection: close\r\n\r\n")
        buf = b""
        while chunk := s.recv(65536):
            buf += chunk
    except OSError:
        return 0
    finally:
        s.close()
    total = 0
    for ln in buf.decode(errors="replace").splitlines():
        if ln.startswith("sidecar_native_requests_total{") and f'op="{op}"' in ln:
            total += int(float(ln.rsplit(" ", 1)[1]))
    return total


WIRE_OPS = ("grpc.SaveState", "grpc.PublishEvent", "grpc.QueryStateAlpha1", "state.save", "publish", "state.query")


def _sidecar_metric(uds: str, prefix: str) -> dict[str, int]:
    """The lines of a native data plane's /metrics that start with ``prefix``: label text ->
    value."""
    import socket as _socket
    s = _socket.socket(_socket.AF_UNIX, _socket.SOCK_STREAM)
    try:
        s.settimeout(10)
        s.connect(uds)
        s.sendall(b"GET /metrics HTTP/1.1\r\nhost: x\r\nconnection: close\r\n\r\n")
        buf = b""
        while chunk := s.recv(65536):
            buf += chunk
    except OSError:
        return {}
    finally:
        s.close()
    out = {}
    for ln in buf.decode(errors="replace").splitlines():
        if ln.startswith(prefix + "{"):
            labels, v = ln.rsplit(" ", 1)
            out[labels[len(prefix):]] = int(float(v))
    return out


def _client_connects(env) -> dict[str, dict[str, int]]:
    """Per app, the outbound connections its sidecars' data planes opened so far (``any`` /
    ``tls``: with a handshake) -- how often a pool had no idle connection."""
    out: dict[str, dict[str, int]] = {}
    for app in (FRONTEND, API, PROC):
        tot = {"any": 0, "tls": 0}
        for r in env.replicas(app):
            for labels, v in _sidecar_metric(r.sidecar_uds, "sidecar_client_connects_total").items():
                tot["tls" if 'transport="tls"' in labels else "any"] += v
        out[app.replace("tasksmanager-", "").replace("backend-", "").replace("-webapp", "")] = tot
    return out


def _api_wire(env) -> dict[str, int]:
    """The API sidecars' data-plane counters of the calls that carry a task: gRPC RPCs
    (``grpc.*``) and the HTTP API operations they run as (``state.save`` / ``publish`` count
    both protocols)."""
    socks = [r.sidecar_uds for r in env.replicas(API)]
    return {op: sum(_sidecar_counter(u, op) for u in socks) for op in WIRE_OPS}


def _wire_delta(w0: dict, w1: dict) -> dict:
    return {k: w1.get(k, 0) - w0.get(k, 0) for k in WIRE_OPS}


def protocol_alt(a: argparse.Namespace, overrides: dict, exe: str, root: str, steps: int, conc: int,
                 rank: int, durable: bool = False) -> dict:
    """The headline's createTask flow with the API's OTHER Dapr protocol (gRPC <-> HTTP), in a
    fresh environment of the same manifest, replicas and CPU caps (no sweep): tasks/s, create
    latency, CPU per task, and the wire counters that show which API carried the calls.
    ``durable``: the SAME protocol with the backing's logs on group commit instead
    (``TT_BACKING_FSYNC=2``, applog.hpp): every state save and publish is acknowledged only once
    fdatasync()ed, as Cosmos and Service Bus acknowledge -- plus the store's sync counts."""
    import psutil

    from aca_dotnet_workshop_amd.platform.background import BackgroundEnvironment
    from aca_dotnet_workshop_amd.platform.manifest import load_manifest
    proto = a.api_protocol if durable else "http" if a.api_protocol == "grpc" else "grpc"
    ov = dict(overrides, backendApiDaprApiProtocol=proto, overdueQuery="equality", overduePageSize=0,
              environmentName=f"cae-{'durable' if durable else 'alt'}-r{rank}")
    m = load_manifest(os.path.join(ROOT, "deploy", "main.yaml"), os.path.join(ROOT, "deploy", "main.parameters.json"), ov)
    env = BackgroundEnvironment(m, os.path.join(root, "durable" if durable else "alt"), log_level="warning")
    fsync0 = os.environ.get("TT_BACKING_FSYNC")
    if durable:
        os.environ["TT_BACKING_FSYNC"] = "2"  # the backing process reads it at start
    try:
        env.start()
        if durable:
            if fsync0 is None:
                os.environ.pop("TT_BACKING_FSYNC", None)
            else:
                os.environ["TT_BACKING_FSYNC"] = fsync0
        ca_file = None
        if a.ingress != "bypass":
            ca_file = str(env.ctl.pki.ca_crt)
            targets = [f"https://127.0.0.1:{env.ctl.apps[FRONTEND].ingress.public_port}"]
            session_url = targets[0]
        else:
            targets = [f"127.0.0.1:{r.app_port}" for r in env.replicas(FRONTEND)]
            session_url = f"http://127.0.0.1:{env.replicas(FRONTEND)[0].app_port}"
        counts = [f"{env.backing_url}/servicebus/taskstracker/counts?entity=tasksavedtopic/subscriptions/{PROC}"]
        cookie, token = _form_session(session_url, "alt@bench.local", ca_file)
        bodies = os.path.join(root, "alt-bodies.txt")
        with open(bodies, "wb") as f:
            f.write(b"\n".join(_form_bodies(a.batch, token, 0)) + b"\n")
        run_form_loadgen(exe, targets, cookie, counts, 2, a.batch, conc, bodies, None, ca_file, a.loadgen_threads)
        me = psutil.Process()
        cpu0 = _cpu_by_role(env.stack)
        t = me.cpu_times()
        cpu0["bench"] = t.user + t.system + t.children_user + t.children_system
        cpu0.update(_ingress_cpu(env))
        w0 = _api_wire(env)
        d0 = _collection_stats(env.backing_url).get("durability") or {}
        dt, rep = run_form_loadgen(exe, targets, cookie, counts, steps, a.batch, conc, bodies, None, ca_file,
                                   a.loadgen_threads)
        w1 = _api_wire(env)
        d1 = _collection_stats(env.backing_url).get("durability") or {}
        cpu1 = _cpu_by_role(env.stack)
        t = me.cpu_times()
        cpu1["bench"] = t.user + t.system + t.children_user + t.children_system
        cpu1.update(_ingress_cpu(env))
        busy = {k: (cpu1.get(k, 0.0) - v) / dt for k, v in cpu0.items()}
        cpu_us = cpu_per_task(busy, a.batch * steps / dt)
        out = {"api_protocol": proto, "value": round(a.batch * steps / dt, 1), "steps": steps,
               "create_latency_p50_ms": rep["latency_ms"]["p50"], "create_latency_p99_ms": rep["latency_ms"]["p99"],
               "cpu_us_per_task": {"total": cpu_us.get("total"),
                                   **{k.replace("tasksmanager-backend-", ""): v
                                      for k, v in (cpu_us.get("by_role") or {}).items() if k.startswith(API)}},
               "api_wire": _wire_delta(w0, w1), "errors": rep.get("errors")}
        if durable:
            syncs = d1.get("syncs", 0) - d0.get("syncs", 0)
            acks = d1.get("acks", 0) - d0.get("acks", 0)
            out["durability"] = {
                "mode": "group commit (fdatasync before every acknowledgement)",
                "fsync_mode": d1.get("fsync_mode"), "state_store_syncs": syncs, "state_store_acks": acks,
                "acks_per_sync": round(acks / syncs, 1) if syncs else None,
                "sync_ms_mean": round((d1.get("sync_ms_total", 0) - d0.get("sync_ms_total", 0)) / syncs, 3) if syncs else None,
                "sync_ms_max": d1.get("sync_ms_max"),
                "unsynced_bytes_at_end": d1.get("written_bytes", 0) - d1.get("synced_bytes", 0),
                "log_file_system": _fs_type(os.path.join(root, "durable"))}
        return out
    except Exception as e:  # reported, not fatal to the headline
        return {"api_protocol": proto, "error": repr(e)[:300]}
    finally:
        env.stop()
        if durable:
            if fsync0 is None:
                os.environ.pop("TT_BACKING_FSYNC", None)
            else:
                os.environ["TT_BACKING_FSYNC"] = fsync0


def reference_envelope(exe: str, root: str, seconds: float, rank: int) -> dict:
    """The reference's own capacity envelope, measured (BASELINE.md "Configured capacity"):
    ``deploy/main.yaml`` with its defaults -- frontend and API at 1..1 replica, the processor at
    1..5 on the KEDA Service Bus rule (10 messages per replica), 0.25 vCPU / 0.5 Gi every
    replica, Cosmos at 4,000 RU/s, mTLS, external HTTPS ingress -- and browser-shaped load: per
    user (a cookie each, so task lists stay bounded) POST /Tasks/Create, then the 302 followed to
    GET /Tasks/Index (the read path, Pages/Tasks/Index.cshtml.cs:48).  Only the KEDA polling
    interval is shortened (5 s instead of ACA's 30 s) so scale-out happens inside the run."""
    import threading

    from aca_dotnet_workshop_amd.platform.background import BackgroundEnvironment
    from aca_dotnet_workshop_amd.platform.manifest import load_manifest
    m = load_manifest(os.path.join(ROOT, "deploy", "main.yaml"), os.path.join(ROOT, "deploy", "main.parameters.json"),
                      {"notifierMode": "log", "kedaPollingIntervalSeconds": 5,
                       "environmentName": f"cae-envelope-r{rank}"})
    env = BackgroundEnvironment(m, os.path.join(root, "envelope"), log_level="warning")
    peak = {"processor": 1}
    stop = threading.Event()

    def watch() -> None:  # the processor replicas KEDA reached
        while not stop.wait(0.5):
            rt = env.ctl.apps.get(PROC) if env.ctl else None
            if rt is not None and rt.current is not None:
                peak["processor"] = max(peak["processor"], len([r for r in rt.current.replicas if r.alive()]))
    try:
        env.start()
        ing = env.ctl.apps[FRONTEND].ingress
        ca = str(env.ctl.pki.ca_crt)
        base = f"https://127.0.0.1:{ing.public_port}"
        cookie, token = _form_session(base, "u0@bench.local", ca)
        af = [c for c in cookie.split("; ") if not c.startswith("TasksCreatedByCookie=")]
        bodies = os.path.join(root, "envelope-bodies.txt")
        with open(bodies, "wb") as f:
            f.write(b"\n".join(_form_bodies(4096, token, 0)) + b"\n")
        counts = [f"{env.backing_url}/servicebus/taskstracker/counts?entity=tasksavedtopic/subscriptions/{PROC}"]
        api_uds = [r.sidecar_uds for r in env.replicas(API)]
        st0 = _collection_stats(env.backing_url).get("throughput", {})
        retry0 = sum(_sidecar_counter(u, "state.throttled_retry") for u in api_uds)
        th = threading.Thread(target=watch, daemon=True)
        th.start()
        steady: dict = {}

        def mark_steady() -> None:
            # the steady window opens at the first 429: the bucket is empty from there on (before
            # it, the load spends the budget an idle bucket holds -- up to a second's worth, which
            # a demand just above the budget takes seconds to drain)
            t_lim = time.perf_counter() + 5.0
            while not stop.wait(0.02):
                st = _collection_stats(env.backing_url).get("throughput", {})
                if st.get("throttled", 0) > st0.get("throttled", 0) or time.perf_counter() > t_lim:
                    steady.update(t=time.perf_counter(), st=st, enq=int(_counts(counts).get("enqueued", 0)),
                                  at_first_429=time.perf_counter() <= t_lim)
                    return
        th2 = threading.Thread(target=mark_steady, daemon=True)
        th2.start()
        enq0 = int(_counts(counts).get("enqueued", 0))
        import subprocess
        cmd = [exe, "--path", "/Tasks/Create", "--bodies", bodies, "--content-type",
               "application/x-www-form-urlencoded", "--header",
               "Cookie: " + "; ".join(["TasksCreatedByCookie={user}"] + af), "--users", "500", "--follow",
               "--concurrency", "16", "--duration", str(seconds), "--expect", "302", "--tls-ca", ca,
               "--until-timeout", "120", "--target", base, *_until(counts)]
        t0 = time.perf_counter()
        p = subprocess.run(cmd, capture_output=True, text=True, timeout=seconds + 600)
        wall = time.perf_counter() - t0
        rep = json.loads(p.stdout.strip().splitlines()[-1]) if p.stdout.strip() else {}
        t_end = time.perf_counter()
        st1 = _collection_stats(env.backing_url).get("throughput", {})
        enq1 = int(_counts(counts).get("enqueued", 0))
        stop.set()
        th2.join(5)
        retries = sum(_sidecar_counter(u, "state.throttled_retry") for u in api_uds) - retry0
        sc = rep.get("status_counts") or {}
        attempts = int(rep.get("requests", 0))
        tasks = int(sc.get("302", 0))  # created (the 302 to the list); a 500 here is a create that failed
        lists_ok = int(sc.get("200", 0))
        ru = float(st1.get("ru_consumed", 0.0)) - float(st0.get("ru_consumed", 0.0))
        el = float(rep.get("elapsed_s") or wall)
        budget = float(st1.get("ru_per_s", 0.0))
        # the steady window: from the first 429 to the end -- RU admitted there over the budget's
        # refill
        sw = None
        if steady and t_end - steady["t"] > 1.0 and budget:
            w = t_end - steady["t"]
            if st1.get("mono") and steady["st"].get("mono"):  # the store's own clock between the two reads
                w = float(st1["mono"]) - float(steady["st"]["mono"])
            ru_s = float(st1.get("ru_consumed", 0.0)) - float(steady["st"].get("ru_consumed", 0.0))
            sw = {"seconds": round(w, 2), "tasks_per_s": round((enq1 - steady["enq"]) / w, 1),
                  "ru_consumed_per_s": round(ru_s / w, 1), "ru_over_budget": round(ru_s / (budget * w), 3),
                  "opens": "at the first 429" if steady.get("at_first_429") else "5 s in (no 429 by then)"}
        by_kind = {k: int(st1.get(f"throttled_{k}", 0) - st0.get(f"throttled_{k}", 0))
                   for k in ("write", "query", "read", "delete")}
        return {"tasks_per_s": round(tasks / el, 1) if el else None, "tasks": tasks, "seconds": round(el, 2),
                "steady_window": sw, "throttled_calls_by_kind": by_kind, "published": enq1 - enq0,
                "create_attempts": attempts, "failed_creates": attempts - tasks, "failed_lists": tasks - lists_ok,
                "errors": rep.get("errors"), "first_error": rep.get("first_error") or None,
                "create_latency_ms": rep.get("latency_ms"), "list_latency_ms": rep.get("follow_latency_ms"),
                "lists_followed": rep.get("follow_requests"), "status_counts": rep.get("status_counts"),
                "ru_per_s_budget": float(st1.get("ru_per_s", 0.0)), "ru_consumed_per_s": round(ru / el, 1) if el else None,
                "ru_per_task": round(ru / tasks, 2) if tasks else None,
                "store_429s": int(st1.get("throttled", 0) - st0.get("throttled", 0)),
                "sidecar_429_retries": retries,
                "budget_over_ru_per_task": round(float(st1.get("ru_per_s", 0.0)) / (ru / tasks), 1) if tasks and ru else None,
                "processor_replicas_reached": peak["processor"],
                "replicas": {"frontend": 1, "api": 1, "processor": "1..5 (KEDA, 10 messages per replica)"},
                "vcpu_per_replica": 0.25, "users": 500, "concurrency": 16,
                "store_429s_per_task": round(int(st1.get("throttled", 0) - st0.get("throttled", 0)) / tasks, 2) if tasks else None,
                # the 429s per charged store call, and how the throttled ones came through: a
                # ticket at its slot (admitted) or early (a second 429 for the same call)
                **_throttle_detail(st0, st1),
                # tasks/s over the rate the budget pays for (budget / RU per task), over the steady
                # window: the whole window also spends the one second of budget the bucket holds
                # when the load starts (an idle bucket refills to it, as Cosmos's burst capacity
                # does) -- that ratio is kept next to it
                "tasks_per_s_over_budget_rate": (sw or {}).get("ru_over_budget"),
                "tasks_per_s_over_budget_rate_whole_window": (
                    round(tasks / el / (float(st1.get("ru_per_s", 0.0)) / (ru / tasks)), 3)
                    if tasks and ru and el and st1.get("ru_per_s") else None),
                "keda_polling_s": 5, "loadgen_exit": p.returncode}
    except Exception as e:  # reported, not fatal to the headline
        return {"error": repr(e)[:500]}
    finally:
        stop.set()
        env.stop()


def _throttle_detail(st0: dict, st1: dict) -> dict:
    d = {k: int(st1.get(k, 0) - st0.get(k, 0)) for k in ("throttled", "calls", "reserved_admits", "early_retries")}
    if not d["calls"]:
        return {}
    first = d["throttled"] - d["early_retries"]  # calls that met a spent budget
    return {"store_calls": d["calls"], "store_calls_throttled_share": round(first / d["calls"], 3),
            "store_429s_per_call": round(d["throttled"] / d["calls"], 3),
            "throttled_calls_admitted_at_slot": d["reserved_admits"], "early_ticket_retries": d["early_retries"]}


def keda_stage(root: str, rank: int, messages: int, polling_s: float = 5.0, cooldown_s: float = 15.0,
               budget_s: float = 360.0) -> dict:
    """The reference's module-9 load test, measured (docs/aca/09-aca-autoscale-keda/index.md:
    192-216): ``deploy/main.yaml`` with its defaults -- the notifier with SendGrid off simulates
    1 s of work per message (TasksNotifierController.cs:60-62), the processor scales 1..5 on the
    KEDA Service Bus rule at 10 messages per replica (processor-backend-service.bicep:159-183) --
    and ``messages`` tasksaved events published at 1 ms intervals (100 every 100 ms) through the
    API's sidecar.  Sampled every 250 ms: the replica timeline 1 -> 5 -> 1, the time to 5
    replicas, the drain time, and the subscription's counters (each message received and
    completed exactly once).  Only KEDA's polling interval (30 s -> ``polling_s``) and cooldown
    (300 s -> ``cooldown_s``) are shortened."""
    import threading

    from aca_dotnet_workshop_amd.platform.background import BackgroundEnvironment
    from aca_dotnet_workshop_amd.platform.manifest import load_manifest
    from aca_dotnet_workshop_amd.web.client import HttpClient
    m = load_manifest(os.path.join(ROOT, "deploy", "main.yaml"), os.path.join(ROOT, "deploy", "main.parameters.json"),
                      {"kedaPollingIntervalSeconds": polling_s, "kedaCooldownPeriodSeconds": cooldown_s,
                       "environmentName": f"cae-keda-r{rank}"})
    env = BackgroundEnvironment(m, os.path.join(root, "keda"), log_level="warning")
    entity = f"tasksavedtopic/subscriptions/{PROC}"
    samples: list[tuple[float, int, int]] = []  # (s since the first publish, replicas, completed)
    stop = threading.Event()
    try:
        env.start()
        counts = f"{env.backing_url}/servicebus/taskstracker/counts?entity={entity}"
        c0 = _counts(counts)
        uds = env.replicas(API)[0].sidecar_uds
        t0 = time.perf_counter()

        def watch() -> None:
            while not stop.wait(0.25):
                rt = env.ctl.apps.get(PROC)
                n = len([r for r in rt.current.replicas if r.alive()]) if rt and rt.current else 0
                try:
                    done = int(_counts(counts).get("completed", 0)) - int(c0.get("completed", 0))
                except Exception:
                    continue
                samples.append((round(time.perf_counter() - t0, 2), n, done))
        th = threading.Thread(target=watch, daemon=True)
        th.start()

        async def publish() -> None:  # 1 ms apart on average, like Service Bus Explorer's sender
            c = HttpClient()
            url = f"unix:{uds}:/v1.0-alpha1/publish/bulk/dapr-pubsub-servicebus/tasksavedtopic"
            try:
                for lo in range(0, messages, 100):
                    entries = [{"entryId": str(i), "contentType": "application/json",
                                "event": {"taskId": f"00000000-0000-4000-8000-{i:012d}", "taskName": f"Load test {i}",
                                          "taskCreatedBy": "load@bench.local", "taskCreatedOn": "2030-01-01T00:00:00",
                                          "taskDueDate": "2030-01-02T00:00:00", "taskAssignedTo": "a@bench.local",
                                          "isCompleted": False, "isOverDue": False}}
                               for i in range(lo, min(messages, lo + 100))]
                    r = await c.post(url, json_body=entries, timeout=60)
                    if r.status != 204:
                        raise RuntimeError(f"bulk publish: {r.status} {r.body[:200]!r}")
                    left = t0 + (lo + 100) / 1000.0 - time.perf_counter()
                    if left > 0:
                        await asyncio.sleep(left)
            finally:
                await c.close()
        asyncio.run(publish())
        sent_s = time.perf_counter() - t0
        while time.perf_counter() - t0 < budget_s:  # drained, then scaled back in to one replica
            time.sleep(0.5)
            if samples and samples[-1][2] >= messages and samples[-1][1] <= 1 and max(s[1] for s in samples) > 1:
                break
        stop.set()
        th.join(5)
        c1 = _counts(counts)
        delta = {k: int(c1.get(k, 0)) - int(c0.get(k, 0)) for k in ("enqueued", "received", "completed", "dead_letter")}
        timeline, last = [], None
        for t, n, _ in samples:
            if n != last:
                timeline.append([t, n])
                last = n
        peak = max((n for _, n, _ in samples), default=0)
        t_peak = next((t for t, n, _ in samples if n == peak), None)
        t_drain = next((t for t, _, done in samples if done >= messages), None)
        t_in = next((t for t, n, _ in samples if t_drain is not None and t >= t_drain and n <= 1), None)
        ev = (env.ctl.apps[PROC].scale_events if env.ctl else [])
        polls = list(env.ctl.apps[PROC].polls) if env.ctl else []
        for _ in range(120):  # the scale-in's event is recorded once its replicas have stopped
            if not polls or any(e["replicas"] <= 1 and e["ts"] > max(p[0] for p in polls if p[4] > 1)
                                for e in ev if any(p[4] > 1 for p in polls)):
                break
            time.sleep(0.25)
            polls = list(env.ctl.apps[PROC].polls)
        wall0 = time.time() - (time.perf_counter() - t0)  # t0 on the wall clock (the polls' clock)
        busy = [p[0] for p in polls if p[1]]
        high = [p[0] for p in polls if p[4] > 1]  # polls that recommended more than one replica
        ins = [e["ts"] for e in ev if high and e["ts"] > high[-1] and e["replicas"] <= 1]
        return {"messages": messages, "published_in_s": round(sent_s, 2), "peak_replicas": peak,
                "polls": len(polls), "last_active_poll_s": round(busy[-1] - wall0, 2) if busy else None,
                "last_scale_out_recommendation_s": round(high[-1] - wall0, 2) if high else None,
                # HPA scale-down stabilization (KEDA cooldown): back to 1 one window after the last
                # poll that asked for more
                "scale_in_after_last_recommendation_s": round(ins[0] - high[-1], 2) if ins else None,
                "time_to_peak_s": t_peak, "drain_s": t_drain, "scaled_in_to_1_s": t_in,
                "replica_timeline": timeline,  # [seconds since the first publish, replicas], on change
                "scale_events": [e["replicas"] for e in ev],
                "counts": delta,
                "exactly_once": delta["enqueued"] == delta["received"] == delta["completed"] == messages
                                and delta["dead_letter"] == 0,
                "rule": "azure-servicebus, messageCount 10, replicas 1..5 (processor-backend-service.bicep:159-183)",
                "work_per_message_ms": 1000, "keda_polling_s": polling_s, "keda_cooldown_s": cooldown_s,
                "reference": "docs/aca/09-aca-autoscale-keda/index.md:192-216 (30 s polling / 300 s cooldown)"}
    except Exception as e:  # reported, not fatal to the headline
        return {"error": repr(e)[:500], "replica_timeline": samples[-20:]}
    finally:
        stop.set()
        env.stop()


PLATFORM_ROLES = ("backing", "ingress", "bench")


def _rank_pids(env) -> dict[str, list[int]]:
    """The rank's processes by side: ``platform`` (this process, ingress, backing services) and
    ``replica`` (every replica with its sidecar and data plane)."""
    pids: dict[str, list[int]] = {"platform": [os.getpid()] + list(_ingress_pid(env).values()), "replica": []}
    st = env.stack
    if st.backing_proc is not None:
        pids["platform"].append(st.backing_proc.pid)
    pids["platform"] += [p.pid for p, _u in st.extra_backing.values()]
    import psutil
    for rs in st.replicas.values():
        for r in rs:
            pids["replica"].append(r.proc.pid)
            try:
                pids["replica"] += [k.pid for k in psutil.Process(r.proc.pid).children(recursive=True)]
            except psutil.Error:
                pass
    return pids


def _enforce_cpusets(env, split, pinned) -> list[str]:
    """Hold every thread of the rank's processes to its side's CPU set (``enforce_cpuset``),
    after the warmup has started the runtimes' own threads (the GPU runtime's among them)."""
    from aca_dotnet_workshop_amd.parallel import enforce_cpuset
    rank = set(pinned) if pinned else None
    moved: list[str] = []
    for side, ps in _rank_pids(env).items():
        want = (split[0] if side == "platform" else split[1]) if split is not None else rank
        if want:
            for pid in ps:
                moved += enforce_cpuset(pid, want)
    return moved


def _platform_cpu(env, split, pinned, busy: dict[str, float]) -> dict:
    """The platform's share of the rank: cores its processes used in the timed region (backing
    services, ingress, this process with its load generators) against the CPUs reserved for
    them, and every thread of the rank's processes checked against its CPU set (the rank's set;
    the platform / replica subset when split): ``outside_rank_set`` counts threads that may run
    elsewhere, ``outside`` names the first of them."""
    from aca_dotnet_workshop_amd.parallel import cpus_allowed
    used = sum(v for k, v in busy.items() if k.split(".")[0].startswith(PLATFORM_ROLES))
    pids = _rank_pids(env)
    rank = set(pinned) if pinned else None
    outside = wrong_side = threads = 0
    names: list[str] = []
    for side, ps in pids.items():
        want = (split[0] if side == "platform" else split[1]) if split is not None else rank
        for pid in ps:
            for tid, cpus in cpus_allowed(pid).items():
                threads += 1
                if rank is not None and not cpus <= rank:
                    outside += 1
                if want is not None and not cpus <= want:
                    wrong_side += 1
                    if len(names) < 8:
                        try:
                            with open(f"/proc/{pid}/task/{tid}/comm") as f:
                                names.append(f"{side}:{f.read().strip()}/{tid}")
                        except OSError:
                            pass
    return {"reserved_cpus": len(split[0]) if split is not None else None, "cores_used": round(used, 2),
            "within_reserve": bool(split is None or used <= len(split[0]) + 0.05),
            "mechanism": (f"pinned: {len(split[0])} of the rank's {len(pinned)} CPUs for backing, ingress and load "
                          f"generator, the other {len(split[1])} for the replicas") if split is not None
            else "shared with the replicas (rank set too small to split)",
            "threads_checked": threads, "outside_rank_set": outside, "outside_own_subset": wrong_side,
            "outside": names}


def _fs_type(path: str) -> str:
    """The file system ``path`` lives on (/proc/mounts, longest mount point): what a sync costs
    there (tmpfs / overlay over one) is part of a durability number."""
    best, fs = "", "?"
    try:
        real = os.path.realpath(path)
        with open("/proc/mounts") as f:
            for ln in f:
                parts = ln.split()
                if len(parts) >= 3 and (real == parts[1] or real.startswith(parts[1].rstrip("/") + "/")) \
                        and len(parts[1]) > len(best):
                    best, fs = parts[1], parts[2]
    except OSError:
        pass
    return fs


def _drop(d: dict | None, *keys: str) -> dict | None:
    """``d`` without ``keys`` (the record's copy of a block whose bulk goes to stderr)."""
    return None if d is None else {k: v for k, v in d.items() if k not in keys}


def record_summary(value: float, cpu_us: dict, sweep: dict | None, browser: dict | None, envelope: dict | None,
                   protocol: str, wire: dict, alt: dict | None, session: dict | None = None,
                   ingest: dict | None = None, platform: dict | None = None, durable: dict | None = None) -> dict:
    """The record's key facts in one small object at the head of ``config`` (the driver keeps
    the head of ``config``: under ~1 KB, so every block keeps only its deciding numbers): CPU
    per task in total and per role, the sweep's percentiles, the browser flow and session, the
    envelope's budget ratio and KEDA's peak, and the API's wire."""
    s: dict = {"tasks_per_s": round(value, 1), "api_protocol": protocol,
               "api_grpc_calls_per_task": None, "cpu_us_per_task": cpu_us.get("total"),
               # the sidecars' Python control planes (~0 µs per task) are left out here
               "cpu_us_per_task_by_role": {k.replace("tasksmanager-", "").replace("backend-", "")
                                           .replace("frontend-webapp", "frontend"): v
                                           for k, v in (cpu_us.get("by_role") or {}).items()
                                           if not k.endswith(".sidecar")}}
    if wire.get("state.save"):
        s["api_grpc_calls_per_task"] = round((wire.get("grpc.SaveState", 0) + wire.get("grpc.PublishEvent", 0))
                                             / wire["state.save"], 2)
    if sweep:
        s["sweep"] = {k: sweep.get(k) for k in ("sweeps", "sweep_p50_ms", "sweep_max_ms", "errors")}
    if browser:
        s["browser_flows_per_s"] = browser.get("flows_per_s")
    if session:
        s["browser_session"] = {k: session.get(k) for k in ("flows_per_s", "errors", "max_page_p99_over_create_p99")}
    if ingest:
        s["external_ingest"] = {k: ingest.get(k) for k in ("msgs_per_s", "all_processed", "dead", "error") if k in ingest}
    if alt:
        s["api_protocol_alt"] = {k: alt.get(k) for k in ("value", "error")
                                 if k in alt} | {"cpu_us_per_task": (alt.get("cpu_us_per_task") or {}).get("total")}
    if durable:
        s["durable"] = {k: durable.get(k) for k in ("value", "create_latency_p99_ms", "error") if k in durable} | {
            "acks_per_sync": (durable.get("durability") or {}).get("acks_per_sync")}
    if platform:
        s["platform_cpu"] = {k: platform.get(k) for k in ("cores_used", "reserved_cpus", "outside_rank_set")}
    if envelope:
        s["envelope"] = {k: envelope.get(k) for k in ("tasks_per_s", "errors", "tasks_per_s_over_budget_rate",
                                                       "store_429s_per_task")}
        k = envelope.get("keda") or {}
        s["keda"] = {x: k.get(x) for x in ("peak_replicas", "time_to_peak_s", "exactly_once")}
    return s


def main_frontend(a: argparse.Namespace, d: Dist, cores: float, pinned) -> None:
    import shutil
    import tempfile

    import psutil

    from aca_dotnet_workshop_amd.native.build import build_dataplane, build_loadgen, build_native
    from aca_dotnet_workshop_amd.platform.background import BackgroundEnvironment
    from aca_dotnet_workshop_amd.platform.manifest import load_manifest
    n = d.world  # the ranks that actually ran (self_launch starts them for --gpus N)
    from aca_dotnet_workshop_amd.parallel import pin_all_threads, split_platform
    # the rank's CPU set split: the platform's processes on PLATFORM_CPUS of them, the replicas
    # on the rest (each process pinned when it is started: parallel.pin_preexec)
    split = split_platform(set(pinned) if pinned else None, a.platform_cpus) if a.platform_split else None
    if split is not None:
        os.environ["TT_PLATFORM_CPUS"] = ",".join(map(str, sorted(split[0])))
        os.environ["TT_REPLICA_CPUS"] = ",".join(map(str, sorted(split[1])))
    fe, api, proc = frontend_topology(cores)
    fe = a.frontend_replicas or fe
    api = a.api_replicas or api
    proc = a.processor_replicas or proc
    conc = a.concurrency or min(512, 48 * fe)
    # per-replica vCPU caps: the rank's CPUs less 2 (backing + load generator), split over the
    # replicas in proportion to each app's measured CPU per created task (app + its sidecar; the
    # API does the most work per task, the processor the least: profiles/r3_mtls_cost.md); each
    # reference app module sets its own resources, so the manifest takes one cap per app
    ingress = a.ingress != "bypass"
    if a.app_cpu:
        caps = {"frontend": a.app_cpu, "api": a.app_cpu, "processor": a.app_cpu}
    else:
        w = CPU_WEIGHT
        if a.cpu_weights:
            w = dict(zip(("frontend", "api", "processor"), (float(x) for x in a.cpu_weights.split(":"))))
        # the platform's own processes are not replicas: the backing services and the load
        # generator, plus the external ingress when load enters through it -- held to their
        # reserve by their own CPU subset when the rank's set can be split (below)
        reserve = 2.0 + (INGRESS_RESERVE if ingress else 0.0)
        if split is not None:
            reserve = float(len(split[0]))
        unit = (cores - reserve) / (fe * w["frontend"] + api * w["api"] + proc * w["processor"])
        caps = {k: round(max(0.25, unit * w[k]), 2) for k in w}
    app_cpu = caps["frontend"]
    for b in (build_native, build_dataplane, build_loadgen):  # once, before any child needs them
        b()
    exe = str(build_loadgen())
    sweep = a.overdue_sweep_ms > 0
    root = tempfile.mkdtemp(prefix="tt-bench-")
    # the environment's processes inherit these: JSON logs to the telemetry dir only (Log
    # Analytics), the rank's own GPU for the store's query path, the sweep's mirrored columns
    os.environ.update({"TT_LOG_CONSOLE": "0", **rank_device_env()})
    if ingress:  # the external ingress's data plane and its event loops (platform/ingress.py)
        os.environ["TT_INGRESS"] = a.ingress
        os.environ.setdefault("TT_INGRESS_THREADS", str(max(1, min(4, round(cores / 8)))))
    if sweep:
        os.environ["TT_QUERY_MIRROR_PATHS"] = "taskDueDate,isCompleted,isOverDue,taskCreatedOn"
    overrides = {"backendApiMinReplicas": api, "backendApiMaxReplicas": api, "frontendMinReplicas": fe,
                 "frontendMaxReplicas": fe, "processorMinReplicas": proc, "processorMaxReplicas": proc,
                 "notifierMode": "log", "cosmosAutoscaleMaxThroughput": a.ru_per_s, "daprMtls": bool(a.mtls),
                 "enforceCpuLimits": bool(a.cpu_limits), "appCpu": app_cpu, "frontendCpu": caps["frontend"],
                 "backendApiCpu": caps["api"], "processorCpu": caps["processor"], "appMemory": "2Gi",
                 "appInsightsSamplingPercentage": a.trace_sampling,
                 "overdueQuery": "range" if sweep else "equality", "overduePageSize": OVERDUE_PAGE if sweep else 0,
                 "overdueMarkChunk": a.mark_chunk, "backendApiDaprApiProtocol": a.api_protocol,
                 "environmentName": f"cae-bench-r{d.rank}"}
    m = load_manifest(os.path.join(ROOT, "deploy", "main.yaml"), os.path.join(ROOT, "deploy", "main.parameters.json"),
                      overrides)
    shared = a.shared_env and d.world > 1
    # --shared-env: every rank's controller hosts one shard of the state store and the broker;
    # the shard URLs are exchanged once the backings are up (platform/controller.py)
    env = BackgroundEnvironment(m, os.path.join(root, "env"), log_level="warning",
                                shard_exchange=d.allgather if shared else None)
    sweeper = None
    try:
        progress(f"environment up: {fe} frontend / {api} API / {proc} processor replicas")
        env.start()
        if split is not None:  # this process (controller, duty-cycle limiter, load generators to come)
            pin_all_threads(split[0])
        lim = env.ctl.limiter.describe()
        fe_ports = [r.app_port for r in env.replicas(FRONTEND)]
        ca_file = None
        if ingress:  # a browser's entry: the frontend's external ingress, HTTPS verified by the env CA
            ing = env.ctl.apps[FRONTEND].ingress
            ca_file = str(env.ctl.pki.ca_crt)
            targets = [f"https://127.0.0.1:{ing.public_port}"]
            session_url = targets[0]
        else:
            targets = [f"127.0.0.1:{p}" for p in fe_ports]
            session_url = f"http://127.0.0.1:{fe_ports[0]}"
        backing = env.backing_url
        shards = env.ctl.shards or [backing]
        entity = "tasksavedtopic/subscriptions/tasksmanager-backend-processor"
        counts_url = [f"{u}/servicebus/taskstracker/counts?entity={entity}" for u in shards]
        cookie, token = _form_session(session_url, "bench@bench.local", ca_file)
        bodies_file = os.path.join(root, "form-bodies.txt")
        with open(bodies_file, "wb") as f:
            f.write(b"\n".join(_form_bodies(a.batch, token, a.past_due_every if sweep else 0)) + b"\n")
        gbase, stride = None, a.batch * d.world
        if shared:  # the subscription's completed counter before anyone sends (global step targets)
            d.barrier()
            gbase = d.broadcast(_counter(counts_url) if d.rank == 0 else None)
        if sweep and (not shared or d.rank == 0):  # one cron trigger per environment
            # running from the warmup on: the timed region sees the steady state of a periodic
            # job (mirror built, device columns and zone maps resident), not its first run
            sweeper = OverdueSweeper(env.replicas(PROC)[0].sidecar_uds, a.overdue_sweep_ms / 1000.0)
            sweeper.start()
        warm = None
        if a.warmup and a.loadgen_threads <= 1:  # one generator process for warmup and timed steps
            progress(f"warmup: {a.warmup} steps")
            warm = WarmLoadgen(_form_loadgen_cmd(exe, targets, cookie, counts_url, a.warmup + a.steps, a.batch, conc,
                                                 bodies_file, (gbase, stride) if shared else None, ca_file),
                               a.warmup, root)
            warm.warmup()
        elif a.warmup:
            progress(f"warmup: {a.warmup} steps")
            run_form_loadgen(exe, targets, cookie, counts_url, a.warmup, a.batch, conc, bodies_file,
                             (gbase, stride) if shared else None, ca_file, a.loadgen_threads)
        # the warmup started every runtime's threads: hold them all to their side's CPU set
        repinned = _enforce_cpusets(env, split, pinned)
        progress(f"timed region: {a.steps} steps of {a.batch}")
        d.barrier()
        device_sync()
        me = psutil.Process()
        cpu0 = _cpu_by_role(env.stack)
        t = me.cpu_times()
        cpu0["bench"] = t.user + t.system + t.children_user + t.children_system
        cpu0.update(_ingress_cpu(env))
        th0 = env.stack.thread_cpu(_ingress_pid(env))
        duty0 = env.ctl.limiter.duty_stats()
        ru0 = _collection_stats(backing).get("throughput", {})
        conn0 = _client_connects(env)
        acc0 = _accel_stats(shards) if sweeper is not None else {}
        wire0 = _api_wire(env)
        if sweeper is not None:
            sweeper.reset()  # sweeps of the timed region only
        wall0 = time.time()
        if warm is not None:
            dt, report = warm.timed()
        else:
            dt, report = run_form_loadgen(exe, targets, cookie, counts_url, a.steps, a.batch, conc, bodies_file,
                                          (gbase + stride * a.warmup, stride) if shared else None, ca_file,
                                          a.loadgen_threads)
        device_sync()
        d.barrier()
        if sweeper is not None:
            sweeper.stop()
        wire = _wire_delta(wire0, _api_wire(env))
        cpu1 = _cpu_by_role(env.stack)
        t = me.cpu_times()
        cpu1["bench"] = t.user + t.system + t.children_user + t.children_system
        cpu1.update(_ingress_cpu(env))
        th1 = env.stack.thread_cpu(_ingress_pid(env))
        hot = hot_threads(th0, th1, dt, top=6)
        # every thread that did work in the timed region: the stderr diagnostics line only
        threads_all = [t for t in hot_threads(th0, th1, dt, top=200) if t[2] >= 0.005]
        throttling = _throttling(duty0, env.ctl.limiter.duty_stats(), dt)
        platform_cpu = _platform_cpu(env, split, pinned, {k: (cpu1.get(k, 0.0) - v) / dt for k, v in cpu0.items()})
        platform_cpu["outside_rank_set"] = int(d.max(platform_cpu["outside_rank_set"]))
        platform_cpu["repinned_before_timed"] = repinned[:8]
        platform_cpu["repinned_threads"] = len(repinned)
        ru1 = _collection_stats(backing).get("throughput", {})
        conn1 = _client_connects(env)
        connects = {k: {t: v[t] - conn0.get(k, {}).get(t, 0) for t in v} for k, v in conn1.items()}
        dt_max = d.max(dt)
        busy = {k: (cpu1.get(k, 0.0) - v) / dt for k, v in cpu0.items()}  # cores busy per role
        util = {k: round(v, 2) for k, v in busy.items()}
        sweep_info = None
        if sweeper is not None:
            acc1 = _accel_stats(shards)  # the timed region's share of the accelerator counters
            acc = {k: (round(v - acc0.get(k, 0), 3) if isinstance(v, (int, float)) and k != "rows" else v)
                   for k, v in acc1.items()}
            sweep_info = {**sweeper.summary(), "period_ms": a.overdue_sweep_ms, "past_due_every": a.past_due_every,
                          "mark_chunk": a.mark_chunk,
                          "page_size": OVERDUE_PAGE,
                          "gpu_queries": acc.get("gpu"), "cpu_queries": acc.get("cpu"),
                          "native_queries": acc.get("native"), "mirror_rows": acc.get("rows"),
                          "shards": len(shards),
                          "store_ms_total": {k2: acc.get(k2) for k2 in ("lock_wait_ms", "sync_ms",
                                                                         "select_and_results_ms", "select_ms",
                                                                         "results_ms", "bg_sync_ms", "bg_syncs", "page_plan_ms",
                                                                         "page_program_ms", "page_host_cpu_ms",
                                                                         "plan_ranks_ms", "plan_tails_ms",
                                                                         "plan_upload_ms", "plan_tail_rows",
                                                                         "plan_rebuilds",
                                                                         "page_zones_ms",
                                                                         "page_kernels_ms", "page_launches",
                                                                         "page_more_ms")}}
        if shared and sweeper is not None:  # the partitioned sweep marks what one store would
            per_step = -(-a.batch // a.past_due_every) if a.past_due_every else 0
            sweep_info["drain"] = sweeper.drain(per_step * d.world * (a.warmup + a.steps))
        delivery = None
        if shared:  # exactly-once across the competing consumers of every rank, over every shard
            c = _counts(counts_url)
            sent = gbase + stride * (a.warmup + a.steps)
            delivery = {"enqueued": c.get("enqueued"), "completed": c.get("completed"), "received": c.get("received"),
                        "dead_lettered": c.get("dead_letter"), "expected": sent,
                        "exactly_once": c.get("completed") == c.get("received") == c.get("enqueued") == sent}
        # the read path at the headline's replica counts: browsers with their own
        # identity cookie (bounded task lists) post Create and follow its 302 to Tasks/Index,
        # which lists the user's tasks through the API (Index.cshtml.cs:48 -> TasksController.Get)
        browser = None
        bsteps = 0 if shared else a.browser_steps if a.browser_steps >= 0 else max(1, a.steps // 4)
        if bsteps:
            progress(f"browser_flow: {bsteps} steps of create + follow to Tasks/Index")
            af = "; ".join(c for c in cookie.split("; ") if not c.startswith("TasksCreatedByCookie="))
            bb = os.path.join(root, "browser-bodies.txt")
            with open(bb, "wb") as f:
                f.write(b"\n".join(_form_bodies(a.batch, token, 0)) + b"\n")
            bdt, brep = run_form_loadgen(exe, targets, f"TasksCreatedByCookie={{user}}; {af}", counts_url, bsteps,
                                         a.batch, conc, bb, None, ca_file, 1,
                                         ["--users", str(BROWSER_USERS), "--follow"])
            sc = brep.get("status_counts") or {}
            browser = {"flows_per_s": round(a.batch * bsteps / bdt, 1), "pages_per_s": round(2 * a.batch * bsteps / bdt, 1),
                       "steps": bsteps, "users": BROWSER_USERS, "concurrency": conc,
                       "create_latency_ms": brep.get("latency_ms"), "list_latency_ms": brep.get("follow_latency_ms"),
                       "lists": brep.get("follow_requests"), "status_counts": sc, "errors": brep.get("errors"),
                       "first_error": brep.get("first_error") or None,
                       "tasks_per_user_at_end": round(a.batch * bsteps / BROWSER_USERS, 1),
                       "flow": "POST /Tasks/Create (302) + GET /Tasks/Index"}
        # the whole browser session at the headline's replica counts: create, list,
        # Edit GET / POST, Complete, Delete, list -- every UI handler and API route of the reference
        session = None
        sflows = 0 if shared else a.session_flows if a.session_flows >= 0 else a.batch
        if sflows:
            progress(f"browser_session: {sflows} flows of 7 pages")
            session = run_session(exe, targets, cookie, token, sflows, conc, root, ca_file, a.batch)
        # §3.4 external-task ingestion: storage queue -> processor -> API -> blob
        ingest = ingest_hot = None
        if a.ingest_messages > 0 and not shared:
            progress(f"external_ingest: {a.ingest_messages} queue messages")
            ingest = external_ingest(env, a.ingest_messages)
            ingest_hot = ingest.pop("hot_threads", None)
        # the same environment, load straight at the API sidecars' invoke (round 2's topology);
        # not in a shared environment (its counters are global: the two loads would mix)
        direct = None
        dsteps = 0 if shared else a.direct_steps if a.direct_steps >= 0 else max(1, a.steps // 4)
        progress(f"timed region done: {dt:.2f} s")
        if dsteps:
            progress(f"api_sidecar_direct: {dsteps} steps")
            socks = [r.sidecar_uds for r in env.replicas(API)]
            jb = os.path.join(root, "json-bodies.jsonl")
            with open(jb, "wb") as f:
                f.write(b"\n".join(_bodies(a.batch)) + b"\n")
            ddt, drep = run_loadgen(exe, socks, counts_url, dsteps, a.batch, conc, jb)
            ddt = d.max(ddt)
            direct = {"value": round(a.batch * dsteps * (d.world if d.world > 1 else 1) / ddt, 2), "steps": dsteps,
                      "create_latency_p50_ms": drep["latency_ms"]["p50"], "create_latency_p99_ms": drep["latency_ms"]["p99"],
                      "note": "same environment, load at the API sidecars' invoke (no frontend, no mTLS hop)"}
        trace = None
        if sweep_info is not None:  # span exporters flush at least once a second
            if not dsteps:
                time.sleep(1.5)
            trace = sweep_trace(str(env.ctl.dir / "telemetry"), sweeper.sampled_trace_ids + sweeper.trace_ids, None)
            # the record keeps the sweep's largest hops; every span goes to the stderr diagnostics
            spans = (trace or {}).get("spans_p50_ms") or {}
            sweep_info["trace_top_spans_p50_ms"] = dict(sorted(spans.items(), key=lambda kv: -kv[1])[:4])
            sweep_info["trace_of"] = "the warmup's sampled sweeps (the timed region's are unsampled)"
        envelope = alt = None
        asteps = 0 if shared else a.alt_steps if a.alt_steps >= 0 else max(2, a.steps // 2)
        if (a.envelope_s > 0 or asteps) and not shared:  # after the headline's environment is down
            env.stop()
        durable = None
        if asteps:
            progress(f"api_protocol_alt: {asteps} steps with the other Dapr protocol")
            alt = protocol_alt(a, overrides, exe, root, asteps, conc, d.rank)
            progress("api_protocol_alt done")
            progress(f"durable: {asteps} steps with the backing's logs on group commit")
            durable = protocol_alt(a, overrides, exe, root, asteps, conc, d.rank, durable=True)
            progress("durable done")
        if a.envelope_s > 0 and not shared:
            if d.rank == 0:
                progress(f"reference envelope: {a.envelope_s:g} s")
                envelope = reference_envelope(exe, root, a.envelope_s, d.rank)
                progress("reference envelope done")
                if a.keda_messages > 0:
                    progress(f"KEDA scale-out: {a.keda_messages} messages with 1 s of work each")
                    envelope["keda"] = keda_stage(root, d.rank, a.keda_messages)
                    progress("KEDA stage done")
            d.barrier()
        total = a.batch * a.steps * (d.world if d.world > 1 else 1)
        value = total / dt_max if dt_max > 0 else 0.0
        p50, p99 = d.max(report["latency_ms"]["p50"]), d.max(report["latency_ms"]["p99"])
        cpu_us = cpu_per_task(busy, a.batch * a.steps / dt)  # this rank's CPU over this rank's tasks
        ru_used = None
        if ru0 and ru1 and "ru_consumed" in ru1:
            ru_used = round((ru1["ru_consumed"] - ru0.get("ru_consumed", 0.0)) / dt, 1)
        if d.rank == 0:
            print(json.dumps({"cpu_cores_busy": util, "total_cores_busy": round(sum(util.values()), 2),
                              "cpu_us_per_task": cpu_us,
                              "cpu_budget_per_rank": round(cores, 2), "loadgen": report,
                              "overdue_sweeps": sweep_info, "sweep_trace": trace, "resource_limits": lim,
                              "sidecar_client_connects": connects, "timed_wall_start": round(wall0, 6),
                              "external_ingest_hot_threads": ingest_hot,
                              "threads": threads_all}), file=sys.stderr, flush=True)
            summary = record_summary(value, cpu_us, sweep_info, browser, envelope, a.api_protocol, wire, alt, session,
                                     ingest, platform_cpu, durable)
            print(json.dumps({
                "metric": "tasks_e2e_per_sec", "value": round(value, 2), "unit": "tasks/s", "n_gpus": n,
                "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(dt_max / a.steps * 1e3, 3),
                "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "n/a (JSON over HTTP)",
                "data": "synthetic createTask form posts",
                "config": {"summary": summary,
                           "model": "tasks-tracker createTask flow, SURVEY §3.1 (frontend -> mTLS -> API -> store + "
                                    "publish -> processor ack)",
                           "api_protocol": a.api_protocol, "api_wire": wire,
                           "global_batch": a.batch * (d.world if d.world > 1 else 1), "seq_len": None,
                           "parallelism": (f"shared-env x{d.world} (store and broker partitioned over {len(shards)} "
                                           f"shards, one per rank; {proc * d.world} competing processor replicas)"
                                           if shared else f"env-per-rank x{d.world if d.world > 1 else 1}"),
                           "delivery": delivery, "launcher": launcher_label(d),
                           "environment": "deploy/main.yaml via the platform controller",
                           "entry": "frontend", "entry_request": "POST /Tasks/Create (form, antiforgery + identity "
                                                                  "cookies) -> 302, redirect not followed",
                           "ingress": (f"external HTTPS ({a.ingress}), {os.environ.get('TT_INGRESS_THREADS')} event "
                                       "loops, certificate verified against the environment CA"
                                       if ingress else "bypassed: the load generator balances over the frontend replicas"),
                           "hot_threads": hot,
                           # outbound connections the sidecars opened in the timed region (tls: a
                           # mesh handshake each): the pools' misses
                           "sidecar_client_connects": connects,
                           "mtls": bool(a.mtls), "ru_per_s": a.ru_per_s or "unlimited", "ru_consumed_per_s": ru_used,
                           "platform_cpu": platform_cpu,
                           "cpu_limits": {"enforced": bool(a.cpu_limits), "vcpu_per_replica": caps,
                                          "mechanism": lim.get("cpu"), "mode": lim.get("mode"),
                                          "throttling_in_timed_region": throttling},
                           "replicas": {"frontend": fe, "api": api, "processor": proc},
                           "notifier": "TasksNotifier:Mode=log (the shipped controller)",
                           "dapr_api_logging": True, "trace_sampling_percent": a.trace_sampling,
                           "concurrency_per_rank": conc, "load_generator": "native" if a.loadgen_threads <= 1 else f"native, {a.loadgen_threads} event loops",
                           "cpu_pinning": pin_label(pinned),
                           "create_latency_p50_ms": round(p50, 3), "create_latency_p99_ms": round(p99, 3),
                           "baseline": "reference publishes no throughput",
                           "step_quantum": f"{a.batch} createTask per step per rank (fixed task quantum)",
                           "timed_region_s": round(dt_max, 3), "log_level": "Information",
                           "log_sink": "structured JSON lines in the environment telemetry dir",
                           # the record stays small (the driver keeps its head): the sweep's store
                           # timings and span dump are in the stderr diagnostics line
                           "overdue_sweeps": _drop(sweep_info, "store_ms_total", "trace_top_spans_p50_ms", "trace_of"),
                           "browser_flow": browser, "browser_session": session,
                           "external_ingest": ingest,
                           "api_sidecar_direct": direct,
                           "api_protocol_alt": alt, "durable": _drop(durable, "api_wire"),
                           "reference_envelope": envelope}}, separators=(",", ":")), flush=True)
    finally:
        if sweeper is not None and sweeper.thread.is_alive():
            sweeper.stop()
        env.stop()
        d.close()
        if not os.environ.get("TT_BENCH_KEEP"):
            shutil.rmtree(root, ignore_errors=True)


if __name__ == "__main__":
    main()
