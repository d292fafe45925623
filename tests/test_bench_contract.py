"""bench.py contract: one JSON line from rank 0 with the fields the driver reads, for a single
process and for a 2-rank torchrun launch over gloo (each rank runs its own environment)."""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
FIELDS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
          "vs_baseline", "dtype", "data", "config"}


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _json_lines(out: str) -> list[dict]:
    return [json.loads(x) for x in out.splitlines() if x.startswith("{") and '"metric"' in x]


def _check(line: dict, n: int, steps: int, warmup: int) -> None:
    assert FIELDS <= set(line)
    assert line["metric"] == "tasks_e2e_per_sec" and line["n_gpus"] == n
    assert line["steps"] == steps and line["warmup"] == warmup
    assert line["value"] > 0 and line["ms_per_step"] > 0 and line["higher_is_better"] is True
    assert line["scaling"] == "weak" and line["vs_baseline"] is None
    assert line["config"]["global_batch"] == 32 * n


def test_bench_single_process():
    env = dict(os.environ, PYTHONPATH=str(ROOT))
    r = subprocess.run([sys.executable, "bench.py", "--steps", "2", "--warmup", "1", "--batch", "32",
                        "--api-replicas", "1", "--processor-replicas", "1", "--envelope-s", "4",
                        "--keda-messages", "300", "--ingest-messages", "64"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1
    _check(lines[0], 1, 2, 1)
    cfg = lines[0]["config"]
    # load enters at the frontend's external HTTPS ingress (native data plane), like a browser's
    assert cfg["entry"] == "frontend" and cfg["ingress"].startswith("external HTTPS (native)")
    # the record's key facts lead config (the driver keeps the line's head), and the line stays small
    assert list(cfg)[0] == "summary" and len(r.stdout.strip().splitlines()[-1]) < 9000
    sm = cfg["summary"]
    # /proc counts CPU in 10 ms ticks: over this run's ~64 timed tasks a cheap role can read 0
    assert sm["cpu_us_per_task"] > 0 and sm["cpu_us_per_task_by_role"]["ingress"] >= 0
    assert set(sm["sweep"]) >= {"sweeps", "sweep_p50_ms", "sweep_max_ms"}
    assert len(json.dumps(sm, separators=(",", ":"))) < 1000, sm  # the driver keeps config's head
    # the reference SDK's wire: every task's save and publish went over the sidecar's gRPC API
    assert cfg["api_protocol"] == sm["api_protocol"] == "grpc"
    w = cfg["api_wire"]
    # (a sweep inside the timed region adds its markoverdue saves, over gRPC too)
    assert w["grpc.PublishEvent"] == w["publish"] == 64 and w["grpc.SaveState"] == w["state.save"] >= 64
    # the whole browser session and the external-task ingestion, at the headline's replica counts
    bs = cfg["browser_session"]
    assert bs["errors"] == 0 and bs["flows"] == 32 and set(bs["latency_ms"]) == {
        "create", "list", "edit_get", "edit_post", "complete", "delete", "list_after"}, bs
    ing = cfg["external_ingest"]
    assert ing["all_processed"] and ing["blobs_written"] == 64 and ing["dead"] == 0, ing
    # the platform's processes on their own CPUs, every thread inside the rank's set
    pc = cfg["platform_cpu"]
    assert pc["outside_rank_set"] == 0 and pc["outside_own_subset"] == 0 and pc["threads_checked"] > 10, pc
    # the same flow with the other protocol, in its own environment: HTTP, no gRPC call
    alt = cfg["api_protocol_alt"]
    assert alt["api_protocol"] == "http" and alt["value"] > 0 and alt["api_wire"]["grpc.SaveState"] == 0
    assert alt["api_wire"]["state.save"] == 32 * alt["steps"]
    # the same flow with the backing's logs on group commit: every acknowledgement after a sync
    dur = cfg["durable"]
    assert dur["value"] > 0 and dur["errors"] == 0 and dur["api_protocol"] == "grpc", dur
    dd = dur["durability"]
    assert dd["fsync_mode"] == 2 and dd["state_store_syncs"] >= 1 and dd["unsynced_bytes_at_end"] == 0, dd
    assert sm["durable"]["value"] == dur["value"]
    sw = cfg["overdue_sweeps"]
    assert len(sw["sweep_ms"]) == sw["sweeps"] and max(sw["sweep_ms"], default=0) == (sw["sweep_max_ms"] or 0)
    assert sw["page_size"] == 4096
    # the busiest threads of the timed region: [role, thread name, cores, kernel share], busiest
    # first
    hot = cfg["hot_threads"]
    assert hot and all(len(h) == 4 and h[2] >= 0 and 0 <= h[3] <= 1 for h in hot)
    assert [h[2] for h in hot] == sorted((h[2] for h in hot), reverse=True)
    # the secondary run inside the reference's envelope: 1/1 replicas, 0.25 vCPU, 4000 RU/s, the
    # create's redirect followed to the task list
    ev = cfg["reference_envelope"]
    assert ev["tasks"] > 0 and ev["ru_per_s_budget"] == 4000.0, ev
    assert ev["lists_followed"] == ev["tasks"] and ev["list_latency_ms"]["p50"] > 0
    assert ev["failed_creates"] + ev["failed_lists"] == ev["errors"]
    assert ev["processor_replicas_reached"] >= 1 and ev["ru_per_task"] > 5
    # the module-9 load test: the backlog scales the processor 1 -> 5 -> 1, each message once
    k = ev["keda"]
    assert k["peak_replicas"] == 5 and k["exactly_once"] and k["counts"]["completed"] == 300, k
    assert k["replica_timeline"][0][1] == 1 and k["replica_timeline"][-1][1] == 1 and k["scaled_in_to_1_s"] > k["drain_s"]


def test_thread_cpu_and_hot_threads():
    """ProcessStack.thread_cpu reads every thread of the given processes; hot_threads ranks the
    deltas by cores busy."""
    import threading
    import time
    sys.path.insert(0, str(ROOT))
    import bench
    from aca_dotnet_workshop_amd.platform.processes import LocalStack
    stack = LocalStack()
    stop = threading.Event()

    def spin():
        while not stop.is_set():
            sum(range(1000))
    t = threading.Thread(target=spin, name="spinner")
    t.start()
    try:
        before = stack.thread_cpu({"self": os.getpid()})
        t0 = time.perf_counter()
        time.sleep(0.5)
        after = stack.thread_cpu({"self": os.getpid()})
        dt = time.perf_counter() - t0
    finally:
        stop.set()
        t.join()
    assert {k[0] for k in after} == {"self"} and len(after) >= 2
    hot = bench.hot_threads(before, after, dt, top=3)
    assert hot[0][0] == "self" and hot[0][2] > 0.3 and hot[0][3] < 0.5  # the spinner: user mode
    assert bench.hot_threads({("a", "x", 1): (1.0, 0.0)}, {("a", "x", 1): (1.5, 0.5), ("b", "y", 2): (0.0, 0.5)},
                             2.0) == [["a", "x", 0.5, 0.5], ["b", "y", 0.25, 1.0]]


def test_bench_api_sidecar_entry_single_process():
    """--entry api-sidecar (round 2's topology, kept as a secondary mode) on one rank."""
    env = dict(os.environ, PYTHONPATH=str(ROOT))
    r = subprocess.run([sys.executable, "bench.py", "--steps", "2", "--warmup", "1", "--batch", "32", "--entry",
                        "api-sidecar", "--api-replicas", "1", "--processor-replicas", "1"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1 and lines[0]["config"]["entry"] == "api-sidecar"
    _check(lines[0], 1, 2, 1)


def test_bench_two_ranks_torchrun():
    env = dict(os.environ, PYTHONPATH=str(ROOT), OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2",
           "--steps", "2", "--warmup", "1", "--batch", "32", "--api-replicas", "1", "--processor-replicas", "1",
           "--envelope-s", "0"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout  # rank 0 only
    # nothing else on stdout (gloo's connection messages go to stderr)
    assert [x for x in r.stdout.splitlines() if x.strip() and not x.startswith("{")] == [], r.stdout
    _check(lines[0], 2, 2, 1)
    # each rank pinned to its own partition of the host (the stack inherits the mask)
    from aca_dotnet_workshop_amd.parallel import cpu_quota, host_topology, one_thread_per_core, partition_cpus
    nodes, core = host_topology()
    part = partition_cpus(set(os.sched_getaffinity(0)), nodes, core, 0, 2)
    want = f"{len(part)} CPUs per rank (NUMA-local whole cores (rank order))" if part else "none"
    q = cpu_quota()
    if part and q is not None and q / 2 <= len(one_thread_per_core(part, core)):  # quota below the cores
        phys = one_thread_per_core(part, core)
        if len(phys) >= 2:
            want = f"{len(phys)} CPUs per rank (NUMA-local whole cores (rank order), one thread per core)"
    assert lines[0]["config"]["cpu_pinning"] == want


def test_bench_gpus_two_without_launcher_self_launches():
    """``bench.py --gpus 2`` run as a plain process (no torchrun): it starts the two ranks itself
    under torch.distributed.run as a child, and the line it relays counts the ranks that ran --
    never one environment's throughput labelled as two."""
    env = dict(os.environ, PYTHONPATH=str(ROOT), OMP_NUM_THREADS="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "2", "--warmup", "1", "--batch", "32",
                        "--api-replicas", "1", "--processor-replicas", "1", "--envelope-s", "0"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    assert [x for x in r.stdout.splitlines() if x.strip() and not x.startswith("{")] == [], r.stdout
    _check(lines[0], 2, 2, 1)
    cfg = lines[0]["config"]
    assert cfg["parallelism"] == "env-per-rank x2"
    assert cfg["launcher"] == "torch.distributed.run, 2 ranks (self-launched by bench.py)"


def test_bench_self_launch_returns_none_for_a_rank_or_one_gpu(monkeypatch):
    sys.path.insert(0, str(ROOT))
    import bench
    monkeypatch.setenv("WORLD_SIZE", "2")
    assert bench.self_launch(2, []) is None  # already a rank
    monkeypatch.delenv("WORLD_SIZE")
    assert bench.self_launch(1, []) is None  # one GPU: runs in this process


def test_bench_shared_env_two_ranks():
    """--shared-env: the state store and the broker are partitioned over both ranks' backings
    (backing/shards.py); the processors of both ranks compete on the ONE subscription (the
    reference's scale axis, processor-backend-service.bicep:159-183), receiving from every shard,
    and every task is delivered and completed once."""
    env = dict(os.environ, PYTHONPATH=str(ROOT), OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2",
           "--steps", "2", "--warmup", "1", "--batch", "32", "--api-replicas", "1", "--processor-replicas", "1",
           "--shared-env", "--overdue-sweep-ms", "0", "--entry", "api-sidecar"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    _check(lines[0], 2, 2, 1)
    cfg = lines[0]["config"]
    assert cfg["parallelism"].startswith("shared-env x2 (store and broker partitioned over 2 shards")
    assert "2 competing processor replicas" in cfg["parallelism"]
    dlv = cfg["delivery"]
    assert dlv["exactly_once"] and dlv["completed"] == dlv["received"] == dlv["expected"] >= 2 * 32 * 3, dlv
    assert dlv["dead_lettered"] == 0


def test_bench_shared_env_frontend_two_ranks():
    """--shared-env at the frontend entry: each rank's platform controller starts its backing,
    the ranks exchange the shard URLs (EnvironmentController.shard_exchange over gloo), and the
    manifest-deployed apps of both ranks run against the partitioned store and broker, with the
    overdue sweep on; every task is delivered and completed exactly once."""
    env = dict(os.environ, PYTHONPATH=str(ROOT), OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2",
           "--steps", "2", "--warmup", "1", "--batch", "32", "--shared-env", "--overdue-sweep-ms", "300"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    _check(lines[0], 2, 2, 1)
    cfg = lines[0]["config"]
    assert cfg["entry"] == "frontend" and cfg["mtls"] is True
    assert cfg["parallelism"].startswith("shared-env x2 (store and broker partitioned over 2 shards")
    dlv = cfg["delivery"]
    assert dlv["exactly_once"] and dlv["completed"] == dlv["expected"] >= 2 * 32 * 3, dlv
    assert cfg["overdue_sweeps"]["shards"] == 2 and cfg["overdue_sweeps"]["errors"] == 0
    drain = cfg["overdue_sweeps"]["drain"]  # batch 32, every 64th past due: 1 per step per rank
    assert drain["expected_past_due"] == 2 * 1 * 3 and drain["exactly_once"], drain


def test_bench_latency_runs():
    """bench_latency.py (SURVEY §7.5's own latency benchmarks): 2-hop CRUD and publish->ack lines."""
    env = dict(os.environ, PYTHONPATH=str(ROOT))
    r = subprocess.run([sys.executable, "bench_latency.py", "--ops", "3", "--events", "3", "--skip-scale"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert [x["metric"] for x in lines] == ["crud_latency_two_sidecar_hops", "publish_to_ack_latency"]
    assert set(lines[0]["ops"]) == {"create", "get", "list", "update", "complete", "delete"}
    assert lines[1]["n"] == 3 and lines[1]["p50_ms"] > 0


def test_parallel_helpers():
    from aca_dotnet_workshop_amd.parallel import Dist, cpu_budget, topology
    assert topology(2) == (1, 1) and topology(16) == (6, 3)
    sizes = [topology(c) for c in (4, 8, 16, 32, 64)]
    assert sizes == sorted(sizes) and sizes[-1] == (8, 5)  # grows with the share, capped like the reference (1..5)
    assert cpu_budget() >= 1
    d = Dist()  # single process: identities
    assert (d.world, d.rank, d.max(3.0), d.sum(2.0)) == (1, 0, 3.0, 2.0)


def test_partition_cpus_numa_and_smt():
    from aca_dotnet_workshop_amd.parallel import host_topology, partition_cpus
    from aca_dotnet_workshop_amd.parallel import _cpulist
    assert _cpulist("0-3,8,10-11\n") == {0, 1, 2, 3, 8, 10, 11}
    # 2 sockets x 64 cores x 2 threads, Linux numbering: socket0 = 0-63 + 128-191
    nodes = [set(range(0, 64)) | set(range(128, 192)), set(range(64, 128)) | set(range(192, 256))]
    core = {c: c % 128 for c in range(256)}
    allowed = set(range(256))
    parts = [partition_cpus(allowed, nodes, core, r, 8) for r in range(8)]
    assert all(len(p) == 32 for p in parts)
    assert set().union(*parts) == allowed and sum(map(len, parts)) == 256  # disjoint cover
    for r, p in enumerate(parts):
        assert p <= nodes[r * 2 // 8]                     # ranks 0-3 on socket 0, 4-7 on socket 1
        assert {c ^ 128 for c in p} == p                  # SMT siblings stay with their core
    # fewer ranks than nodes: whole nodes; a quota-restricted affinity mask is respected
    assert partition_cpus(allowed, nodes, core, 1, 2) == nodes[1]
    sub = set(range(0, 16))
    assert partition_cpus(sub, nodes, core, 1, 2) == set(range(8, 16))
    assert partition_cpus({0, 1}, nodes, core, 1, 4) is None  # too small to pin
    assert partition_cpus(allowed, nodes, core, 0, 1) is None
    ns, cr = host_topology()  # real sysfs of this host: readable, every allowed CPU mapped
    assert set(cr) == set(os.sched_getaffinity(0))


def test_one_thread_per_core():
    from aca_dotnet_workshop_amd.parallel import one_thread_per_core
    core = {c: c % 128 for c in range(256)}  # Linux numbering: cpu c and c + 128 share a core
    assert one_thread_per_core(set(range(0, 64)) | set(range(128, 192)), core) == set(range(64))
    assert one_thread_per_core({130, 131, 3}, core) == {130, 3}  # core 2 via its second thread


def test_rank_device_env():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    assert b.rank_device_env({"WORLD_SIZE": "8", "LOCAL_RANK": "3"}) == {"HIP_VISIBLE_DEVICES": "3"}
    assert b.rank_device_env({"WORLD_SIZE": "1", "LOCAL_RANK": "0"}) == {}
    assert b.rank_device_env({"WORLD_SIZE": "2", "LOCAL_RANK": "1", "HIP_VISIBLE_DEVICES": "5"}) == {}


def test_sweep_trace_summarises_the_sweeps_spans(tmp_path):
    """bench.sweep_trace: the sweeps are sampled traces; their spans (any process, any file)
    become per-hop medians in the order of the first sweep, plus the store's numeric hop stamps;
    spans of other traces are ignored."""
    sys.path.insert(0, str(ROOT))
    from bench import sweep_trace

    def span(tid, role, kind, name, ts, ms, attrs=None):
        return json.dumps({"type": "span", "role": role, "kind": kind, "name": name, "traceId": tid, "spanId": os.urandom(8).hex(),
                           "parentId": None, "ts": ts, "durationMs": ms, **({"attributes": attrs} if attrs else {})})
    a, b, other = "a" * 32, "b" * 32, "c" * 32
    (tmp_path / "spans-proc-1-x.jsonl").write_text("\n".join([
        span(a, "proc", "server", "POST /job", 1.0, 20.0), span(b, "proc", "server", "POST /job", 2.0, 30.0),
        span(other, "proc", "server", "POST /job", 3.0, 999.0)]) + "\n")
    (tmp_path / "spans-backing-2-x.jsonl").write_text("\n".join([
        span(a, "backing", "server", "POST query", 1.1, 4.0, {"since_front_forwarded_ms": 0.5, "bytes": 10}),
        span(b, "backing", "server", "POST query", 2.1, 6.0, {"since_front_forwarded_ms": 0.7})]) + "\n")
    got = sweep_trace(str(tmp_path), [a, b])
    assert got["sweeps_traced"] == 2
    assert list(got["spans_p50_ms"]) == ["proc server POST /job", "backing server POST query"]
    assert got["spans_p50_ms"]["proc server POST /job"] == 30.0  # upper median of 2
    assert got["stamps_p50_ms"] == {"backing server POST query since_front_forwarded_ms": 0.7}
    assert sweep_trace(str(tmp_path), []) is None
