"""Scale-out coordination -- the parallelism the reference actually has.

The reference has no data/tensor/pipeline parallelism; its scaling axis is horizontal replica
scale-out: KEDA adds processor replicas that compete for one Service Bus subscription
(bicep/modules/container-apps/processor-backend-service.bicep:159-183).  In this framework that
lives in the platform (``platform/scaler.py``, ``platform/controller.py``); this module holds
the multi-rank side used by ``bench.py`` when the driver launches one process per GPU:

* ``Dist`` -- rank coordination over ``torch.distributed`` with the gloo backend (barriers and
  max/sum reductions of scalars; the workload moves JSON over HTTP, no tensors, so RCCL has
  nothing to carry -- SURVEY.md §5 "Distributed communication backend");
* ``cpu_budget`` / ``topology`` -- each rank runs its own environment (weak scaling, like adding
  Container Apps environments) sized to its share of the host's CPUs;
* ``pin_rank`` / ``partition_cpus`` -- NUMA- and core-aware CPU partitions, one per rank on a
  host, so N environments do not migrate across each other's cores and sockets;
* ``cgroup_throttling`` -- CFS quota throttling counters for the bench report.
"""
from __future__ import annotations

import os
import sys

__all__ = ["Dist", "cpu_budget", "cpu_quota", "one_thread_per_core", "topology", "cgroup_throttling",
           "partition_cpus", "pin_rank", "gpu_numa_nodes", "PIN_INFO", "split_platform", "affinity_from_env",
           "pin_preexec", "pin_all_threads", "cpus_allowed"]


class Dist:
    """Rank coordination over torch.distributed (gloo: this workload has no tensors)."""

    def __init__(self) -> None:
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.pg = None
        if self.world > 1:
            import torch.distributed as dist
            # gloo announces its peer connections on fd 1; rank 0's stdout carries exactly one
            # JSON result line (the bench contract), so route that chatter to stderr
            sys.stdout.flush()
            saved = os.dup(1)
            os.dup2(2, 1)
            try:
                dist.init_process_group("gloo", init_method="env://")
            finally:
                os.dup2(saved, 1)
                os.close(saved)
            self.pg = dist

    def barrier(self) -> None:
        if self.pg is not None:
            self.pg.barrier()

    def max(self, v: float) -> float:
        if self.pg is None:
            return v
        import torch
        t = torch.tensor([v], dtype=torch.float64)
        self.pg.all_reduce(t, op=self.pg.ReduceOp.MAX)
        return float(t.item())

    def sum(self, v: float) -> float:
        if self.pg is None:
            return v
        import torch
        t = torch.tensor([v], dtype=torch.float64)
        self.pg.all_reduce(t, op=self.pg.ReduceOp.SUM)
        return float(t.item())

    def broadcast(self, obj, src: int = 0):
        """``obj`` of rank ``src`` on every rank (a picklable object over gloo)."""
        if self.pg is None:
            return obj
        box = [obj]
        self.pg.broadcast_object_list(box, src=src)
        return box[0]

    def allgather(self, obj) -> list:
        """Every rank's ``obj``, in rank order (picklable objects over gloo)."""
        if self.pg is None:
            return [obj]
        out = [None] * self.world
        self.pg.all_gather_object(out, obj)
        return out

    def close(self) -> None:
        if self.pg is not None:
            self.pg.destroy_process_group()


def _cpulist(text: str) -> set[int]:
    """Kernel cpulist syntax (``0-3,8,10-11``) -> CPU ids."""
    out: set[int] = set()
    for part in text.strip().split(","):
        if part:
            lo, _, hi = part.partition("-")
            out.update(range(int(lo), int(hi or lo) + 1))
    return out


def host_topology() -> tuple[list[set[int]], dict[int, int]]:
    """(NUMA nodes as CPU sets, CPU -> first SMT sibling) from sysfs; one node and no SMT
    grouping when sysfs does not say."""
    nodes, core = [], {}
    base = "/sys/devices/system/node"
    try:
        for d in sorted(os.listdir(base)):
            if d.startswith("node") and d[4:].isdigit():
                nodes.append(_cpulist(open(f"{base}/{d}/cpulist").read()))
    except OSError:
        pass
    for c in os.sched_getaffinity(0):
        try:
            core[c] = min(_cpulist(open(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list").read()))
        except (OSError, ValueError):
            core[c] = c
    return [n for n in nodes if n], core


def partition_cpus(allowed: set[int], nodes: list[set[int]], core: dict[int, int],
                   local_rank: int, local_world: int, min_cpus: int = 2) -> set[int] | None:
    """The CPUs of one rank when ``local_world`` ranks share a host: ranks are spread over the
    NUMA nodes (each rank's processes -- API/processor replicas, sidecars, backing, load
    generator -- talk over loopback/UDS, so keeping them on one socket keeps that traffic in
    one L3/memory domain), and each node's CPUs are cut into contiguous runs of whole cores
    (SMT siblings stay together, so two ranks never share a physical core).  ``None`` when a
    rank would get fewer than ``min_cpus`` CPUs (no pinning then)."""
    if local_world <= 1:
        return None
    nodes = [n & allowed for n in nodes if n & allowed] or [set(allowed)]
    if local_world < len(nodes):  # fewer ranks than nodes: each rank takes whole nodes
        lo, hi = local_rank * len(nodes) // local_world, (local_rank + 1) * len(nodes) // local_world
        cpus = set().union(*nodes[lo:hi])
        return cpus if len(cpus) >= min_cpus else None
    node = local_rank * len(nodes) // local_world
    peers = [r for r in range(local_world) if r * len(nodes) // local_world == node]
    k, i = len(peers), peers.index(local_rank)
    order = sorted(nodes[node], key=lambda c: (core.get(c, c), c))
    cpus = set(order[i * len(order) // k:(i + 1) * len(order) // k])
    return cpus if len(cpus) >= min_cpus else None


PIN_INFO: dict[str, str] = {}  # how the last pin_rank chose its CPUs (for the bench report)


def one_thread_per_core(cpus: set[int], core: dict[int, int]) -> set[int]:
    """The first hardware thread of every physical core in ``cpus`` (``core``: CPU -> its
    core's first sibling, ``host_topology``); a core whose first sibling is outside ``cpus``
    keeps its lowest CPU in the set."""
    by_core: dict[int, int] = {}
    for c in sorted(cpus):
        by_core.setdefault(core.get(c, c), c)
    return set(by_core.values())


def gpu_numa_nodes(sysfs: str = "/sys/class/drm") -> list[int]:
    """NUMA node of every AMD GPU, in PCI address order -- the order HIP numbers the devices (a
    rank with ``HIP_VISIBLE_DEVICES=<local rank>`` drives the ``<local rank>``-th).  -1 where
    sysfs has no node.  Read from sysfs only: no HIP context is opened."""
    out: dict[str, int] = {}
    try:
        names = os.listdir(sysfs)
    except OSError:
        return []
    for d in names:
        if not (d.startswith("card") and d[4:].isdigit()):
            continue
        dev = os.path.join(sysfs, d, "device")
        try:
            if open(os.path.join(dev, "vendor")).read().strip() != "0x1002":
                continue
            bdf = os.path.basename(os.path.realpath(dev))
            node = int(open(os.path.join(dev, "numa_node")).read().strip())
        except (OSError, ValueError):
            continue
        out[bdf] = node
    return [out[k] for k in sorted(out)]


def rank_gpu_node(local_rank: int, nodes: list[set[int]], gpu_nodes: list[int] | None = None) -> int | None:
    """Index into ``nodes`` of the NUMA node the rank's GPU hangs off, when known."""
    gpu_nodes = gpu_numa_nodes() if gpu_nodes is None else gpu_nodes
    visible = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("ROCR_VISIBLE_DEVICES")
    idx = local_rank
    if visible:
        ids = [x for x in visible.split(",") if x.strip().isdigit()]
        if ids:
            idx = int(ids[0]) if len(ids) == 1 else int(ids[local_rank % len(ids)])
    if not gpu_nodes or idx >= len(gpu_nodes) or gpu_nodes[idx] < 0 or gpu_nodes[idx] >= len(nodes):
        return None
    return gpu_nodes[idx]


def pin_rank(local_rank: int, local_world: int, spec: str | None = None,
             gpu_nodes: list[int] | None = None) -> set[int] | None:
    """Pin this process (and every child it starts later) to its rank's CPU partition.
    ``spec`` (default ``$TT_BENCH_PIN``): ``0`` never pins; otherwise the rank's CPUs come from
    the NUMA node of its own GPU when sysfs names one (``gpu_numa_nodes``), shared with the
    other ranks whose GPUs sit on that node (whole cores each); without that, ranks split the
    nodes (``partition_cpus``) and a single rank takes its first node.  ``<n>`` > 1 (single
    rank): only n CPUs of that node; ``phys``: the same set, one hardware thread per physical
    core -- the default (``1``/``auto``) when the CPU quota's share of this rank is no more
    than the set's physical cores.  On the MI355X box one stack on one socket ran +24 % vs
    unpinned (profiles/r2_rank_pinning.md), one thread per core of that socket another +6 %
    (16-CPU quota, 64 cores: profiles/r3_cpu_envelope.md)."""
    spec = os.environ.get("TT_BENCH_PIN", "1") if spec is None else spec
    PIN_INFO.clear()
    if spec == "0":
        return None
    nodes, core = host_topology()
    allowed = set(os.sched_getaffinity(0))
    gnodes = gpu_numa_nodes() if gpu_nodes is None else gpu_nodes
    mine = rank_gpu_node(local_rank, nodes, gnodes)
    cpus = None
    if mine is not None and nodes[mine] & allowed:
        # the ranks whose GPUs share my node split its CPUs, whole cores each
        peers = [r for r in range(max(1, local_world)) if rank_gpu_node(r, nodes, gnodes) == mine]
        if local_rank not in peers:
            peers = [local_rank]
        order = sorted(nodes[mine] & allowed, key=lambda c: (core.get(c, c), c))
        k, i = len(peers), peers.index(local_rank)
        cpus = set(order[i * len(order) // k:(i + 1) * len(order) // k])
        if local_world <= 1 and spec.isdigit() and int(spec) > 1:
            cpus = set(order[:int(spec)])
        PIN_INFO["mode"] = f"GPU-local NUMA node {mine}, whole cores"
        if len(cpus) < 2:
            cpus = None
    if cpus is None and local_world > 1:
        cpus = partition_cpus(allowed, nodes, core, local_rank, local_world)
        PIN_INFO["mode"] = "NUMA-local whole cores (rank order)"
    elif cpus is None and (spec in ("1", "auto", "node", "phys") or spec.isdigit() and int(spec) > 1):
        first = next((n & allowed for n in nodes if n & allowed), allowed)
        order = sorted(first, key=lambda c: (core.get(c, c), c))
        cpus = set(order if spec in ("1", "auto", "node", "phys") else order[:int(spec)])
        PIN_INFO["mode"] = "first NUMA node, whole cores"
    if cpus and spec in ("1", "auto"):
        # default: one thread per core when the job's CPU quota (this rank's share) does not
        # even cover the set's physical cores -- siblings would only split the quota's time
        q = cpu_quota()
        if q is not None and q / max(1, local_world) <= len(one_thread_per_core(cpus, core)):
            spec = "phys"
    if cpus and spec == "phys":
        # one hardware thread per physical core: under a CPU quota smaller than the set, busy
        # threads never share a core with a sibling (SMT halves each one's speed while both
        # still draw on the quota)
        primary = one_thread_per_core(cpus, core)
        if len(primary) >= 2:
            cpus = primary
            PIN_INFO["mode"] = PIN_INFO.get("mode", "first NUMA node") + ", one thread per core"
    if cpus:
        os.sched_setaffinity(0, cpus)
    return cpus


def split_platform(cpus: set[int] | None, n: int) -> tuple[set[int], set[int]] | None:
    """Reserve ``n`` CPUs of a rank's set for the platform's own processes (backing services,
    ingress, load generator, the controller) and give the replicas the rest, so neither side can
    run on the other's CPUs: a rank's platform is held to its reserve the way its replicas are
    held to their caps (the ACA environment's infrastructure is not billed to the apps either).
    None when the set is too small to split (fewer than ``n`` + 2 CPUs)."""
    if not cpus or n <= 0 or len(cpus) < n + 2:
        return None
    order = sorted(cpus)
    return set(order[-n:]), set(order[:-n])


def affinity_from_env(role: str) -> set[int] | None:
    """``TT_PLATFORM_CPUS`` / ``TT_REPLICA_CPUS`` (comma-separated CPU ids) for ``role``
    (``platform`` | ``replica``): the CPUs a process the platform starts is pinned to."""
    raw = os.environ.get("TT_PLATFORM_CPUS" if role == "platform" else "TT_REPLICA_CPUS", "")
    try:
        cpus = {int(x) for x in raw.split(",") if x.strip()}
    except ValueError:
        return None
    return cpus or None


def pin_preexec(role: str):
    """A ``preexec_fn`` pinning the child (and every thread it will start) to ``role``'s CPUs,
    or None when no such split is configured."""
    cpus = affinity_from_env(role)
    if not cpus:
        return None

    def pin() -> None:
        try:
            os.sched_setaffinity(0, cpus)
        except OSError:
            pass
    return pin


def pin_all_threads(cpus: set[int]) -> None:
    """Pin every thread of this process (those already running too) to ``cpus``."""
    for t in os.listdir("/proc/self/task"):
        try:
            os.sched_setaffinity(int(t), cpus)
        except OSError:
            pass


class hold_affinity:
    """``with hold_affinity(): <GPU runtime init>`` -- the runtime may widen the calling
    thread's CPU set (and so every thread started from it later); on exit every thread of this
    process is put back on the set it had on entry."""

    def __enter__(self):
        try:
            self.cpus = set(os.sched_getaffinity(0))
        except OSError:
            self.cpus = None
        return self

    def __exit__(self, *exc) -> None:
        if self.cpus and any(c != self.cpus for c in cpus_allowed(os.getpid()).values()):
            pin_all_threads(self.cpus)


def enforce_cpuset(pid: int, cpus: set[int]) -> list[str]:
    """Re-pin every thread of ``pid`` allowed outside ``cpus`` back into them, the way a cgroup
    cpuset holds all of a container's threads (an affinity inherited at fork does not hold a
    runtime that sets its own threads' affinity). Returns ``comm/tid`` of each thread moved."""
    moved = []
    for tid, allowed in cpus_allowed(pid).items():
        if allowed <= cpus:
            continue
        try:
            os.sched_setaffinity(tid, cpus)
        except OSError:
            continue
        try:
            with open(f"/proc/{pid}/task/{tid}/comm") as f:
                name = f.read().strip()
        except OSError:
            name = "?"
        moved.append(f"{name}/{tid}")
    return moved


def cpus_allowed(pid: int) -> dict[int, set[int]]:
    """tid -> the CPUs each thread of ``pid`` may run on (``Cpus_allowed_list``)."""
    out: dict[int, set[int]] = {}
    try:
        tids = os.listdir(f"/proc/{pid}/task")
    except OSError:
        return out
    for t in tids:
        try:
            with open(f"/proc/{pid}/task/{t}/status") as f:
                for ln in f:
                    if ln.startswith("Cpus_allowed_list:"):
                        cpus: set[int] = set()
                        for part in ln.split(":", 1)[1].strip().split(","):
                            if "-" in part:
                                a, b = part.split("-")
                                cpus.update(range(int(a), int(b) + 1))
                            elif part:
                                cpus.add(int(part))
                        out[int(t)] = cpus
                        break
        except (OSError, ValueError):
            continue
    return out


def cpu_quota() -> float | None:
    """The cgroup (v2, else v1) CPU quota in CPUs, None when unlimited or unreadable."""
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if quota == "max" else int(quota) / int(period)
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            p = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            return q / p if q > 0 else None
        except (OSError, ValueError):
            return None


def cpu_budget() -> float:
    """CPUs this process may use: cgroup v2/v1 quota, else the affinity mask (a GPU box's
    ``nproc`` shows the whole machine while the job gets a share of it)."""
    n = float(len(os.sched_getaffinity(0)))
    q = cpu_quota()
    return min(n, q) if q is not None else n


def topology(cores: float) -> tuple[int, int]:
    """Replica counts for one rank's environment.  Per-task CPU measured on the stack
    (docs/PERFORMANCE.md): the Python API app is the costliest hop, then the processor app;
    sidecar data planes and the backing front are native and cheap."""
    api = max(1, min(8, int(cores / 2.6)))
    proc = max(1, min(5, int(cores // 5)))
    return max(api, 2 if cores >= 6 else 1), max(proc, 2 if cores >= 6 else 1)


def cgroup_throttling() -> dict[str, int]:
    """cgroup v2 ``cpu.stat`` throttling counters (the job's CPU quota being hit stalls every
    thread of the job until the next CFS period)."""
    out = {}
    try:
        for line in open("/sys/fs/cgroup/cpu.stat"):
            k, v = line.split()
            if k in ("nr_periods", "nr_throttled", "throttled_usec"):
                out[k] = int(v)
    except (OSError, ValueError):
        pass
    return out
