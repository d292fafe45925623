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
* ``cgroup_throttling`` -- CFS quota throttling counters for the bench report.
"""
from __future__ import annotations

import os
import sys

__all__ = ["Dist", "cpu_budget", "topology", "cgroup_throttling"]


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

    def close(self) -> None:
        if self.pg is not None:
            self.pg.destroy_process_group()


def cpu_budget() -> float:
    """CPUs this process may use: cgroup v2/v1 quota, else the affinity mask (a GPU box's
    ``nproc`` shows the whole machine while the job gets a share of it)."""
    n = float(len(os.sched_getaffinity(0)))
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, int(quota) / int(period))
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            p = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                n = min(n, q / p)
        except (OSError, ValueError):
            pass
    return n


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
