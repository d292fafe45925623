"""Per-replica resource limits: the Consumption workload profile's ``cpu`` / ``memory``
(0.25 vCPU / 0.5 Gi for every app: reference bicep/modules/container-apps/
processor-backend-service.bicep:143-146, webapi-backend-service.bicep:124-127,
webapp-frontend-service.bicep:84-87).

A replica is the process group of its sidecar (sidecar + native data plane + app).  Two
enforcement mechanisms, chosen at start-up and reported in the environment status:

* ``cgroup2`` -- a delegated cgroup v2 subtree is writable: one cgroup per replica with
  ``cpu.max`` (quota per 100 ms period) and ``memory.max``; the kernel throttles and
  OOM-kills, the controller sees the dead replica and restarts it (``ReplicaOOMKilled``
  when ``memory.events`` counted an OOM kill).
* ``cgroup1-cpu`` -- no delegated v2 subtree, but a writable cgroup v1 ``cpu`` hierarchy (a
  root container on a v1 host): one cgroup per replica with ``cpu.cfs_quota_us`` -- the same
  kernel CFS bandwidth control as ``cpu.max`` -- and memory by the watchdog below.
* ``watchdog`` -- no writable cgroup at all (unprivileged containers): memory is
  enforced by the controller, which sums the RSS of the replica's processes every
  supervision tick and kills + restarts a replica above its limit (``ReplicaOOMKilled``),
  like ACA restarting an OOM-killed container; CPU is enforced, when enabled, by a duty-cycle
  throttle: SIGSTOP the group once it has used its quota of the current period, SIGCONT at the
  next -- otherwise only accounted.  The period is 20 ms (``TT_CPU_PERIOD_MS``), five times
  finer than CFS's 100 ms, so a throttled replica stalls for at most a few ms instead of tens;
  its CPU time is read per thread from ``/proc/<pid>/task/<tid>/schedstat`` (nanoseconds)
  because ``/proc/<pid>/stat`` counts 10 ms clock ticks -- as coarse as the period itself.
  The duty cycle runs on a native thread (``native/src/dutycycle.hpp``: eight checks per period
  on an absolute clock, so a stopped replica resumes at the period boundary however busy the
  controller's Python threads are); ``TT_CPU_DUTY=python`` keeps the controller's own tick.

``environment.resourceLimits`` in the manifest: ``{memory: true|false, cpu: true|false}``
(both enforced in ``deploy/main.yaml``; the controller's own default without the key is memory
enforced, CPU accounted).  ``describe()`` reports which mechanism is in force.
"""
from __future__ import annotations

import os
import signal
import time
from dataclasses import dataclass, field
from pathlib import Path

import psutil

CGROUP_ROOT = Path("/sys/fs/cgroup")
PERIOD_S = max(0.005, float(os.environ.get("TT_CPU_PERIOD_MS", "20")) / 1000.0)
TREE_REFRESH_S = 0.5  # how often a replica's process / thread list is re-read


def parse_memory(v: str | int | float) -> int:
    """``0.5Gi`` / ``512Mi`` / ``1G`` / bytes -> bytes."""
    s = str(v).strip()
    units = {"Ki": 1 << 10, "Mi": 1 << 20, "Gi": 1 << 30, "Ti": 1 << 40, "K": 10 ** 3, "M": 10 ** 6, "G": 10 ** 9,
             "T": 10 ** 12}
    for u in sorted(units, key=len, reverse=True):
        if s.endswith(u):
            return int(float(s[:-len(u)]) * units[u])
    return int(float(s))


@dataclass
class Limits:
    cpu: float           # cores
    memory: int          # bytes

    @classmethod
    def from_spec(cls, spec: dict) -> "Limits":
        r = spec.get("resources") or {}
        return cls(float(r.get("cpu", 0.25)), parse_memory(r.get("memory", "0.5Gi")))


def tree(pid: int) -> list[psutil.Process]:
    try:
        p = psutil.Process(pid)
        return [p] + p.children(recursive=True)
    except psutil.Error:
        return []


def rss(procs: list[psutil.Process]) -> int:
    total = 0
    for p in procs:
        try:
            total += p.memory_info().rss
        except psutil.Error:
            pass
    return total


def cpu_seconds(procs: list[psutil.Process]) -> float:
    total = 0.0
    for p in procs:
        try:
            t = p.cpu_times()
            total += t.user + t.system
        except psutil.Error:
            pass
    return total


def cgroup1_cpu() -> Path | None:
    """This process's writable cgroup v1 ``cpu`` directory (CFS bandwidth control), if any."""
    try:
        rel = next((ln.split(":", 2)[2].strip() for ln in Path("/proc/self/cgroup").read_text().splitlines()
                    if ln.split(":", 2)[1] in ("cpu", "cpu,cpuacct", "cpuacct,cpu")), None)
        for mount in ("cpu", "cpu,cpuacct"):
            base = CGROUP_ROOT / mount
            if rel is not None and (base / "cpu.cfs_quota_us").exists():
                d = base / rel.lstrip("/")
                if (d / "cpu.cfs_quota_us").exists() and os.access(d, os.W_OK):
                    return d
    except (OSError, IndexError):
        pass
    return None


def delegated_cgroup() -> Path | None:
    """This process's cgroup v2 directory when we may create children with cpu+memory."""
    try:
        if not (CGROUP_ROOT / "cgroup.controllers").exists():
            return None
        rel = next((ln.split("::", 1)[1].strip() for ln in Path("/proc/self/cgroup").read_text().splitlines()
                    if ln.startswith("0::")), None)
        if rel is None:
            return None
        base = CGROUP_ROOT / rel.lstrip("/")
        ctrls = (base / "cgroup.controllers").read_text().split()
        if "cpu" not in ctrls or "memory" not in ctrls or not os.access(base, os.W_OK):
            return None
        return base
    except OSError:
        return None


@dataclass
class ReplicaState:
    name: str
    pid: int
    limits: Limits
    cgroup: Path | None = None
    period_start: float = field(default_factory=time.monotonic)
    period_cpu: float = 0.0
    stopped: bool = False
    throttled_periods: int = 0
    peak_rss: int = 0
    cpu_cgroup: Path | None = None   # cgroup v1 cpu directory (mode cgroup1-cpu)
    clock: "ThreadClock | None" = None


class ThreadClock:
    """CPU seconds a replica has used, at nanosecond resolution: the per-thread CPU time of
    every thread of the replica's processes (``/proc/<pid>/task/<tid>/schedstat``, read in one
    native call), summed as deltas so a thread that exits keeps what it used.  Threads found
    after the first read count from zero (they started inside the window)."""

    def __init__(self, pid: int, reader) -> None:
        self.pid = pid
        self.reader = reader
        self.fds: dict[tuple[int, int], int] = {}
        self.last: dict[tuple[int, int], int] = {}
        self.total_ns = 0
        self.refreshed = 0.0
        self._first = True

    def refresh(self, now: float) -> None:
        seen = set()
        for p in tree(self.pid):
            try:
                tids = os.listdir(f"/proc/{p.pid}/task")
            except OSError:
                continue
            for t in tids:
                key = (p.pid, int(t))
                seen.add(key)
                if key in self.fds:
                    continue
                try:
                    self.fds[key] = os.open(f"/proc/{p.pid}/task/{t}/schedstat", os.O_RDONLY)
                except OSError:
                    continue
                if not self._first:
                    self.last[key] = 0
        for key in [k for k in self.fds if k not in seen]:
            self._drop(key)
        self._first = False
        self.refreshed = now

    def _drop(self, key) -> None:
        try:
            os.close(self.fds.pop(key))
        except OSError:
            pass
        self.last.pop(key, None)

    def seconds(self, now: float) -> float:
        if now - self.refreshed >= TREE_REFRESH_S:
            self.refresh(now)
        keys = list(self.fds)
        vals = self.reader([self.fds[k] for k in keys])
        for k, v in zip(keys, vals):
            if v < 0:
                self._drop(k)
                continue
            prev = self.last.get(k)
            if prev is not None and v > prev:
                self.total_ns += v - prev
            self.last[k] = v
        return self.total_ns / 1e9

    def close(self) -> None:
        for key in list(self.fds):
            self._drop(key)


def _schedstat_reader():
    """The native per-thread CPU reader, if this kernel exposes schedstat (else None)."""
    try:
        if not os.path.exists(f"/proc/self/task/{os.getpid()}/schedstat"):
            return None
        from .. import native
        return native.load().schedstat_ns
    except Exception:
        return None


class ResourceLimiter:
    def __init__(self, env_name: str, enforce_memory: bool = True, enforce_cpu: bool = False,
                 cgroup_base: Path | None = None, allow_cgroup: bool = True) -> None:
        self.enforce_memory = enforce_memory
        self.enforce_cpu = enforce_cpu
        base = cgroup_base if cgroup_base is not None else (delegated_cgroup() if allow_cgroup else None)
        self.mode = "cgroup2" if base is not None else "watchdog"
        self.root: Path | None = None
        self.cpu_root: Path | None = None  # cgroup v1 cpu hierarchy (mode cgroup1-cpu)
        if base is not None:
            self.root = base / f"tt-{env_name}"
            try:
                self.root.mkdir(exist_ok=True)
                (self.root / "cgroup.subtree_control").write_text("+cpu +memory")
            except OSError:
                self.mode, self.root = "watchdog", None
        if self.mode == "watchdog" and enforce_cpu and allow_cgroup and cgroup_base is None:
            v1 = cgroup1_cpu()
            if v1 is not None:
                try:
                    self.cpu_root = v1 / f"tt-{env_name}"
                    self.cpu_root.mkdir(exist_ok=True)
                    self.mode = "cgroup1-cpu"
                except OSError:
                    self.cpu_root = None
        self.replicas: dict[str, ReplicaState] = {}
        self._reader = _schedstat_reader() if self.mode == "watchdog" and enforce_cpu else None
        self.duty = None  # the native duty cycle (dutycycle.hpp), when it can run here
        if self._reader is not None and os.environ.get("TT_CPU_DUTY", "native").lower() != "python":
            try:
                from .. import native
                self.duty = native.load().DutyCycle(PERIOD_S)
                self.duty.start()
            except Exception:
                self.duty = None

    def describe(self) -> dict:
        acct = "per-thread schedstat ns" if self._reader else "process clock ticks"
        if self.duty is not None:
            acct += ", native thread"
        cpu = {"cgroup2": "cgroup cpu.max", "cgroup1-cpu": "cgroup v1 cpu.cfs_quota_us",
               "watchdog": f"duty-cycle throttle (SIGSTOP/SIGCONT, {PERIOD_S * 1000:g} ms period, {acct})"}[self.mode] \
            if self.enforce_cpu else "accounted"
        mem = ("cgroup memory.max" if self.mode == "cgroup2" else "RSS watchdog + restart") if self.enforce_memory \
            else "accounted"
        return {"mode": self.mode, "cpu": cpu, "memory": mem}

    # -- lifecycle -------------------------------------------------------------------------
    def add(self, name: str, pid: int, limits: Limits) -> ReplicaState:
        st = self.replicas[name] = ReplicaState(name, pid, limits)
        if self.root is not None:
            cg = self.root / name
            try:
                cg.mkdir(exist_ok=True)
                if self.enforce_cpu:
                    (cg / "cpu.max").write_text(f"{max(1000, int(limits.cpu * 100000))} 100000")
                if self.enforce_memory:
                    (cg / "memory.max").write_text(str(limits.memory))
                st.cgroup = cg
                self._adopt(st)
            except OSError:
                st.cgroup = None
        elif self.cpu_root is not None:
            cg = self.cpu_root / name
            try:
                cg.mkdir(exist_ok=True)
                (cg / "cpu.cfs_period_us").write_text("100000")
                (cg / "cpu.cfs_quota_us").write_text(str(max(1000, int(limits.cpu * 100000))))
                st.cpu_cgroup = cg
                self._adopt_v1(st)
            except OSError:
                st.cpu_cgroup = None
        if self.duty is not None:
            self.duty.add(name, pid, limits.cpu)
            return st
        if self._reader is not None:
            st.clock = ThreadClock(pid, self._reader)
        st.period_cpu = self._used(st, time.monotonic())
        return st

    def _used(self, st: ReplicaState, now: float) -> float:
        return st.clock.seconds(now) if st.clock is not None else cpu_seconds(tree(st.pid))

    def _adopt_v1(self, st: ReplicaState) -> None:
        for p in tree(st.pid):
            try:
                (st.cpu_cgroup / "cgroup.procs").write_text(str(p.pid))
            except OSError:
                pass

    def remove(self, name: str) -> None:
        st = self.replicas.pop(name, None)
        if st is None:
            return
        if self.duty is not None:
            self.duty.remove(name)
        if st.stopped:
            self._signal(st, signal.SIGCONT)
        if st.clock is not None:
            st.clock.close()
        for cg in (st.cgroup, st.cpu_cgroup):
            if cg is not None:
                try:
                    cg.rmdir()
                except OSError:
                    pass

    def _adopt(self, st: ReplicaState) -> None:
        """Move the replica's processes (children started since) into its cgroup."""
        for p in tree(st.pid):
            try:
                (st.cgroup / "cgroup.procs").write_text(str(p.pid))
            except OSError:
                pass

    def _signal(self, st: ReplicaState, sig: int) -> None:
        try:
            os.killpg(st.pid, sig)  # replicas run in their own session / process group
        except (ProcessLookupError, PermissionError):
            pass

    # -- supervision tick: memory ---------------------------------------------------------------
    def check_memory(self) -> list[tuple[str, int]]:
        """Replicas over their memory limit, killed now: [(name, rss bytes)]."""
        out = []
        for st in list(self.replicas.values()):
            if st.cgroup is not None:
                self._adopt(st)
                try:
                    ev = dict(ln.split() for ln in (st.cgroup / "memory.events").read_text().splitlines())
                    if int(ev.get("oom_kill", 0)):
                        out.append((st.name, st.limits.memory))
                except (OSError, ValueError):
                    pass
                continue
            if st.cpu_cgroup is not None:
                self._adopt_v1(st)  # children the replica started since (its app, the data plane)
            used = rss(tree(st.pid))
            st.peak_rss = max(st.peak_rss, used)
            if self.enforce_memory and used > st.limits.memory:
                self._signal(st, signal.SIGCONT)
                self._signal(st, signal.SIGKILL)
                out.append((st.name, used))
        return out

    # -- CPU duty cycle (watchdog mode) ----------------------------------------------------------
    def throttle_tick(self, now: float | None = None) -> None:
        """Call every few ms: stop a replica's group once it has used ``cpu x PERIOD_S`` CPU
        seconds in the current period, resume it when the next period starts."""
        if not self.enforce_cpu or self.mode != "watchdog" or self.duty is not None:
            return
        now = time.monotonic() if now is None else now
        for st in list(self.replicas.values()):
            used = self._used(st, now)
            if now - st.period_start >= PERIOD_S:
                # unused quota does not carry over; an overrun does (paid off in later periods)
                quota = st.limits.cpu * (now - st.period_start)
                overrun = max(0.0, (used - st.period_cpu) - quota)
                st.period_cpu = used - overrun  # the next period starts with the debt already spent
                st.period_start = now
                if st.stopped:
                    self._signal(st, signal.SIGCONT)
                    st.stopped = False
                continue
            if not st.stopped and used - st.period_cpu >= st.limits.cpu * PERIOD_S:
                self._signal(st, signal.SIGSTOP)
                st.stopped = True
                st.throttled_periods += 1

    def throttled_periods(self, name: str) -> int:
        if self.duty is not None:
            return int((self.duty.stats().get(name) or {}).get("throttled_periods", 0))
        st = self.replicas.get(name)
        return st.throttled_periods if st else 0

    def duty_stats(self) -> dict[str, dict]:
        """Per replica: periods throttled, CPU and stopped seconds (native duty cycle only)."""
        return dict(self.duty.stats()) if self.duty is not None else {}

    def release_all(self) -> None:
        for name in list(self.replicas):
            self.remove(name)
        if self.duty is not None:
            self.duty.stop()
        for root in (self.root, self.cpu_root):
            if root is not None:
                try:
                    root.rmdir()
                except OSError:
                    pass
