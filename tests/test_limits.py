"""Per-replica resource limits (platform/limits.py): the Consumption profile's 0.25 vCPU /
0.5 Gi (reference processor-backend-service.bicep:143-146).  Exercised here in watchdog mode
(no delegated cgroup in CI): the memory watchdog kills a replica over its limit, the CPU
duty-cycle throttle holds a busy loop near its quota."""
import os
import subprocess
import sys
import time

import pytest

from aca_dotnet_workshop_amd.platform.limits import Limits, ResourceLimiter, cpu_seconds, parse_memory, tree


def _spawn(code):
    return subprocess.Popen([sys.executable, "-c", code], start_new_session=True)


def test_parse_memory():
    assert parse_memory("0.5Gi") == 512 << 20
    assert parse_memory("256Mi") == 256 << 20
    assert parse_memory("1G") == 10 ** 9
    assert parse_memory(1024) == 1024


def test_memory_watchdog_kills_replica_over_limit():
    p = _spawn("import time\nx = bytearray(160 << 20)\nfor i in range(0, len(x), 4096): x[i] = 1\ntime.sleep(30)")
    lim = ResourceLimiter("t", enforce_memory=True, allow_cgroup=False)
    try:
        lim.add("hog-0", p.pid, Limits(0.25, parse_memory("64Mi")))
        assert lim.describe()["memory"] == "RSS watchdog + restart"
        killed = []
        deadline = time.time() + 20
        while not killed and time.time() < deadline:
            killed = lim.check_memory()
            time.sleep(0.1)
        assert killed and killed[0][0] == "hog-0" and killed[0][1] > (64 << 20)
        assert p.wait(10) == -9
    finally:
        if p.poll() is None:
            p.kill()
        lim.release_all()


def test_memory_under_limit_is_left_alone():
    p = _spawn("import time\ntime.sleep(30)")
    lim = ResourceLimiter("t", enforce_memory=True, allow_cgroup=False)
    try:
        lim.add("small-0", p.pid, Limits(0.25, parse_memory("0.5Gi")))
        for _ in range(5):
            assert lim.check_memory() == []
            time.sleep(0.05)
        assert p.poll() is None and lim.replicas["small-0"].peak_rss > 0
    finally:
        p.kill()
        lim.release_all()


@pytest.mark.parametrize("duty", ["native", "python"])
def test_cpu_throttle_holds_quota(duty, monkeypatch):
    """The duty cycle on its native thread (dutycycle.hpp; ``throttle_tick`` is then a no-op)
    and the controller's own Python tick hold a busy loop at its quota."""
    monkeypatch.setenv("TT_CPU_DUTY", duty)
    p = _spawn("while True: pass")
    lim = ResourceLimiter("t", enforce_cpu=True, allow_cgroup=False)
    try:
        assert (lim.duty is not None) == (duty == "native")
        lim.add("busy-0", p.pid, Limits(0.25, parse_memory("0.5Gi")))
        c0, t0 = cpu_seconds(tree(p.pid)), time.monotonic()
        while time.monotonic() - t0 < 3.0:
            lim.throttle_tick()
            time.sleep(0.005)
        used = cpu_seconds(tree(p.pid)) - c0
        wall = time.monotonic() - t0
        assert 0.15 < used / wall < 0.35, used / wall  # ~0.25 cores, not 1.0
        assert lim.throttled_periods("busy-0") >= 50  # 20 ms periods: a short stall each, not a long one
        d = lim.describe()
        assert d["mode"] == "watchdog" and "20 ms period" in d["cpu"] and "schedstat" in d["cpu"], d
        assert ("native thread" in d["cpu"]) == (duty == "native")
        if duty == "native":
            st = lim.duty_stats()["busy-0"]
            assert 0.5 < st["stopped_seconds"] and 0.4 < st["cpu_seconds"] < 1.2, st
    finally:
        lim.release_all()
        os.killpg(p.pid, 9)
        p.wait()


@pytest.mark.parametrize("duty", ["native", "python"])
def test_cpu_throttle_counts_threads_started_later(duty, monkeypatch):
    """A replica whose process starts busy threads after it was added: their CPU counts (the
    per-thread clock picks new threads up from zero) and the group is held at its quota."""
    monkeypatch.setenv("TT_CPU_DUTY", duty)
    p = _spawn("import threading, time\ntime.sleep(0.3)\n"
               "def spin():\n    while True: pass\n"
               "[threading.Thread(target=spin, daemon=True).start() for _ in range(2)]\nwhile True: time.sleep(1)")
    lim = ResourceLimiter("t2", enforce_cpu=True, allow_cgroup=False)
    try:
        lim.add("busy-1", p.pid, Limits(0.5, parse_memory("0.5Gi")))
        time.sleep(0.6)  # the spinning threads exist now (the GIL holds them near 1 core)
        c0, t0 = cpu_seconds(tree(p.pid)), time.monotonic()
        while time.monotonic() - t0 < 3.0:
            lim.throttle_tick()
            time.sleep(0.005)
        used = cpu_seconds(tree(p.pid)) - c0
        assert used / (time.monotonic() - t0) < 0.7
    finally:
        lim.release_all()
        os.killpg(p.pid, 9)
        p.wait()


def test_cpu_quota_by_cgroup_v1_when_writable():
    """Where a cgroup v1 ``cpu`` hierarchy is writable (a root container on a v1 host), the
    replica gets CFS bandwidth control -- the kernel holds it at its share, no signals."""
    from aca_dotnet_workshop_amd.platform.limits import cgroup1_cpu, delegated_cgroup
    if delegated_cgroup() is not None or cgroup1_cpu() is None:
        pytest.skip("no writable cgroup v1 cpu hierarchy here (or v2 is delegated)")
    p = _spawn("while True: pass")
    lim = ResourceLimiter("tv1", enforce_cpu=True)
    try:
        assert lim.describe() == {"mode": "cgroup1-cpu", "cpu": "cgroup v1 cpu.cfs_quota_us",
                                  "memory": "RSS watchdog + restart"}
        st = lim.add("busy-0", p.pid, Limits(0.25, parse_memory("0.5Gi")))
        assert (st.cpu_cgroup / "cpu.cfs_quota_us").read_text().strip() == "25000"
        c0, t0 = cpu_seconds(tree(p.pid)), time.monotonic()
        time.sleep(2.0)
        used = cpu_seconds(tree(p.pid)) - c0
        assert used / (time.monotonic() - t0) < 0.35
    finally:
        lim.release_all()
        os.killpg(p.pid, 9)
        p.wait()
