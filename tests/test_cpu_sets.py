"""The rank's CPU split (parallel.split_platform / pin_preexec / enforce_cpuset): the platform's
processes on their reserve, the replicas on the rest, and a thread that left its set (a runtime
setting its own threads' affinity) put back."""
import os
import subprocess
import sys
import threading

import pytest

from aca_dotnet_workshop_amd.parallel import (cpus_allowed, enforce_cpuset, pin_all_threads, pin_preexec,
                                              split_platform)

ALL = set(os.sched_getaffinity(0))


def test_split_platform_reserves_the_top_cpus():
    assert split_platform(set(range(16)), 4) == ({12, 13, 14, 15}, set(range(12)))
    assert split_platform(set(range(5)), 4) is None  # too small: shared
    assert split_platform(None, 4) is None and split_platform(set(range(16)), 0) is None


@pytest.mark.skipif(len(ALL) < 2, reason="needs two CPUs")
def test_pin_preexec_pins_the_child_and_its_threads(monkeypatch):
    one = min(ALL)
    monkeypatch.setenv("TT_PLATFORM_CPUS", str(one))
    code = ("import os, threading; t = threading.Thread(target=lambda: print(sorted(os.sched_getaffinity(0))));"
            "t.start(); t.join(); print(sorted(os.sched_getaffinity(0)))")
    out = subprocess.run([sys.executable, "-c", code], preexec_fn=pin_preexec("platform"), capture_output=True,
                         text=True, timeout=60).stdout.split("\n")
    assert out[:2] == [f"[{one}]", f"[{one}]"]
    monkeypatch.delenv("TT_PLATFORM_CPUS")
    assert pin_preexec("platform") is None


@pytest.mark.skipif(len(ALL) < 2, reason="needs two CPUs")
def test_enforce_cpuset_moves_a_thread_that_escaped():
    one = {min(ALL)}
    p = subprocess.Popen([sys.executable, "-c", "import sys, threading, time; "
                          "[threading.Thread(target=time.sleep, args=(30,), daemon=True).start() for _ in range(3)];"
                          "print('up', flush=True); sys.stdin.read()"],
                         stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
    try:
        assert p.stdout.readline().strip() == "up"
        tids = sorted(cpus_allowed(p.pid))
        assert len(tids) >= 4
        for t in tids:  # the process is pinned, one thread then widened again (as a runtime may)
            os.sched_setaffinity(t, one)
        os.sched_setaffinity(tids[-1], ALL)
        moved = enforce_cpuset(p.pid, one)
        assert len(moved) == 1 and moved[0].endswith(f"/{tids[-1]}")
        assert all(c == one for c in cpus_allowed(p.pid).values())
        assert enforce_cpuset(p.pid, one) == []  # nothing left outside
    finally:
        p.stdin.close()
        p.kill()
        p.wait()


def test_pin_all_threads_covers_running_threads():
    stop = threading.Event()
    t = threading.Thread(target=stop.wait, daemon=True)
    t.start()
    try:
        pin_all_threads(ALL)  # this process's own set: a no-op that must reach every thread
        assert all(c == ALL for c in cpus_allowed(os.getpid()).values())
    finally:
        stop.set()
        t.join()


@pytest.mark.skipif(len(ALL) < 2, reason="needs two CPUs")
def test_hold_affinity_puts_every_thread_back():
    """A runtime that widens the calling thread's set (the GPU runtime's first call does) and
    starts threads from it: on leaving ``hold_affinity`` every thread of the process is back on
    the set it had on entry."""
    code = """
import os, threading, time
from aca_dotnet_workshop_amd.parallel import hold_affinity, cpus_allowed
one = {min(os.sched_getaffinity(0))}
os.sched_setaffinity(0, one)
ev = threading.Event()
with hold_affinity():
    os.sched_setaffinity(0, set(range(os.cpu_count())) & set(%r))  # the runtime widens it
    t = threading.Thread(target=ev.wait, daemon=True)
    t.start()                                  # ... and starts a thread with the wide set
print(sorted({c for s in cpus_allowed(os.getpid()).values() for c in s}) == sorted(one))
ev.set()
""" % (sorted(ALL),)
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60,
                         env={**os.environ, "PYTHONPATH": os.path.dirname(os.path.dirname(__file__))})
    assert out.stdout.strip() == "True", out.stderr[-2000:]
