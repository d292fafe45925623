"""The reference's overdue flow on the GPU (VERDICT r1 "next round" #1): cron -> processor ->
``GET /api/overduetasks?limit=`` -> API sidecar -> backing query planner -> gfx950 columnar
scan over a >=1M-task collection -> paged ``markoverdue`` bulk saves, repeated until a short
page.  The collection's writes stay on the native document store (its column mirror is
maintained in C++), and the result must equal the native engine's own answer."""
import asyncio
import os
import json
import time
from datetime import timedelta

import pytest

from aca_dotnet_workshop_amd.models import format_fixed, today
from aca_dotnet_workshop_amd.platform.inproc import InProcessEnvironment, tasks_tracker_specs

from helpers import run
from test_e2e_inproc import API, PROC, _task_doc

N_TASKS = int(os.environ.get("TT_TEST_SWEEP_TASKS", "1000000"))
PAST_EVERY = 101  # ~1% of the tasks are past due


@pytest.mark.gpu
def test_gpu_overdue_sweep_over_a_million_tasks(monkeypatch):
    _sweep(monkeypatch, "gpu", N_TASKS, 2000)


def test_cpu_overdue_sweep(monkeypatch):
    """The same flow without a GPU: the planner runs the program on the host executor
    (native/src/cpuscan.hpp), paged by 50, through the native list codecs of the apps."""
    _sweep(monkeypatch, "cpu", 30_000, 50)


def _sweep(monkeypatch, accel: str, n_tasks: int, page_size: int) -> None:
    monkeypatch.setenv("TT_QUERY_ACCEL", accel)
    monkeypatch.setenv("TT_QUERY_MIRROR_PATHS", "taskDueDate,isCompleted,isOverDue")
    N_TASKS = n_tasks

    async def main():
        env = InProcessEnvironment()
        await env.start_backing()
        try:
            for s in tasks_tracker_specs(frontend=False, api={"OverdueTasks:Query": "range"},
                                         processor={"OverdueTasks:PageSize": page_size}):
                await env.add_app(s)
            await env.wait_ready()
            st = env.backing.store("taskstracker-state-store", "tasksmanagerdb", "taskscollection")
            past = [format_fixed(today() - timedelta(days=d)) for d in (1, 2, 9)]
            future = [format_fixed(today() + timedelta(days=d)) for d in range(1, 60)]
            t0 = time.perf_counter()
            want = 0
            for i in range(N_TASKS):
                if i % PAST_EVERY == 0:
                    k, v = _task_doc(i, past[i % 3], done=i % 7 == 0)
                    want += i % 7 != 0
                else:
                    k, v = _task_doc(i, future[i % 59])
                st.set(k, v)
            print(f"seeded {N_TASKS} tasks in {time.perf_counter() - t0:.1f}s, {want} past due and open", flush=True)
            assert st.mirror_stats()["rows"] == N_TASKS  # mirrored from the first write
            c = env.replicas[PROC][0].client
            t0 = time.perf_counter()
            res = await c.invoke_method("POST", PROC, "ScheduledTasksManager", {})
            dt = time.perf_counter() - t0
            print(f"sweep: {res} in {dt:.2f}s", flush=True)
            assert res["markedOverdue"] == want and res["pages"] == want // page_size + 1
            acc = env.backing.accel("taskstracker-state-store", "tasksmanagerdb", "taskscollection")
            assert acc.stats[accel] >= res["pages"] and acc.stats["fallback"] == 0
            q = {"filter": {"EQ": {"isOverDue": True}}}
            assert len(json.loads(st.query(json.dumps(q)))["results"]) == want
            # nothing left: the next run retrieves an empty page
            res = await c.invoke_method("POST", PROC, "ScheduledTasksManager", {})
            assert res["markedOverdue"] == 0 and res["retrieved"] == 0
        finally:
            await env.stop()
    run(asyncio.wait_for(main(), 110))


def _created_order_case(monkeypatch, accel: str) -> None:
    """Range mode answers ``GET /api/overduetasks`` oldest first by ``TaskCreatedOn`` (reference
    ``.OrderBy(o => o.TaskCreatedOn)``, TasksStoreManager.cs:136): the store picks the page with
    ``ORDER BY taskCreatedOn`` over the stored round-trip strings (seven fractional digits, so
    string order IS DateTime order, ``TaskModel.to_store_json``) -- the page is exactly the
    oldest tasks by DateTime, in DateTime order.  An update to an old task re-appends its mirror
    row at the end; it must still come back in its creation-time position."""
    import random
    from datetime import datetime

    from aca_dotnet_workshop_amd.models.dotnet import format_roundtrip
    monkeypatch.setenv("TT_QUERY_ACCEL", accel)
    monkeypatch.setenv("TT_QUERY_ACCEL_MIN_DOCS", "0")
    monkeypatch.setenv("TT_QUERY_MIRROR_PATHS", "taskDueDate,isCompleted,isOverDue,taskCreatedOn")
    rnd = random.Random(5)
    base = datetime(2025, 3, 1, 8, 0, 0)
    n = 3000
    # creation times shuffled against insertion order, several per second, some on whole seconds
    stamps = [base + timedelta(seconds=i // 4, microseconds=[0, 100000, 500000, 120000][i % 4]) for i in range(n)]
    rnd.shuffle(stamps)
    due = format_fixed(today() - timedelta(days=2))

    async def main():
        env = InProcessEnvironment()
        await env.start_backing()
        try:
            for s in tasks_tracker_specs(frontend=False, api={"OverdueTasks:Query": "range"},
                                         processor={"OverdueTasks:PageSize": 100}):
                await env.add_app(s)
            await env.wait_ready()
            st = env.backing.store("taskstracker-state-store", "tasksmanagerdb", "taskscollection")
            for i, t in enumerate(stamps):
                k, v = _task_doc(i, due)
                st.set(k, v.replace('"2024-01-01T00:00:00"', f'"{format_roundtrip(t)}Z"'))  # as the API stores it
            c = env.replicas[PROC][0].client
            oldest = min(range(n), key=lambda i: stamps[i])
            # an update to the oldest task: a new mirror row at the end of the collection
            tid = f"00000000-0000-4000-8000-{oldest:012d}"
            await c.invoke_method("PUT", API, f"api/tasks/{tid}",
                                  {"taskId": tid, "taskName": "renamed", "taskAssignedTo": "b@x", "taskDueDate": due})
            r = await c.invoke_method_raw("GET", API, "api/overduetasks?limit=250")
            assert r.status == 200 and r.headers.get("x-tt-more-results") == "true"
            got = json.loads(r.body)
            # the page: exactly the 250 oldest by DateTime, in DateTime order (the reference's OrderBy)
            want = sorted(range(n), key=lambda i: stamps[i])[:250]
            assert [t["taskId"] for t in got] == [f"00000000-0000-4000-8000-{i:012d}" for i in want]
            assert got[0]["taskName"] == "renamed"
            from aca_dotnet_workshop_amd.models import parse_datetime
            created = [parse_datetime(t["taskCreatedOn"]) for t in got]
            assert created == sorted(created) and [c.replace(tzinfo=None) for c in created] == [stamps[i] for i in want]
            # the API answers in System.Text.Json's form (trimmed fraction), not the store's
            assert all(".0000000" not in t["taskCreatedOn"] and len(t["taskCreatedOn"]) <= 27 for t in got)
            acc = env.backing.accel("taskstracker-state-store", "tasksmanagerdb", "taskscollection")
            assert acc.stats[accel] >= 1 and acc.stats["fallback"] == 0
        finally:
            await env.stop()
    run(asyncio.wait_for(main(), 110))


def test_cpu_range_page_is_oldest_first(monkeypatch):
    _created_order_case(monkeypatch, "cpu")


@pytest.mark.gpu
def test_gpu_range_page_is_oldest_first(monkeypatch):
    _created_order_case(monkeypatch, "gpu")
