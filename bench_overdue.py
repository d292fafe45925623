#!/usr/bin/env python3
"""The overdue sweep as the application runs it, on a large task collection.

cron-equivalent trigger -> processor ``POST /ScheduledTasksManager`` -> API
``GET /api/overduetasks?limit=`` (``OverdueTasks:Query=range``) -> API sidecar -> backing
query planner -> columnar mirror sync + gfx950 scan / ordering kernels -> paged
``markoverdue`` bulk saves, until a short page (reference flow:
Controllers/ScheduledTasksManagerController.cs:19-46, Services/TasksStoreManager.cs:104-149).

Seeds ``--tasks`` documents straight into the document store (``--past-every``: one in N is
due before today and open), runs ``--sweeps`` full sweeps (the first marks every past-due
task; later ones find an empty page after re-seeding ``--reseed`` new past-due tasks) and
prints one JSON line with per-sweep wall time, pages, tasks marked and the accelerator's
query counts.  Run under ``rocprofv3 --kernel-trace --stats`` for the kernel trace of the
app-driven sweep (profiles/r2_overdue_sweep.md).

    python bench_overdue.py --tasks 1000000 --accel gpu
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import sys
import time
from datetime import timedelta

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

API = "tasksmanager-backend-api"
PROC = "tasksmanager-backend-processor"
COLL = ("taskstracker-state-store", "tasksmanagerdb", "taskscollection")


def task_doc(i: int, due: str, done: bool = False) -> tuple[str, str]:
    tid = f"00000000-0000-4000-8000-{i:012d}"
    return f"{API}||{tid}", (
        '{"taskId":"%s","taskName":"seed %d","taskCreatedBy":"seed%d@x","taskCreatedOn":"2024-01-01T00:00:00",'
        '"taskDueDate":"%s","taskAssignedTo":"a@x","isCompleted":%s,"isOverDue":false}'
        % (tid, i, i % 97, due, "true" if done else "false"))


async def main(a: argparse.Namespace) -> dict:
    os.environ["TT_QUERY_ACCEL"] = a.accel
    os.environ["TT_QUERY_MIRROR_PATHS"] = "taskDueDate,isCompleted,isOverDue"
    os.environ.setdefault("TT_LOG_CONSOLE", "0")
    from aca_dotnet_workshop_amd.models import format_fixed, today
    from aca_dotnet_workshop_amd.platform.inproc import InProcessEnvironment, tasks_tracker_specs
    from aca_dotnet_workshop_amd.telemetry.logging import configure_logging
    configure_logging("bench-overdue")
    env = InProcessEnvironment()
    await env.start_backing()
    try:
        for s in tasks_tracker_specs(frontend=False, api={"OverdueTasks:Query": "range", "Logging:LogLevel:Default": "Warning"},
                                     processor={"OverdueTasks:PageSize": a.page, "Logging:LogLevel:Default": "Warning"}):
            await env.add_app(s)
        await env.wait_ready()
        st = env.backing.store(*COLL)
        past = [format_fixed(today() - timedelta(days=d)) for d in (1, 2, 9)]
        future = [format_fixed(today() + timedelta(days=d)) for d in range(1, 60)]
        t0 = time.perf_counter()
        want = 0
        for i in range(a.tasks):
            if i % a.past_every == 0:
                k, v = task_doc(i, past[i % 3], done=i % 7 == 0)
                want += i % 7 != 0
            else:
                k, v = task_doc(i, future[i % 59])
            st.set(k, v)
        seed_s = time.perf_counter() - t0
        c = env.replicas[PROC][0].client
        sweeps = []
        nxt = a.tasks
        for n in range(a.sweeps):
            if n:  # new past-due tasks arrive between runs (through the store, mirrored natively)
                for _ in range(a.reseed):
                    k, v = task_doc(nxt, past[nxt % 3])
                    st.set(k, v)
                    nxt += 1
            t = time.perf_counter()
            res = await c.invoke_method("POST", PROC, "ScheduledTasksManager", {})
            sweeps.append({"s": round(time.perf_counter() - t, 4), "pages": res["pages"], "marked": res["markedOverdue"]})
        acc = env.backing.accel(*COLL)
        out = {"tasks": a.tasks, "past_due_open": want, "seed_s": round(seed_s, 2), "page": a.page, "accel": a.accel,
               "sweeps": sweeps, "accelerator": dict(acc.stats), "mirror": dict(st.mirror_stats())}
        assert sweeps[0]["marked"] == want, (sweeps[0], want)
        return out
    finally:
        await env.stop()


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--tasks", type=int, default=1_000_000)
    ap.add_argument("--past-every", type=int, default=101)
    ap.add_argument("--page", type=int, default=2000)
    ap.add_argument("--sweeps", type=int, default=5)
    ap.add_argument("--reseed", type=int, default=1000)
    ap.add_argument("--accel", default="gpu", choices=("gpu", "cpu", "off"))
    print(json.dumps(asyncio.run(main(ap.parse_args()))), flush=True)
