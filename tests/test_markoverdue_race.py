"""``POST api/overduetasks/markoverdue`` against concurrent completions.

The reference's ``MarkOverdueTasks`` saves the processor's copy of every task with
``IsOverDue = true`` and no ETag (TasksStoreManager.cs:141-149): a ``PUT .../markcomplete``
that lands between the cron job's ``GET api/overduetasks`` and its ``markoverdue`` is
overwritten with ``isCompleted: false``.  Here the API re-reads the tasks (state bulk get),
marks only the stored tasks still open and not yet overdue, each save guarded by the ETag it
read (first-write), and re-applies on a conflict.  Both sidecar data planes.
"""
import asyncio
from datetime import timedelta

import pytest

from aca_dotnet_workshop_amd.models import format_fixed, today
from aca_dotnet_workshop_amd.platform.inproc import InProcessEnvironment, tasks_tracker_specs

from helpers import run

API = "tasksmanager-backend-api"


async def _env(plane: str) -> InProcessEnvironment:
    env = InProcessEnvironment()
    await env.start_backing()
    for s in tasks_tracker_specs(frontend=False, api={"OverdueTasks:Query": "range"}):
        s.env["TT_SIDECAR_DATAPLANE"] = plane
        await env.add_app(s)
    await env.wait_ready()
    return env


async def _create(c, n: int, due: str) -> list[str]:
    ids = []
    for i in range(n):
        r = await c.invoke_method_raw("POST", API, "api/tasks", {"taskName": f"race {i}", "taskCreatedBy": "race@x",
                                                                 "taskDueDate": due, "taskAssignedTo": "a@x"})
        assert r.status == 201
        ids.append(r.headers["location"].rsplit("/", 1)[1])
    return ids


@pytest.mark.parametrize("plane", ["python", "native"])
def test_markoverdue_never_reverts_a_completion(plane):
    async def main():
        env = await _env(plane)
        try:
            c = env.replicas[API][0].client
            yesterday = format_fixed(today() - timedelta(days=1))
            for rnd in range(3):
                ids = await _create(c, 30, yesterday)
                page = [t for t in await c.invoke_method("GET", API, "api/overduetasks?limit=1000")
                        if t["taskId"] in set(ids)]
                assert len(page) == 30 and not any(t["isCompleted"] for t in page)  # the sweep's snapshot
                done = set(ids[rnd::2])
                # the race: completions land while the stale snapshot is being marked
                rs = await asyncio.gather(*(c.invoke_method_raw("PUT", API, f"api/tasks/{t}/markcomplete")
                                            for t in done),
                                          c.invoke_method_raw("POST", API, "api/overduetasks/markoverdue", page))
                assert [r.status for r in rs] == [200] * len(rs)
                # the same stale snapshot once more, after every completion: the reference would
                # now write isCompleted=false back over each of them
                r = await c.invoke_method_raw("POST", API, "api/overduetasks/markoverdue", page)
                assert r.status == 200
                for t in ids:
                    got = await c.invoke_method("GET", API, f"api/tasks/{t}")
                    if t in done:
                        assert got["isCompleted"] is True, got  # never reverted
                    else:
                        assert got["isOverDue"] is True and got["isCompleted"] is False, got  # none left unmarked
                    assert got["taskName"].startswith("race ")
        finally:
            await env.stop()
    run(main())


@pytest.mark.parametrize("plane", ["python", "native"])
def test_markoverdue_marks_the_stored_task_not_the_callers_copy(plane):
    """An edit between the query and the mark (a rename) survives: the flag is set on the stored
    document, and a task deleted in between is skipped rather than re-created."""
    async def main():
        env = await _env(plane)
        try:
            c = env.replicas[API][0].client
            ids = await _create(c, 3, format_fixed(today() - timedelta(days=1)))
            page = [t for t in await c.invoke_method("GET", API, "api/overduetasks?limit=1000") if t["taskId"] in ids]
            upd = {"taskId": ids[0], "taskName": "renamed meanwhile", "taskDueDate": page[0]["taskDueDate"],
                   "taskAssignedTo": "a@x"}
            assert (await c.invoke_method_raw("PUT", API, f"api/tasks/{ids[0]}", upd)).status == 200
            assert (await c.invoke_method_raw("DELETE", API, f"api/tasks/{ids[1]}")).status == 200
            assert (await c.invoke_method_raw("POST", API, "api/overduetasks/markoverdue", page)).status == 200
            t0 = await c.invoke_method("GET", API, f"api/tasks/{ids[0]}")
            assert t0["taskName"] == "renamed meanwhile" and t0["isOverDue"] is True
            assert (await c.invoke_method_raw("GET", API, f"api/tasks/{ids[1]}")).status == 404
            assert (await c.invoke_method("GET", API, f"api/tasks/{ids[2]}"))["isOverDue"] is True
        finally:
            await env.stop()
    run(main())
