"""Backend API contract tests (reference SURVEY.md §2.11; module-1 acceptance check:
``GET /api/tasks?createdBy=tjoudeh@bitoftech.net`` returns 10 tasks,
docs/aca/01-deploy-api-to-aca/index.md:532-534)."""
import uuid
from datetime import timedelta

from aca_dotnet_workshop_amd.models import TaskModel, format_fixed, today
from aca_dotnet_workshop_amd.services.backend_api import FakeTasksManager, create_app
from aca_dotnet_workshop_amd.utils.config import Configuration

from helpers import run, served

SEED = "tjoudeh@bitoftech.net"


def _app(env="Production", manager=None):
    cfg = Configuration([{"Environment": env}])
    return create_app(config=cfg, manager=manager or FakeTasksManager())


def test_seeded_tasks_and_ordering():
    async def main():
        async with served(_app()) as (base, c):
            r = await c.get(f"{base}/api/tasks?createdBy={SEED}")
            assert r.status == 200
            tasks = r.json()
            assert len(tasks) == 10
            # newest first (TaskCreatedOn = UtcNow + i minutes)
            assert [t["taskName"] for t in tasks] == [f"Task number: {i}" for i in range(9, -1, -1)]
            assert set(tasks[0]) == {"taskId", "taskName", "taskCreatedBy", "taskCreatedOn", "taskDueDate",
                                     "taskAssignedTo", "isCompleted", "isOverDue"}
            assert tasks[0]["taskCreatedOn"].endswith("Z")
            # query parameter binding is case-insensitive like ASP.NET
            r = await c.get(f"{base}/api/tasks/?createdby={SEED}")
            assert len(r.json()) == 10
            r = await c.get(f"{base}/api/tasks")
            assert r.json() == []
    run(main())


def test_crud_roundtrip():
    async def main():
        async with served(_app()) as (base, c):
            body = {"taskName": "write tests", "taskCreatedBy": "a@b.com", "taskDueDate": "2030-01-02T00:00:00",
                    "taskAssignedTo": "c@d.com"}
            r = await c.post(f"{base}/api/tasks", json_body=body)
            assert r.status == 201 and r.body == b""
            loc = r.headers["location"]
            assert loc.startswith("/api/tasks/")
            tid = loc.rsplit("/", 1)[1]
            uuid.UUID(tid)
            r = await c.get(f"{base}{loc}")
            assert r.status == 200
            t = r.json()
            assert t["taskName"] == "write tests" and t["taskDueDate"] == "2030-01-02T00:00:00"
            assert t["isCompleted"] is False
            upd = {"taskId": tid, "taskName": "renamed", "taskDueDate": "2030-02-03T00:00:00", "taskAssignedTo": "x@y.z"}
            r = await c.put(f"{base}/api/tasks/{tid}", json_body=upd)
            assert r.status == 200
            r = await c.put(f"{base}/api/tasks/{tid}/markcomplete")
            assert r.status == 200
            t = (await c.get(f"{base}/api/tasks/{tid}")).json()
            assert (t["taskName"], t["taskAssignedTo"], t["isCompleted"]) == ("renamed", "x@y.z", True)
            r = await c.delete(f"{base}/api/tasks/{tid}")
            assert r.status == 200
            assert (await c.get(f"{base}/api/tasks/{tid}")).status == 404
            assert (await c.delete(f"{base}/api/tasks/{tid}")).status == 404
            missing = str(uuid.uuid4())
            assert (await c.put(f"{base}/api/tasks/{missing}", json_body=upd)).status == 400
            assert (await c.put(f"{base}/api/tasks/{missing}/markcomplete")).status == 400
            assert (await c.get(f"{base}/api/tasks/not-a-guid")).status == 400
            # body validation
            assert (await c.post(f"{base}/api/tasks", body=b"{bad json", headers={"Content-Type": "application/json"})).status == 400
            assert (await c.post(f"{base}/api/tasks", body=b"x=1", headers={"Content-Type": "text/plain"})).status == 415
            assert (await c.request("PATCH", f"{base}/api/tasks")).status == 405
    run(main())


def test_overdue_endpoints_with_fake():
    mgr = FakeTasksManager(seed=False)
    y = today() - timedelta(days=1)

    async def main():
        async with served(_app(manager=mgr)) as (base, c):
            for i, due in enumerate([y, y, today(), y]):
                await c.post(f"{base}/api/tasks", json_body={"taskName": f"t{i}", "taskCreatedBy": "u@x",
                                                             "taskDueDate": format_fixed(due), "taskAssignedTo": "a@x"})
            tasks = (await c.get(f"{base}/api/tasks?createdBy=u@x")).json()
            t3 = [t for t in tasks if t["taskName"] == "t3"][0]
            await c.put(f"{base}/api/tasks/{t3['taskId']}/markcomplete")
            due = (await c.get(f"{base}/api/overduetasks")).json()
            assert [t["taskName"] for t in due] == ["t0", "t1"]  # ascending by creation, open only
            r = await c.post(f"{base}/api/overduetasks/markoverdue", json_body=due)
            assert r.status == 200
            assert (await c.get(f"{base}/api/overduetasks")).json() == []
            tasks = {t["taskName"]: t for t in (await c.get(f"{base}/api/tasks?createdBy=u@x")).json()}
            assert tasks["t0"]["isOverDue"] and tasks["t1"]["isOverDue"] and not tasks["t2"]["isOverDue"]
    run(main())


def test_openapi_only_in_development():
    async def main():
        async with served(_app("Development")) as (base, c):
            r = await c.get(f"{base}/openapi/v1.json")
            assert r.status == 200
            doc = r.json()
            assert "/api/tasks/{taskId}" in doc["paths"]
            assert set(doc["paths"]["/api/tasks/{taskId}"]) == {"get", "put", "delete"}
            assert "TaskModel" in doc["components"]["schemas"]
        async with served(_app("Production")) as (base, c):
            assert (await c.get(f"{base}/openapi/v1.json")).status == 404
    run(main())


def test_taskmodel_wire_format():
    t = TaskModel.from_wire({"TaskName": "x", "taskDueDate": "2024-05-01", "taskCreatedOn": "2024-05-01T10:11:12.1234567Z"})
    w = t.to_wire()
    assert w["taskName"] == "x"
    assert w["taskDueDate"] == "2024-05-01T00:00:00"
    assert w["taskCreatedOn"] == "2024-05-01T10:11:12.123456Z"
    assert w["taskId"] == "00000000-0000-0000-0000-000000000000"
