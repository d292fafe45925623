"""End-to-end tests over the in-process environment (3 apps + 3 sidecars + backing
services), one per workshop module acceptance check:

M3 invoke through the sidecar; M4 state API (bulk save 204, get, ETag, query, key
prefix); M5 publish -> processor delivery; M6 queue -> processor -> API + blob; M7 cron
-> overdue job; plus the frontend pages and trace propagation (M8)."""
import asyncio
import base64
import json
import re
from datetime import timedelta

from aca_dotnet_workshop_amd.models import format_fixed, today
from aca_dotnet_workshop_amd.platform.inproc import InProcessEnvironment, tasks_tracker_specs
from aca_dotnet_workshop_amd.sidecar import from_dict

from helpers import run

API = "tasksmanager-backend-api"
PROC = "tasksmanager-backend-processor"
WEB = "tasksmanager-frontend-webapp"


async def _env(**kw):
    env = InProcessEnvironment(**{k: v for k, v in kw.items() if k in ("extra_components", "policy")})
    await env.start_backing()
    for s in tasks_tracker_specs(processor=kw.get("processor"), frontend=kw.get("frontend", True)):
        await env.add_app(s)
    await env.wait_ready()
    return env


async def _until(pred, timeout=5.0, step=0.02):
    loop = asyncio.get_running_loop()
    end = loop.time() + timeout
    while loop.time() < end:
        v = await pred()
        if v:
            return v
        await asyncio.sleep(step)
    raise AssertionError("condition not met in time")


def test_invoke_state_pubsub_flow():
    async def main():
        env = await _env(frontend=False)
        try:
            c = env.replicas[PROC][0].client  # any app's sidecar can invoke the API by app-id
            r = await c.invoke_method_raw("POST", API, "api/tasks",
                                          {"taskName": "Email", "taskCreatedBy": "me@x", "taskDueDate": "2030-01-02T00:00:00",
                                           "taskAssignedTo": "you@x"})
            assert r.status == 201
            tid = r.headers["location"].rsplit("/", 1)[1]
            tasks = await c.invoke_method("GET", API, "api/tasks?createdBy=me@x")
            assert [t["taskId"] for t in tasks] == [tid]
            # the stored document lives under the API's key prefix in the "Cosmos" account
            st = env.backing.store("taskstracker-state-store", "tasksmanagerdb", "taskscollection")
            assert st.get(f"{API}||{tid}") is not None
            # tasksavedtopic -> processor subscription (named after the processor app-id) -> completed
            b = env.backing.broker("taskstracker")

            async def delivered():  # plane-agnostic: consumers may run in the native data plane
                return b.counts("tasksavedtopic/subscriptions/" + PROC)["completed"] >= 1
            await _until(delivered)
            cnt = b.counts("tasksavedtopic/subscriptions/" + PROC)
            assert cnt["completed"] == 1 and cnt["active"] == 0
            # assignee change republishes, same assignee (case-insensitive) does not
            await c.invoke_method("PUT", API, f"api/tasks/{tid}", {"taskId": tid, "taskName": "Email", "taskDueDate":
                                  "2030-01-02T00:00:00", "taskAssignedTo": "YOU@x"})
            await c.invoke_method("PUT", API, f"api/tasks/{tid}", {"taskId": tid, "taskName": "Email", "taskDueDate":
                                  "2030-01-02T00:00:00", "taskAssignedTo": "other@x"})
            await _until(lambda: _async(b.counts("tasksavedtopic/subscriptions/" + PROC)["completed"] == 2))
            await asyncio.sleep(0.1)
            assert b.counts("tasksavedtopic/subscriptions/" + PROC)["enqueued"] == 2
            # delete -> 200 then 404 (store-backed API reports missing tasks, §2.12 #4)
            assert (await c.invoke_method_raw("DELETE", API, f"api/tasks/{tid}")).status == 200
            assert (await c.invoke_method_raw("DELETE", API, f"api/tasks/{tid}")).status == 404
            # unknown app-id -> 500 ERR_DIRECT_INVOKE
            r = await c.invoke_method_raw("GET", "no-such-app", "x")
            assert r.status == 500 and r.json()["errorCode"] == "ERR_DIRECT_INVOKE"
        finally:
            await env.stop()
    run(main())


async def _async(v):
    return v


def test_state_api_module4():
    """M4: bulk save -> 204, get by key, etag conflicts -> 409, transactions, query."""
    async def main():
        env = await _env(frontend=False)
        try:
            sc = env.replicas[API][0].client
            http, base = sc.http, sc.base
            r = await http.post(base + "/v1.0/state/statestore", json_body=[
                {"key": "Book1", "value": {"title": "Parallel and High Performance Computing", "author": "Robert Robey"}},
                {"key": "Book2", "value": {"title": "Software Engineering Best Practices", "author": "Capers Jones"}},
                {"key": "Book3", "value": {"title": "The Art of Computer Programming", "author": "Donald Knuth"}}])
            assert r.status == 204
            r = await http.get(base + "/v1.0/state/statestore/Book3")
            assert r.status == 200 and r.json()["author"] == "Donald Knuth"
            etag = r.headers["etag"]
            assert (await http.get(base + "/v1.0/state/statestore/Missing")).status == 204
            ok = await http.post(base + "/v1.0/state/statestore", json_body=[{"key": "Book3", "value": 1, "etag": etag}])
            assert ok.status == 204
            stale = await http.post(base + "/v1.0/state/statestore", json_body=[{"key": "Book3", "value": 2, "etag": etag}])
            assert stale.status == 409
            r = await http.post(base + "/v1.0/state/statestore/bulk", json_body={"keys": ["Book1", "Nope"]})
            items = r.json()
            assert items[0]["data"]["author"] == "Robert Robey" and "data" not in items[1]
            r = await http.post(base + "/v1.0/state/statestore/transaction", json_body={"operations": [
                {"operation": "upsert", "request": {"key": "Book4", "value": {"author": "Knuth"}}},
                {"operation": "delete", "request": {"key": "Book2"}}]})
            assert r.status == 204
            r = await http.post(base + "/v1.0-alpha1/state/statestore/query",
                                json_body={"filter": {"EQ": {"author": "Knuth"}}})
            assert [x["key"] for x in r.json()["results"]] == ["Book4"]
            # store scoped to the API only (components/dapr-statestore-cosmos.yaml scopes)
            pc = env.replicas[PROC][0].client
            r = await pc.http.get(pc.base + "/v1.0/state/statestore/Book1")
            assert r.status == 400 and r.json()["errorCode"] == "ERR_STATE_STORE_NOT_FOUND"
            # keys are stored as <app-id>||<key>
            st = env.backing.store("taskstracker-state-store", "tasksmanagerdb", "taskscollection")
            assert st.get(f"{API}||Book1") is not None and st.get("Book1") is None
            meta = (await http.get(base + "/v1.0/metadata")).json()
            assert meta["id"] == API and {"name": "statestore", "type": "state.azure.cosmosdb", "version": "v1"} in meta["components"]
        finally:
            await env.stop()
    run(main())


def test_queue_binding_to_blob_module6():
    async def main():
        env = await _env(frontend=False)
        try:
            payload = {"taskName": "Task from queue", "taskAssignedTo": "a@b.com", "taskCreatedBy": "ext@x",
                       "taskDueDate": "2030-05-01T00:00:00"}
            b64 = base64.b64encode(json.dumps(payload).encode())
            env.backing.broker("storage-taskstrackerstorage").send("external-tasks-queue", b64)
            env.backing.waiters.notify("storage-taskstrackerstorage|external-tasks-queue")
            c = env.replicas[PROC][0].client

            async def created():
                ts = await c.invoke_method("GET", API, "api/tasks?createdBy=ext@x")
                return ts if ts else None
            tasks = await _until(created)
            tid = tasks[0]["taskId"]
            blob = env.backing.blob_root / "taskstrackerstorage" / "externaltaskscontainer" / f"{tid}.json"
            await _until(lambda: _async(blob.exists()))
            stored = json.loads(blob.read_text())
            assert stored["taskId"] == tid and stored["taskName"] == "Task from queue"
            await _until(lambda: _async(
                env.backing.broker("storage-taskstrackerstorage").counts("external-tasks-queue")["completed"] == 1))
        finally:
            await env.stop()
    run(main())


def test_cron_overdue_job_module7():
    fast_cron = from_dict({"apiVersion": "dapr.io/v1alpha1", "kind": "Component", "metadata": {"name": "FastCron"},
                           "spec": {"type": "bindings.cron", "version": "v1", "metadata": [
                               {"name": "schedule", "value": "@every 200ms"}, {"name": "route", "value": "/ScheduledTasksManager"},
                               {"name": "singleReplica", "value": "true"}]},
                           "scopes": [PROC]})

    async def main():
        env = await _env(frontend=False, extra_components=[fast_cron])
        try:
            c = env.replicas[PROC][0].client
            y = format_fixed(today() - timedelta(days=1))
            for name, due in (("late", y), ("future", format_fixed(today() + timedelta(days=3)))):
                await c.invoke_method("POST", API, "api/tasks", {"taskName": name, "taskCreatedBy": "cron@x",
                                                                 "taskDueDate": due, "taskAssignedTo": "a@x"})

            async def marked():
                ts = {t["taskName"]: t for t in await c.invoke_method("GET", API, "api/tasks?createdBy=cron@x")}
                return ts if ts["late"]["isOverDue"] else None
            ts = await _until(marked, timeout=8)
            assert ts["future"]["isOverDue"] is False
            assert await c.invoke_method("GET", API, "api/overduetasks") == []
            cron = env.sidecar(PROC).bindings["FastCron"]
            assert cron.fired >= 1
        finally:
            await env.stop()
    run(main())


def test_frontend_pages_flow():
    async def main():
        env = await _env(frontend=True)
        try:
            web = env.url(WEB)
            http = env.http
            r = await http.get(web + "/Tasks/Index")
            assert r.status == 302 and r.headers["location"] == "/"
            r = await http.post(web + "/", body=b"TasksCreatedBy=ui%40user.com",
                                headers={"Content-Type": "application/x-www-form-urlencoded"})
            assert r.status == 302 and "TasksCreatedByCookie=ui@user.com" in r.headers["set-cookie"]
            cookie = "TasksCreatedByCookie=ui@user.com"
            r = await http.get(web + "/Tasks/Create", headers={"Cookie": cookie})
            assert r.status == 200
            # client-side validation: unobtrusive data-val rules + message spans + the script
            # (the reference's asp-validation-for + _ValidationScriptsPartial, Create.cshtml:13-29,45)
            assert 'name="TaskAdd.TaskName"' in r.text and 'data-val="true"' in r.text
            assert 'data-val-required="The Task Name field is required."' in r.text
            assert 'data-val-email="The Assigned To field is not a valid e-mail address."' in r.text
            assert 'data-valmsg-for="TaskAdd.TaskDueDate"' in r.text and '<script src="/js/validation.js">' in r.text
            assert (await http.get(web + "/js/validation.js")).status == 200
            af_cookie = re.search(r"\.AspNetCore\.Antiforgery=([0-9a-f]+)", r.headers["set-cookie"]).group(1)
            token = re.search(r'name="__RequestVerificationToken" value="([0-9a-f]+)"', r.text).group(1)
            cookies = f"{cookie}; .AspNetCore.Antiforgery={af_cookie}"
            form_h = {"Cookie": cookies, "Content-Type": "application/x-www-form-urlencoded"}
            # missing required fields -> page re-rendered with validation messages
            r = await http.post(web + "/Tasks/Create", body=f"__RequestVerificationToken={token}&TaskAdd.TaskName=",
                                headers=form_h)
            assert r.status == 200 and "The Task Name field is required." in r.text
            assert 'class="field-validation-error text-danger" data-valmsg-for="TaskAdd.TaskName"' in \
                " ".join(r.text.split())
            # no antiforgery token -> 400
            r = await http.post(web + "/Tasks/Create", body=b"TaskAdd.TaskName=x", headers=form_h)
            assert r.status == 400
            body = (f"__RequestVerificationToken={token}&TaskAdd.TaskName=Buy+milk&TaskAdd.TaskDueDate=2030-06-07"
                    f"&TaskAdd.TaskAssignedTo=bob%40x.com")
            r = await http.post(web + "/Tasks/Create", body=body, headers=form_h)
            assert r.status == 302 and r.headers["location"] == "/Tasks/Index"
            r = await http.get(web + "/Tasks/Index", headers={"Cookie": cookies})
            assert "Buy milk" in r.text and "07-06-2030" in r.text and "Tasks for (ui@user.com)" in r.text
            tid = re.search(r'data-task-id="([0-9a-f-]+)"', r.text).group(1)
            r = await http.get(web + f"/Tasks/Edit/{tid}", headers={"Cookie": cookies})
            assert r.status == 200 and 'value="2030-06-07"' in r.text
            body = (f"__RequestVerificationToken={token}&TaskUpdate.TaskId={tid}&TaskUpdate.TaskName=Buy+oat+milk"
                    f"&TaskUpdate.TaskDueDate=2030-06-08&TaskUpdate.TaskAssignedTo=bob%40x.com")
            assert (await http.post(web + f"/Tasks/Edit/{tid}", body=body, headers=form_h)).status == 302
            r = await http.post(web + f"/Tasks/Index?handler=complete&id={tid}",
                                body=f"__RequestVerificationToken={token}", headers=form_h)
            assert r.status == 302
            r = await http.get(web + "/Tasks/Index", headers={"Cookie": cookies})
            assert "Buy oat milk" in r.text and "checked" in r.text
            r = await http.post(web + f"/Tasks/Index?handler=delete&id={tid}",
                                body=f"__RequestVerificationToken={token}", headers=form_h)
            r = await http.get(web + "/Tasks/Index", headers={"Cookie": cookies})
            assert "Buy oat milk" not in r.text
            assert (await http.get(web + "/css/site.css")).status == 200
            assert (await http.get(web + "/Privacy")).status == 200
        finally:
            await env.stop()
    run(main())


def test_trace_propagates_through_sidecars_and_pubsub():
    async def main():
        env = await _env(frontend=False)
        try:
            c = env.replicas[API][0].client
            from aca_dotnet_workshop_amd.telemetry import tracing
            tr = tracing.Tracer("test-client")
            with tr.start_span("root", "client") as root:
                await c.invoke_method("POST", API, "api/tasks", {"taskName": "traced", "taskCreatedBy": "t@x",
                                                                 "taskDueDate": "2030-01-01T00:00:00", "taskAssignedTo": "a@x"})
            psc = env.sidecar(PROC)
            await _until(lambda: _async(any(s["name"].startswith("pubsub/") and s["traceId"] == root.trace_id
                                            for s in psc.tracer.exporter.memory)))
            api_spans = env.sidecar(API).tracer.exporter.memory
            assert any(s["traceId"] == root.trace_id and s["kind"] == "server" for s in api_spans)
        finally:
            await env.stop()
    run(main())


def _fast_cron(schedule="@every 200ms"):
    return from_dict({"apiVersion": "dapr.io/v1alpha1", "kind": "Component", "metadata": {"name": "FastCron"},
                      "spec": {"type": "bindings.cron", "version": "v1", "metadata": [
                          {"name": "schedule", "value": schedule}, {"name": "route", "value": "/ScheduledTasksManager"},
                          {"name": "singleReplica", "value": "true"}]},
                      "scopes": [PROC]})


def _task_doc(i, due, done=False, overdue=False):
    tid = f"00000000-0000-4000-8000-{i:012d}"
    return f"{API}||{tid}", (
        '{"taskId":"%s","taskName":"seed %d","taskCreatedBy":"seed%d@x","taskCreatedOn":"2024-01-01T00:00:00",'
        '"taskDueDate":"%s","taskAssignedTo":"a@x","isCompleted":%s,"isOverDue":%s}'
        % (tid, i, i % 97, due, "true" if done else "false", "true" if overdue else "false"))


async def _range_sweep_env(monkeypatch, accel, page, processor=None):
    monkeypatch.setenv("TT_QUERY_ACCEL", accel)
    monkeypatch.setenv("TT_QUERY_ACCEL_MIN_DOCS", "50")
    env = InProcessEnvironment(extra_components=[_fast_cron()])
    await env.start_backing()
    for s in tasks_tracker_specs(frontend=False, api={"OverdueTasks:Query": "range"},
                                 processor={"OverdueTasks:PageSize": page, **(processor or {})}):
        await env.add_app(s)
    await env.wait_ready()
    return env


def test_cron_range_sweep_marks_every_past_due_task(monkeypatch):
    """OverdueTasks:Query=range + paged cron sweep (SURVEY §2.12 #7 fixed): tasks due before
    today -- at any time of day, any number of days back -- are marked overdue page by page by
    the cron job through API -> sidecar -> backing, where the filter runs on the columnar
    accelerator (CPU executor here, gfx950 kernels in the GPU test); completed and future tasks
    stay untouched, and tasks created after the mirror exists are swept too."""
    async def main():
        env = await _range_sweep_env(monkeypatch, "cpu", 7)
        try:
            st = env.backing.store("taskstracker-state-store", "tasksmanagerdb", "taskscollection")
            past = [format_fixed(today() - timedelta(days=d, hours=-h)) for d in (1, 2, 30) for h in (0, 13)]
            fut = format_fixed(today() + timedelta(days=2))
            want = set()
            for i in range(120):
                k, v = _task_doc(i, past[i % len(past)] if i % 3 else fut, done=i % 10 == 1)
                st.set(k, v)
                if i % 3 and i % 10 != 1:
                    want.add(k.split("||")[1])
            c = env.replicas[PROC][0].client

            async def swept():
                res = json.loads(st.query(json.dumps({"filter": {"EQ": {"isOverDue": True}}})))["results"]
                out = {r["data"]["taskId"] for r in res}
                return out if out == want else None
            await _until(swept, timeout=15)
            # a task created through the API afterwards (mirror already built) is swept as well
            r = await c.invoke_method_raw("POST", API, "api/tasks", {"taskName": "late", "taskCreatedBy": "n@x",
                                                                      "taskDueDate": past[-1], "taskAssignedTo": "a@x"})
            tid = r.headers["location"].rsplit("/", 1)[1]
            want.add(tid)
            await _until(swept, timeout=15)
            assert await c.invoke_method("GET", API, "api/overduetasks?limit=5") == []
            acc = env.backing.accel("taskstracker-state-store", "tasksmanagerdb", "taskscollection")
            assert acc.stats["cpu"] >= 2 and acc.stats["fallback"] == 0
        finally:
            await env.stop()
    run(main())


def test_cron_sweep_marks_in_concurrent_chunks(monkeypatch):
    """OverdueTasks:MarkChunk: a page's overdue list goes to markoverdue in concurrent calls of at
    most that many tasks (disjoint), with the same end state as the reference's single call:
    every open past-due task overdue, nothing else touched."""
    async def main():
        env = await _range_sweep_env(monkeypatch, "cpu", 60, {"OverdueTasks:MarkChunk": 7})
        try:
            st = env.backing.store("taskstracker-state-store", "tasksmanagerdb", "taskscollection")
            past = format_fixed(today() - timedelta(days=1))
            fut = format_fixed(today() + timedelta(days=2))
            want = set()
            for i in range(150):
                k, v = _task_doc(i, past if i % 5 else fut, done=i % 11 == 3)
                st.set(k, v)
                if i % 5 and i % 11 != 3:
                    want.add(k.split("||")[1])

            async def swept():
                res = json.loads(st.query(json.dumps({"filter": {"EQ": {"isOverDue": True}}})))["results"]
                out = {r["data"]["taskId"] for r in res}
                return out if out == want else None
            await _until(swept, timeout=15)
            res = json.loads(st.query(json.dumps({"filter": {"EQ": {"isCompleted": True}}})))["results"]
            assert all(not r["data"]["isOverDue"] for r in res)
        finally:
            await env.stop()
    run(main())
