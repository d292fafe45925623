"""Backend processor (app-id ``tasksmanager-backend-processor``, no ingress).

Endpoints (reference SURVEY.md §2.2, §2.11):

* ``POST /api/tasksnotifier/tasksaved`` -- subscriber of ``tasksavedtopic`` on both
  ``dapr-pubsub-servicebus`` and ``taskspubsub`` (reference
  Controllers/TasksNotifierController.cs:23-32).  Modes (``TasksNotifier:Mode``):
    - ``log`` (default, the shipped controller): log and return 200 with a message;
    - ``sendgrid-binding`` (reference docs/aca/06-aca-dapr-bindingsapi/TasksNotifierController.cs:22-77):
      if ``SendGrid:IntegrationEnabled`` send the e-mail through the ``sendgrid`` output
      binding, otherwise simulate ``SendGrid:SimulatedDelayMs`` (1000) of work -- the load
      the KEDA scale-out test relies on; failures return 400 so the broker retries;
    - ``sendgrid-api`` (reference docs/aca/05-aca-dapr-pubsubapi/TasksNotifierController-SendGrid.cs):
      call the SendGrid-compatible HTTP API directly with ``SendGrid:ApiKey``.
* ``POST /ExternalTasksProcessor/process`` -- storage-queue input binding handler
  (reference Controllers/ExternalTasksProcessorController.cs:22-53): create the task via
  the API, then archive it to ``externaltasksblobstore`` as ``<taskId>.json``.  Exceptions
  propagate as 500 so the queue message is retried.  Deviation: the
  blob is named after the id the API actually stored (parsed from its ``Location``
  header), so the archive and the store agree.
* ``POST /ScheduledTasksManager`` -- cron handler (reference
  Controllers/ScheduledTasksManagerController.cs:19-46): fetch yesterday's open tasks,
  keep those with ``runAt.Date > dueDate.Date``, mark them overdue.  With
  ``OverdueTasks:PageSize`` > 0 it sweeps page by page (``GET /api/overduetasks?limit=``)
  until a short page: the API's ``OverdueTasks:Query=range`` mode answers with every open
  task due before today, filtered in the store (GPU columnar scan in the backing services).
  ``OverdueTasks:MarkChunk`` (default 256; 0 = the reference's one call) marks a page in
  concurrent calls of at most that many tasks.
* ``GET /dapr/subscribe`` -- ``MapSubscribeHandler`` (reference Program.cs:33).
"""
from __future__ import annotations

import asyncio
import base64
import json
import logging
import uuid
from datetime import datetime
from pathlib import Path

from ...models import TaskModel, json_array_chunks, naive_utc, overdue_filter_chunks, overdue_filter_wire, task_model_name, tasks_from_json, utcnow
from ...sdk import SidecarClient, cloud_events_middleware, map_subscribe_handler, topic
from ...sdk.client import InvocationError, RawJsonBytes, client_from_config, native_route_failure
from ...web.app import WebApp, read_model
from ...web.http import Request, Response, empty, json_response, text_response
from ..hosting import create_host, map_openapi, run_host

ROLE = "tasksmanager-backend-processor"
API_APP_ID = "tasksmanager-backend-api"
CONTENT_ROOT = Path(__file__).parent
OUTPUT_BINDING_NAME = "externaltasksblobstore"
OUTPUT_BINDING_OPERATION = "create"

log_notifier = logging.getLogger("TasksNotifierController")
log_external = logging.getLogger("ExternalTasksProcessorController")
log_sched = logging.getLogger("ScheduledTasksManagerController")

# consecutive empty pages the API still reports more matches for, before the sweep stops
EMPTY_MORE_LIMIT = 3


# TasksNotifierController.TaskSaved's log line and answer (TasksNotifierController.cs:26-32): the
# Python handler and the app host's native route (apphost.hpp processor_notify) use this text
NOTIFY_LOG = "Started processing message with Task Name '%s'"
# ScheduledTasksManagerController's log lines (ScheduledTasksManagerController.cs:22-40), shared
# with the app host's native sweep route (apphost.hpp processor_sweep)
LOG_TRIGGERED = "ScheduledTasksManager::Timer Services triggered at: %s"
LOG_RETRIEVED = "ScheduledTasksManager::completed query state store for tasks, retrieved tasks count: %d"
LOG_MARKING = "ScheduledTasksManager::marking %d as overdue tasks"
MORE_HEADER = "x-tt-more-results"


def register_controllers(app: WebApp, client: SidecarClient) -> None:
    cfg = app.config
    api_app_id = cfg.get_str("Processor:BackendApiAppId", API_APP_ID)

    # -- TasksNotifierController ----------------------------------------------
    if (cfg.get_str("TasksNotifier:Mode") or "log").lower() == "log":
        # the app host's I/O thread answers the log-mode notification itself when it can: the
        # same native envelope unwrap and binding check, log line and 200 as below
        app.services.setdefault("native_routes", []).append({
            "kind": "processor_notify", "method": "POST", "path": "/api/tasksnotifier/tasksaved",
            "route": "/api/tasksnotifier/tasksaved",
            "cfg": {"log_category": log_notifier.name, "log_notify": NOTIFY_LOG, "log_notify_args": "name",
                    "status": 200, "content_type": "text/plain; charset=utf-8"}})

    @app.route("/api/tasksnotifier/tasksaved", ("POST",), name="TaskSaved", tag="TasksNotifier", body=TaskModel)
    @topic("dapr-pubsub-servicebus", "tasksavedtopic")
    @topic("taskspubsub", "tasksavedtopic")
    async def task_saved(req: Request) -> Response:
        mode = (cfg.get_str("TasksNotifier:Mode") or "log").lower()
        if mode == "log":  # the shipped controller needs the name only: a native binding check
            ctype = req.content_type
            name = task_model_name(req.body) if not ctype or "json" in ctype else None
            if name is not None:
                log_notifier.info(NOTIFY_LOG, name)
                return text_response(NOTIFY_LOG % name)
        t: TaskModel = await read_model(req, TaskModel)
        log_notifier.info(NOTIFY_LOG, t.task_name)
        if mode == "log":
            return text_response(NOTIFY_LOG % t.task_name)
        ok = await send_email(t)
        return empty(200) if ok else Response(b"Failed to send an email", 400, None, "text/plain")

    async def send_email(t: TaskModel) -> bool:
        mode = (cfg.get_str("TasksNotifier:Mode") or "log").lower()
        subject = f"Task '{t.task_name}' is assigned to you!"
        due = naive_utc(t.task_due_date)
        text = (f"Task '{t.task_name}' is assigned to you. Task should be completed by the end of: "
                f"{due.day:02d}/{due.month:02d}/{due.year:04d}")
        try:
            if mode == "sendgrid-api":
                from ...backing.client import BackingClient
                bc = BackingClient(cfg.get_str("SendGrid:Endpoint"), http=client.http)
                await bc.sendgrid_send({"personalizations": [{"to": [{"email": t.task_assigned_to,
                                                                       "name": t.task_assigned_to}], "subject": subject}],
                                        "from": {"email": cfg.get_str("SendGrid:FromEmail", "noreply@taskstracker.local"),
                                                 "name": "Tasks Tracker Notification"},
                                        "content": [{"type": "text/plain", "value": text},
                                                    {"type": "text/html", "value": text}]},
                                       cfg.get_str("SendGrid:ApiKey"))
            elif cfg.get_bool("SendGrid:IntegrationEnabled"):
                await client.invoke_binding("sendgrid", "create", text,
                                            {"emailTo": t.task_assigned_to, "emailToName": t.task_assigned_to,
                                             "subject": subject})
            else:
                log_notifier.info("Simulate slow processing for email sending for Email with Email subject '%s' "
                                  "Email to: '%s'", subject, t.task_assigned_to)
                await asyncio.sleep(cfg.get_int("SendGrid:SimulatedDelayMs", 1000) / 1000.0)
            log_notifier.info("Email with subject '%s' sent to: '%s' successfully", subject, t.task_assigned_to)
            return True
        except Exception as e:
            log_notifier.error("Failed to send email with subject '%s' To: '%s': %s", subject, t.task_assigned_to, e)
            return False

    # -- ExternalTasksProcessorController --------------------------------------
    @app.route("/ExternalTasksProcessor/process", ("POST",), name="ProcessTaskAndStore", tag="ExternalTasksProcessor",
               body=TaskModel)
    async def process_task_and_store(req: Request) -> Response:
        t: TaskModel = await read_model(req, TaskModel)
        log_external.info("Started processing external task message from storage queue. Task Name: '%s'", t.task_name)
        t.task_id = uuid.uuid4()
        t.task_created_on = utcnow()
        r = await client.invoke_method_raw("POST", api_app_id, "api/tasks", t)
        if r.status >= 300:
            raise InvocationError(r.status, r.body, f"invoke {api_app_id}/api/tasks")
        loc = r.headers.get("location", "")
        try:
            t.task_id = uuid.UUID(loc.rstrip("/").rsplit("/", 1)[-1])
        except ValueError:
            pass
        log_external.info("Saved external task to the state store successfully. Task name: '%s', Task Id: '%s'",
                          t.task_name, t.task_id)
        await client.invoke_binding(OUTPUT_BINDING_NAME, OUTPUT_BINDING_OPERATION, t, {"blobName": f"{t.task_id}.json"})
        log_external.info("Invoked output binding '%s' for external task. Task name: '%s', Task Id: '%s'",
                          OUTPUT_BINDING_NAME, t.task_name, t.task_id)
        return empty(200)

    # -- ScheduledTasksManagerController ---------------------------------------
    # OverdueTasks:PageSize > 0 (with the API's OverdueTasks:Query=range): sweep page by page
    # -- a marked page drops out of the API's filter, so each request asks for the next one
    page = cfg.get_int("OverdueTasks:PageSize", 0)
    max_pages = cfg.get_int("OverdueTasks:MaxPages", 100000)
    # OverdueTasks:MarkChunk > 0: a page's overdue list goes to markoverdue in concurrent
    # calls of at most this many tasks (disjoint: the same end state as one call, which is
    # what the reference makes -- 0), so the API's replicas and their sidecars share the work
    chunk = cfg.get_int("OverdueTasks:MarkChunk", 256)
    overdue_path = "api/overduetasks" + (f"?limit={page}" if page > 0 else "")
    mark_path = "api/overduetasks/markoverdue"
    sweep_what = {"overdue": f"invoke {api_app_id}/{overdue_path}", "mark": f"invoke {api_app_id}/{mark_path}"}
    ep = client.native_endpoint() if chunk > 0 and hasattr(client, "native_endpoint") else None
    if ep is not None and ep.get("protocol", "http") == "http":
        # the job on the app host's I/O thread: the same loop, filter, chunks, log lines and summary
        app.services.setdefault("native_routes", []).append({
            "kind": "processor_sweep", "method": "POST", "path": "/ScheduledTasksManager",
            "route": "/ScheduledTasksManager",
            "cfg": {"sidecar": ep["sidecar"], "token": ep["token"], "timeout": ep["timeout"],
                    "overdue_target": f"{ep['prefix']}/v1.0/invoke/{api_app_id}/method/{overdue_path}",
                    "mark_target": f"{ep['prefix']}/v1.0/invoke/{api_app_id}/method/{mark_path}",
                    "page": page, "max_pages": max_pages, "chunk": chunk, "empty_more_limit": EMPTY_MORE_LIMIT,
                    "more_header": MORE_HEADER, "log_category": log_sched.name,
                    "log_triggered": LOG_TRIGGERED, "log_retrieved": LOG_RETRIEVED.replace("%d", "%s"),
                    "log_marking": LOG_MARKING.replace("%d", "%s"),
                    "status": 200, "content_type": "application/json; charset=utf-8"}})

    @app.route("/ScheduledTasksManager", ("POST",), name="CheckOverDueTasksJob", tag="ScheduledTasksManager")
    async def check_overdue_tasks_job(req: Request) -> Response:
        note = req.state.get("tt_native") or ""
        if note.startswith("resume "):
            # the native route ran the job up to a page its filter does not read: go on from there
            st = json.loads(base64.b64decode(note[7:]))
            run_at = datetime.fromisoformat(st["runAt"])
            retrieved, marked, pages, empty_more = st["retrieved"], st["marked"], st["pages"], st["emptyMore"]
            t_query, t_mark = float(st["queryS"]), float(st["markS"])
        else:
            failed = native_route_failure(req, sweep_what)
            if failed is not None:  # a call the native route made failed: the same error
                raise failed
            run_at = utcnow()
            log_sched.info(LOG_TRIGGERED, run_at)
            retrieved = marked = pages = empty_more = 0
            t_query = t_mark = 0.0  # wall time of the job's two hops (returned for attribution)
        run_day = naive_utc(run_at).date().isoformat()
        clock = asyncio.get_running_loop().time
        while pages < max_pages:
            pages += 1
            path = overdue_path
            t0 = clock()
            r = await client.invoke_method_raw("GET", api_app_id, path)
            t_query += clock() - t0
            if r.status >= 300:
                raise InvocationError(r.status, r.body, f"invoke {api_app_id}/{path}")
            # the page bound and filtered in one native pass (with MarkChunk, also cut into the
            # markoverdue chunks); any other shape binds with TaskModel
            parts = None
            if (fast := overdue_filter_chunks(r.body, run_day, chunk) if r.body and chunk > 0 else None) is not None:
                n_page, n_overdue, parts = fast
                overdue = parts[0] if len(parts) == 1 else None
            elif (fast := overdue_filter_wire(r.body, run_day) if r.body else None) is not None:
                n_page, n_overdue, overdue = fast
            else:
                tasks = tasks_from_json(r.body or b"[]")
                overdue = [t for t in tasks if naive_utc(run_at).date() > naive_utc(t.task_due_date).date()]
                n_page, n_overdue = len(tasks), len(overdue)
            retrieved += n_page
            log_sched.info(LOG_RETRIEVED, n_page)
            if n_overdue:
                log_sched.info(LOG_MARKING, n_overdue)
                if parts is None and isinstance(overdue, bytes) and 0 < chunk < n_overdue:
                    parts = json_array_chunks(overdue, chunk)
                t0 = clock()
                if parts and len(parts) > 1:
                    results = await asyncio.gather(*(client.invoke_method("POST", api_app_id, mark_path,
                                                                          RawJsonBytes(p)) for p in parts),
                                                   return_exceptions=True)
                    for res in results:  # every call has finished: the first failure fails the job
                        if isinstance(res, BaseException):
                            raise res
                else:
                    data = RawJsonBytes(overdue) if isinstance(overdue, bytes) else overdue
                    await client.invoke_method("POST", api_app_id, mark_path, data)
                t_mark += clock() - t0
                marked += n_overdue
            if page <= 0:
                break
            more = (r.headers.get(MORE_HEADER) or "").lower()
            if more:  # the API says whether the store holds more matches than this page
                # a short (even empty) page with more matches: rows that changed after the
                # store's selection were skipped -- ask again; a page of nothing to mark stops
                if more != "true" or (n_page and not n_overdue):
                    break
                if not n_page:  # empty yet "more": a few retries, paced, then stop (no hot loop)
                    empty_more += 1
                    if empty_more >= EMPTY_MORE_LIMIT:
                        break
                    await asyncio.sleep(0.005 * empty_more)
                else:
                    empty_more = 0
            elif n_page < page or not n_overdue:
                break
        return json_response({"runAt": run_at.isoformat(), "retrieved": retrieved, "markedOverdue": marked,
                              "pages": pages, "emptyMorePages": empty_more, "queryMs": round(t_query * 1e3, 2),
                              "markMs": round(t_mark * 1e3, 2)})


def create_app(argv: list[str] | None = None, client: SidecarClient | None = None, config=None,
               overrides: dict | None = None) -> WebApp:
    app = create_host(ROLE, CONTENT_ROOT, argv, config=config, overrides=overrides)
    app.openapi_info = {"title": "TasksTracker.Processor.Backend.Svc | v1", "version": "1.0.0"}
    client = client or client_from_config(app.config)
    app.services["dapr"] = client
    app.use(cloud_events_middleware())  # app.UseCloudEvents()
    register_controllers(app, client)
    map_subscribe_handler(app)          # app.MapSubscribeHandler()
    map_openapi(app)

    async def _close() -> None:
        await client.close()
    app.on_shutdown.append(_close)
    return app


def main(argv: list[str] | None = None) -> None:
    import sys
    run_host(create_app(sys.argv[1:] if argv is None else argv))


if __name__ == "__main__":
    main()
