"""Backend API (app-id ``tasksmanager-backend-api``).

Routes (reference SURVEY.md §2.11):

=======  ==================================  ======================================  ==========================
verb     route                               result                                  reference
=======  ==================================  ======================================  ==========================
GET      /api/tasks?createdBy=               200 [TaskModel] newest first            TasksController.cs:20-24
GET      /api/tasks/{taskId}                 200 TaskModel / 404 / 400 bad guid      TasksController.cs:26-32
POST     /api/tasks                          201 + Location, empty body              TasksController.cs:34-46
PUT      /api/tasks/{taskId}                 200 / 400                               TasksController.cs:48-59
PUT      /api/tasks/{taskId}/markcomplete    200 / 400                               TasksController.cs:61-67
DELETE   /api/tasks/{taskId}                 200 / 404                               TasksController.cs:69-75
GET      /api/overduetasks                   200 [TaskModel] oldest first            OverdueTasksController.cs:20-24
POST     /api/overduetasks/markoverdue       200                                     OverdueTasksController.cs:26-32
GET      /openapi/v1.json                    OpenAPI (Development only)              Program.cs:16,21-24
=======  ==================================  ======================================  ==========================

The manager implementation is chosen by ``TasksManager:Backend`` (``fake`` | ``store``).
The reference hard-wires the fake (Program.cs:13) while its module-4 docs wire the
store (docs/aca/04-aca-dapr-stateapi/Program-dotnet9.cs:7-9); here the default is
``store`` when a sidecar is configured (``DAPR_HTTP_PORT`` / ``TT_SIDECAR_UDS``) and
``fake`` otherwise, so ``python -m ...backend_api`` alone reproduces module 1.
"""
from __future__ import annotations

import logging
import os
import uuid
from pathlib import Path

from ...models import TaskAddModel, TaskModel, TaskUpdateModel, tasks_to_json
from ...models.dotnet import is_guid
from ...sdk.client import client_from_config, native_route_failure
from ...web.app import WebApp, read_model
from ...web.http import HTTPError, Request, Response, empty
from ..hosting import create_host, map_openapi, run_host
from .managers import FakeTasksManager, TasksManager, TasksStoreManager

ROLE = "tasksmanager-backend-api"
CONTENT_ROOT = Path(__file__).parent
log = logging.getLogger("TasksController")
MORE_HEADER = "x-tt-more-results"  # GET api/overduetasks?limit= in range mode: the store has more matches


def _task_id(req: Request) -> uuid.UUID:
    raw = req.path_params["taskId"]
    if not is_guid(raw):
        raise HTTPError(400, detail={"taskId": [f"The value '{raw}' is not valid."]})
    return uuid.UUID(raw.strip("{}"))


def _json(body: bytes, status: int = 200) -> Response:
    return Response(body, status, None, "application/json; charset=utf-8")


# TasksController.Post's answer (TasksController.cs:44): ``CreatedAtAction`` -> 201 + Location.
# The Python handler and the app host's native route (apphost.hpp) both answer from these.
CREATED_STATUS = 201
CREATED_LOCATION = "/api/tasks/%s"


def register_controllers(app: WebApp, manager: TasksManager) -> None:
    fast_list = getattr(manager, "tasks_by_creator_json", None)
    list_native = getattr(manager, "native_list_route", None)
    if os.environ.get("TT_READ_PATH", "").lower() == "bind":  # A/B: bind a TaskModel per task
        fast_list = list_native = None
    overdue_native = getattr(manager, "native_overdue_route", None)
    overdue_spec = overdue_native() if overdue_native is not None and getattr(manager, "overdue_page_json", None) \
        else None
    overdue_what = overdue_spec.pop("what") if overdue_spec else {}
    if overdue_spec:
        # GET api/overduetasks on the app host's I/O thread: the manager's range query and log line
        overdue_spec["cfg"].update({"status": 200, "content_type": "application/json; charset=utf-8",
                                    "more_header": MORE_HEADER})
        app.services.setdefault("native_routes", []).append(overdue_spec)
    list_spec = list_native() if fast_list is not None and list_native is not None else None
    list_what = list_spec.pop("what") if list_spec else {}
    if list_spec:
        # GET api/tasks on the app host's I/O thread: the manager's query, the same codec
        list_spec["cfg"].update({"status": 200, "content_type": "application/json; charset=utf-8"})
        app.services.setdefault("native_routes", []).append(list_spec)
    # -- TasksController (reference Controllers/TasksController.cs) --------------
    @app.route("/api/tasks", ("GET",), name="GetTasks", query=["createdBy"], tag="Tasks",
               responses={200: [TaskModel]})
    async def get_tasks(req: Request) -> Response:
        failed = native_route_failure(req, list_what) if list_what else None
        if failed is not None:  # the native route's query failed: the SDK's error
            raise failed
        created_by = req.query_get("createdBy") or ""
        if fast_list is not None:
            body = await fast_list(created_by)
            if body is not None:
                return _json(body)
        return _json(tasks_to_json(await manager.get_tasks_by_creator(created_by)))

    fast_get = getattr(manager, "get_task_json", None)
    fast_update = getattr(manager, "update_task_from_body", None)
    fast_complete = getattr(manager, "mark_task_completed_fast", None)
    task_routes = getattr(manager, "native_task_routes", None)
    task_what: dict[str, dict] = {}
    for spec in (task_routes() if task_routes is not None and os.environ.get("TT_READ_PATH", "").lower() != "bind"
                 else []):
        # GET / PUT / PUT markcomplete / DELETE api/tasks/{id} on the app host's I/O thread: the
        # same codec passes, sidecar calls, log lines and answers as the handlers below
        task_what[spec["kind"]] = spec.pop("what")
        spec["cfg"].update({"status": 200, "content_type": "application/json; charset=utf-8"})
        app.services.setdefault("native_routes", []).append(spec)

    def _failed(req: Request, kind: str) -> None:
        what = task_what.get(kind)
        failed = native_route_failure(req, what, req.path_params.get("taskId")) if what else None
        if failed is not None:  # the native route's sidecar call failed: the SDK's error
            raise failed

    @app.route("/api/tasks/{taskId}", ("GET",), name="GetTask", tag="Tasks", responses={200: TaskModel, 404: None})
    async def get_task(req: Request) -> Response:
        _failed(req, "api_get")
        tid = _task_id(req)
        if fast_get is not None:  # the stored document -> TaskModel JSON in one native pass
            body = await fast_get(tid)
            if body is not False:
                return empty(404) if body is None else _json(body)
        t = await manager.get_task_by_id(tid)
        if t is None:
            return empty(404)
        return _json(t.model_dump_json(by_alias=True).encode())

    fast_create = getattr(manager, "create_new_task_from_body", None)
    fast_mark = getattr(manager, "mark_overdue_from_body", None)
    fast_page = getattr(manager, "overdue_page_json", None)
    native = getattr(manager, "native_create_route", None)
    spec = native() if fast_create is not None and native is not None else None
    create_what = spec.pop("what") if spec else {}
    if spec:
        spec["cfg"].update({"status": CREATED_STATUS, "location": CREATED_LOCATION, "location_args": "id"})
        # the app host's I/O thread serves POST api/tasks end to end when it can: the same
        # native codec, log lines, state save and event as create_new_task_from_body, the same
        # 201; the rest (bodies for the general binder, sampled traces, a failed sidecar call)
        # comes to this handler
        app.services.setdefault("native_routes", []).append(spec)

    @app.route("/api/tasks", ("POST",), name="CreateTask", tag="Tasks", body=TaskAddModel, responses={201: None})
    async def post_task(req: Request) -> Response:
        failed = native_route_failure(req, create_what) if create_what else None
        if failed is not None:  # the native route's save or publish failed: the SDK's error
            raise failed
        ctype = req.content_type
        if fast_create is not None and (not ctype or "json" in ctype):  # one native pass over the body
            tid = await fast_create(req.body)
            if tid is not None:
                return Response(b"", CREATED_STATUS, [("Location", CREATED_LOCATION % tid)])
        m: TaskAddModel = await read_model(req, TaskAddModel)
        tid = await manager.create_new_task(m.task_name, m.task_created_by, m.task_assigned_to, m.task_due_date)
        return Response(b"", CREATED_STATUS, [("Location", CREATED_LOCATION % tid)])

    @app.route("/api/tasks/{taskId}", ("PUT",), name="UpdateTask", tag="Tasks", body=TaskUpdateModel,
               responses={200: None, 400: None})
    async def put_task(req: Request) -> Response:
        _failed(req, "api_update")
        tid = _task_id(req)
        ctype = req.content_type
        if fast_update is not None and (not ctype or "json" in ctype):  # binder + RMW codec, one pass each
            ok = await fast_update(tid, req.body)
            if ok is not None:
                return empty(200) if ok else empty(400)
        m: TaskUpdateModel = await read_model(req, TaskUpdateModel)
        ok = await manager.update_task(tid, m.task_name, m.task_assigned_to, m.task_due_date)
        return empty(200) if ok else empty(400)

    @app.route("/api/tasks/{taskId}/markcomplete", ("PUT",), name="MarkComplete", tag="Tasks",
               responses={200: None, 400: None})
    async def mark_complete(req: Request) -> Response:
        _failed(req, "api_complete")
        tid = _task_id(req)
        ok = await fast_complete(tid) if fast_complete is not None else None
        if ok is None:
            ok = await manager.mark_task_completed(tid)
        return empty(200) if ok else empty(400)

    @app.route("/api/tasks/{taskId}", ("DELETE",), name="DeleteTask", tag="Tasks", responses={200: None, 404: None})
    async def delete_task(req: Request) -> Response:
        _failed(req, "api_delete")
        ok = await manager.delete_task(_task_id(req))
        return empty(200) if ok else empty(404)

    # -- OverdueTasksController (reference Controllers/OverdueTasksController.cs) --
    @app.route("/api/overduetasks", ("GET",), name="GetOverdueTasks", tag="OverdueTasks", query=["limit"],
               responses={200: [TaskModel]})
    async def get_overdue(req: Request) -> Response:
        failed = native_route_failure(req, overdue_what) if overdue_what else None
        if failed is not None:  # the native route's query failed: the SDK's error
            raise failed
        raw = req.query_get("limit") or ""
        limit = int(raw) if raw.isdigit() else None  # page size of the range sweep (OverdueTasks:Query=range)
        if fast_page is not None:
            made = await fast_page(limit)
            if made is not None:
                # the sweep pages until the store reports no more matches, not until a short page:
                # rows changed since the store's selection are skipped and shorten a page
                resp = _json(made[0])
                resp.headers.append((MORE_HEADER, "true" if made[1] else "false"))
                return resp
        return _json(tasks_to_json(await manager.get_yesterdays_due_tasks(limit)))

    mark_native = getattr(manager, "native_markoverdue_route", None)
    mark_spec = mark_native() if mark_native is not None and fast_mark is not None else None
    mark_what = mark_spec.pop("what") if mark_spec else {}
    if mark_spec:
        # POST markoverdue on the app host's I/O thread: the same binder, conditional mark pass,
        # log lines and bulk save as mark_overdue_from_body
        mark_spec["cfg"].update({"status": 200})
        app.services.setdefault("native_routes", []).append(mark_spec)

    @app.route("/api/overduetasks/markoverdue", ("POST",), name="MarkOverdue", tag="OverdueTasks",
               body=[TaskModel], responses={200: None})
    async def mark_overdue(req: Request) -> Response:
        failed = native_route_failure(req, mark_what) if mark_what else None
        if failed is not None:  # the native route's bulk get or save failed: the SDK's error
            raise failed
        ctype = req.content_type
        if fast_mark is not None and (not ctype or "json" in ctype) and await fast_mark(req.body):
            return empty(200)
        tasks = await read_model(req, [TaskModel])
        await manager.mark_overdue_tasks(tasks)
        return empty(200)


def select_manager(config) -> TasksManager:
    backend = (config.get_str("TasksManager:Backend") or "").lower()
    has_sidecar = bool(config.get_str("DAPR_HTTP_PORT") or config.get_str("TT_SIDECAR_UDS")
                       or config.get_str("DAPR_HTTP_ENDPOINT"))
    if not backend:
        backend = "store" if has_sidecar else "fake"
    if backend == "fake":
        return FakeTasksManager()
    if backend == "store":
        return TasksStoreManager.from_config(client_from_config(config), config)
    raise ValueError(f"unknown TasksManager:Backend {backend!r}")


def create_app(argv: list[str] | None = None, manager: TasksManager | None = None, config=None,
               overrides: dict | None = None) -> WebApp:
    app = create_host(ROLE, CONTENT_ROOT, argv, config=config, overrides=overrides)
    app.openapi_info = {"title": "TasksTracker.TasksManager.Backend.Api | v1", "version": "1.0.0"}
    if manager is None:
        manager = select_manager(app.config)
    app.services["tasks_manager"] = manager
    register_controllers(app, manager)
    map_openapi(app)
    return app


def main(argv: list[str] | None = None) -> None:
    import sys
    run_host(create_app(sys.argv[1:] if argv is None else argv))


if __name__ == "__main__":
    main()
