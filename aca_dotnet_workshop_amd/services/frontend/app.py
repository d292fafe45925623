"""Web portal (app-id ``tasksmanager-frontend-webapp``, external ingress).

Razor-Pages equivalent rendered with Jinja2 (reference SURVEY.md §2.3):

==================================  ==========================================================
page                                reference
==================================  ==========================================================
``GET/POST /``                      Pages/Index.cshtml(.cs): e-mail form -> ``TasksCreatedByCookie``
``GET /Tasks/Index``                Pages/Tasks/Index.cshtml(.cs):23-55 (cookie or redirect to /)
``POST /Tasks/Index?handler=...``   OnPostDeleteAsync / OnPostCompleteAsync (:57-71)
``GET/POST /Tasks/Create``          Pages/Tasks/Create.cshtml(.cs) with ``[Required]`` validation
``GET/POST /Tasks/Edit/{id:guid}``  Pages/Tasks/Edit.cshtml(.cs)
``/Privacy``, ``/Error``            Pages/Privacy, Pages/Error (RequestId = trace id)
==================================  ==========================================================

Backend access (``Frontend:BackendMode``):
* ``dapr`` (default; reference Index.cshtml.cs:48) -- ``DaprClient.InvokeMethodAsync`` via the sidecar;
* ``http`` (module-2 variant, reference docs/aca/02-aca-comm/Tasks.Index.cshtml.cs:20-48) -- a
  named HTTP client on ``BackendApiConfig:BaseUrlExternalHttp`` (required in this mode, as the
  reference's startup check, Program.cs:15-27).

Antiforgery: like Razor Pages, POSTs to ``/Tasks/*`` must carry a token bound to the
antiforgery cookie; the landing page opts out (``[IgnoreAntiforgeryToken]``, Index.cshtml.cs:7).
"""
from __future__ import annotations

import hashlib
import json
import hmac
import logging
import os
import secrets
from pathlib import Path
from typing import Any
from urllib.parse import quote

from jinja2 import Environment, FileSystemLoader, select_autoescape

from ...models import FIELD_DISPLAY, REQUIRED_FIELDS, TaskModel, parse_datetime, tasks_from_json
from ...models.dotnet import is_guid, naive_utc
from ...sdk import SidecarClient
from ...sdk.client import RawJson, native_route_failure
from ...web.app import WebApp
from ...web.client import HttpClient
from ...web.http import HTTPError, Request, Response, redirect
from ..hosting import create_host, run_host

ROLE = "tasksmanager-frontend-webapp"
API_APP_ID = "tasksmanager-backend-api"
COOKIE = "TasksCreatedByCookie"
AF_COOKIE = ".AspNetCore.Antiforgery"
AF_FIELD = "__RequestVerificationToken"
HERE = Path(__file__).parent
log = logging.getLogger("Frontend")


class BackendGateway:
    """The two ways the reference's pages reach the API."""

    def __init__(self, mode: str, client: SidecarClient | None, base_url: str | None) -> None:
        self.mode = mode
        self.dapr = client
        self.base = (base_url or "").rstrip("/")
        self.http = HttpClient() if mode == "http" else None

    async def call(self, method: str, path: str, data: Any = None) -> Any:
        if self.mode == "dapr":
            return await self.dapr.invoke_method(method, API_APP_ID, path, data)
        import json
        from ...sdk.client import InvocationError, to_jsonable
        body = json.dumps(to_jsonable(data)).encode() if data is not None else None
        r = await self.http.request(method, f"{self.base}/{path.lstrip('/')}", body=body,
                                    headers={"Content-Type": "application/json"} if body else None)
        if r.status >= 300:
            raise InvocationError(r.status, r.body, f"{method} {path}")
        return r.json() if r.body else None

    async def close(self) -> None:
        if self.dapr is not None:
            await self.dapr.close()
        if self.http is not None:
            await self.http.close()


class Antiforgery:
    def __init__(self, key: bytes) -> None:
        self.key = key

    def token_for(self, cookie: str) -> str:
        return hmac.new(self.key, cookie.encode(), hashlib.sha256).hexdigest()

    def ensure_cookie(self, req: Request, resp: Response) -> str:
        c = req.cookies.get(AF_COOKIE)
        if not c:
            c = secrets.token_hex(16)
            resp.set_cookie(AF_COOKIE, c, httponly=True, samesite="strict")
        return c

    def validate(self, req: Request, form: dict[str, str]) -> bool:
        c = req.cookies.get(AF_COOKIE)
        t = form.get(AF_FIELD) or req.headers.get("requestverificationtoken")
        return bool(c and t and hmac.compare_digest(self.token_for(c), t))


def _fmt_date(dt) -> str:
    d = naive_utc(dt)
    return f"{d.day:02d}-{d.month:02d}-{d.year:04d}"


def _input_date(dt) -> str:
    d = naive_utc(dt)
    return f"{d.year:04d}-{d.month:02d}-{d.day:02d}"


# CreateModel.OnPostAsync's answer (Create.cshtml.cs:50, ``RedirectToPage("./Index")``): the
# page's handler and the app host's native route (apphost.hpp frontend_create) both use it
CREATED_REDIRECT = (302, "/Tasks/Index")


def create_app(argv: list[str] | None = None, client: SidecarClient | None = None, config=None,
               overrides: dict | None = None) -> WebApp:
    app = create_host(ROLE, HERE, argv, config=config, overrides=overrides)
    cfg = app.config
    mode = (cfg.get_str("Frontend:BackendMode") or "dapr").lower()
    base = cfg.get_str("BackendApiConfig:BaseUrlExternalHttp")
    if mode == "http" and not base:
        raise RuntimeError("BackendApiConfig:BaseUrlExternalHttp is not defined in App Settings.")
    gw = BackendGateway(mode, client or (SidecarClient() if mode == "dapr" else None), base)
    app.services["backend"] = gw
    af = Antiforgery((cfg.get_str("Frontend:AntiforgeryKey") or secrets.token_hex(32)).encode())
    env = Environment(loader=FileSystemLoader(str(HERE / "templates")), autoescape=select_autoescape(["html"]))
    env.filters["ddmmyyyy"] = _fmt_date
    env.filters["inputdate"] = _input_date
    app.mount_static("/", HERE / "wwwroot")
    from .rows import RowRenderer
    rows = RowRenderer(env)  # Tasks/Index's rows compiled from the template's own task_row macro
    if os.environ.get("TT_READ_PATH", "").lower() == "bind":  # A/B: TaskModel per task + template loop
        rows.ok = False

    def render(req: Request, name: str, status: int = 200, **ctx: Any) -> Response:
        resp = Response(b"", status, None, "text/html; charset=utf-8")
        cookie = af.ensure_cookie(req, resp)
        ctx.setdefault("title", "Tasks Tracker")
        html = env.get_template(name).render(af_field=AF_FIELD, af_token=af.token_for(cookie), request=req, **ctx)
        resp.body = html.encode()
        return resp

    def require_af(req: Request, form: dict[str, str]) -> None:
        if not af.validate(req, form):
            raise HTTPError(400, detail="The antiforgery token could not be validated.")

    # non-development: exception handler page (reference Program.cs:32-37)
    if not app.is_development:
        async def error_page(req: Request, nxt) -> Response:
            try:
                resp = await nxt(req)
            except HTTPError:
                raise
            except Exception:
                log.exception("unhandled error on %s", req.path)
                return render(req, "error.html", 500, request_id=req.state.get("trace_id", ""))
            return resp
        app.use(error_page)

    # -- Index (landing) --------------------------------------------------------
    @app.route("/", ("GET",), name="Index", include_in_schema=False)
    async def index_get(req: Request) -> Response:
        return render(req, "index.html")

    @app.route("/", ("POST",), name="IndexPost", include_in_schema=False)
    async def index_post(req: Request) -> Response:
        email = req.form().get("TasksCreatedBy", "").strip()
        resp = redirect("/Tasks/Index")
        if email:
            resp.set_cookie(COOKIE, email)
        return resp

    # -- Tasks/Index ----------------------------------------------------------
    @app.route("/Tasks/Index", ("GET",), name="TasksIndex", include_in_schema=False)
    @app.route("/Tasks", ("GET",), name="TasksIndexShort", include_in_schema=False)
    async def tasks_index(req: Request) -> Response:
        created_by = req.cookies.get(COOKIE)
        if not created_by:
            return redirect("/")
        failed = native_route_failure(req, {"invoke": f"invoke {API_APP_ID}/api/tasks?createdBy={quote(created_by)}"})
        if failed is not None:  # the native route's invoke failed: the SDK's error, as below
            raise failed
        data = await gw.call("GET", f"api/tasks?createdBy={quote(created_by)}")
        fast = rows.render(data)
        if fast is not None:
            return render(req, "tasks_index.html", rows_html=fast, created_by=created_by)
        return render(req, "tasks_index.html", tasks=tasks_from_json(data), created_by=created_by)

    index_form = _native_fn("frontend_index_form") if mode == "dapr" else None
    edit_form = _native_fn("frontend_edit_form") if mode == "dapr" else None

    @app.route("/Tasks/Index", ("POST",), name="TasksIndexPost", include_in_schema=False)
    async def tasks_index_post(req: Request) -> Response:
        failed = native_route_failure(req, {"invoke": "invoke {key}"}, _index_invoke_path(req))
        if failed is not None:  # the native route's invoke failed: the SDK's error, as below
            raise failed
        if index_form is not None and index_form(req.body, (req.headers.get("cookie") or "").encode(), af.key) is True:
            form = {}  # the antiforgery check passed in the native pass; handler and id from the query
        else:
            form = req.form()
            require_af(req, form)
        handler = (req.query_get("handler") or form.get("handler") or "").lower()
        tid = req.query_get("id") or form.get("id") or ""
        if not is_guid(tid):
            raise HTTPError(400, detail="invalid id")
        if handler == "delete":
            await gw.call("DELETE", f"api/tasks/{tid}")
        elif handler == "complete":
            await gw.call("PUT", f"api/tasks/{tid}/markcomplete")
        else:
            raise HTTPError(400, detail=f"unknown handler {handler!r}")
        return redirect("/Tasks/Index")

    # -- Tasks/Create -----------------------------------------------------------
    @app.route("/Tasks/Create", ("GET",), name="TasksCreate", include_in_schema=False)
    async def create_get(req: Request) -> Response:
        if not req.cookies.get(COOKIE):
            return redirect("/")
        return render(req, "tasks_create.html", values={}, errors={}, display=FIELD_DISPLAY)

    fast_form = _native_form() if mode == "dapr" else None
    create_what = {"invoke": f"invoke {API_APP_ID}/api/tasks"}
    ep = gw.dapr.native_endpoint() if fast_form is not None and isinstance(gw.dapr, SidecarClient) else None
    if ep is not None:
        # the app host's I/O thread serves this post end to end when it can: the same native
        # form binding as below, the same invoke through the sidecar, the same 302; the rest
        # (binding errors, bad tokens, sampled traces, a failed invoke) comes to this handler
        app.services.setdefault("native_routes", []).append({
            "kind": "frontend_create", "method": "POST", "path": "/Tasks/Create", "route": "/Tasks/Create",
            "cfg": {"sidecar": ep["sidecar"], "token": ep["token"], "timeout": ep["timeout"],
                    "af_key": af.key.decode(), "af_cookie": AF_COOKIE, "id_cookie": COOKIE,
                    "invoke_target": f"{ep['prefix']}/v1.0/invoke/{API_APP_ID}/method/api/tasks",
                    "status": CREATED_REDIRECT[0], "location": CREATED_REDIRECT[1]}})

    if ep is not None and rows.ok:
        # GET Tasks/Index on the app host's I/O thread: the same cookies, the same invoke, the
        # page from the templates' own pieces (rows.py); the rest -- no identity, a new
        # antiforgery cookie, an answer outside the rows' shape, a failed invoke -- comes here
        page = rows.page_pieces(env, "tasks_index.html", af_field=AF_FIELD, request=None, title="Tasks Tracker")
        if page is not None:
            app.services.setdefault("native_routes", []).append({
                "kind": "frontend_list", "method": "GET", "path": "/Tasks/Index", "route": "/Tasks/Index",
                "cfg": {"sidecar": ep["sidecar"], "token": ep["token"], "timeout": ep["timeout"],
                        "af_key": af.key.decode(), "af_cookie": AF_COOKIE, "id_cookie": COOKIE,
                        "list_target": f"{ep['prefix']}/v1.0/invoke/{API_APP_ID}/method/api/tasks?createdBy=",
                        "status": 200, "content_type": "text/html; charset=utf-8", "page": json.dumps(page),
                        **{k: json.dumps(v) for k, v in rows.row_pieces().items()}}})

    @app.route("/Tasks/Create", ("POST",), name="TasksCreatePost", include_in_schema=False)
    async def create_post(req: Request) -> Response:
        failed = native_route_failure(req, create_what)
        if failed is not None:  # the native route's invoke failed: the SDK's error, as below
            raise failed
        if fast_form is not None:  # form, cookies, antiforgery and binding in one native pass
            made = fast_form(req.body, (req.headers.get("cookie") or "").encode(), af.key)
            if made is not None and made[0]:
                await gw.call("POST", "api/tasks", RawJson(made[1].decode()))
                return redirect(CREATED_REDIRECT[1], CREATED_REDIRECT[0])
        form = req.form()
        require_af(req, form)
        values, errors = _bind(form, "TaskAdd")
        if errors:
            return render(req, "tasks_create.html", 200, values=values, errors=errors, display=FIELD_DISPLAY)
        created_by = req.cookies.get(COOKIE)
        if created_by:
            await gw.call("POST", "api/tasks", {"taskName": values["taskName"], "taskCreatedBy": created_by,
                                                "taskDueDate": values["taskDueDate"], "taskAssignedTo": values["taskAssignedTo"]})
        return redirect(CREATED_REDIRECT[1], CREATED_REDIRECT[0])

    # -- Tasks/Edit ---------------------------------------------------------------
    if ep is not None:
        # the Edit page and the Index / Edit posts on the app host's I/O thread: the same cookies,
        # antiforgery check and form binding (formcodec.hpp), the same invoke, the same page from
        # the template's own pieces (rows.py edit_page_pieces) or 302; the rest comes here
        inv = f"{ep['prefix']}/v1.0/invoke/{API_APP_ID}/method/api/tasks/"
        common = {"sidecar": ep["sidecar"], "token": ep["token"], "timeout": ep["timeout"], "af_key": af.key.decode(),
                  "af_cookie": AF_COOKIE, "id_cookie": COOKIE, "invoke_target": inv}
        edit_page = rows.edit_page_pieces(env, "tasks_edit.html", af_field=AF_FIELD, request=None, title="Tasks Tracker",
                                          errors={}, display=FIELD_DISPLAY)
        if edit_page is not None and rows.ok:
            app.services.setdefault("native_routes", []).append({
                "kind": "frontend_edit_get", "method": "GET", "path": "/Tasks/Edit/{id}", "route": "/Tasks/Edit/{id}",
                "cfg": {**common, "status": 200, "content_type": "text/html; charset=utf-8", "page": json.dumps(edit_page)}})
        if edit_form is not None:
            app.services.setdefault("native_routes", []).append({
                "kind": "frontend_edit", "method": "POST", "path": "/Tasks/Edit/{id}", "route": "/Tasks/Edit/{id}",
                "cfg": {**common, "status": 302, "location": "/Tasks/Index"}})
        if index_form is not None:
            app.services.setdefault("native_routes", []).append({
                "kind": "frontend_index_post", "method": "POST", "path": "/Tasks/Index", "route": "/Tasks/Index",
                "cfg": {**common, "status": 302, "location": "/Tasks/Index"}})

    @app.route("/Tasks/Edit/{id:guid}", ("GET",), name="TasksEdit", include_in_schema=False)
    async def edit_get(req: Request) -> Response:
        if not req.cookies.get(COOKIE):
            return redirect("/")
        path = f"api/tasks/{req.path_params['id']}"
        failed = native_route_failure(req, {"invoke": f"invoke {API_APP_ID}/{path}"})
        if failed is not None:  # the native route's invoke failed: the SDK's error, as below
            raise failed
        data = await gw.call("GET", path)
        if not data:
            return render(req, "not_found.html", 404)
        values = rows.edit_values(data) if rows.ok else None  # the plain shape: no TaskModel
        if values is None:
            t = TaskModel.model_validate(data)
            values = {"taskId": str(t.task_id), "taskName": t.task_name, "taskAssignedTo": t.task_assigned_to,
                      "taskDueDate": _input_date(t.task_due_date)}
        return render(req, "tasks_edit.html", values=values, errors={}, display=FIELD_DISPLAY)

    @app.route("/Tasks/Edit/{id:guid}", ("POST",), name="TasksEditPost", include_in_schema=False)
    async def edit_post(req: Request) -> Response:
        failed = native_route_failure(req, {"invoke": "invoke {key}"}, _edit_invoke_path(req))
        if failed is not None:  # the native route's invoke failed: the SDK's error, as below
            raise failed
        if edit_form is not None:  # antiforgery, binding and the PUT body in one native pass
            made = edit_form(req.body, (req.headers.get("cookie") or "").encode(), af.key, str(req.path_params["id"]))
            if made is not None:
                if not made[0]:
                    raise HTTPError(400, detail="The antiforgery token could not be validated.")
                await gw.call("PUT", f"api/tasks/{made[2]}", RawJson(made[1].decode()))
                return redirect("/Tasks/Index")
        form = req.form()
        require_af(req, form)
        values, errors = _bind(form, "TaskUpdate")
        values["taskId"] = form.get("TaskUpdate.TaskId") or str(req.path_params["id"])
        if errors:
            return render(req, "tasks_edit.html", 200, values=values, errors=errors, display=FIELD_DISPLAY)
        await gw.call("PUT", f"api/tasks/{values['taskId']}", {"taskId": values["taskId"], "taskName": values["taskName"],
                                                              "taskDueDate": values["taskDueDate"],
                                                              "taskAssignedTo": values["taskAssignedTo"]})
        return redirect("/Tasks/Index")

    # -- Privacy / Error -----------------------------------------------------------
    @app.route("/Privacy", ("GET",), name="Privacy", include_in_schema=False)
    async def privacy(req: Request) -> Response:
        return render(req, "privacy.html", title="Privacy Policy")

    @app.route("/Error", ("GET",), name="Error", include_in_schema=False)
    async def error(req: Request) -> Response:
        return render(req, "error.html", request_id=req.state.get("trace_id", ""))

    app.on_shutdown.append(gw.close)
    return app


def _native_fn(name: str):
    """A form codec of the native module (formcodec.hpp via module.cpp), or None without it."""
    try:
        from ...native import load
        return getattr(load(), name)
    except Exception:
        return None


def _index_invoke_path(req: Request) -> str:
    """The SDK's InvocationError text for tasks_index_post's invoke (its path)."""
    if not req.state.get("tt_native"):
        return ""
    handler = (req.query_get("handler") or "").lower()
    tid = req.query_get("id") or ""
    return f"{API_APP_ID}/api/tasks/{tid}" + ("/markcomplete" if handler == "complete" else "")


def _edit_invoke_path(req: Request) -> str:
    """The SDK's InvocationError text for edit_post's invoke (its path: the form's TaskId, else
    the route's id)."""
    if not req.state.get("tt_native"):
        return ""
    tid = req.form().get("TaskUpdate.TaskId") or str(req.path_params.get("id"))
    return f"{API_APP_ID}/api/tasks/{tid}"


def _native_form():
    """``native/src/formcodec.hpp``'s Create-post binder, or None without the native module: it
    answers exactly like the page below for the posts it accepts and declines the rest."""
    try:
        from ...native import load
        return load().frontend_create_form
    except Exception:
        return None


def _bind(form: dict[str, str], prefix: str) -> tuple[dict[str, Any], dict[str, str]]:
    """Razor model binding for ``TaskAdd.*`` / ``TaskUpdate.*`` fields + ``[Required]``."""
    values: dict[str, Any] = {}
    errors: dict[str, str] = {}
    for field in REQUIRED_FIELDS:
        raw = form.get(f"{prefix}.{field[0].upper()}{field[1:]}", "").strip()
        values[field] = raw
        if not raw:
            errors[field] = f"The {FIELD_DISPLAY[field]} field is required."
    if values.get("taskDueDate") and "taskDueDate" not in errors:
        try:
            values["taskDueDate"] = parse_datetime(values["taskDueDate"]).strftime("%Y-%m-%dT%H:%M:%S")
        except ValueError:
            errors["taskDueDate"] = f"The value '{values['taskDueDate']}' is not valid for {FIELD_DISPLAY['taskDueDate']}."
    return values, errors


def main(argv: list[str] | None = None) -> None:
    import sys
    run_host(create_app(sys.argv[1:] if argv is None else argv))


if __name__ == "__main__":
    main()
