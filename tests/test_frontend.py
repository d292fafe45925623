"""Frontend variants: module-2 direct HTTP mode (named HttpClient on BaseUrlExternalHttp) and
the production error page."""
import json

import pytest

from aca_dotnet_workshop_amd.services.backend_api import FakeTasksManager
from aca_dotnet_workshop_amd.services.backend_api import create_app as api_app
from aca_dotnet_workshop_amd.services.frontend import create_app as fe_app
from aca_dotnet_workshop_amd.utils.config import Configuration

from helpers import run, served


def test_http_mode_requires_base_url():
    with pytest.raises(RuntimeError, match="BaseUrlExternalHttp"):
        fe_app(config=Configuration([{"Frontend": {"BackendMode": "http"}}]))


def test_http_mode_lists_seeded_tasks():
    async def main():
        async with served(api_app(config=Configuration([{}]), manager=FakeTasksManager())) as (api, _):
            cfg = Configuration([{"Frontend": {"BackendMode": "http"}, "BackendApiConfig": {"BaseUrlExternalHttp": api}}])
            async with served(fe_app(config=cfg)) as (web, c):
                r = await c.get(web + "/Tasks/Index", headers={"Cookie": "TasksCreatedByCookie=tjoudeh@bitoftech.net"})
                assert r.status == 200 and r.text.count("Task number:") == 10
    run(main())


def test_error_page_outside_development():
    async def main():
        cfg = Configuration([{"Environment": "Production", "Frontend": {"BackendMode": "http"},
                              "BackendApiConfig": {"BaseUrlExternalHttp": "http://127.0.0.1:9"}}])
        async with served(fe_app(config=cfg)) as (web, c):
            r = await c.get(web + "/Tasks/Index", headers={"Cookie": "TasksCreatedByCookie=a@b"})
            assert r.status == 500 and "An error occurred while processing your request." in r.text
    run(main())


# -- the native Create-post binder (native/src/formcodec.hpp) against the page's Python path ----
from hypothesis import given, settings  # noqa: E402
from hypothesis import strategies as st  # noqa: E402


class _Capture:
    """The frontend's sidecar: records the invoke it was asked to make, answers 201."""

    def __init__(self):
        from aca_dotnet_workshop_amd.web.client import ClientResponse
        from aca_dotnet_workshop_amd.web.http import Headers
        self.resp = ClientResponse(201, Headers({"location": "/api/tasks/x"}), b"")
        self.calls = []

    async def request(self, method, url, *, headers=None, body=None, json_body=None, timeout=None):
        self.calls.append((method, url, body))
        return self.resp

    async def close(self):
        pass


def _post(native: bool, body: bytes, cookie: str):
    import json

    from aca_dotnet_workshop_amd.sdk.client import SidecarClient
    from aca_dotnet_workshop_amd.services.frontend import app as fe
    from aca_dotnet_workshop_amd.web.http import Headers, Request
    cap = _Capture()
    real = fe._native_form
    if not native:
        fe._native_form = lambda: None
    try:
        app = fe.create_app([], client=SidecarClient("unix:/nonexistent:", http=cap),
                            overrides={"Frontend:AntiforgeryKey": "k3y"})
    finally:
        fe._native_form = real
    req = Request("POST", "/Tasks/Create", Headers({"content-type": "application/x-www-form-urlencoded",
                                                    "cookie": cookie}), body, None, "HTTP/1.1")
    try:
        resp = run(app(req))
    except Exception as e:  # the page's HTTPError (400) surfaces the same way on both paths
        return ("error", getattr(e, "status", None)), cap.calls
    sent = [(m, u, json.loads(b)) for m, u, b in cap.calls]
    return (resp.status, resp.header("location")), sent


_TOKEN = None


def _token(cookie_value: str) -> str:
    from aca_dotnet_workshop_amd.services.frontend.app import Antiforgery
    return Antiforgery(b"k3y").token_for(cookie_value)


_text = st.text(alphabet=st.characters(blacklist_categories=("Cs",)), max_size=12)
_dates = st.one_of(st.sampled_from(["2030-01-01", "2024-02-29", "2023-02-29", "2030-01-01T10:20", "2030-1-1",
                                    "2030-01-01T10:20:30.1234567", "2030-01-01Z", " 2030-01-01", "", "x"]), _text)


@settings(max_examples=300, deadline=None)
@given(_text, _dates, _text, st.sampled_from(["a@b.c", "", "x%40y", "bad%zz"]), st.booleans(), st.booleans(),
       st.sampled_from(["", "&junk", "&TaskAdd.TaskName=second", "&noequals"]))
def test_native_create_post_decides_like_the_page(name, due, assignee, who, good_token, plus, extra):
    """Every post the native binder accepts is sent exactly as the Python page sends it (same
    TaskAddModel fields, same redirect); what it declines goes to the page unchanged."""
    from urllib.parse import quote, quote_plus
    q = quote_plus if plus else quote
    af = "c0ffee"
    tok = _token(af) if good_token else "0" * 64
    body = (f"__RequestVerificationToken={tok}&TaskAdd.TaskName={q(name)}&TaskAdd.TaskDueDate={q(due)}"
            f"&TaskAdd.TaskAssignedTo={q(assignee)}{extra}").encode()
    cookie = f"TasksCreatedByCookie={who}; .AspNetCore.Antiforgery={af}"
    assert _post(True, body, cookie) == _post(False, body, cookie)


def test_native_create_post_is_taken_for_a_browser_post():
    from aca_dotnet_workshop_amd import native
    body = (f"__RequestVerificationToken={_token('c0ffee')}&TaskAdd.TaskName=Buy+milk&TaskAdd.TaskDueDate=2030-01-01"
            "&TaskAdd.TaskAssignedTo=a%40b.c").encode()
    made = native.load().frontend_create_form(body, b"TasksCreatedByCookie=me%40x.y; .AspNetCore.Antiforgery=c0ffee",
                                              b"k3y")
    import json
    assert made[0] and json.loads(made[1]) == {"taskName": "Buy milk", "taskCreatedBy": "me@x.y",
                                               "taskDueDate": "2030-01-01T00:00:00", "taskAssignedTo": "a@b.c"}


def _row_renderer():
    import os

    from jinja2 import Environment, FileSystemLoader, select_autoescape

    import aca_dotnet_workshop_amd.services.frontend.app as fa
    from aca_dotnet_workshop_amd.services.frontend.rows import RowRenderer
    env = Environment(loader=FileSystemLoader(os.path.join(os.path.dirname(fa.__file__), "templates")),
                      autoescape=select_autoescape(["html"]))
    env.filters["ddmmyyyy"] = fa._fmt_date
    env.filters["inputdate"] = fa._input_date
    return env, RowRenderer(env)


from hypothesis import given, settings  # noqa: E402
from hypothesis import strategies as st  # noqa: E402


@settings(max_examples=150, deadline=None)
@given(st.lists(st.tuples(st.text(max_size=12), st.text(max_size=12), st.booleans(), st.booleans(),
                          st.datetimes(), st.uuids()), max_size=6))
def test_task_rows_fast_path_equals_the_template(rows):
    """Tasks/Index's rows compiled from the task_row macro (services/frontend/rows.py) render
    byte for byte what the template renders from bound TaskModels, escaping included."""
    from aca_dotnet_workshop_amd.models import TaskModel
    env, r = _row_renderer()
    assert r.ok
    tpl = env.get_template("tasks_index.html")
    items = [TaskModel(task_id=u, task_name=n, task_assigned_to=a, task_due_date=due, is_completed=c,
                       is_over_due=o).to_wire() for n, a, c, o, due, u in rows]
    items = json.loads(json.dumps(items))  # as the SDK hands the API's answer to the page
    fast = r.render(items)
    assert fast is not None
    ctx = dict(af_field="f", af_token="t", request=None, created_by="u@x", title="T")
    assert tpl.render(rows_html=fast, **ctx) == tpl.render(tasks=[TaskModel.model_validate(d) for d in items], **ctx)


def test_task_rows_fast_path_declines_other_shapes():
    _, r = _row_renderer()
    good = {"taskId": "0f8fad5b-d9cb-469f-a165-70867728950e", "taskName": "n", "taskAssignedTo": "a",
            "taskDueDate": "2026-01-02T00:00:00", "isCompleted": False, "isOverDue": False}
    assert r.render([good]) is not None
    for bad in ({**good, "taskId": good["taskId"].upper()}, {**good, "taskDueDate": "2026-01-02T00:00:00+02:00"},
                {**good, "isCompleted": 0}, {**good, "taskName": None}, "x"):
        assert r.render([good, bad]) is None
