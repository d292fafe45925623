"""The native TaskModel codec (native/src/taskcodec.hpp) against the pydantic binder it shortcuts.

Invariant: for any body, the codec either declines (``None``: the general binder decides) or
produces exactly what binding the body with ``TaskAddModel`` and serialising the new
``TaskModel`` for the store (``to_store_json``) produces -- and it declines every body the binder rejects (400)."""
import json
import uuid

import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from aca_dotnet_workshop_amd.models import TaskAddModel, TaskModel, create_task_wire, parse_datetime

pytestmark = pytest.mark.skipif(create_task_wire(b"{}") is None, reason="native module not built")


def _reference(body: bytes, made) -> bytes | None:
    """What the pydantic path produces for ``body`` with the codec's id and timestamp."""
    try:
        m = TaskAddModel.model_validate(json.loads(body))
        created = json.loads(made[3])["taskCreatedOn"] if made else "2030-01-01T00:00:00Z"
        t = TaskModel(task_id=uuid.UUID(made[0]) if made else uuid.uuid4(), task_name=m.task_name,
                      task_created_by=m.task_created_by, task_created_on=parse_datetime(created),
                      task_due_date=m.task_due_date, task_assigned_to=m.task_assigned_to)
        return t.to_store_json().encode()  # the stored form: taskCreatedOn round-trip ("O")
    except Exception:  # rejected by the binder (400) or unserialisable (500)
        return None


def _check(body: bytes) -> bool:
    made = create_task_wire(body)
    ref = _reference(body, made)
    if made is None:
        return False
    assert ref is not None, f"codec accepted a body the binder rejects: {body!r}"
    assert made[3] == ref, (body, made[3], ref)
    doc = json.loads(made[3])
    assert made[1] == doc["taskName"] and made[2] == doc["taskAssignedTo"] and made[0] == doc["taskId"]
    assert json.loads(made[4]) == [{"key": made[0], "value": doc}]
    return True


def _body(**kw) -> bytes:
    base = {"taskName": "Task 1", "taskCreatedBy": "b@example.com", "taskDueDate": "2030-01-01T00:00:00",
            "taskAssignedTo": "a@example.com"}
    base.update(kw)
    return json.dumps({k: v for k, v in base.items() if v is not ...}).encode()


@pytest.mark.parametrize("body", [
    _body(),
    _body(taskDueDate="2030-01-01"),
    _body(taskDueDate="2030-01-01T10:20"),
    _body(taskDueDate="2030-01-01 10:20:30"),
    _body(taskDueDate="2030-01-01T10:20:30.1200000"),
    _body(taskDueDate="2030-01-01T10:20:30,000001Z"),
    _body(taskDueDate="2024-02-29T00:00:00z"),
    _body(taskDueDate="2030-01-01T00:00:00.123456789"),
    _body(taskName='quote " backslash \\ tab \t nl \n bell \x07 del \x7f', taskAssignedTo="é ✓ 😀  "),
    _body(taskName=...),
    _body(taskDueDate=...),
    _body(extra="ignored", another=True, third=None),
    b'{"taskName":"\\u00e9\\ud83d\\ude00","taskDueDate":"2030-01-01T00:00:00"}',
    b' {"taskName" : "spaced" ,\n "taskDueDate":"2030-01-01"} ',
    b"{}",
])
def test_codec_matches_binder(body):
    assert _check(body), f"codec declined a plain body: {body!r}"


@pytest.mark.parametrize("body", [
    _body(TaskName="case"),                      # remapped case-insensitively by the binder
    _body(task_name="snake"),                    # populate_by_name
    _body(taskDueDate="2030-01-01T00:00:00+02:00"),
    _body(taskDueDate=" 2030-01-01"),            # stripped by the binder
    _body(taskDueDate="2030-02-30"),             # invalid day -> 400
    _body(taskDueDate="2023-02-29"),
    _body(taskDueDate="0000-01-01"),
    _body(taskDueDate="2030-01-01T24:00:00"),
    _body(taskDueDate="2030-01-01T00:00:00.1234567890"),
    _body(taskDueDate="not a date"),
    _body(taskDueDate=20300101),
    _body(taskName=None),
    _body(taskName=7),
    _body(count=3),                              # numbers: the binder's JSON parser decides
    _body(nested={"a": [1]}),
    b'{"taskName":"a","taskName":"b"}',          # duplicate: json.loads keeps the last
    b'{"taskName":"raw\tcontrol"}',              # invalid JSON (strict)
    b'{"taskName":"\\ud800"}',                   # lone surrogate
    b'{"taskName":"\xff"}',                      # invalid UTF-8
    b'\xef\xbb\xbf{"taskName":"bom"}',
    b'[]', b'"x"', b'', b'{', b'{"taskName":"x"} trailing',
])
def test_codec_declines_what_it_does_not_decide(body):
    assert create_task_wire(body) is None
    _check(body)  # (and the invariant holds trivially)


def test_ids_are_random_v4_and_created_is_now():
    from datetime import datetime, timezone
    ids = set()
    for _ in range(2000):
        made = create_task_wire(_body())
        u = uuid.UUID(made[0])
        assert u.version == 4 and u.variant == uuid.RFC_4122 and str(u) == made[0]
        ids.add(made[0])
    assert len(ids) == 2000
    created = parse_datetime(json.loads(made[3])["taskCreatedOn"])
    assert abs((datetime.now(timezone.utc) - created).total_seconds()) < 5


_text = st.text(st.characters(blacklist_categories=("Cs",)), max_size=12)
_date = st.one_of(
    st.datetimes(min_value=__import__("datetime").datetime(1, 1, 1)).map(lambda d: d.isoformat()),
    st.from_regex(r"\A\d{4}-\d{2}-\d{2}([T ]\d{2}:\d{2}(:\d{2}([.,]\d{1,10})?)?)?([Zz]|[+-]\d{2}:?\d{2})?\Z"),
    _text)


@settings(max_examples=400, deadline=None)
@given(st.dictionaries(st.sampled_from(["taskName", "taskCreatedBy", "taskAssignedTo", "TaskName", "x"]),
                       st.one_of(_text, st.none(), st.booleans(), st.integers()), max_size=4), _date)
def test_codec_fuzz_parity(fields, due):
    fields["taskDueDate"] = due
    _check(json.dumps(fields).encode())
    _check(json.dumps(fields, ensure_ascii=False).encode())


def test_api_uses_codec_and_general_binder():
    """POST /api/tasks: plain bodies take the native pass, others the binder (same responses)."""
    import asyncio

    from aca_dotnet_workshop_amd.sdk.client import SidecarClient
    from aca_dotnet_workshop_amd.services.backend_api.app import create_app
    from aca_dotnet_workshop_amd.services.backend_api.managers import TasksStoreManager
    from aca_dotnet_workshop_amd.web.client import ClientResponse
    from aca_dotnet_workshop_amd.web.http import Headers, Request

    sent = []

    class Http:
        async def request(self, method, url, *, headers=None, body=None, json_body=None, timeout=None):
            sent.append((url.split(":", 2)[-1], body))
            return ClientResponse(204, Headers({}), b"")

        async def close(self):
            pass

    app = create_app([], manager=TasksStoreManager(SidecarClient("unix:/x:", http=Http())))

    async def post(body, ctype="application/json"):
        return await app(Request("POST", "/api/tasks", Headers({"content-type": ctype}), body, None, "HTTP/1.1"))

    async def main():
        r1 = await post(_body())
        r2 = await post(_body(TaskName="Cased", taskName=...))
        r3 = await post(_body(taskDueDate="2030-02-30"))
        r4 = await post(_body(), "text/plain")
        return r1, r2, r3, r4
    r1, r2, r3, r4 = asyncio.run(main())
    assert r1.status == 201 and r2.status == 201 and r3.status == 400 and r4.status == 415
    tid = dict(r1.headers)["Location"].rsplit("/", 1)[1]
    (p1, save1), (p2, pub1), (p3, save2), (p4, pub2) = sent
    assert p1 == "/v1.0/state/statestore" and p2 == "/v1.0/publish/dapr-pubsub-servicebus/tasksavedtopic"
    assert json.loads(save1)[0]["key"] == tid and json.loads(pub1)["taskId"] == tid
    assert json.loads(pub2)["taskName"] == "Cased"   # the binder's remapping
    assert set(json.loads(pub1)) == set(json.loads(pub2))


# ---------------------------------------------------------------------- the processor's side
def _native():
    from aca_dotnet_workshop_amd.native import load
    return load()


def _envelope(data, **kw):
    ce = {"specversion": "1.0", "id": "e1", "source": "tasksmanager-backend-api", "type": "com.dapr.event.sent",
          "topic": "tasksavedtopic", "pubsubname": "dapr-pubsub-servicebus", "datacontenttype": "application/json",
          "traceparent": "00-4bf92f3577b34da6a3ce929d0e0e4736-00f067aa0ba902b7-00", "data": data}
    ce.update(kw)
    return json.dumps(ce).encode()


_TASK = {"taskId": "0f8fad5b-d9cb-469f-a165-70867728950e", "taskName": "Task 1", "taskCreatedBy": "b@x",
         "taskCreatedOn": "2030-01-01T00:00:00.1234567Z", "taskDueDate": "2030-01-02T00:00:00",
         "taskAssignedTo": "a@x", "isCompleted": False, "isOverDue": False}


@pytest.mark.parametrize("data", [_TASK, {"a": ["x", None, True, {"b": "é\n\""}]}, [], {}])
def test_cloudevent_unwrap_matches_python(data):
    body = _envelope(data, extra={"k": "v"})
    u = _native().cloudevent_unwrap(body)
    ce = json.loads(body)
    assert u is not None
    assert json.loads(u[0]) == ce.pop("data") and u[1] == "application/json" and u[2] == ce


@pytest.mark.parametrize("body", [
    _envelope({"n": 1}),                                   # numbers: Python's parser decides
    _envelope("text", datacontenttype="text/plain"),
    json.dumps({"specversion": "1.0", "data_base64": "eyJ9"}).encode(),
    b'{"data":{},"data":{}}', b"[]", b"{", _envelope(_TASK, id=5),
])
def test_cloudevent_unwrap_declines(body):
    assert _native().cloudevent_unwrap(body) is None


def _model_ref(body: bytes):
    try:
        return TaskModel.model_validate(json.loads(body)).task_name
    except Exception:
        return None


@pytest.mark.parametrize("kw", [{}, {"taskId": "0F8FAD5B-D9CB-469F-A165-70867728950E"}, {"isCompleted": True},
                                {"taskCreatedOn": "2030-01-01"}, {"extra": "x"}])
def test_task_model_name_matches_binder(kw):
    body = json.dumps({**_TASK, **kw}).encode()
    assert _native().task_model_name(body) == _model_ref(body) == "Task 1"


@pytest.mark.parametrize("kw", [{"taskId": "{0f8fad5b-d9cb-469f-a165-70867728950e}"}, {"taskId": "nope"},
                                {"isCompleted": "true"}, {"isCompleted": 1}, {"taskDueDate": "2030-13-01"},
                                {"TaskName": "x"}, {"task_name": "x"}, {"taskName": None}])
def test_task_model_name_declines(kw):
    assert _native().task_model_name(json.dumps({**_TASK, **kw}).encode()) is None


@settings(max_examples=300, deadline=None)
@given(st.dictionaries(st.sampled_from(list(_TASK) + ["TaskName", "x"]),
                       st.one_of(_text, st.none(), st.booleans(), _date, st.uuids().map(str)), max_size=8))
def test_task_model_name_fuzz(fields):
    body = json.dumps(fields).encode()
    got = _native().task_model_name(body)
    if got is not None:
        assert got == _model_ref(body), body


# ---------------------------------------------------------------------- the overdue sweep's lists
def _binder_list(body: bytes):
    try:
        return [TaskModel.model_validate(x) for x in json.loads(body)]
    except Exception:
        return None


def _check_lists(tasks_json: bytes, run_day: str) -> None:
    from datetime import date

    from aca_dotnet_workshop_amd.models import mark_overdue_wire, naive_utc, overdue_filter_wire
    ref = _binder_list(tasks_json)
    if not isinstance(json.loads(tasks_json), list):
        ref = None
    made = mark_overdue_wire(tasks_json)
    if made is not None:
        assert ref is not None, f"accepted a list the binder rejects: {tasks_json!r}"
        want = [{"key": str(t.task_id), "value": {**t.to_wire(), "isOverDue": True}} for t in ref]
        assert made[0] == [str(t.task_id) for t in ref] and json.loads(made[1]) == want
    f = overdue_filter_wire(tasks_json, run_day)
    if f is not None:
        assert ref is not None
        day = date.fromisoformat(run_day)
        keep = [t.to_wire() for t in ref if day > naive_utc(t.task_due_date).date()]
        assert f[0] == len(ref) and f[1] == len(keep) and json.loads(f[2]) == keep


@pytest.mark.parametrize("tasks", [
    [], [_TASK], [_TASK, {**_TASK, "taskId": "0F8FAD5B-D9CB-469F-A165-70867728950F", "taskDueDate": "2029-12-31Z"}],
    [{"taskName": "defaults only"}], [{**_TASK, "isOverDue": True, "extra": "x"}],
])
def test_overdue_lists_match_binder(tasks):
    body = json.dumps(tasks).encode()
    for day in ("2030-01-02", "2030-01-03", "2000-01-01"):
        _check_lists(body, day)
    assert _native().tasks_mark_overdue(body) is not None


@pytest.mark.parametrize("body", [b"{}", b"[1]", b'[{"TaskName":"x"}]', b'[{"taskId":"nope"}]', b'[{"isOverDue":"yes"}]',
                                  json.dumps([_TASK, {**_TASK, "taskDueDate": "2030-02-30"}]).encode()])
def test_overdue_lists_decline(body):
    assert _native().tasks_mark_overdue(body) is None and _native().tasks_overdue_filter(body, "2030-01-01") is None


@settings(max_examples=200, deadline=None)
@given(st.lists(st.dictionaries(st.sampled_from(list(_TASK) + ["x"]),
                                st.one_of(_text, st.booleans(), _date, st.uuids().map(str)), max_size=8), max_size=4),
       st.dates().map(lambda d: d.isoformat()))
def test_overdue_lists_fuzz(tasks, day):
    _check_lists(json.dumps(tasks).encode(), day)
    _check_lists(json.dumps(tasks, ensure_ascii=False).encode(), day)


@pytest.mark.parametrize("results", [[], None, [{"key": "a", "data": _TASK, "etag": "1"}, {"key": "b", "data": None}],
                                     [{"key": "c", "data": {**_TASK, "taskId": _TASK["taskId"].upper()}}]])
def test_query_results_to_tasks(results):
    from aca_dotnet_workshop_amd.models import tasks_from_query_wire
    body = json.dumps({"results": results, "token": "100"}).encode()
    made = tasks_from_query_wire(body)
    want = [TaskModel.model_validate(r["data"]).to_wire() for r in results or [] if r.get("data") is not None]
    assert made is not None and made[0] == len(want) and json.loads(made[1]) == want and made[2] is True


def test_query_results_ordered_by_created_datetime():
    """``by_created``: DateTime order, not string order -- System.Text.Json trims the fraction,
    so "...:42Z" < "...:42.1Z" < "...:42.12Z" chronologically although not as strings."""
    from aca_dotnet_workshop_amd.models import tasks_from_query_wire
    stamps = ["2026-01-02T03:04:42.12Z", "2026-01-02T03:04:42Z", "2026-01-01T23:59:59.9999Z",
              "2026-01-02T03:04:42.1Z", "2026-01-02T03:04:43Z", "2026-01-02T03:04:42.12Z"]
    results = [{"key": str(i), "data": {**_TASK, "taskId": f"00000000-0000-0000-0000-00000000000{i}",
                                        "taskCreatedOn": t}} for i, t in enumerate(stamps)]
    made = tasks_from_query_wire(json.dumps({"results": results}).encode(), by_created=True)
    got = [(t["taskCreatedOn"], t["taskId"][-1]) for t in json.loads(made[1])]
    want = sorted(((TaskModel.model_validate(r["data"]), r["key"]) for r in results),
                  key=lambda x: x[0].task_created_on)
    assert [k for _, k in got] == [k for _, k in want]  # stable: the two equal stamps keep their order
    assert made[2] is False


@settings(max_examples=150, deadline=None)
@given(st.lists(st.tuples(st.integers(0, 3), st.integers(0, 59), st.integers(0, 999999), st.integers(0, 6),
                          st.booleans()), min_size=1, max_size=25))
def test_query_results_created_order_matches_datetime_order(stamps):
    """The page codec's numeric DateTime key (taskcodec.hpp created_key) orders like the
    TaskModel's DateTime (UTC and unspecified kinds on one clock), stably, for any mix of
    fraction lengths and UTC markers."""
    from aca_dotnet_workshop_amd.models import naive_utc, tasks_from_query_wire
    texts = []
    for day, sec, us, digits, z in stamps:
        frac = f"{us:06d}"[:digits]
        texts.append(f"2026-03-{10 + day:02d}T11:22:{sec:02d}" + (f".{frac}" if digits else "") + ("Z" if z else ""))
    results = [{"key": str(i), "data": {**_TASK, "taskId": f"00000000-0000-0000-0000-{i:012d}", "taskCreatedOn": t}}
               for i, t in enumerate(texts)]
    made = tasks_from_query_wire(json.dumps({"results": results}).encode(), by_created=True)
    got = [int(t["taskId"][-12:]) for t in json.loads(made[1])]
    want = [i for i, _ in sorted(enumerate(results),
                                 key=lambda x: naive_utc(TaskModel.model_validate(x[1]["data"]).task_created_on))]
    assert got == want
    # descending (GET api/tasks: newest first) equals the binder path's stable reverse sort
    # (managers.get_tasks_by_creator: ``tasks.sort(key=_created_key, reverse=True)``), byte for byte
    from aca_dotnet_workshop_amd.models import tasks_to_json
    from aca_dotnet_workshop_amd.services.backend_api.managers import _created_key
    body = json.dumps({"results": results + [{"key": "gone", "data": None}]}).encode()
    made = tasks_from_query_wire(body, by_created=True, descending=True)
    ref = [TaskModel.model_validate(r["data"]) for r in results]
    ref.sort(key=_created_key, reverse=True)
    assert made[1] == tasks_to_json(ref)


def _store_page(datas: list, token: str | None, keys: list[str] | None = None) -> bytes:
    """A query page laid out as the backing's page assembly writes it (DocStore::mirror_results):
    compact, key / data / etag per result, then the token."""
    parts = []
    for i, d in enumerate(datas):
        k = json.dumps(keys[i] if keys else f"k{i}")
        parts.append('{"key":' + k + ',"data":' + d + ',"etag":"' + str(i + 1) + '"}')
    return ('{"results":[' + ",".join(parts) + "]" + (',"token":' + json.dumps(token) if token is not None else "")
            + "}").encode()


@settings(max_examples=300, deadline=None)
@given(st.lists(st.tuples(_text, _text, _text, st.datetimes(min_value=__import__("datetime").datetime(1, 1, 1)),
                          st.datetimes(min_value=__import__("datetime").datetime(1, 1, 1)), st.booleans(),
                          st.booleans(), st.booleans(), st.uuids()), max_size=12),
       st.one_of(st.none(), st.just(""), st.text("0123456789", min_size=1, max_size=4)),
       st.booleans(), st.booleans())
def test_query_results_in_the_store_layout_read_in_one_pass(rows, token, by_created, descending):
    """The page as the backing writes it is read in one pass (taskcodec.hpp fast_query_tasks):
    the same tasks, order, bytes and continuation flag as the value-tree reader gives for the same
    page re-spaced (which that pass declines) -- for any names (a page with an escaped one goes
    to the tree whole), upper-case ids, any dates."""
    from aca_dotnet_workshop_amd.models import tasks_from_query_wire
    datas = []
    for name, by, to, created, due, done, over, upper, uid in rows:
        t = TaskModel(task_id=str(uid).upper() if upper else str(uid), task_name=name, task_created_by=by,
                      task_created_on=created, task_due_date=due, task_assigned_to=to, is_completed=done,
                      is_over_due=over)
        datas.append(t.to_store_json())
    page = _store_page(datas, token)
    spaced = json.dumps(json.loads(page)).encode()  # ", " / ": " separators: not the store's layout
    fast = tasks_from_query_wire(page, by_created=by_created, descending=descending)
    tree = tasks_from_query_wire(spaced, by_created=by_created, descending=descending)
    assert fast is not None and fast == tree
    assert fast[2] == bool(token)
    plain = b"\\" not in page  # no escaped (or control) character anywhere
    assert _native().tasks_query_in_store_layout(page) == plain
    assert not _native().tasks_query_in_store_layout(spaced) or not datas


@settings(max_examples=200, deadline=None)
@given(st.lists(st.tuples(_text, st.datetimes(min_value=__import__("datetime").datetime(1, 1, 1)),
                          st.datetimes(min_value=__import__("datetime").datetime(2000, 1, 1),
                                       max_value=__import__("datetime").datetime(2040, 1, 1)),
                          st.booleans(), st.uuids()), max_size=12),
       st.dates(min_value=__import__("datetime").date(2000, 1, 1), max_value=__import__("datetime").date(2040, 1, 1)),
       st.integers(1, 5))
def test_overdue_filter_of_the_api_page_in_one_pass(rows, day, chunk):
    """The processor's filter over the API's overdue page (the page exactly as the API answers:
    taskcodec.hpp fast_overdue_filter) gives what the value-tree reader gives for the same page
    re-spaced: counts, kept tasks and chunk boundaries, byte for byte; and the binder agrees."""
    page_tasks = [TaskModel(task_id=uid, task_name=name, task_created_on=created, task_due_date=due,
                            is_completed=done).to_json() for name, created, due, done, uid in rows]
    page = ("[" + ",".join(page_tasks) + "]").encode()
    spaced = json.dumps(json.loads(page)).encode()
    run_day = day.isoformat()
    assert _native().tasks_overdue_filter(page, run_day) == _native().tasks_overdue_filter(spaced, run_day)
    assert (_native().tasks_overdue_filter_chunks(page, run_day, chunk)
            == _native().tasks_overdue_filter_chunks(spaced, run_day, chunk))
    _check_lists(page, run_day)


@settings(max_examples=200, deadline=None)
@given(st.lists(st.tuples(_text, st.datetimes(min_value=__import__("datetime").datetime(1, 1, 1)),
                          st.booleans(), st.booleans(), st.uuids(), st.sampled_from(["", "7", "123"]),
                          st.booleans()), max_size=10))
def test_conditional_mark_of_the_bulk_get_in_one_pass(rows):
    """markoverdue's conditional save over the sidecar's bulk-get answer laid out as the data
    plane writes it (taskcodec.hpp fast_conditional_mark) equals the value-tree reader's answer
    for the same text re-spaced: the same bulk body, ids and skips (deleted, completed and
    already-overdue tasks; empty ETags)."""
    parts = []
    for name, created, done, over, uid, etag, gone in rows:
        if gone:
            parts.append('{"key":' + json.dumps(str(uid)) + "}")
            continue
        t = TaskModel(task_id=uid, task_name=name, task_created_on=created, is_completed=done, is_over_due=over)
        parts.append('{"key":' + json.dumps(str(uid)) + ',"data":' + t.to_store_json() + ',"etag":'
                     + json.dumps(etag) + "}")
    got = ("[" + ",".join(parts) + "]").encode()
    spaced = json.dumps(json.loads(got)).encode()
    fast, tree = _native().tasks_conditional_mark(got), _native().tasks_conditional_mark(spaced)
    assert fast is not None and fast == tree


def test_query_results_one_pass_declines_other_layouts():
    """Anything but the store's exact layout goes to the value tree, with the same answer."""
    from aca_dotnet_workshop_amd.models import tasks_from_query_wire
    t = TaskModel.model_validate(_TASK).to_store_json()
    pages = [_store_page([t], "7"), _store_page([t, t.replace('"isOverDue":false', '"isOverDue":false,"x":"y"')], None),
             _store_page([t], None).replace(b'"etag":"1"', b'"etag":"1","extra":1'),
             _store_page([t], None).replace(b'{"results":', b'{"metadata":{},"results":'),
             _store_page([], "9"), b'{"results":[]}', b'{"results":null}']
    for page in pages:
        want = tasks_from_query_wire(json.dumps(json.loads(page)).encode(), by_created=True)
        assert tasks_from_query_wire(page, by_created=True) == want, page


@pytest.mark.parametrize("body", [b"[]", b'{"results": 5}', b'{"results": [{"data": "text"}]}',
                                  json.dumps({"results": [{"data": {"TaskName": "x"}}]}).encode()])
def test_query_results_decline(body):
    from aca_dotnet_workshop_amd.models import tasks_from_query_wire
    assert tasks_from_query_wire(body) is None



@settings(max_examples=200, deadline=None)
@given(st.lists(st.recursive(st.none() | st.booleans() | st.integers() | st.text(max_size=8),
                             lambda ch: st.lists(ch, max_size=3) | st.dictionaries(st.text(max_size=4), ch, max_size=3),
                             max_leaves=6), max_size=30), st.integers(1, 9), st.booleans())
def test_json_array_chunks_regroups_the_items(items, n, spaced):
    """models.json_array_chunks (native): the items of a JSON array, in order, in arrays of at most
    n; each item's text is kept (raw slices), so the chunks parse back to the same items."""
    from aca_dotnet_workshop_amd.models import json_array_chunks
    body = json.dumps(items, separators=(", ", ": ") if spaced else (",", ":"), ensure_ascii=False).encode()
    chunks = json_array_chunks(body, n)
    parsed = [json.loads(c) for c in chunks]
    assert all(1 <= len(c) <= n for c in parsed) and sum(parsed, []) == items
    assert json_array_chunks(b'{"a": 1}', n) is None and json_array_chunks(b"[1,", n) is None


@settings(max_examples=100, deadline=None)
@given(st.lists(st.tuples(st.sampled_from(["2026-10-15T00:00:00", "2026-10-16T23:59:59.5Z", "2026-10-17T00:00:00",
                                           "2026-10-18T08:00:00"]),
                          st.text(max_size=6), st.booleans()), max_size=40), st.integers(1, 9))
def test_overdue_filter_chunks_equals_filter_then_chunk(rows, n):
    """models.overdue_filter_chunks (one native pass) gives the processor exactly what
    overdue_filter_wire followed by json_array_chunks gives: the page size, the kept count, and
    the kept tasks' canonical TaskModel JSON cut into arrays of at most n."""
    import uuid
    from aca_dotnet_workshop_amd.models import json_array_chunks, overdue_filter_chunks, overdue_filter_wire
    tasks = [{"taskId": str(uuid.UUID(int=i + 1)), "taskName": name, "taskCreatedBy": "c@x",
              "taskCreatedOn": "2026-10-14T10:00:00", "taskDueDate": due, "taskAssignedTo": "a@x",
              "isCompleted": done, "isOverDue": False} for i, (due, name, done) in enumerate(rows)]
    body = json.dumps(tasks).encode()
    n_page, n_kept, kept = overdue_filter_wire(body, "2026-10-17")
    got = overdue_filter_chunks(body, "2026-10-17", n)
    assert got[0] == n_page == len(tasks) and got[1] == n_kept
    assert got[2] == (json_array_chunks(kept, n) if n_kept else [])
    assert [t["taskId"] for p in got[2] for t in json.loads(p)] == \
        [t["taskId"] for t in tasks if t["taskDueDate"][:10] < "2026-10-17"]


def test_conditional_mark_falls_back_when_the_native_codec_declines():
    """A markoverdue page holding a stored document the native codec turns down (a null string,
    a duplicate key, an offset date form) is marked by the Python twin instead of failing the
    whole chunk; a document that does not bind as a TaskModel at all is skipped and
    the rest of the page is still marked."""
    from aca_dotnet_workshop_amd.models.task import _lists, conditional_mark_wire

    def task(**kw):
        d = {"taskId": str(uuid.uuid4()), "taskName": "n", "taskCreatedBy": "a@x",
             "taskCreatedOn": "2024-01-01T00:00:00.0000000Z", "taskDueDate": "2024-01-02T00:00:00",
             "taskAssignedTo": "b@x", "isCompleted": False, "isOverDue": False}
        d.update(kw)
        return d
    ok, null_name, offset, done = task(), task(taskAssignedTo=None), task(taskDueDate="2024-01-02T00:00:00+00:00"), \
        task(isCompleted=True)
    rows = [{"key": t["taskId"], "data": t, "etag": str(i)} for i, t in enumerate((ok, null_name, offset, done))]
    rows.append({"key": "gone", "data": None})
    got = json.dumps(rows).encode()
    assert _lists()[2](got) is None  # the native codec declines this page
    ids, bulk, skipped = conditional_mark_wire(got)
    assert ids == [ok["taskId"], offset["taskId"]] and skipped == 3
    items = json.loads(bulk)
    assert [i["key"] for i in items] == ids and all(i["value"]["isOverDue"] for i in items)
    assert [i["etag"] for i in items] == ["0", "2"] and all(i["options"] == {"concurrency": "first-write"} for i in items)


# ------------------------------------------------------- the API's read-modify-writes (r6)
def _update_ref(body: bytes):
    from aca_dotnet_workshop_amd.models import TaskUpdateModel
    try:
        return TaskUpdateModel.model_validate(json.loads(body))
    except Exception:
        return None


def _check_edit(stored: dict, body: bytes | None) -> None:
    """task_update_bind / task_edit / task_json against TaskUpdateModel + TaskModel: the same
    document written back (to_store_json), the same GET answer (to_json)."""
    from aca_dotnet_workshop_amd.models import format_datetime
    n = _native()
    raw = json.dumps(stored, ensure_ascii=False).encode()
    try:
        ref = TaskModel.model_validate(stored)
    except Exception:
        ref = None
    got = n.task_json(raw)
    if got is not None:
        assert ref is not None and got.decode() == ref.to_json(), (stored, got)
    done = n.task_edit(raw, True, None)
    if done is not None:
        assert ref is not None
        want = ref.model_copy()
        want.is_completed = True
        assert done[0].decode() == want.to_store_json() and done[1] == str(ref.task_id)
        assert done[2] == ref.task_assigned_to
    if body is None:
        return
    upd = n.task_update_bind(body)
    m = _update_ref(body)
    if upd is not None:
        assert m is not None, body
        assert (upd[0], upd[1]) == (m.task_name, m.task_assigned_to) and upd[2] == format_datetime(m.task_due_date)
        made = n.task_edit(raw, False, upd)
        if made is not None:
            assert ref is not None
            want = ref.model_copy()
            want.task_name, want.task_assigned_to, want.task_due_date = m.task_name, m.task_assigned_to, m.task_due_date
            assert made[0].decode() == want.to_store_json(), (stored, body)


_UPD = {"taskId": "0f8fad5b-d9cb-469f-a165-70867728950e", "taskName": "edited ✓ 'q' \"x\"",
        "taskDueDate": "2030-02-01T00:00:00", "taskAssignedTo": "Other@x"}


@pytest.mark.parametrize("stored", [_TASK, {**_TASK, "taskId": _TASK["taskId"].upper(), "isOverDue": True},
                                    {**_TASK, "taskCreatedOn": "2030-01-01T00:00:00Z", "taskDueDate": "2030-01-02"},
                                    {"taskName": "defaults only"}, {**_TASK, "extra": "x"}])
@pytest.mark.parametrize("body", [_UPD, {**_UPD, "taskDueDate": "2030-02-01"}, {"taskName": "only a name"},
                                  {**_UPD, "taskDueDate": "2030-02-01T10:11:12.5Z", "x": None}])
def test_rmw_codecs_match_the_models(stored, body):
    _check_edit(stored, json.dumps(body, ensure_ascii=False).encode())
    assert _native().task_update_bind(json.dumps(body).encode()) is not None


@pytest.mark.parametrize("body", [b"[]", b'{"taskname":"x"}', b'{"task_name":"x"}', b'{"taskDueDate":"2030-02-30"}',
                                  b'{"taskId":"nope"}', b'{"taskName":1}', b'{"taskDueDate":"2030-02-01T00:00:00+02:00"}'])
def test_update_bind_declines_what_it_does_not_decide(body):
    assert _native().task_update_bind(body) is None


@settings(max_examples=200, deadline=None)
@given(st.dictionaries(st.sampled_from(list(_TASK) + ["x"]), st.one_of(_text, st.booleans(), _date, st.uuids().map(str)),
                       max_size=8),
       st.dictionaries(st.sampled_from(list(_UPD) + ["y"]), st.one_of(_text, st.booleans(), _date, st.uuids().map(str)),
                       max_size=5))
def test_rmw_codecs_fuzz(stored, body):
    _check_edit(stored, json.dumps(body).encode())
    _check_edit(stored, json.dumps(body, ensure_ascii=False).encode())
