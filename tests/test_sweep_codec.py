"""The overdue sweep's one-pass protobuf hops (native/src/sweepcodec.hpp) and the sidecar's
one-pass query encoder (daprpb.hpp ``query_response_pb``) against the chains they shortcut.

Invariant: each one-pass function either declines (``None``: the app host runs the chain) or
returns exactly the chain's answer, byte for byte:

* ``tasks_from_query_pb(pb)``            == ``tasks_from_query(dapr_pb_query_json(pb))``
* ``tasks_conditional_mark_pb(pb, st)``  == ``dapr_pb_save_state_bulk(st, conditional_mark(bulk_state_json(pb)))``
* ``tasks_mark_overdue_ids(body)``       == ``tasks_mark_overdue(body)``'s ids
* ``dapr_pb_query_from_json(json)``      == the QueryStateResponse of the JSON's results (data compacted)

and it reads the layouts the services actually exchange (the store's, the API's) in one pass.
"""
import json
import uuid
from datetime import datetime

import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from aca_dotnet_workshop_amd.models import TaskModel, create_task_wire

pytestmark = pytest.mark.skipif(create_task_wire(b"{}") is None, reason="native module not built")

_text = st.text(st.characters(blacklist_categories=("Cs",)), max_size=10)
_dt = st.datetimes(min_value=datetime(1, 1, 1))


def _n():
    from aca_dotnet_workshop_amd.native import load
    return load()


def _varint(n: int) -> bytes:
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        out.append(b | (0x80 if n else 0))
        if not n:
            return bytes(out)


def _lf(f: int, v: bytes) -> bytes:
    return _varint(f << 3 | 2) + _varint(len(v)) + v


def _s(f: int, v: bytes) -> bytes:
    return _lf(f, v) if v else b""


def _item(key: bytes, data: bytes, etag: bytes, error: bytes = b"") -> bytes:
    return _lf(1, _s(1, key) + _s(2, data) + _s(3, etag) + _s(4, error))


def _task(name, by, to, created, due, done, over, uid, upper=False) -> bytes:
    return TaskModel(task_id=str(uid).upper() if upper else str(uid), task_name=name, task_created_by=by,
                     task_created_on=created, task_due_date=due, task_assigned_to=to, is_completed=done,
                     is_over_due=over).to_store_json().encode()


@settings(max_examples=300, deadline=None)
@given(st.lists(st.tuples(_text, _text, _text, _dt, _dt, st.booleans(), st.booleans(), st.booleans(), st.uuids(),
                          st.sampled_from([b"", b"1", b"77"]), st.sampled_from(["ok", "ok", "ok", "gone", "spaced"])),
                max_size=10),
       st.sampled_from([b"", b"3"]), st.booleans(), st.booleans())
def test_query_pb_tasks_equals_the_chain(rows, token, by_created, descending):
    n = _n()
    items, escaped = [], False
    for name, by, to, created, due, done, over, upper, uid, etag, how in rows:
        data = b"" if how == "gone" else _task(name, by, to, created, due, done, over, uid, upper)
        if how == "spaced":
            data = json.dumps(json.loads(data)).encode()
        escaped |= b"\\" in data
        items.append(_item(str(uid).encode(), data, etag))
    msg = b"".join(items) + _s(2, token)
    js = n.dapr_pb_query_json(msg)
    chain = n.tasks_from_query(js, by_created, descending) if js is not None else None
    fast = n.tasks_from_query_pb(msg, by_created, descending)
    assert fast is None or fast == chain
    # the store's own layout (no deleted item, no re-spaced task, no escaped character) is read in one pass
    if all(r[-1] == "ok" for r in rows) and not escaped:
        assert fast is not None and fast == chain


@settings(max_examples=300, deadline=None)
@given(st.lists(st.tuples(_text, _dt, st.booleans(), st.booleans(), st.uuids(), st.sampled_from([b"", b"7", b"123"]),
                          st.sampled_from(["ok", "ok", "ok", "gone", "null", "spaced", "error"])), max_size=10),
       st.sampled_from(["statestore", "s"]))
def test_conditional_mark_pb_equals_the_chain(rows, store):
    n = _n()
    items, escaped = [], False
    for name, created, done, over, uid, etag, how in rows:
        data = _task(name, "b@x", "a@x", created, created, done, over, uid)
        escaped |= b"\\" in data
        if how == "gone":
            data = b""
        elif how == "null":
            data = b"null"
        elif how == "spaced":
            data = json.dumps(json.loads(data)).encode()
        items.append(_item(str(uid).encode(), data, etag, b"boom" if how == "error" else b""))
    msg = b"".join(items)
    fast = n.tasks_conditional_mark_pb(msg, store)
    js = n.dapr_pb_bulk_state_json(msg)
    cm = n.tasks_conditional_mark(js) if js is not None else None
    if cm is None:
        assert fast is None
        return
    ids, bulk, skipped = cm
    save = n.dapr_pb_save_state_bulk(store, bulk) if ids else None
    if fast is not None:
        assert fast[1] == ids and fast[2] == skipped
        if ids:
            assert fast[0] == save
    if all(r[-1] in ("ok", "gone", "null") for r in rows) and not escaped:
        assert fast is not None


@settings(max_examples=300, deadline=None)
@given(st.lists(st.tuples(_text, _dt, _dt, st.booleans(), st.uuids(), st.booleans()), max_size=10),
       st.booleans())
def test_mark_overdue_ids_equals_the_binder(rows, spaced):
    n = _n()
    tasks = [TaskModel(task_id=str(uid).upper() if upper else str(uid), task_name=name, task_created_on=c,
                       task_due_date=d, is_completed=done).to_json() for name, c, d, done, uid, upper in rows]
    body = ("[" + ",".join(tasks) + "]").encode()
    if spaced:
        body = json.dumps(json.loads(body)).encode()
    fast = n.tasks_mark_overdue_ids(body)
    ref = n.tasks_mark_overdue(body)
    assert fast is None or (ref is not None and fast == ref[0])
    if not spaced and b"\\" not in body:
        assert fast is not None and fast == ref[0]


@pytest.mark.parametrize("body", [b"", b"[", b"[1]", b'[{"taskId":"x"}]', b"{}", b'[{"a":1}]'])
def test_mark_overdue_ids_declines(body):
    assert _n().tasks_mark_overdue_ids(body) is None


def _compact(s: str) -> str:
    out, in_str, esc = [], False, False
    for ch in s:
        if in_str:
            out.append(ch)
            if esc:
                esc = False
            elif ch == "\\":
                esc = True
            elif ch == '"':
                in_str = False
        elif ch == '"':
            in_str = True
            out.append(ch)
        elif ch not in " \n\r\t":
            out.append(ch)
    return "".join(out)


def _query_pb_ref(text: bytes) -> bytes:
    doc = json.loads(text)
    out = b""
    for r in doc.get("results") or []:
        data = b""
        if r.get("data") is not None:
            raw = json.dumps(r["data"], ensure_ascii=False, separators=(", ", ": "), indent=None)
            data = _compact(raw).encode()
        out += _item((r.get("key") or "").encode(), data, (r.get("etag") or "").encode(),
                     (r.get("error") or "").encode())
    if doc.get("token"):
        out += _s(2, doc["token"].encode())
    return out


_json_val = st.recursive(st.none() | st.booleans() | st.integers(-9, 99) | _text,
                         lambda ch: st.lists(ch, max_size=3) | st.dictionaries(_text, ch, max_size=3), max_leaves=6)


@settings(max_examples=300, deadline=None)
@given(st.lists(st.tuples(st.text("abc-0123", max_size=8), _json_val, st.text("0123456789", max_size=3),
                          st.booleans()), max_size=8),
       st.text("0123456789", max_size=3), st.sampled_from([(",", ":"), (", ", ": ")]), st.booleans())
def test_query_response_pb_equals_the_results(rows, token, seps, indent):
    """The sidecar's encoder (one pass, strings skipped 16 bytes a step, compact data kept as
    is) writes each result's key, compacted data and etag, and the token -- for compact and
    spaced / indented answers alike."""
    doc = {"results": [{"key": k, "data": d, "etag": e} if present else {"key": k, "etag": e}
                       for k, d, e, present in rows], "token": token}
    text = json.dumps(doc, ensure_ascii=False, separators=seps, indent=2 if indent else None).encode()
    got = _n().dapr_pb_query_from_json(text)
    assert got is not None and got == _query_pb_ref(text)


@pytest.mark.parametrize("text", [b'{"results":[{"key":"a\\"b","data":1}]}', b'{"metadata":{},"results":[]}',
                                  b'{"results":[{"key":"a","data":1,"x":2}]}', b"[", b'{"results":[}'])
def test_query_response_pb_declines(text):
    assert _n().dapr_pb_query_from_json(text) is None


def test_the_sweeps_real_page_goes_one_pass_end_to_end():
    """A page as the backing answers it, through the sidecar's encoder and the app host's reader:
    the API's page, byte for byte what the chain gives."""
    n = _n()
    datas = [_task(f"t{i}", "b@x", "a@x", datetime(2026, 10, 17, 10, 0, i % 60, i), datetime(2026, 10, 16), False,
                   False, uuid.UUID(int=i + 1)) for i in range(50)]
    text = ('{"results":[' + ",".join(f'{{"key":"k{i}","data":{d.decode()},"etag":"{i + 1}"}}' for i, d in enumerate(datas))
            + '],"token":""}').encode()
    pb = n.dapr_pb_query_from_json(text)
    fast = n.tasks_from_query_pb(pb, True, False)
    assert fast is not None and fast == n.tasks_from_query(text, True, False) and fast[0] == 50
