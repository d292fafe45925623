"""Native document store + broker engine tests (unit + property tests against a
brute-force Python model of the query semantics)."""
import json
import time

import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from aca_dotnet_workshop_amd import native

N = native.load()


def test_set_get_etag_concurrency():
    s = N.DocStore()
    e1 = s.set("k", json.dumps({"a": 1}))
    v, e = s.get("k")
    assert json.loads(v) == {"a": 1} and e == e1
    e2 = s.set("k", json.dumps({"a": 2}), etag=e1)
    assert e2 != e1
    with pytest.raises(N.EtagMismatch):
        s.set("k", "{}", etag=e1)  # stale etag
    with pytest.raises(N.EtagMismatch):
        s.set("k", "{}", first_write=True)  # first-write on existing key without etag
    s.set("new", "{}", first_write=True)
    with pytest.raises(N.EtagMismatch):
        s.delete("k", etag=e1)
    assert s.delete("k", etag=e2) is True
    assert s.get("k") is None
    assert s.delete("k") is False
    with pytest.raises(ValueError):
        s.set("bad", "{not json")


def test_ttl_expiry():
    s = N.DocStore()
    s.set("t", "1", ttl_ms=50)
    assert s.get("t") is not None
    time.sleep(0.08)
    assert s.get("t") is None


def test_transaction_all_or_nothing():
    s = N.DocStore()
    e = s.set("a", "1")
    with pytest.raises(N.EtagMismatch):
        s.transact([N.TxOp(False, "b", "2"), N.TxOp(False, "a", "3", etag="999")])
    assert s.get("b") is None and s.get("a")[0] == "1"
    s.transact([N.TxOp(False, "b", "2"), N.TxOp(True, "a", etag=e)])
    assert s.get("a") is None and s.get("b")[0] == "2"


def _docs():
    return [
        {"taskCreatedBy": "a@x", "taskDueDate": "2024-05-01T00:00:00", "n": 3, "isCompleted": False},
        {"taskCreatedBy": "b@x", "taskDueDate": "2024-05-02T00:00:00", "n": 1, "isCompleted": True},
        {"taskCreatedBy": "a@x", "taskDueDate": "2024-05-02T00:00:00", "n": 2, "isCompleted": False, "nested": {"k": "v"}},
    ]


def test_query_filters_sort_page_prefix():
    s = N.DocStore()
    for i, d in enumerate(_docs()):
        s.set(f"app||{i}", json.dumps(d))
    s.set("other||9", json.dumps({"taskCreatedBy": "a@x"}))

    def q(query, prefix="app||"):
        return json.loads(s.query(json.dumps(query), prefix))

    r = q({"filter": {"EQ": {"taskCreatedBy": "a@x"}}})
    assert [x["key"] for x in r["results"]] == ["0", "2"]
    assert r["results"][0]["data"]["n"] == 3 and "etag" in r["results"][0]
    r = q({"filter": {"AND": [{"EQ": {"taskCreatedBy": "a@x"}}, {"EQ": {"taskDueDate": "2024-05-02T00:00:00"}}]}})
    assert [x["key"] for x in r["results"]] == ["2"]
    r = q({"filter": {"OR": [{"EQ": {"n": 1}}, {"IN": {"n": [3, 7]}}]}})
    assert [x["key"] for x in r["results"]] == ["0", "1"]
    r = q({"filter": {"EQ": {"nested.k": "v"}}})
    assert [x["key"] for x in r["results"]] == ["2"]
    r = q({"sort": [{"key": "n", "order": "DESC"}]})
    assert [x["data"]["n"] for x in r["results"]] == [3, 2, 1]
    r = q({"sort": [{"key": "n"}], "page": {"limit": 2}})
    assert [x["data"]["n"] for x in r["results"]] == [1, 2] and r["token"] == "2"
    r = q({"sort": [{"key": "n"}], "page": {"limit": 2, "token": "2"}})
    assert [x["data"]["n"] for x in r["results"]] == [3] and "token" not in r
    r = q({"filter": {"GT": {"n": 1}}})
    assert sorted(x["data"]["n"] for x in r["results"]) == [2, 3]
    r = q({"filter": {"NEQ": {"isCompleted": True}}})
    assert [x["key"] for x in r["results"]] == ["0", "2"]
    assert len(q({}, prefix="")["results"]) == 4
    with pytest.raises(ValueError):
        q({"filter": {"LIKE": {"n": 1}}})
    with pytest.raises(ValueError):
        q({"filter": {"AND": []}})


def test_secondary_index_used_and_maintained():
    s = N.DocStore("", 0, 8)
    for i in range(100):
        s.set(f"k{i}", json.dumps({"owner": f"u{i % 10}", "i": i}))
    r = json.loads(s.query(json.dumps({"filter": {"EQ": {"owner": "u3"}}})))
    assert [x["data"]["i"] for x in r["results"]] == list(range(3, 100, 10))
    assert "owner" in s.indexed_paths()
    assert s.stats()["indexed_queries"] >= 1
    s.set("k3", json.dumps({"owner": "u4", "i": 3}))  # move between index buckets
    s.delete("k13")
    r = json.loads(s.query(json.dumps({"filter": {"EQ": {"owner": "u3"}}})))
    assert [x["data"]["i"] for x in r["results"]] == [i for i in range(3, 100, 10) if i not in (3, 13)]


def test_growth_keeps_lookups_order_and_counts():
    """The document map grows a shard at a time (native/src/shardedmap.hpp): across many growth
    steps every key stays reachable, deletes and updates are exact, ``len`` counts the live
    documents, and an unsorted query still answers in insertion order."""
    s = N.DocStore("", 0, 1 << 30)  # no secondary index: the scan path walks the whole map
    n = 20000
    keys = [f"app||{(i * 7919) % 100003:06d}-{i}" for i in range(n)]
    for i, k in enumerate(keys):
        s.set(k, json.dumps({"i": i}))
    assert len(s) == n
    for k in keys[::3]:
        assert s.delete(k) is True
    s.set(keys[1], json.dumps({"i": 1, "updated": True}))
    live = [i for i in range(n) if i % 3]
    assert len(s) == len(live)
    assert s.get(keys[0]) is None and json.loads(s.get(keys[1])[0])["updated"] is True
    assert all(json.loads(s.get(keys[i])[0])["i"] == i for i in live[::97])
    r = json.loads(s.query(json.dumps({"filter": {"GT": {"i": -1}}}), "app||"))
    assert [x["data"]["i"] for x in r["results"]] == live


def test_persistence_and_compaction(tmp_path):
    p = str(tmp_path / "state.log")
    s = N.DocStore(p)
    e = None
    for i in range(200):
        e = s.set("hot", json.dumps({"v": i}))
    s.set("cold", '"x"')
    s.delete("cold")
    s.set("keep", "[1,2]")
    del s
    s2 = N.DocStore(p)
    assert s2.get("hot") == ('{"v": 199}', e)
    assert s2.get("cold") is None and s2.get("keep")[0] == "[1,2]"
    before = s2.stats()["log_bytes"]
    s2.compact()
    assert s2.stats()["log_bytes"] < before
    del s2
    s3 = N.DocStore(p)
    assert s3.get("hot")[1] == e and len(s3) == 2
    # new writes keep increasing etags after recovery
    assert int(s3.set("hot", "{}")) > int(e)


# --- property test: native query == brute-force Python evaluation -------------
scalars = st.one_of(st.none(), st.booleans(), st.integers(-3, 3), st.sampled_from(["a", "b", "c"]))
docs_st = st.lists(st.fixed_dictionaries({}, optional={"f": scalars, "g": scalars}), max_size=25)


def leaf():
    path = st.sampled_from(["f", "g"])
    return st.one_of(
        st.builds(lambda p, v: {"EQ": {p: v}}, path, scalars),
        st.builds(lambda p, v: {"NEQ": {p: v}}, path, scalars),
        st.builds(lambda p, vs: {"IN": {p: vs}}, path, st.lists(scalars, min_size=1, max_size=3)),
        st.builds(lambda p, v: {"GT": {p: v}}, path, st.integers(-3, 3)),
        st.builds(lambda p, v: {"LTE": {p: v}}, path, st.integers(-3, 3)),
    )


filters_st = st.recursive(leaf(), lambda inner: st.one_of(
    st.builds(lambda xs: {"AND": xs}, st.lists(inner, min_size=1, max_size=3)),
    st.builds(lambda xs: {"OR": xs}, st.lists(inner, min_size=1, max_size=3))), max_leaves=6)

_MISSING = object()


def _jeq(a, b):
    if isinstance(a, bool) or isinstance(b, bool):
        return type(a) is type(b) and a == b
    return a == b


def _py_eval(f, d):
    (op, arg), = f.items()
    if op == "AND":
        return all(_py_eval(x, d) for x in arg)
    if op == "OR":
        return any(_py_eval(x, d) for x in arg)
    (path, val), = arg.items()
    v = d.get(path, _MISSING)
    if op == "EQ":
        return v is not _MISSING and _jeq(v, val)
    if op == "NEQ":
        return v is _MISSING or not _jeq(v, val)
    if op == "IN":
        return v is not _MISSING and any(_jeq(v, x) for x in val)
    if v is _MISSING or isinstance(v, bool) or not isinstance(v, int):
        return False
    return v > val if op == "GT" else v <= val


@settings(max_examples=200, deadline=None)
@given(docs_st, filters_st, st.integers(1, 4))
def test_query_matches_bruteforce(docs, flt, threshold):
    s = N.DocStore("", 0, threshold)  # small threshold -> exercises the index planner too
    for i, d in enumerate(docs):
        s.set(str(i), json.dumps(d))
    got = [int(x["key"]) for x in json.loads(s.query(json.dumps({"filter": flt})))["results"]]
    want = [i for i, d in enumerate(docs) if _py_eval(flt, d)]
    assert got == want


# --- broker -------------------------------------------------------------------
def test_broker_fanout_and_competing_consumers():
    b = N.Broker()
    b.create_subscription("tasksavedtopic", "processor")
    b.create_subscription("tasksavedtopic", "audit")
    for i in range(5):
        b.publish("tasksavedtopic", json.dumps({"i": i}).encode())
    # two competing receivers on one subscription never see the same message
    r1 = b.receive("tasksavedtopic/subscriptions/processor", 3)
    r2 = b.receive("tasksavedtopic/subscriptions/processor", 3)
    got = [json.loads(m.body)["i"] for m in r1 + r2]
    assert got == [0, 1, 2, 3, 4]
    assert b.counts("tasksavedtopic/subscriptions/audit")["active"] == 5
    for m in r1 + r2:
        assert b.complete("tasksavedtopic/subscriptions/processor", m.lock_token)
    c = b.counts("tasksavedtopic/subscriptions/processor")
    assert (c["active"], c["locked"], c["completed"]) == (0, 0, 5)
    # topic without subscriptions drops messages (Service Bus semantics)
    assert b.publish("nosubs", b"x") == 0


def test_broker_abandon_lock_expiry_and_dead_letter():
    b = N.Broker()
    b.create_subscription("t", "s", N.QueueOptions(lock_ms=60000, max_delivery=3))
    p = "t/subscriptions/s"
    b.publish("t", b"m")
    m = b.receive(p)[0]
    assert m.delivery_count == 1
    assert b.abandon(p, m.lock_token)
    m = b.receive(p, 1, 30)[0]
    assert m.delivery_count == 2
    assert not b.complete(p, "bogus")
    # lock expiry makes it visible again
    time.sleep(0.05)
    m = b.receive(p, 1, 30)[0]
    assert m.delivery_count == 3
    time.sleep(0.06)
    assert b.receive(p) == []  # 3rd delivery expired -> max delivery -> DLQ
    c = b.counts(p)
    assert c["dead_letter"] == 1 and c["active"] == 0
    dl = b.drain_dead_letters(p)
    assert dl[0][2] == b"m" and dl[0][3] == "MaxDeliveryCountExceeded"
    b.publish("t", b"n")
    m = b.receive(p)[0]
    assert b.dead_letter(p, m.lock_token, "bad payload")
    assert b.drain_dead_letters(p)[0][3] == "bad payload"


def test_broker_delay_ttl_renew_queue():
    b = N.Broker()
    b.create_queue("q", N.QueueOptions(lock_ms=40))
    b.send("q", b"later", delay_ms=60)
    b.send("q", b"short", ttl_ms=1)
    time.sleep(0.01)
    assert b.receive("q") == []  # 'short' expired, 'later' not yet visible
    c = b.counts("q")
    assert c["scheduled"] == 1
    time.sleep(0.07)
    m = b.receive("q")[0]
    assert m.body == b"later"
    assert b.renew("q", m.lock_token, 1000)
    time.sleep(0.06)
    assert b.receive("q") == []  # renewed lock still held
    assert b.complete("q", m.lock_token)


def test_broker_persistence(tmp_path):
    p = str(tmp_path / "bus.log")
    b = N.Broker(p)
    b.create_subscription("t", "s")
    for i in range(3):
        b.publish("t", str(i).encode())
    m = b.receive("t/subscriptions/s")[0]
    b.complete("t/subscriptions/s", m.lock_token)
    b.send("q", b"queued")
    del b
    b2 = N.Broker(p)
    got = [x.body for x in b2.receive("t/subscriptions/s", 10)]
    assert got == [b"1", b"2"]
    assert b2.receive("q")[0].body == b"queued"
