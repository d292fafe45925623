"""Backing-services parity between the Python handlers and the native HTTP front
(native/src/backingfront.hpp): document CRUD with ETags, publish / long-poll receive /
settle / counts, RBAC decisions, non-UTF-8 bodies, and collections mirrored by the columnar
query accelerator keeping their writes on the native front."""
import asyncio
import time

import pytest

from aca_dotnet_workshop_amd.backing.client import BackingClient, BackingError, EtagConflict
from aca_dotnet_workshop_amd.backing.server import serve_backing
from aca_dotnet_workshop_amd.web import HttpClient

from helpers import run

FRONTS = ["python", "native"]


class Backing:
    def __init__(self, front, monkeypatch, policy=None):
        monkeypatch.setenv("TT_BACKING_FRONT", front)
        self.policy = policy

    async def __aenter__(self):
        ready = asyncio.get_running_loop().create_future()
        self.stop = asyncio.Event()
        self.task = asyncio.ensure_future(serve_backing("127.0.0.1", 0, None, self.policy, ready.set_result, self.stop))
        port = await asyncio.wait_for(ready, 20)
        self.base = f"http://127.0.0.1:{port}"
        return self

    async def __aexit__(self, *exc):
        self.stop.set()
        await asyncio.wait_for(self.task, 20)


@pytest.mark.parametrize("front", FRONTS)
def test_documents(front, monkeypatch):
    async def main():
        async with Backing(front, monkeypatch) as b:
            c = BackingClient(b.base, identity="x")
            e1 = await c.doc_put("acct", "db", "c", "k/1 é", '{"a": 1}')
            got = await c.doc_get("acct", "db", "c", "k/1 é")
            assert got == (b'{"a": 1}', e1) or got[1] == e1
            with pytest.raises(EtagConflict):
                await c.doc_put("acct", "db", "c", "k/1 é", "2", etag="bogus")
            with pytest.raises(EtagConflict):
                await c.doc_put("acct", "db", "c", "k/1 é", "2", first_write=True)
            e2 = await c.doc_put("acct", "db", "c", "k/1 é", "2", etag=e1)
            assert e2 != e1
            assert await c.doc_get("acct", "db", "c", "missing") is None
            with pytest.raises(EtagConflict):
                await c.doc_delete("acct", "db", "c", "k/1 é", etag=e1)
            assert await c.doc_delete("acct", "db", "c", "k/1 é") is True
            assert await c.doc_delete("acct", "db", "c", "k/1 é") is False
            with pytest.raises(BackingError) as ei:
                await c.doc_put("acct", "db", "c", "bad", "{not json")
            assert ei.value.status == 400
            # query (always Python) sees documents written through the front
            await c.doc_put("acct", "db", "c", "q1", '{"n": 5}')
            res = await c.doc_query("acct", "db", "c", b'{"filter": {"EQ": {"n": 5}}}')
            assert b'"q1"' in res
            # bulk save (multi-item state saves): per-item etags, 412 on any etag conflict
            res = await c.doc_bulk_set("acct", "db", "c", [{"key": f"b{i}", "value": '{"i": %d}' % i, "etag": None,
                                                             "firstWrite": False, "ttlMs": 0} for i in range(3)])
            assert [x["key"] for x in res] == ["b0", "b1", "b2"] and all(x.get("etag") for x in res)
            with pytest.raises(EtagConflict):
                await c.doc_bulk_set("acct", "db", "c", [{"key": "b0", "value": "1", "etag": "nope"}])
            assert (await c.doc_get("acct", "db", "c", "b2"))[0] == b'{"i": 2}'
            # bulk get (the read half of markoverdue's conditional save): request order, etags,
            # a missing key without data
            got = await c.doc_bulk_get("acct", "db", "c", ["b2", "missing", "b0"])
            etag_b0 = (await c.doc_get("acct", "db", "c", "b0"))[1]
            assert got == [{"key": "b2", "data": {"i": 2}, "etag": got[0]["etag"]}, {"key": "missing"},
                           {"key": "b0", "data": {"i": 0}, "etag": etag_b0}]
            fs = (await c.http.get(b.base + "/admin/front")).json()
            assert fs["front"] == front
            if front == "native":
                assert fs["requests"]["doc.put"] >= 4 and fs["requests"]["doc.get"] >= 2
                assert fs["requests"]["doc.bulkget"] == 1
            await c.http.close()
    run(main())


@pytest.mark.parametrize("front", FRONTS)
def test_bulk_set_items_fail_alone_and_persist(front, monkeypatch, tmp_path):
    """A bulk save is not atomic: an item with a failed ETag precondition or invalid JSON fails
    alone (412 wins over 400), the others are applied in order -- the native front writes the
    whole batch under one store lock with one log write -- and the batch survives a restart of
    the store from its log."""
    import json as _json

    items = [{"key": "a", "value": '{"v": 1}'}, {"key": "a", "value": '{"v": 2}'},
             {"key": "b", "value": '{"v": 3}', "etag": "nope"}, {"key": "c", "value": "{not json"},
             {"key": "d", "value": {"v": [4]}}, {"key": "e", "value": '"x"', "firstWrite": True}]

    class Persisted(Backing):
        async def __aenter__(self):
            ready = asyncio.get_running_loop().create_future()
            self.stop = asyncio.Event()
            self.task = asyncio.ensure_future(serve_backing("127.0.0.1", 0, str(tmp_path), None, ready.set_result,
                                                            self.stop))
            self.base = f"http://127.0.0.1:{await asyncio.wait_for(ready, 20)}"
            return self

    async def main():
        async with Persisted(front, monkeypatch) as b:
            c = BackingClient(b.base, identity="x")
            await c.doc_put("acct", "db", "c", "seed", "0")
            r = await c.http.post(b.base + "/cosmos/acct/db/c/bulkset", body=_json.dumps(items).encode(),
                                  headers={"Content-Type": "application/json"})
            assert r.status == 412
            out = r.json()
            assert [o["key"] for o in out] == ["a", "a", "b", "c", "d", "e"]
            assert [o.get("error") for o in out] == [None, None, "etag", "invalid", None, None]
            assert int(out[1]["etag"]) > int(out[0]["etag"])
            assert (await c.doc_get("acct", "db", "c", "a"))[0] == b'{"v": 2}'
            assert await c.doc_get("acct", "db", "c", "b") is None
            assert await c.doc_get("acct", "db", "c", "c") is None
            assert _json.loads((await c.doc_get("acct", "db", "c", "d"))[0]) == {"v": [4]}
            r = await c.http.post(b.base + "/cosmos/acct/db/c/bulkset", headers={"Content-Type": "application/json"},
                                  body=_json.dumps([{"key": "f", "value": "1"}, {"key": "g", "value": "{"}]).encode())
            assert r.status == 400 and [o.get("error") for o in r.json()] == [None, "invalid"]
            await c.http.close()
        async with Persisted(front, monkeypatch) as b:  # replayed from the log
            c = BackingClient(b.base, identity="x")
            assert (await c.doc_get("acct", "db", "c", "a"))[0] == b'{"v": 2}'
            assert (await c.doc_get("acct", "db", "c", "e"))[0] == b'"x"'
            assert (await c.doc_get("acct", "db", "c", "f"))[0] == b"1"
            assert await c.doc_get("acct", "db", "c", "b") is None
            await c.http.close()
    run(main())


def test_ttl_writes_store_the_same_bytes_as_native_writes(monkeypatch):
    """A bulk item with a TTL is stored by the Python handlers (the native front leaves TTL
    writes to them), one without by the native front: the same value text is stored either way
    -- numbers as sent (1e3 stays 1e3), escapes as sent (\u00e9 stays escaped)."""
    import json as _json
    raw = b'{"n": 1e3, "f": -0.5E+2, "s": "caf\\u00e9 \\ud83d\\ude00", "big": 12345678901234567890}'

    async def main():
        async with Backing("native", monkeypatch) as b:
            c = BackingClient(b.base, identity="x")
            await c.doc_put("acct", "db", "c", "seed", "0")  # the collection exists: the front takes plain writes
            for key, ttl in (("plain", 0), ("ttl", 60000)):
                body = b'[{"key": "%s", "value": %s, "etag": null, "firstWrite": false, "ttlMs": %d}]' % (
                    key.encode(), raw, ttl)
                r = await c.http.post(b.base + "/cosmos/acct/db/c/bulkset", body=body,
                                      headers={"Content-Type": "application/json"})
                assert r.status == 200, r.body
            plain = (await c.doc_get("acct", "db", "c", "plain"))[0]
            ttl = (await c.doc_get("acct", "db", "c", "ttl"))[0]
            assert plain == ttl == b'{"n":1e3,"f":-0.5E+2,"s":"caf\\u00e9 \\ud83d\\ude00","big":12345678901234567890}'
            assert _json.loads(ttl)["s"] == "caf\u00e9 \U0001F600"
            fs = (await c.http.get(b.base + "/admin/front")).json()
            assert fs["requests"]["doc.bulkset"] == 1 and fs["requests"]["forwarded"] >= 1  # one each way
            await c.http.close()
    run(main())


@pytest.mark.parametrize("front", FRONTS)
def test_transactions_store_the_same_bytes_as_saves(front, monkeypatch):
    """A transaction's values are stored as the request's own compact bytes, like a save's: 1e3
    stays 1e3, escapes stay escaped, a 20-digit integer keeps every digit (the
    transaction route re-serialised them through json.dumps)."""
    raw = b'{"n": 1e3, "f": -0.5E+2, "s": "caf\\u00e9 \\ud83d\\ude00", "big": 12345678901234567890}'
    want = b'{"n":1e3,"f":-0.5E+2,"s":"caf\\u00e9 \\ud83d\\ude00","big":12345678901234567890}'

    async def main():
        async with Backing(front, monkeypatch) as b:
            c = BackingClient(b.base, identity="x")
            await c.doc_put("acct", "db", "c", "seed", "0")
            r = await c.http.post(b.base + "/cosmos/acct/db/c/bulkset", headers={"Content-Type": "application/json"},
                                  body=b'[{"key": "saved", "value": %s}]' % raw)
            assert r.status == 200, r.body
            body = (b'{"ops": [{"op": "upsert", "key": "tx", "value": %s}, {"op": "delete", "key": "seed"}, '
                    b'{"op": "upsert", "key": "tx-text", "value": "[1.50, \\"x\\"]"}]}' % raw)
            r = await c.http.post(b.base + "/cosmos/acct/db/c/transaction", body=body,
                                  headers={"Content-Type": "application/json"})
            assert r.status == 204, r.body
            assert (await c.doc_get("acct", "db", "c", "saved"))[0] == want
            assert (await c.doc_get("acct", "db", "c", "tx"))[0] == want
            assert (await c.doc_get("acct", "db", "c", "tx-text"))[0] == b'[1.50, "x"]'  # a string holds JSON text
            assert await c.doc_get("acct", "db", "c", "seed") is None
            await c.http.close()
    run(main())


def test_tx_values_scanner():
    from aca_dotnet_workshop_amd import native
    N = native.load()
    assert N.tx_values(b'{"ops": [{"value": {"a" : 1e3}}, {"op": "delete"}, {"value": "\\"t\\""}]}') == \
        ['{"a":1e3}', "null", '"t"']
    assert N.tx_values(b'{"x": 1}') is None and N.tx_values(b"[1]") is None and N.tx_values(b"{bad") is None


@pytest.mark.parametrize("front", FRONTS)
def test_messaging_and_long_poll(front, monkeypatch):
    async def main():
        async with Backing(front, monkeypatch) as b:
            c = BackingClient(b.base, identity="x")
            await c.sb_create_subscription("ns", "t", "s", lock_ms=60000, max_delivery=2)
            ent = "t/subscriptions/s"
            # a receive parked before the publish wakes up promptly
            t0 = time.monotonic()
            recv = asyncio.ensure_future(c.sb_receive("ns", ent, 5, 0, 3000))
            await asyncio.sleep(0.1)
            await c.sb_publish("ns", "t", b'{"x": 1}', "application/json", {"k": "v"})
            msgs = await recv
            assert time.monotonic() - t0 < 1.5
            assert len(msgs) == 1 and msgs[0]["body"] == '{"x": 1}' and msgs[0]["props"] == {"k": "v"}
            assert msgs[0]["deliveryCount"] == 1
            # abandon -> redelivered, then complete
            res = await c.sb_settle("ns", ent, abandon=[{"token": msgs[0]["lockToken"]}])
            assert res["abandon"] == [True]
            again = await c.sb_receive("ns", ent, 5, 0, 1000)
            assert again[0]["deliveryCount"] == 2
            res = await c.sb_settle("ns", ent, complete=[again[0]["lockToken"], "nope"])
            assert res["complete"] == [True, False]
            cnt = await c.sb_counts("ns", ent)
            assert cnt["completed"] == 1 and cnt["active"] == 0 and cnt["enqueued"] == 1
            # binary payloads travel base64-encoded
            await c.sb_publish("ns", "t", b"\xff\x00\x01", "application/octet-stream")
            m = (await c.sb_receive("ns", ent, 1, 0, 1000))[0]
            assert "bodyB64" in m and m["contentType"] == "application/octet-stream"
            # an empty long-poll returns [] after its wait
            await c.sb_settle("ns", ent, complete=[m["lockToken"]])
            t0 = time.monotonic()
            assert await c.sb_receive("ns", ent, 1, 0, 300) == []
            assert 0.25 < time.monotonic() - t0 < 2.0
            await c.http.close()
    run(main())


@pytest.mark.parametrize("front", FRONTS)
def test_storage_queue(front, monkeypatch):
    """The storage queue the processor's input binding reads (backing/server.py _storage_routes):
    put, long-poll receive woken by a put, the visibility timeout, release, delete, counts and
    non-UTF-8 bodies -- the same answers on both fronts, and the native front serving them."""
    async def main():
        async with Backing(front, monkeypatch) as b:
            c = BackingClient(b.base, identity="x")
            await c.queue_put("acct", "q", b"first")  # the account's broker is made by Python's route
            assert (await c.queue_get("acct", "q", 1, 30000))[0]["body"] == "first"
            t0 = time.monotonic()
            recv = asyncio.ensure_future(c.queue_get("acct", "q", 5, 60, 3000))
            await asyncio.sleep(0.1)
            mid = await c.queue_put("acct", "q", b"eyJhIjoxfQ==")
            msgs = await recv
            assert time.monotonic() - t0 < 1.5
            assert [(m["messageId"], m["body"], m["dequeueCount"]) for m in msgs] == [(mid, "eyJhIjoxfQ==", 1)]
            assert msgs[0]["insertionMs"] > 0 and msgs[0]["popReceipt"]
            await asyncio.sleep(0.1)  # its 60 ms visibility timeout elapses: it is back
            again = await c.queue_get("acct", "q", 5, 30000)
            assert [(m["messageId"], m["dequeueCount"]) for m in again] == [(mid, 2)]
            assert await c.queue_release("acct", "q", again[0]["popReceipt"], 0)  # visible again now
            third = await c.queue_get("acct", "q", 5, 30000, 1000)
            assert third[0]["dequeueCount"] == 3
            assert await c.queue_delete("acct", "q", third[0]["popReceipt"])
            assert not await c.queue_delete("acct", "q", third[0]["popReceipt"])
            assert not await c.queue_release("acct", "q", "no-such-receipt", 0)
            await c.queue_put("acct", "q", b"\xff\x00")
            m = (await c.queue_get("acct", "q", 1, 30000))[0]
            assert "body" not in m and m["bodyB64"] == "/wA="
            assert await c.queue_delete("acct", "q", m["popReceipt"])
            t0 = time.monotonic()
            assert await c.queue_get("acct", "q", 1, 30000, 300) == []  # an empty long poll ends at its wait
            assert 0.25 < time.monotonic() - t0 < 2.0
            cnt = await c.queue_count("acct", "q")
            assert (cnt["active"], cnt["locked"], cnt["enqueued"], cnt["completed"]) == (0, 1, 3, 2)  # "first" held
            h = HttpClient()
            # a value the Python route parses its own way goes to it (numofmessages=0: no messages)
            r = await h.get(b.base + "/storage/acct/queues/q/messages?numofmessages=0&waitMs=0",
                            headers={"x-tt-identity": "x"})
            assert r.status == 200 and r.json() == []
            stats = (await h.get(b.base + "/admin/front")).json()
            if front == "native":
                req = stats["requests"]
                assert req["queue.put"] >= 2 and req["queue.get"] >= 5 and req["queue.delete"] == 3
                assert req["queue.update"] == 2
            await h.close()
            await c.http.close()
    run(main())


@pytest.mark.parametrize("front", FRONTS)
def test_blobs(front, monkeypatch):
    """The output binding's blobs: a put on either front, read back, listed, counted (the front's
    name set follows Python's deletes too); names Python resolves its own way stay with it."""
    async def main():
        async with Backing(front, monkeypatch) as b:
            c = BackingClient(b.base, identity="x")
            assert await c.blob_count("sa", "box") == 0
            r1 = await c.blob_put("sa", "box", "t1.json", b'{"a": 1}', "application/json")
            assert r1 == {"blobURL": "/storage/sa/blobs/box/t1.json"}
            await c.blob_put("sa", "box", "dir/t2.json", b"\xff\x00", "application/octet-stream")
            await c.blob_put("sa", "box", "t1.json", b'{"a": 2}', "application/json")  # overwrite
            assert await c.blob_get("sa", "box", "t1.json") == b'{"a": 2}'
            assert await c.blob_get("sa", "box", "dir/t2.json") == b"\xff\x00"
            assert sorted(x["name"] for x in await c.blob_list("sa", "box")) == ["dir/t2.json", "t1.json"]
            assert await c.blob_count("sa", "box") == 2 and await c.blob_count("sa", "box", "dir/") == 1
            assert await c.blob_delete("sa", "box", "t1.json")
            assert await c.blob_count("sa", "box") == 1
            with pytest.raises(BackingError) as ei:  # escapes the container: Python's 400 on both
                await c.blob_put("sa", "box", "../../escape", b"x")
            assert ei.value.status == 400
            await c.blob_put("sa", "box", "a/./b.json", b"{}")  # a dot segment: Python's route
            assert await c.blob_count("sa", "box") == 2
            stats = (await c.http.get(b.base + "/admin/front")).json()
            if front == "native":
                assert stats["requests"]["blob.put"] == 3 and stats["requests"]["blob.count"] >= 4
            await c.http.close()
    run(main())


@pytest.mark.parametrize("front", FRONTS)
def test_abandoned_long_poll_takes_no_messages(front, monkeypatch):
    """A receiver that disconnects in the middle of its long poll (its process died) must not get
    -- and lock -- the next message: a live receiver gets it at once, not after the lock expires."""
    async def main():
        async with Backing(front, monkeypatch) as b:
            c = BackingClient(b.base, identity="x")
            await c.sb_create_subscription("ns", "t2", "s", lock_ms=60000, max_delivery=5)
            host, port = b.base.rsplit(":", 1)
            r, w = await asyncio.open_connection("127.0.0.1", int(port))
            w.write(b"POST /servicebus/ns/receive?entity=t2/subscriptions/s&max=5&lockMs=60000&waitMs=10000 HTTP/1.1\r\n"
                    b"host: x\r\nx-tt-identity: x\r\ncontent-length: 0\r\n\r\n")
            await w.drain()
            await asyncio.sleep(0.2)   # parked
            w.close()                  # the receiver dies
            await asyncio.sleep(0.3)
            await c.sb_publish("ns", "t2", b'{"x": 1}', "application/json")
            t0 = time.monotonic()
            msgs = await c.sb_receive("ns", "t2/subscriptions/s", 5, 60000, 3000)
            assert len(msgs) == 1 and msgs[0]["deliveryCount"] == 1 and time.monotonic() - t0 < 1.5
            await c.http.close()
    run(main())


@pytest.mark.parametrize("front", FRONTS)
def test_rbac(front, monkeypatch):
    policy = {"mode": "enforce", "keys": {"cosmos/acct": "masterkey"},
              "roleAssignments": [
                  {"principal": "api-mi", "role": "Cosmos DB Built-in Data Contributor", "scope": "cosmos/acct"},
                  {"principal": "api-mi", "role": "Azure Service Bus Data Sender", "scope": "servicebus/ns/topics/t"},
                  {"principal": "proc-mi", "role": "Azure Service Bus Data Receiver", "scope": "servicebus/ns/topics/t"},
                  {"principal": "admin", "role": "Owner", "scope": ""}]}

    async def main():
        async with Backing(front, monkeypatch, policy) as b:
            admin, api = BackingClient(b.base, identity="admin"), BackingClient(b.base, identity="api-mi")
            proc, anon = BackingClient(b.base, identity="proc-mi"), BackingClient(b.base, identity="")
            keyed = BackingClient(b.base, identity="", key="masterkey")
            await admin.sb_create_subscription("ns", "t", "proc")
            await admin.doc_put("acct", "db", "c", "seed", "0")  # engines exist -> front serves
            await api.doc_put("acct", "db", "c", "k", "1")
            await keyed.doc_put("acct", "db", "c", "k2", "2")
            for call in (anon.doc_put("acct", "db", "c", "k", "1"), proc.doc_get("acct", "db", "c", "k"),
                         proc.sb_publish("ns", "t", b"x"), api.sb_receive("ns", "t/subscriptions/proc")):
                with pytest.raises(BackingError) as ei:
                    await call
                assert ei.value.status == 403
                assert b"not authorized" in ei.value.body
            await api.sb_publish("ns", "t", b"x")
            assert len(await proc.sb_receive("ns", "t/subscriptions/proc")) == 1
            await admin.queue_put("sa", "q", b"m")  # the account's broker exists -> front serves
            for call in (proc.queue_put("sa", "q", b"m"), anon.queue_get("sa", "q")):
                with pytest.raises(BackingError) as ei:
                    await call
                assert ei.value.status == 403 and b"not authorized" in ei.value.body
            assert len(await admin.queue_get("sa", "q")) == 1
            # a policy change at runtime reaches the front
            h = HttpClient()
            r = await h.put(b.base + "/admin/policy", json_body={"mode": "open"})
            assert r.status in (200, 204)
            await anon.doc_put("acct", "db", "c", "k3", "3")
            await h.close()
            for c in (admin, api, proc, anon, keyed):
                await c.http.close()
    run(main())


def test_accelerator_keeps_writes_native(monkeypatch):
    """Once the columnar accelerator mirrors a collection its writes still go through the
    native front: the DocStore appends mirror rows itself, and queries see every write
    (updates, deletes, TTL writes turning the accelerator off) made through either front."""
    monkeypatch.setenv("TT_QUERY_ACCEL", "cpu")
    monkeypatch.setenv("TT_QUERY_ACCEL_MIN_DOCS", "10")

    async def main():
        async with Backing("native", monkeypatch) as b:
            c = BackingClient(b.base, identity="x")
            for i in range(40):
                await c.doc_put("acct", "db", "c", f"k{i}", '{"n": %d}' % i)
            q = b'{"filter": {"GT": {"n": 30}}}'
            assert (await c.doc_query("acct", "db", "c", q)).count(b'"key"') == 9  # builds the mirror
            puts0 = (await c.http.get(b.base + "/admin/front")).json()["requests"]["doc.put"]
            for i in range(40, 60):
                await c.doc_put("acct", "db", "c", f"k{i}", '{"n": %d}' % i)
            await c.doc_put("acct", "db", "c", "k31", '{"n": 1}')  # update drops out of the range
            await c.doc_delete("acct", "db", "c", "k35")
            await c.doc_bulk_set("acct", "db", "c", [{"key": "k2", "value": '{"n": 99}', "etag": None,
                                                      "firstWrite": False, "ttlMs": 0}])
            fs = (await c.http.get(b.base + "/admin/front")).json()
            assert fs["requests"]["doc.put"] - puts0 == 21  # still served natively
            res = await c.doc_query("acct", "db", "c", q)
            assert res.count(b'"key"') == 28 and b'"k31"' not in res and b'"k2"' in res
            st = (await c.doc_stats("acct", "db", "c"))["accelerator"]
            assert st["cpu"] == 2 and st["rows"] == 59 and st["mirror"]["on"] == 1
            # a TTL write turns the mirror off; the native engine answers from then on
            await c.doc_put("acct", "db", "c", "t1", '{"n": 77}', ttl_ms=60000)
            res = await c.doc_query("acct", "db", "c", q)
            assert res.count(b'"key"') == 29
            st = (await c.doc_stats("acct", "db", "c"))["accelerator"]
            assert st["cpu"] == 2 and st["mirror"]["disabled"] == 1
            await c.http.close()
    run(main())


@pytest.mark.parametrize("front", FRONTS)
def test_provisioned_throughput_429(front, monkeypatch):
    """RU token bucket shared by both fronts: 429 with x-ms-retry-after-ms / Retry-After when spent;
    a rejected call is given a reserved slot behind the earlier waiters (the hints are spaced by
    its RU / the rate) and a ticket; the backing client retries at the hint with the ticket."""
    async def main():
        async with Backing(front, monkeypatch) as b:
            c = BackingClient(b.base, identity="x")
            await c.doc_set_throughput("acct", "db", "c", 10.0)
            await asyncio.sleep(1.05)  # the bucket starts empty: a second of refill
            h = HttpClient()
            statuses, hints = [], []
            for i in range(5):
                r = await h.put(f"{b.base}/cosmos/acct/db/c/docs/k{i}", body=b'{"a": 1}',
                                headers={"Content-Type": "application/json", "x-tt-identity": "x"})
                statuses.append(r.status)
                if r.status == 429:
                    hints.append(int(r.headers["x-ms-retry-after-ms"]))
                    assert int(r.headers["retry-after"]) >= 1 and int(r.headers["x-tt-ru-ticket"]) > 0
            assert statuses == [200, 200, 429, 429, 429]
            # 5 RU each at 10 RU/s: the waiters' slots are 500 ms apart, not one shared deficit
            assert len(hints) == 3 and all(abs(b - a - 500) <= 20 for a, b in zip(hints, hints[1:])), hints
            await c.doc_put("acct", "db", "c", "late", '{"a": 2}')  # retried transparently
            assert c.throttled_retries >= 1
            st = await c.doc_stats("acct", "db", "c")
            assert st["throughput"]["ru_per_s"] == 10.0 and st["throughput"]["throttled"] >= 1
            await c.doc_set_throughput("acct", "db", "c", 0)  # unlimited again
            for i in range(20):
                await c.doc_put("acct", "db", "c", f"u{i}", "1")
            await h.close()
            await c.http.close()
    run(main())


@pytest.mark.parametrize("front", FRONTS)
def test_throttled_retry_at_the_hint_without_a_ticket_gets_in(front, monkeypatch):
    """a client that follows only the Cosmos contract -- retry after
    x-ms-retry-after-ms, no ticket -- is admitted at its slot: the reservation is bound to the
    request (method + target), so the same request claims it; an early retry is told the time
    left without a second reservation.  Tickets are random, and another request presenting a
    ticket it did not get is not admitted on it."""
    async def main():
        async with Backing(front, monkeypatch) as b:
            c = BackingClient(b.base, identity="x")
            await c.doc_set_throughput("acct", "db", "c", 20.0)
            await asyncio.sleep(1.05)  # the bucket starts empty: a second of refill
            h = HttpClient()
            hd = {"Content-Type": "application/json", "x-tt-identity": "x"}
            for i in range(4):  # spend the bucket (5 RU each at 20 RU/s)
                r = await h.put(f"{b.base}/cosmos/acct/db/c/docs/p{i}", body=b'{"a": 1}', headers=hd)
                assert r.status == 200
            url = f"{b.base}/cosmos/acct/db/c/docs/lone"
            r = await h.put(url, body=b'{"a": 1}', headers=hd)
            assert r.status == 429
            hint, ticket = int(r.headers["x-ms-retry-after-ms"]), int(r.headers["x-tt-ru-ticket"])
            assert 150 <= hint <= 300, hint
            # someone else's request presenting that ticket: not admitted on it (its own 429)
            r2 = await h.put(f"{b.base}/cosmos/acct/db/c/docs/thief", body=b'{"a": 1}',
                             headers={**hd, "x-tt-ru-ticket": str(ticket)})
            assert r2.status == 429 and r2.headers["x-tt-ru-ticket"] != str(ticket)
            # an early retry of the same request, no ticket: the time left, same reservation
            r3 = await h.put(url, body=b'{"a": 1}', headers=hd)
            assert r3.status == 429 and int(r3.headers["x-ms-retry-after-ms"]) <= hint
            assert r3.headers.get("x-tt-ru-ticket") == str(ticket)
            await asyncio.sleep(hint / 1000 + 0.01)
            r4 = await h.put(url, body=b'{"a": 1}', headers=hd)  # at the hint, no ticket
            assert r4.status == 200, (r4.status, r4.headers)
            st = (await c.doc_stats("acct", "db", "c"))["throughput"]
            assert st["reserved_admits"] == 1 and st["early_retries"] == 1 and st["throttled_write"] == 2
            assert st["open_reservations"] == 1  # the thief's own, unclaimed
            await h.close()
            await c.http.close()
    run(main())


def test_unclaimed_reservations_lapse_and_refund():
    """A reservation whose caller gave up lapses kTicketTtlS after its slot and its RU go back to
    the bucket; admitted RU never exceed the budget's refill over the window (+ one call): the
    bucket starts empty (ru_consumed <= budget x window)."""
    import threading
    import time as _t

    from aca_dotnet_workshop_amd import native
    N = native.load()
    s = N.DocStore()
    s.set_throughput(200.0)
    t0 = _t.monotonic()
    admitted = [0.0]
    stop = threading.Event()

    def worker(w):
        i = 0
        while not stop.is_set():
            i += 1
            ticket, bind = 0, f"PUT /w{w}/{i}"
            while not stop.is_set():
                wait, ticket = s.charge(5.0, ticket, bind, 1)
                if not wait:
                    admitted[0] += 5.0
                    break
                _t.sleep(wait / 1000)
    ts = [threading.Thread(target=worker, args=(w,)) for w in range(8)]
    for t in ts:
        t.start()
    _t.sleep(1.5)
    stop.set()
    for t in ts:
        t.join()
    window = _t.monotonic() - t0
    st = s.throughput_stats()
    assert st["ru_consumed"] == pytest.approx(admitted[0])
    assert st["ru_consumed"] <= 200.0 * window + 5.0, (st, window)
    assert st["throttled"] > 0 and st["reserved_admits"] > 0
    # reservations of callers that gave up lapse after the ticket TTL and refund their RU
    s.set_throughput(10.0, 0.2)
    _t.sleep(1.0)  # a second of refill into the empty bucket
    assert s.charge(10.0, 0, "PUT /a", 1) == (0, 0)  # that second of budget
    wait, ticket = s.charge(5.0, 0, "PUT /b", 1)  # reserved 500 ms ahead, never claimed
    assert wait >= 400 and ticket > 0
    _t.sleep(0.8)  # slot + TTL passed: ~8 RU refilled less the 5 reserved, plus the 5 refunded
    assert s.charge(7.5, 0, "PUT /c", 1)[0] == 0  # without the refund: ~3 RU, a 429
    st = s.throughput_stats()
    assert st["lapsed_reservations"] == 1 and st["refunded_ru"] == 5.0 and st["open_reservations"] == 0


def test_indexed_queries_run_on_the_native_front(monkeypatch):
    """A query the hash indexes answer (backing/accel.py ``indexable``: the list of a creator's
    tasks) runs on the native front's loop; the answers equal the Python handler's, and every
    other query (scans the accelerator may take, boolean equality, sampled traces) still goes to
    Python.  The front's choice is the planner's ``indexable`` rule."""
    import json as _json

    from aca_dotnet_workshop_amd.backing.accel import indexable
    filters = [{"EQ": {"who": "u1"}}, {"EQ": {"done": True}}, {"IN": {"who": ["u1", "u3"]}}, {"IN": {"who": [None, False]}},
               {"AND": [{"EQ": {"done": False}}, {"EQ": {"who": "u2"}}]}, {"AND": [{"EQ": {"done": False}}]},
               {"OR": [{"EQ": {"who": "u1"}}, {"EQ": {"n": 3}}]}, {"OR": [{"EQ": {"who": "u1"}}, {"GT": {"n": 3}}]},
               {"GT": {"n": 2}}, {}, {"eq": {"who": "u2"}}]
    queries = [{"filter": f} for f in filters] + [
        {"filter": {"EQ": {"who": "u1"}}, "sort": [{"key": "n", "order": "DESC"}], "page": {"limit": 2}},
        {"filter": {"EQ": {"who": "u1"}}, "sort": [{"key": "n"}], "page": {"limit": 2, "token": "2"}}]

    async def answers(front):
        async with Backing(front, monkeypatch) as b:
            c = BackingClient(b.base, identity="x")
            for i in range(12):
                await c.doc_put("acct", "db", "c", f"p||k{i}", _json.dumps({"who": f"u{i % 4}", "n": i % 5,
                                                                             "done": i % 3 == 0}))
            out = []
            for q in queries:
                out.append(_json.loads(await c.doc_query("acct", "db", "c", _json.dumps(q).encode(), "p||")))
            for kw in ({"sortkeys": True},):
                r = await c.http.post(b.base + "/cosmos/acct/db/c/query?prefix=p%7C%7C&project=sortkeys",
                                      body=_json.dumps(queries[-2]).encode(), headers={"x-tt-identity": "x"})
                out.append(r.json())
            sampled = await c.http.post(b.base + "/cosmos/acct/db/c/query", body=_json.dumps(queries[0]).encode(),
                                        headers={"x-tt-identity": "x", "traceparent": "00-" + "a" * 32 + "-" + "b" * 16 + "-01"})
            out.append(sampled.json())
            fs = (await c.http.get(b.base + "/admin/front")).json()
            await c.http.close()
            return out, fs
    py, _ = run(answers("python"))
    nat, fs = run(answers("native"))
    assert nat == py
    want_native = sum(1 for q in queries if indexable(q["filter"])) + 1  # + the sort-keys projection
    assert fs["requests"].get("doc.query", 0) == want_native, (fs["requests"], want_native)
    # the rest ran on the front's query worker (the Python planner called from C++), not
    # through the Python server: the sampled one too, which records the store's spans there
    assert fs["requests"].get("doc.query_worker", 0) == len(queries) + 1 - (want_native - 1), fs["requests"]
