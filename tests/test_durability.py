"""Group commit (applog.hpp fsync_mode 2, ``TT_BACKING_FSYNC=2``): every acknowledged write is
on the device -- the acknowledgement waits for the fdatasync that covers it -- while the writes
of a sync period share one fdatasync; the native front's answers and the Python-path writes both
wait; the log replays after a restart, compaction included."""
import asyncio
import json
import threading

import pytest

from aca_dotnet_workshop_amd.backing.client import BackingClient
from aca_dotnet_workshop_amd.backing.server import serve_backing
from aca_dotnet_workshop_amd.native import load

from helpers import run


def _n():
    return load()


def test_group_commit_acknowledges_after_sync_and_batches(tmp_path):
    N = _n()
    s = N.DocStore(str(tmp_path / "c.log"), 2)
    assert s.group_commit()
    n_threads, per = 8, 200

    def writer(t):
        for i in range(per):
            s.set(f"k{t}-{i}", json.dumps({"t": t, "i": i}))
            st = s.commit_stats()
            # returned from set(): its record is covered by a completed sync
            assert st["synced_bytes"] >= 1
    ths = [threading.Thread(target=writer, args=(t,)) for t in range(n_threads)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    st = s.commit_stats()
    assert st["acks"] == n_threads * per and st["synced_bytes"] == st["written_bytes"] > 0
    # concurrent writers share syncs (8 threads: never more syncs than writes, usually far fewer)
    assert 1 <= st["syncs"] <= n_threads * per
    del s
    s2 = N.DocStore(str(tmp_path / "c.log"), 2)  # replayed
    assert json.loads(s2.get("k7-199")[0]) == {"t": 7, "i": 199}


def test_group_commit_across_compaction(tmp_path):
    N = _n()
    s = N.DocStore(str(tmp_path / "c.log"), 2)
    for i in range(300):
        s.set("same", json.dumps({"i": i}))  # rewrites of one key: compaction material
    s.compact()
    for i in range(10):
        s.set(f"after{i}", "1")  # waits on marks past the compaction: must not hang
    st = s.commit_stats()
    assert st["synced_bytes"] == st["written_bytes"]
    del s
    s2 = N.DocStore(str(tmp_path / "c.log"), 2)
    assert json.loads(s2.get("same")[0]) == {"i": 299} and s2.get("after9")[0] == "1"


def test_other_modes_need_no_committer(tmp_path):
    N = _n()
    for mode in (0, 1):
        s = N.DocStore(str(tmp_path / f"m{mode}.log"), mode)
        assert not s.group_commit()
        s.set("a", "1")
        assert s.commit_stats()["syncs"] == 0
    b = N.Broker(str(tmp_path / "b.log"), 2)
    assert b.group_commit()


@pytest.mark.parametrize("front", ["native", "python"])
def test_backing_writes_answer_once_durable(front, monkeypatch, tmp_path):
    monkeypatch.setenv("TT_BACKING_FRONT", front)
    monkeypatch.setenv("TT_BACKING_FSYNC", "2")

    async def main():
        ready = asyncio.get_running_loop().create_future()
        stop = asyncio.Event()
        task = asyncio.ensure_future(serve_backing("127.0.0.1", 0, str(tmp_path), None, ready.set_result, stop))
        base = f"http://127.0.0.1:{await asyncio.wait_for(ready, 20)}"
        c = BackingClient(base, identity="x")
        try:
            await asyncio.gather(*(c.doc_put("acct", "db", "c", f"k{i}", json.dumps({"i": i})) for i in range(64)))
            res = await c.doc_bulk_set("acct", "db", "c", [{"key": f"b{i}", "value": "1"} for i in range(5)])
            assert all(x.get("etag") for x in res)
            assert await c.doc_delete("acct", "db", "c", "k0") is True
            stats = (await c.http.get(base + "/cosmos/acct/db/c/stats", headers={"x-tt-identity": "x"})).json()
            d = stats["durability"]
            assert d["fsync_mode"] == 2 and d["group_commit"]
            # every answered write was covered by a sync: nothing written is left unsynced
            assert d["synced_bytes"] == d["written_bytes"] > 0 and d["acks"] >= 66
            assert d["syncs"] >= 1
        finally:
            await c.http.close()
            stop.set()
            await asyncio.wait_for(task, 20)
        # a fresh process replays what was acknowledged
        ready = asyncio.get_running_loop().create_future()
        stop = asyncio.Event()
        task = asyncio.ensure_future(serve_backing("127.0.0.1", 0, str(tmp_path), None, ready.set_result, stop))
        base = f"http://127.0.0.1:{await asyncio.wait_for(ready, 20)}"
        c = BackingClient(base, identity="x")
        try:
            assert json.loads((await c.doc_get("acct", "db", "c", "k63"))[0]) == {"i": 63}
            assert await c.doc_get("acct", "db", "c", "k0") is None
        finally:
            await c.http.close()
            stop.set()
            await asyncio.wait_for(task, 20)
    run(main())
