"""The partitioned shared environment (backing/shards.py; VERDICT r2 "partitioned shared env"):
documents and messages spread over several backing processes by partition-key hash, the
cross-partition query merged page by page with a composite continuation token, transactions
held to one partition, the broker's receivers draining every shard exactly once, and the
native data plane routing with the same hash as the Python client."""
import asyncio
import json
import os
import socket
import subprocess
import sys
import urllib.request
from pathlib import Path

import pytest

from aca_dotnet_workshop_amd.backing.client import BackingClient, BackingError
from aca_dotnet_workshop_amd.backing.shards import (ShardedBackingClient, decode_token, encode_token, fnv1a64,
                                                    merge_pages, shard_of)
from aca_dotnet_workshop_amd.platform.processes import LocalStack

from helpers import run

ROOT = Path(__file__).resolve().parents[1]
ACCT, DB, COLL = "taskstracker-state-store", "tasksmanagerdb", "taskscollection"
PREFIX = "tasksmanager-backend-api||"


def test_fnv1a64_reference_vectors():
    assert fnv1a64(b"") == 0xcbf29ce484222325
    assert fnv1a64(b"a") == 0xaf63dc4c8601ec8c
    assert fnv1a64("foobar") == 0x85944171f73967e8
    assert shard_of("anything", 1) == 0 and {shard_of(f"k{i}", 4) for i in range(64)} == {0, 1, 2, 3}


def test_token_roundtrip_and_rejection():
    assert encode_token([None, None]) is None
    t = encode_token([3, None, 0])
    assert decode_token(t, 3) == [3, None, 0] and decode_token(None, 3) == [0, 0, 0]
    for bad in ("42", t + "x", encode_token([1, 2])):
        with pytest.raises(BackingError) as e:
            decode_token(bad, 3)
        assert e.value.status == 400


def test_merge_pages_offsets():
    """A shard whose page was only partly used resumes at its offset; a shard that returned its
    last matches and had them all taken is exhausted."""
    q = {"sort": [{"key": "v", "order": "ASC"}], "page": {"limit": 3}}
    pages = [(0, {"results": [{"key": "a", "data": {"v": 1}}, {"key": "b", "data": {"v": 5}}], "token": "2"}),
             (1, {"results": [{"key": "c", "data": {"v": 2}}, {"key": "d", "data": {"v": 3}}]}),
             (2, None)]
    out = merge_pages(q, pages, [0, 0, None])
    assert [r["key"] for r in out["results"]] == ["a", "c", "d"]
    assert decode_token(out["token"], 3) == [1, None, None]
    # a missing sort path sorts like null (first), DESC reverses, ties go in shard order
    q2 = {"sort": [{"key": "v", "order": "DESC"}]}
    pages2 = [(0, {"results": [{"key": "x", "data": {"v": 1}}, {"key": "m", "data": {}}]}),
              (1, {"results": [{"key": "y", "data": {"v": 1}}]})]
    assert [r["key"] for r in merge_pages(q2, pages2, [0, 0])["results"]] == ["x", "y", "m"]


def test_merge_pages_stops_where_a_short_shard_page_runs_out():
    """A k-way PAGED merge: shard 0 sent a short page (its mirror skipped stale
    rows) with a token, so its unfetched matches may sort before shard 1's -- the merged page
    ends when shard 0's entries run out, and shard 0 resumes at the position IT named."""
    q = {"sort": [{"key": "v", "order": "ASC"}], "page": {"limit": 3}}
    pages = [(0, {"results": [{"key": "a", "data": {"v": 1}}], "token": "3"}),
             (1, {"results": [{"key": "c", "data": {"v": 2}}, {"key": "d", "data": {"v": 3}},
                              {"key": "e", "data": {"v": 4}}], "token": "3"})]
    out = merge_pages(q, pages, [0, 0])
    assert [r["key"] for r in out["results"]] == ["a"]
    assert decode_token(out["token"], 2) == [3, 0]
    # an empty page with a token: nothing can be merged yet, but the shard still moves on
    pages = [(0, {"results": [], "token": "6"}), pages[1]]
    out = merge_pages(q, pages, [3, 0])
    assert out["results"] == [] and decode_token(out["token"], 2) == [6, 0]


def _task(i: int) -> dict:
    return {"taskId": f"00000000-0000-4000-8000-{i:012d}", "taskName": f"Task {i % 17}",
            "taskCreatedBy": f"user{i % 5}@x", "taskCreatedOn": f"2026-10-{1 + i % 28:02d}T{i // 3600 % 24:02d}:{i % 60:02d}:{i // 60 % 60:02d}",
            "taskDueDate": f"2026-10-{1 + (i * 7) % 28:02d}T00:00:00", "taskAssignedTo": "a@x",
            "isCompleted": i % 9 == 0, "isOverDue": i % 11 == 0}


async def _pages(client, q: dict) -> list[str]:
    keys, token = [], None
    for _ in range(1000):
        qq = json.loads(json.dumps(q))
        if token:
            qq.setdefault("page", {})["token"] = token
        res = json.loads(await client.doc_query(ACCT, DB, COLL, json.dumps(qq).encode(), PREFIX))
        keys += [r["key"] for r in res["results"]]
        token = res.get("token")
        if not token:
            return keys
    raise AssertionError("paging did not end")


@pytest.fixture(scope="module")
def backings(tmp_path_factory):
    """Three shard backings (columnar accelerator on, CPU executor) and one single store."""
    base = tmp_path_factory.mktemp("shards")
    stacks = []
    try:
        for i in range(4):
            env = {"TT_QUERY_ACCEL": "cpu", "TT_QUERY_ACCEL_MIN_DOCS": "0",
                   "TT_QUERY_MIRROR_PATHS": "taskDueDate,isCompleted,isOverDue,taskCreatedOn"} if i < 3 else {}
            s = LocalStack(root=base / f"s{i}", env=env)
            s.start_backing()
            stacks.append(s)
        yield [s.backing_url for s in stacks]
    finally:
        for s in stacks:
            s.stop()


def test_partitioned_store_matches_one_store(backings):
    async def main():
        sh = ShardedBackingClient(backings[:3], identity="platform-admin")
        one = BackingClient(backings[3], identity="platform-admin")
        try:
            docs = {f"{PREFIX}{_task(i)['taskId']}": _task(i) for i in range(600)}
            items = [{"key": k, "value": json.dumps(v)} for k, v in docs.items()]
            for lo in range(0, len(items), 100):
                await sh.doc_bulk_set(ACCT, DB, COLL, items[lo:lo + 100])
                await one.doc_bulk_set(ACCT, DB, COLL, items[lo:lo + 100])
            # every document on the shard its key hashes to, and only there
            for k in list(docs)[:60]:
                home = shard_of(k, 3)
                for i, c in enumerate(sh.shards):
                    assert (await c.doc_get(ACCT, DB, COLL, k) is not None) == (i == home)
            per = [(await c.doc_stats(ACCT, DB, COLL))["docs"] for c in sh.shards]
            assert sum(per) == 600 and min(per) > 120, per
            got = await sh.doc_bulk_get(ACCT, DB, COLL, list(docs)[:50] + ["missing"])
            assert [g["key"] for g in got] == list(docs)[:50] + ["missing"] and "data" not in got[-1]
            # the overdue sweep's query (range + ORDER BY taskCreatedOn + page), page by page
            sweep = {"filter": {"AND": [{"LT": {"taskDueDate": "2026-10-15T00:00:00"}}, {"EQ": {"isCompleted": False}},
                                        {"EQ": {"isOverDue": False}}]},
                     "sort": [{"key": "taskCreatedOn", "order": "ASC"}], "page": {"limit": 37}}
            a, b = await _pages(sh, sweep), await _pages(one, sweep)
            assert a == b and len(a) > 100
            desc = dict(sweep, sort=[{"key": "taskCreatedOn", "order": "DESC"}], page={"limit": 64})
            assert await _pages(sh, desc) == await _pages(one, desc)
            eq = {"filter": {"EQ": {"taskCreatedBy": "user3@x"}}, "page": {"limit": 25}}
            assert sorted(await _pages(sh, eq)) == sorted(await _pages(one, eq))
            assert sorted(await _pages(sh, {"filter": {"EQ": {"taskName": "Task 4"}}})) == \
                sorted(await _pages(one, {"filter": {"EQ": {"taskName": "Task 4"}}}))
            # transactions stay within one partition
            k0 = next(k for k in docs if shard_of(k, 3) == 0)
            k1 = next(k for k in docs if shard_of(k, 3) == 1)
            with pytest.raises(BackingError) as e:
                await sh.doc_transaction(ACCT, DB, COLL, [{"op": "delete", "key": k0}, {"op": "delete", "key": k1}])
            assert e.value.status == 400
            await sh.doc_transaction(ACCT, DB, COLL, [{"op": "upsert", "key": k0, "value": json.dumps({"x": 1})}])
            assert json.loads((await sh.doc_get(ACCT, DB, COLL, k0))[0]) == {"x": 1}
            # provisioned throughput is split over the partitions
            r = await sh.doc_set_throughput(ACCT, DB, COLL, 3000)
            assert r["perShard"] == 1000.0
            await sh.doc_set_throughput(ACCT, DB, COLL, 0)
        finally:
            await sh.close()
            await one.close()
    run(main())


def test_partitioned_broker_exactly_once(backings):
    async def main():
        sh = ShardedBackingClient(backings[:3], identity="platform-admin")
        try:
            await sh.sb_create_topic("ns1", "t")
            await sh.sb_create_subscription("ns1", "t", "g", 30000, 5)
            for i in range(90):
                await sh.sb_publish("ns1", "t", json.dumps({"i": i}).encode(), message_id=f"m{i}")
            await sh.sb_publish_batch("ns1", "t", [{"body": json.dumps({"i": 90 + i}), "contentType": "application/json",
                                                   "entryId": f"e{i}"} for i in range(30)])
            per = [(await c.sb_counts("ns1", "t/subscriptions/g"))["enqueued"] for c in sh.shards]
            assert sum(per) == 120 and min(per) > 15, per
            seen: list[int] = []
            for _ in range(200):
                msgs = await sh.sb_receive("ns1", "t/subscriptions/g", 16, 30000, 50)
                if not msgs and len(seen) >= 120:
                    break
                seen += [json.loads(m["body"])["i"] if "body" in m else None for m in msgs]
                res = await sh.sb_settle("ns1", "t/subscriptions/g", complete=[m["lockToken"] for m in msgs])
                assert all(res["complete"])
            assert sorted(seen) == list(range(120))
            c = await sh.sb_counts("ns1", "t/subscriptions/g")
            assert c["completed"] == c["received"] == 120, c
        finally:
            await sh.close()
    run(main())


def test_native_data_plane_routes_with_the_same_hash(tmp_path, backings):
    """An API replica whose sidecar runs the native data plane over two shards: the documents it
    saves land where the Python client's hash says, its publishes spread over both brokers, and
    the cross-partition query of GET /api/tasks?createdBy= (fanned out and merged by the data
    plane) returns every task."""
    urls = backings[:2]
    stack = LocalStack(root=tmp_path / "app")
    try:
        stack.start_backing()  # the replica's home backing (Key Vault, Storage, ...)
        for fam in ("COSMOS", "SERVICEBUS"):
            stack.base_env[f"TT_BACKING_SHARDS_{fam}"] = ",".join(urls)
        api = stack.start_replica("tasksmanager-backend-api", {"Logging:LogLevel:Default": "Warning"})
        stack.wait_ready()

        async def main():
            from aca_dotnet_workshop_amd.web.client import HttpClient
            http = HttpClient()
            sh = ShardedBackingClient(urls, identity="platform-admin")
            try:
                await sh.sb_create_topic("taskstracker", "tasksavedtopic")  # the processor's subscription
                await sh.sb_create_subscription("taskstracker", "tasksavedtopic", "tasksmanager-backend-processor")
                base = f"unix:{api.sidecar_uds}:/v1.0/invoke/tasksmanager-backend-api/method/api/tasks"
                ids = []
                for i in range(40):
                    body = json.dumps({"taskName": f"n{i}", "taskCreatedBy": "route@x", "taskAssignedTo": "a@x",
                                       "taskDueDate": "2030-01-01T00:00:00"}).encode()
                    r = await http.request("POST", base, body=body, headers=[("Content-Type", "application/json")])
                    assert r.status == 201, r.body
                    ids.append(r.headers["location"].rsplit("/", 1)[1])
                for tid in ids:
                    k = f"{PREFIX}{tid}"
                    assert await sh.shards[shard_of(k, 2)].doc_get(ACCT, DB, COLL, k) is not None
                    assert await sh.shards[1 - shard_of(k, 2)].doc_get(ACCT, DB, COLL, k) is None
                r = await http.request("GET", base + "?createdBy=route@x")
                assert r.status == 200 and sorted(t["taskId"] for t in json.loads(r.body)) == sorted(ids)
                ent = "tasksavedtopic/subscriptions/tasksmanager-backend-processor"
                per = [(await c.sb_counts("taskstracker", ent))["enqueued"] for c in sh.shards]
                assert sum(per) >= 40 and min(per) > 0, per
                # the Service Bus partitionKey metadata pins messages to one shard
                pub = f"unix:{api.sidecar_uds}:/v1.0/publish/dapr-pubsub-servicebus/tasksavedtopic"
                for i in range(12):
                    r = await http.request("POST", pub + "?metadata.partitionKey=tenant-7", body=b'{"n": 1}',
                                           headers=[("Content-Type", "application/json")])
                    assert r.status == 204, r.body
                after = [(await c.sb_counts("taskstracker", ent))["enqueued"] for c in sh.shards]
                home = shard_of("tenant-7", 2)
                assert after[home] - per[home] == 12 and after[1 - home] == per[1 - home], (per, after)
                # an empty partitionKey is no key (like shards.py): routed by each event's id
                for i in range(24):
                    r = await http.request("POST", pub + "?metadata.partitionKey=", body=b'{"n": 2}',
                                           headers=[("Content-Type", "application/json")])
                    assert r.status == 204, r.body
                final = [(await c.sb_counts("taskstracker", ent))["enqueued"] for c in sh.shards]
                assert all(final[i] > after[i] for i in range(2)), (after, final)
            finally:
                await sh.close()
                await http.close()
        run(main())
    finally:
        stack.stop()


def test_native_cross_partition_query_pages_match_one_store(tmp_path, backings):
    """The native data plane's cross-partition state query (dataplane.cpp state_query_sharded):
    every shard answers its sorted page as sort keys only, the sidecar k-way merges them and
    fetches just the merged page's documents.  Page by page -- ASC, DESC, unsorted, two sort
    keys, continuation tokens -- the results equal one store's; a token from the Python merge
    is accepted; rows moved are counted per phase."""
    urls = backings[:3]
    stack = LocalStack(root=tmp_path / "xq")
    try:
        stack.start_backing()
        stack.base_env["TT_BACKING_SHARDS_COSMOS"] = ",".join(urls)
        api = stack.start_replica("tasksmanager-backend-api", {"Logging:LogLevel:Default": "Warning"})
        stack.wait_ready()

        async def main():
            from aca_dotnet_workshop_amd.web.client import HttpClient
            http = HttpClient()
            sh = ShardedBackingClient(urls, identity="platform-admin")
            one = BackingClient(backings[3], identity="platform-admin")
            try:
                docs = {}
                for i in range(300):
                    t = _task(50_000 + i)
                    t["taskCreatedBy"] = "xq@x"
                    t["rank"] = i % 7  # ties across shards for the two-key sort
                    docs[f"{PREFIX}{t['taskId']}"] = t
                items = [{"key": k, "value": json.dumps(v)} for k, v in docs.items()]
                await sh.doc_bulk_set(ACCT, DB, COLL, items)
                await one.doc_bulk_set(ACCT, DB, COLL, items)
                qurl = f"unix:{api.sidecar_uds}:/v1.0-alpha1/state/statestore/query"

                async def via_sidecar(q):
                    keys, token, pages = [], None, 0
                    while True:
                        qq = json.loads(json.dumps(q))
                        if token:
                            qq.setdefault("page", {})["token"] = token
                        r = await http.request("POST", qurl, body=json.dumps(qq).encode(),
                                               headers=[("Content-Type", "application/json")])
                        assert r.status == 200, r.body
                        res = json.loads(r.body)
                        assert all(x["data"]["taskCreatedBy"] == "xq@x" and x["etag"] for x in res["results"])
                        keys += [x["key"] for x in res["results"]]
                        token, pages = res.get("token"), pages + 1
                        if not token:
                            return keys, pages

                flt = {"AND": [{"EQ": {"taskCreatedBy": "xq@x"}}, {"LT": {"taskDueDate": "2026-10-20T00:00:00"}}]}
                for sort, limit in (([{"key": "taskCreatedOn", "order": "ASC"}], 23),
                                    ([{"key": "taskCreatedOn", "order": "DESC"}], 64),
                                    ([{"key": "rank"}, {"key": "taskCreatedOn", "order": "DESC"}], 17)):
                    q = {"filter": flt, "sort": sort, "page": {"limit": limit}}
                    got, pages = await via_sidecar(q)
                    want = await _pages(one, q)  # the store strips the key prefix
                    assert got == want and len(got) > 100 and pages >= len(got) // limit, (sort, len(got), len(want))
                unsorted, _ = await via_sidecar({"filter": flt, "page": {"limit": 40}})
                assert sorted(unsorted) == sorted(await _pages(one, {"filter": flt}))
                # a continuation token issued by the Python plane's merge resumes natively
                q = {"filter": flt, "sort": [{"key": "taskCreatedOn"}], "page": {"limit": 30}}
                first = json.loads(await sh.doc_query(ACCT, DB, COLL, json.dumps(q).encode(), PREFIX))
                q2 = dict(q, page={"limit": 30, "token": first["token"]})
                r = await http.request("POST", qurl, body=json.dumps(q2).encode(),
                                       headers=[("Content-Type", "application/json")])
                py2 = json.loads(await sh.doc_query(ACCT, DB, COLL, json.dumps(q2).encode(), PREFIX))
                assert [x["key"] for x in json.loads(r.body)["results"]] == [x["key"] for x in py2["results"]]
                bad = await http.request("POST", qurl, body=json.dumps(dict(q, page={"limit": 5, "token": "42"})).encode(),
                                         headers=[("Content-Type", "application/json")])
                assert bad.status == 400
                m = (await http.request("GET", f"unix:{api.sidecar_uds}:/metrics")).body.decode()
                keys_moved = int(m.split('phase="keys"} ')[1].split()[0])
                docs_moved = int(m.split('phase="documents"} ')[1].split()[0])
                assert 0 < docs_moved <= keys_moved
            finally:
                await sh.close()
                await one.close()
                await http.close()
        run(main())
    finally:
        stack.stop()


def _sweep_env(tmp: Path, name: str, shard_urls: list[str] | None, single_url: str | None):
    """An API (range overdue query) + processor (pages of 50) pair over either the shards or one
    backing; returns (stack, processor sidecar socket)."""
    stack = LocalStack(root=tmp / name)
    if shard_urls:
        stack.start_backing()  # home services; the store and the broker are the shards
        for fam in ("COSMOS", "SERVICEBUS"):
            stack.base_env[f"TT_BACKING_SHARDS_{fam}"] = ",".join(shard_urls)
    else:
        stack.base_env["TT_BACKING_URL"] = single_url
        stack.backing_url = single_url
    cfg = {"Logging:LogLevel:Default": "Warning", "TasksNotifier:Mode": "log"}
    stack.start_replica("tasksmanager-backend-api", {**cfg, "OverdueTasks:Query": "range"})
    proc = stack.start_replica("tasksmanager-backend-processor", {**cfg, "OverdueTasks:PageSize": "50"})
    stack.wait_ready()
    return stack, proc.sidecar_uds


@pytest.fixture(params=[2, 8], ids=["2shards", "8shards"])
def sweep_backings(tmp_path, request):
    """Fresh backings for the sweep test: N shards and one single store (columnar CPU path)."""
    stacks = []
    try:
        for i in range(request.param + 1):
            st = LocalStack(root=tmp_path / f"b{i}", env={"TT_QUERY_ACCEL": "cpu", "TT_QUERY_ACCEL_MIN_DOCS": "0",
                                                          "TT_QUERY_MIRROR_PATHS": "taskDueDate,isCompleted,isOverDue,taskCreatedOn"})
            st.start_backing()
            stacks.append(st)
        yield [st.backing_url for st in stacks]
    finally:
        for st in stacks:
            st.stop()


def test_sharded_overdue_sweep_marks_the_same_tasks_as_one_store(tmp_path, sweep_backings):
    """The cron job (processor -> API range query -> cross-partition merge of both shards'
    columnar pages -> markoverdue bulk save routed per shard) marks exactly the tasks a
    single-store environment marks, page by page across the shards."""
    from datetime import datetime, timedelta
    past = (datetime.utcnow() - timedelta(days=3)).strftime("%Y-%m-%dT00:00:00")
    future = (datetime.utcnow() + timedelta(days=3)).strftime("%Y-%m-%dT00:00:00")
    docs = {}
    for i in range(400):
        t = _task(10_000 + i)
        t["taskDueDate"] = past if i % 3 else future
        t["isCompleted"], t["isOverDue"] = i % 7 == 0, i % 11 == 0
        docs[f"{PREFIX}{t['taskId']}"] = t
    want = {k for k, t in docs.items() if t["taskDueDate"] == past and not t["isCompleted"] and not t["isOverDue"]}
    stacks = []
    try:
        async def load(client):
            items = [{"key": k, "value": json.dumps(v)} for k, v in docs.items()]
            await client.doc_bulk_set("taskstracker-state-store", DB, COLL, items)
            await client.close()
        backings = sweep_backings
        n = len(backings) - 1
        run(load(ShardedBackingClient(backings[:n], identity="platform-admin")))
        one_url = backings[n]
        run(load(BackingClient(one_url, identity="platform-admin")))
        results = []
        for name, shard_urls, single in (("sharded", backings[:n], None), ("single", None, one_url)):
            stack, sock = _sweep_env(tmp_path, name, shard_urls, single)
            stacks.append(stack)

            async def sweep(sock=sock):
                from aca_dotnet_workshop_amd.web.client import HttpClient
                http = HttpClient()
                try:
                    r = await http.request("POST", f"unix:{sock}:/v1.0/invoke/tasksmanager-backend-processor/method/"
                                           "ScheduledTasksManager", body=b"{}",
                                           headers=[("Content-Type", "application/json")], timeout=120)
                    assert r.status == 200, r.body
                    return json.loads(r.body)
                finally:
                    await http.close()
            results.append(run(sweep()))

        async def marked(client):
            try:
                got = await client.doc_bulk_get("taskstracker-state-store", DB, COLL, sorted(want))
                return {g["key"] for g in got if g.get("data") and g["data"].get("isOverDue")}
            finally:
                await client.close()
        sharded = run(marked(ShardedBackingClient(backings[:n], identity="platform-admin")))
        single = run(marked(BackingClient(one_url, identity="platform-admin")))
        assert sharded == single == want, (len(sharded), len(single), len(want))
        assert results[0]["markedOverdue"] == results[1]["markedOverdue"] == len(want)
        assert results[0]["pages"] >= len(want) // 50  # paged through the merged order
        per_shard = {shard_of(k, n) for k in want}
        assert per_shard == set(range(n))
    finally:
        for st in stacks:
            st.stop()


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_shared_env_four_ranks_exactly_once():
    """Four ranks, one partitioned environment: every rank hosts one shard of the store and of
    the broker; the four processors compete on the one subscription over all four shards and
    every task is delivered and completed exactly once (bench.py --shared-env, gloo)."""
    env = dict(os.environ, PYTHONPATH=str(ROOT), OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "4",
           "--steps", "2", "--warmup", "1", "--batch", "24", "--api-replicas", "1", "--processor-replicas", "1",
           "--shared-env", "--overdue-sweep-ms", "0", "--entry", "api-sidecar", "--split-backing", "0"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{") and '"metric"' in x]
    assert len(line) == 1
    cfg = line[0]["config"]
    assert cfg["parallelism"].startswith("shared-env x4 (store and broker partitioned over 4 shards")
    dlv = cfg["delivery"]
    assert dlv["exactly_once"] and dlv["completed"] == dlv["expected"] == 4 * 24 * 3, dlv
    assert dlv["dead_lettered"] == 0


@pytest.mark.slow
def test_shared_env_eight_ranks_exactly_once():
    """The whole machine: eight ranks (one per GPU of an MI355X node), one partitioned
    environment -- each rank hosts one shard of the store and of the broker, the eight
    processors compete on the one subscription over all eight shards -- and every task is
    delivered and completed exactly once (bench.py --shared-env over gloo, small batch)."""
    env = dict(os.environ, PYTHONPATH=str(ROOT), OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "8",
           "--steps", "2", "--warmup", "1", "--batch", "16", "--api-replicas", "1", "--processor-replicas", "1",
           "--shared-env", "--overdue-sweep-ms", "0", "--entry", "api-sidecar", "--split-backing", "0"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=1200)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{") and '"metric"' in x]
    assert len(line) == 1
    cfg = line[0]["config"]
    assert cfg["parallelism"].startswith("shared-env x8 (store and broker partitioned over 8 shards")
    dlv = cfg["delivery"]
    assert dlv["exactly_once"] and dlv["completed"] == dlv["expected"] == 8 * 16 * 3, dlv
    assert dlv["dead_lettered"] == 0


@pytest.mark.slow
def test_shared_env_frontend_eight_ranks_exactly_once():
    """The headline's own topology at eight ranks: ``bench.py --gpus 8 --shared-env`` started
    WITHOUT a launcher (it self-launches the ranks), load at every rank's frontend through its
    external HTTPS ingress, sidecar mTLS, the manifest's CPU caps, and the overdue cron sweep
    through the data plane's native cross-partition merge; every task is delivered and
    completed exactly once and the sweeps run without error."""
    env = dict(os.environ, PYTHONPATH=str(ROOT), OMP_NUM_THREADS="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, "bench.py", "--gpus", "8", "--steps", "2", "--warmup", "1", "--batch", "16",
           "--shared-env", "--overdue-sweep-ms", "500", "--past-due-every", "4"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=1500)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{") and '"metric"' in x]
    assert len(line) == 1 and line[0]["n_gpus"] == 8
    cfg = line[0]["config"]
    assert cfg["entry"] == "frontend" and cfg["mtls"] is True and cfg["ingress"].startswith("external HTTPS (native)")
    assert cfg["launcher"] == "torch.distributed.run, 8 ranks (self-launched by bench.py)"
    assert cfg["parallelism"].startswith("shared-env x8 (store and broker partitioned over 8 shards")
    dlv = cfg["delivery"]
    assert dlv["exactly_once"] and dlv["completed"] == dlv["expected"] == 8 * 16 * 3, dlv
    assert dlv["dead_lettered"] == 0
    sw = cfg["overdue_sweeps"]
    assert sw["shards"] == 8 and sw["errors"] == 0, sw
    # every past-due task of every rank is marked exactly once over the 8 shards, as one store
    # marks them (the sweeps of the run, then sweeps until one marks nothing)
    drain = sw["drain"]
    assert drain["expected_past_due"] == 8 * 4 * 3 and drain["exactly_once"], drain
    # no thread of any rank's processes may run outside that rank's CPU set (the max over ranks)
    pc = cfg["platform_cpu"]
    assert pc["outside_rank_set"] == 0 and pc["threads_checked"] > 0, pc
