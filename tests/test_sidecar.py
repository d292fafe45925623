"""Sidecar semantics: component loading (both dialects, scopes, secret references),
pub/sub delivery outcomes (2xx / RETRY / DROP / 400 / 404, dead-letter topic), input
binding acknowledgement, API and mesh tokens, bulk publish, cron parsing."""
import asyncio
import json
from datetime import datetime, timezone
from pathlib import Path

import pytest

from aca_dotnet_workshop_amd.backing import BackingServices
from aca_dotnet_workshop_amd.sdk import SidecarClient, cloud_events_middleware, map_subscribe_handler, topic
from aca_dotnet_workshop_amd.sidecar import NameResolver, Sidecar, from_dict, load_paths
from aca_dotnet_workshop_amd.sidecar.components import ComponentError
from aca_dotnet_workshop_amd.utils.cron import CronError, CronSchedule, parse_duration
from aca_dotnet_workshop_amd.web import HttpClient, HttpServer, Response, WebApp, empty, json_response

from helpers import run

ROOT = Path(__file__).resolve().parents[1]


def test_load_both_dialects_and_scopes():
    comps, subs, _ = load_paths([ROOT / "deploy" / "components"])
    by = {c.name: c for c in comps}
    assert by["statestore"].type == "state.azure.cosmosdb" and by["statestore"].scopes == ["tasksmanager-backend-api"]
    assert by["ScheduledTasksManager"].type == "bindings.cron"
    assert not by["taskspubsub"].scopes  # unscoped: loaded by every app
    aca, _, _ = load_paths([ROOT / "deploy" / "aca-components"])
    q = {c.name: c for c in aca}["containerapps-bindings-in-storagequeue"]
    assert q.dialect == "aca" and q.secret_store == "secretstoreakv"
    assert [i.secret_name for i in q.items if i.secret_name] == ["external-azure-storage-key"]
    assert q.in_scope("tasksmanager-backend-processor") and not q.in_scope("tasksmanager-backend-api")
    with pytest.raises(ComponentError):
        from_dict({"kind": "Widget"})


def _inline(name, type_, meta, **extra):
    d = {"apiVersion": "dapr.io/v1alpha1", "kind": "Component", "metadata": {"name": name},
         "spec": {"type": type_, "version": "v1", "metadata": [{"name": k, **v} if isinstance(v, dict) else
                                                              {"name": k, "value": v} for k, v in meta.items()]}}
    d.update(extra)
    return from_dict(d)


class Harness:
    """Backing services + one app + its sidecar, all in-process over TCP."""

    def __init__(self, app: WebApp, components, app_id="testapp", **sc_kw):
        self.app, self.components, self.app_id, self.sc_kw = app, components, app_id, sc_kw

    async def __aenter__(self):
        loop = asyncio.get_running_loop()
        self.backing = BackingServices()
        self.bsrv = HttpServer(self.backing.build_app(), loop)
        self.burl = f"http://127.0.0.1:{await self.bsrv.listen_tcp('127.0.0.1', 0)}"
        self.asrv = HttpServer(self.app, loop)
        await self.app.startup()
        self.app_port = await self.asrv.listen_tcp("127.0.0.1", 0)
        self.sc = Sidecar(self.app_id, app_port=self.app_port, http_port=0, components=self.components,
                          resolver=NameResolver(), backing_url=self.burl, **self.sc_kw)
        await self.sc.start()
        self.base = f"http://127.0.0.1:{self.sc.bound_http_port}"
        self.http = HttpClient()
        await asyncio.wait_for(self.sc.app_ready.wait(), 10)
        return self

    async def __aexit__(self, *exc):
        await self.sc.stop(1.0)
        await self.asrv.close(1.0)
        await self.bsrv.close(1.0)
        await self.http.close()


async def _until(pred, timeout=5.0):
    end = asyncio.get_running_loop().time() + timeout
    while asyncio.get_running_loop().time() < end:
        if pred():
            return True
        await asyncio.sleep(0.02)
    raise AssertionError("timeout")


def test_pubsub_delivery_outcomes():
    app = WebApp("sub")
    app.use(cloud_events_middleware())
    seen: dict[str, list] = {"ok": [], "retry": [], "drop": [], "fail400": [], "gone": [], "dlq": []}
    attempts = {"fail400": 0}

    def handler(kind, resp):
        async def h(req):
            seen[kind].append(req.json())
            return resp() if callable(resp) else resp
        return h

    def fail_twice():
        attempts["fail400"] += 1
        return Response(b"", 400) if attempts["fail400"] <= 2 else empty(200)

    for kind, resp, extra in (("ok", json_response({"status": "SUCCESS"}), {}),
                              ("retry", json_response({"status": "RETRY"}), {}),
                              ("drop", json_response({"status": "DROP"}), {"dead_letter_topic": "poison"}),
                              ("fail400", fail_twice, {}),
                              ("gone", empty(404), {}),
                              ("dlq", empty(200), {})):
        fn = handler(kind, resp)
        topic("bus", kind, **extra)(fn)
        app.add_route(f"/{kind}", fn, ("POST",))
    fn = handler("dlq", empty(200))
    topic("bus", "poison")(fn)
    app.add_route("/poison", fn, ("POST",))
    map_subscribe_handler(app)
    bus = _inline("bus", "pubsub.azure.servicebus", {"connectionString": "Endpoint=sb://ns1.servicebus.windows.net/",
                                                      "maxDeliveryCount": "3"})

    async def main():
        async with Harness(app, [bus]) as h:
            for t in ("ok", "retry", "drop", "fail400", "gone"):
                r = await h.http.post(f"{h.base}/v1.0/publish/bus/{t}", json_body={"topic": t})
                assert r.status == 204
            b = h.backing.broker("ns1")

            def counts(t):
                return b.counts(f"{t}/subscriptions/testapp")
            await _until(lambda: counts("ok")["completed"] == 1)
            assert seen["ok"] == [{"topic": "ok"}]  # CloudEvent unwrapped to data by the middleware
            await _until(lambda: counts("retry")["dead_letter"] == 1)  # RETRY x maxDeliveryCount -> DLQ
            assert len(seen["retry"]) == 3
            await _until(lambda: len(seen["dlq"]) == 1)  # DROP with deadLetterTopic -> forwarded
            assert counts("drop")["completed"] == 1 and counts("drop")["dead_letter"] == 0
            await _until(lambda: counts("fail400")["completed"] == 1)  # 400 -> redelivered until success
            assert attempts["fail400"] == 3
            await _until(lambda: counts("gone")["dead_letter"] == 1)  # 404 -> dropped to DLQ, no retry
            assert len(seen["gone"]) == 1
            # bulk publish
            r = await h.http.post(f"{h.base}/v1.0-alpha1/publish/bulk/bus/ok",
                                  json_body=[{"entryId": str(i), "event": {"i": i}, "contentType": "application/json"}
                                             for i in range(5)])
            assert r.status == 204
            await _until(lambda: counts("ok")["completed"] == 6)
            # unknown pubsub -> 404
            assert (await h.http.post(f"{h.base}/v1.0/publish/nope/x", json_body={})).status == 404
            meta = (await h.http.get(f"{h.base}/v1.0/metadata")).json()
            assert {s["topic"] for s in meta["subscriptions"]} >= {"ok", "retry", "poison"}
    run(main())


def test_input_binding_ack_and_redelivery():
    app = WebApp("binder")
    calls = []

    async def handler(req):
        calls.append(json.loads(req.body))
        return empty(500) if len(calls) == 1 else empty(200)
    app.add_route("/jobs", handler, ("POST",))
    q = _inline("jobs", "bindings.azure.storagequeues", {"storageAccount": "acct", "queue": "q1", "decodeBase64": "true",
                                                         "visibilityTimeout": "100ms", "pollingInterval": "200ms"})
    unrouted = _inline("unrouted", "bindings.azure.storagequeues", {"storageAccount": "acct", "queue": "q2"})

    async def main():
        async with Harness(app, [q, unrouted]) as h:
            assert h.sc.input_bindings == ["jobs"]  # OPTIONS /unrouted -> 404: binding not started
            import base64
            h.backing.broker("storage-acct").send("q1", base64.b64encode(b'{"n": 1}'))
            h.backing.waiters.notify("storage-acct|q1")
            await _until(lambda: len(calls) == 2, timeout=5)  # first delivery failed -> reappeared
            await _until(lambda: h.backing.broker("storage-acct").counts("q1")["completed"] == 1)
            # output binding on the same component type
            r = await h.http.post(f"{h.base}/v1.0/bindings/unrouted", json_body={"operation": "create", "data": {"x": 1}})
            assert r.status == 204
            assert h.backing.broker("storage-acct").counts("q2")["active"] == 1
            r = await h.http.post(f"{h.base}/v1.0/bindings/unrouted", json_body={"operation": "delete"})
            assert r.status == 400
    run(main())


def test_input_binding_slow_or_failing_delivery_does_not_stall_the_queue():
    """the poller delivers each message on its own slot and refills freed
    slots at once -- one slow delivery (the app holds it 1.5 s) and one failing delivery (500,
    redelivered after the visibility timeout) do not delay the other messages, which are all
    delivered and deleted while the slow one is still running."""
    import base64
    import time as _t
    app = WebApp("binder")
    done: dict[int, float] = {}
    attempts: dict[int, int] = {}
    release = asyncio.Event()

    async def handler(req):
        n = json.loads(req.body)["n"]
        attempts[n] = attempts.get(n, 0) + 1
        if n == 0:  # the slow one
            await asyncio.wait_for(release.wait(), 5)
        if n == 1 and attempts[n] == 1:  # the failing one: 500 once, then fine
            return empty(500)
        done.setdefault(n, _t.monotonic())
        return empty(200)
    app.add_route("/jobs", handler, ("POST",))
    q = _inline("jobs", "bindings.azure.storagequeues", {"storageAccount": "acct", "queue": "q1", "decodeBase64": "true",
                                                         "visibilityTimeout": "300ms", "pollingInterval": "200ms",
                                                         "concurrency": "4"})

    async def main():
        async with Harness(app, [q]) as h:
            b = h.backing.broker("storage-acct")
            t0 = _t.monotonic()
            for n in range(40):
                b.send("q1", base64.b64encode(json.dumps({"n": n}).encode()))
            h.backing.waiters.notify("storage-acct|q1")
            # 38 fast messages through 3 free slots (the 4th is held by the slow one), long before it ends
            await _until(lambda: len([x for x in done if x >= 2]) == 38, timeout=5)
            assert 0 not in done and all(done[x] - t0 < 1.5 for x in done if x >= 2)
            await _until(lambda: 1 in done, timeout=5)  # the failed one came back after its visibility timeout
            assert attempts[1] == 2 and done[1] - t0 >= 0.3
            release.set()
            await _until(lambda: 0 in done and b.counts("q1")["completed"] == 40, timeout=5)
            # (the slow one outlived its 300 ms visibility timeout, so it was handed out again --
            # at-least-once, as the storage queue promises -- and still only 40 were completed)
    run(main())


def test_secret_references_and_stores(tmp_path):
    secrets_file = tmp_path / "secrets.json"
    secrets_file.write_text(json.dumps({"db": {"key": "s3cr3t"}, "plain": "p"}))
    store = _inline("localsecrets", "secretstores.local.file", {"secretsFile": str(secrets_file), "nestedSeparator": ":"})
    state = _inline("kv", "state.in-memory", {"password": {"secretKeyRef": {"name": "db:key", "key": "db:key"}}},
                    auth={"secretStore": "localsecrets"})
    app = WebApp("s")

    async def main():
        async with Harness(app, [store, state]) as h:
            assert h.sc.components["kv"].metadata["password"] == "s3cr3t"
            r = await h.http.get(f"{h.base}/v1.0/secrets/localsecrets/plain")
            assert r.json() == {"plain": "p"}
            r = await h.http.get(f"{h.base}/v1.0/secrets/localsecrets/bulk")
            assert r.json()["db:key"] == {"db:key": "s3cr3t"}
            assert (await h.http.get(f"{h.base}/v1.0/secrets/none/x")).status == 401
    run(main())


def test_api_token_and_scoping():
    app = WebApp("t")
    kv = _inline("kv", "state.in-memory", {}, scopes=["other-app"])
    kv2 = _inline("kv2", "state.in-memory", {"keyPrefix": "none"})

    async def main():
        async with Harness(app, [kv, kv2], api_token="tok") as h:
            assert (await h.http.get(f"{h.base}/v1.0/state/kv2/a")).status == 401
            hdr = {"dapr-api-token": "tok"}
            assert (await h.http.get(f"{h.base}/v1.0/healthz")).status == 204  # health is exempt
            r = await h.http.post(f"{h.base}/v1.0/state/kv", json_body=[{"key": "a", "value": 1}], headers=hdr)
            assert r.status == 400  # out of scope -> not loaded
            c = SidecarClient(h.base, api_token="tok")
            await c.save_state("kv2", "a", {"v": 1})
            assert await c.get_state("kv2", "a") == {"v": 1}
            st = h.sc.state_stores["kv2"]
            assert st.store.get("a") is not None  # keyPrefix none -> raw key
            await c.close()
    run(main())


def test_cron_parser():
    s = CronSchedule.parse("5 0 * * *")
    t = datetime(2024, 5, 1, 12, 0, tzinfo=timezone.utc)
    assert s.next_after(t) == datetime(2024, 5, 2, 0, 5, tzinfo=timezone.utc)
    assert CronSchedule.parse("*/15 * * * * *").next_after(t).second == 15
    assert CronSchedule.parse("0 0 1 JAN *").next_after(t) == datetime(2025, 1, 1, tzinfo=timezone.utc)
    wk = CronSchedule.parse("0 9 * * MON-FRI").next_after(datetime(2024, 5, 3, 10, 0, tzinfo=timezone.utc))  # Fri
    assert wk == datetime(2024, 5, 6, 9, 0, tzinfo=timezone.utc)
    assert CronSchedule.parse("@every 1m30s").next_after(t) == datetime(2024, 5, 1, 12, 1, 30, tzinfo=timezone.utc)
    assert CronSchedule.parse("@daily").next_after(t) == datetime(2024, 5, 2, tzinfo=timezone.utc)
    # dom + dow both restricted: OR semantics
    either = CronSchedule.parse("0 0 13 * FRI")
    assert either.next_after(datetime(2024, 5, 1, tzinfo=timezone.utc)) == datetime(2024, 5, 3, tzinfo=timezone.utc)
    assert parse_duration("500ms").total_seconds() == 0.5
    for bad in ("* * *", "61 * * * *", "x * * * *", "@every 0s"):
        with pytest.raises(CronError):
            CronSchedule.parse(bad)


def test_cloudevent_envelope():
    from aca_dotnet_workshop_amd.sidecar import make_cloudevent
    ce = make_cloudevent(b'{"a":1}', "application/json", "ps", "t", "app", "00-" + "1" * 32 + "-" + "2" * 16 + "-01")
    assert ce["specversion"] == "1.0" and ce["data"] == {"a": 1} and ce["pubsubname"] == "ps" and ce["topic"] == "t"
    assert ce["type"] == "com.dapr.event.sent" and ce["traceparent"].startswith("00-111")
    assert make_cloudevent(b"hi", "text/plain", "ps", "t", "app", None)["data"] == "hi"
    assert "data_base64" in make_cloudevent(b"\x00\x01", "application/octet-stream", "ps", "t", "app", None)


def test_cron_single_replica_lease():
    """``singleReplica: "true"``: several replicas of the processor run the same cron binding, and
    each tick is delivered by exactly one of them (a first-write lease document per tick in the
    state store) -- the scale-out vs. periodic-job conflict the reference leaves open
    (docs/aca/07-aca-cron-bindings/index.md:234)."""
    comp = _inline("tick", "bindings.cron", {"schedule": "@every 200ms", "singleReplica": "true"})
    hits: list[tuple[str, str]] = []

    def app(tag):
        a = WebApp(f"cron-{tag}")

        async def on_tick(req):
            hits.append((tag, req.headers.get("x-fire-time") or req.headers.get("fireTime") or
                         json.dumps(sorted(req.headers.items()))))
            return empty(200)
        a.add_route("/tick", on_tick, ("POST",))
        return a

    async def main():
        loop = asyncio.get_running_loop()
        backing = BackingServices()
        bsrv = HttpServer(backing.build_app(), loop)
        burl = f"http://127.0.0.1:{await bsrv.listen_tcp('127.0.0.1', 0)}"
        servers, cars = [], []
        for tag in "abc":
            a = app(tag)
            s = HttpServer(a, loop)
            await a.startup()
            port = await s.listen_tcp("127.0.0.1", 0)
            sc = Sidecar("proc", app_port=port, http_port=0, components=[comp], resolver=NameResolver(),
                         backing_url=burl, identity="proc", instance=f"proc-{tag}")
            await sc.start()
            servers.append(s)
            cars.append(sc)
        await asyncio.sleep(2.1)
        for sc in cars:
            await sc.stop(1.0)
        for s in servers:
            await s.close(1.0)
        await bsrv.close(1.0)
        fired = sum(b.fired for sc in cars for b in sc.bindings.values())
        assert 7 <= fired <= 12, fired                   # ~10 ticks in 2 s, each fired once
        assert len(hits) == fired                        # every claimed tick was delivered once
        assert len({t for t, _ in hits}) >= 1
    run(main())
