"""Backing-services emulator: one process standing in for the cloud services the
reference's Dapr components talk to:

============================  =================================  ==========================================
reference service             component type(s)                  emulated here by
============================  =================================  ==========================================
Cosmos DB (SQL API)           state.azure.cosmosdb               ``/cosmos``  -> native ``DocStore``
Redis (``dapr init``)          state.redis, pubsub.redis          ``/cosmos`` + ``/servicebus`` namespaces ``redis-*``
Service Bus topics/subs        pubsub.azure.servicebus(.topics)   ``/servicebus`` -> native ``Broker``
Storage Queue                  bindings.azure.storagequeues       ``/storage/.../queues`` -> native ``Broker``
Blob Storage                   bindings.azure.blobstorage         ``/storage/.../blobs`` -> files
Key Vault                      secretstores.azure.keyvault        ``/keyvault``
SendGrid                       bindings.twilio.sendgrid           ``/sendgrid`` -> outbox (JSONL)
============================  =================================  ==========================================

Long-poll receive (``waitMs``) gives push-like latency without busy polling.  All state
is persisted under ``--data-dir`` when given (append-only logs + files), so restarting
the emulator keeps tasks, queued messages, blobs and secrets.
"""
from __future__ import annotations

import argparse
import asyncio
import base64
import concurrent.futures
import json
import logging
import os
import re
import sys
import tempfile
import time
from pathlib import Path
from typing import Any

from .. import native
from ..telemetry import configure, configure_logging
from ..telemetry.tracing import parse_traceparent, tracer
from ..telemetry.profiler import maybe_profile
from ..utils import gctrace
from ..web.app import WebApp
from ..web.http import HTTPError, Request, Response, empty, json_response, problem
from .accel import CollectionAccelerator, accelerator_from_env, mirror_paths_from_env
from .auth import AccessPolicy

log = logging.getLogger("backing")
_SAFE = re.compile(r"[^A-Za-z0-9._-]")


def _safe(name: str) -> str:
    return _SAFE.sub("_", name)


class Waiters:
    """Per-entity wake-ups for long-poll receivers (replace-on-notify events)."""

    def __init__(self) -> None:
        self._ev: dict[str, asyncio.Event] = {}
        self.listeners: list[Any] = []  # e.g. the native front's parked receives

    def notify(self, key: str) -> None:
        ev = self._ev.pop(key, None)
        if ev is not None:
            ev.set()
        for fn in self.listeners:
            fn(key)

    async def wait(self, key: str, timeout: float) -> None:
        ev = self._ev.get(key)
        if ev is None:
            ev = self._ev[key] = asyncio.Event()
        try:
            await asyncio.wait_for(ev.wait(), timeout)
        except asyncio.TimeoutError:
            pass


def _encode_body(body: bytes) -> dict[str, str]:
    try:
        return {"body": body.decode("utf-8")}
    except UnicodeDecodeError:
        return {"bodyB64": base64.b64encode(body).decode()}


def _decode_body(entry: dict[str, Any]) -> bytes:
    if "bodyB64" in entry:
        return base64.b64decode(entry["bodyB64"])
    b = entry.get("body", "")
    if isinstance(b, str):
        return b.encode()
    return json.dumps(b).encode()


class BackingServices:
    def __init__(self, data_dir: str | None = None, policy: AccessPolicy | None = None, fsync: int = 0) -> None:
        self.N = native.load()
        self.data_dir = Path(data_dir) if data_dir else None
        self._tmp = None
        if self.data_dir is None:
            self._tmp = tempfile.TemporaryDirectory(prefix="tt-backing-")
            self.blob_root = Path(self._tmp.name) / "blobs"
        else:
            self.data_dir.mkdir(parents=True, exist_ok=True)
            self.blob_root = self.data_dir / "storage"
        self.policy = policy or AccessPolicy()
        self.fsync = fsync
        self.stores: dict[tuple[str, str, str], Any] = {}
        self.accel_mode, self.accel_min_docs = accelerator_from_env()
        self.mirror_paths = mirror_paths_from_env()
        # blocking query work (columnar mirror sync, GPU kernels, native scans) runs here, never
        # on the event loop; the per-collection accelerator lock serialises GPU use
        self.query_pool = concurrent.futures.ThreadPoolExecutor(max_workers=4, thread_name_prefix="tt-query")
        self.accels: dict[tuple[str, str, str], CollectionAccelerator] = {}
        self.brokers: dict[str, Any] = {}
        self.waiters = Waiters()
        self.vaults: dict[str, dict[str, str]] = {}
        self.outbox: list[dict[str, Any]] = []
        self.front = None
        self._load_vaults()

    # -- native front --------------------------------------------------------------
    def attach_front(self, front) -> None:
        """Let the native HTTP front (native/src/backingfront.hpp) serve hot routes against
        this process's engines.  Engines created later are attached on creation."""
        self.front = front
        for (a, d, c), s in self.stores.items():
            front.attach_store(a, d, c, s)
        for ns, b in self.brokers.items():
            front.attach_broker(ns, b)
        self._push_policy()
        self.waiters.listeners.append(lambda key: front.notify(*key.split("|", 1)))
        front.set_blob_root(str(self.blob_root))

    def _push_policy(self) -> None:
        if self.front is None:
            return
        from .auth import ROLE_ACTIONS
        grants = [(a.principal, a.scope, sorted(ROLE_ACTIONS.get(a.role, set()))) for a in self.policy.assignments]
        self.front.set_policy(self.policy.mode, list(self.policy.keys.items()), grants)

    # -- engines ---------------------------------------------------------------
    def _path(self, *parts: str) -> str:
        # TT_BACKING_LOGS=0: documents and messages kept in memory only (a measurement switch:
        # what the append logs cost the write path)
        if self.data_dir is None or os.environ.get("TT_BACKING_LOGS", "1") == "0":
            return ""
        p = self.data_dir.joinpath(*[_safe(x) for x in parts])
        p.parent.mkdir(parents=True, exist_ok=True)
        return str(p)

    def store(self, account: str, db: str, coll: str):
        key = (account, db, coll)
        s = self.stores.get(key)
        if s is None:
            s = self.stores[key] = self.N.DocStore(self._path("cosmos", account, db, coll + ".log"), self.fsync)
            self.accel(account, db, coll).attach(s)
            if self.front is not None:
                self.front.attach_store(account, db, coll, s)
        return s

    def run_query(self, account: str, db: str, coll: str, raw: bytes, prefix: str, sort_keys: bool,
                  traceparent: str = "", sent_mono: str = "", front_mono: str = "") -> tuple[int, bytes, list]:
        """A state query of the collection, after admission (auth and RU charge are the
        caller's): the planner sends it to the columnar / GPU accelerator or the native engine.
        Returns (200, result JSON, headers) -- the result-size RU are debited here -- or (400,
        the error, []).  Blocking; runs on the query pool (the Python route) or on the native
        front's query worker (backingfront.hpp ``set_query_fn``), with no HTTP hop in between.
        A sampled caller (the data plane passes the trace on for queries) gets the store's share
        as spans: the query, and the planner + page run inside it."""
        s = self.store(account, db, coll)
        a = self.accel(account, db, coll)
        tp = parse_traceparent(traceparent) if traceparent else None
        span = tracer().start_span("POST query", "server", parent=tp, activate=False) if tp and tp[2] else None
        if span is not None:  # the hops before this call, from the callers' monotonic stamps
            now = time.monotonic()
            for k, at in (("since_sidecar_sent_ms", sent_mono), ("since_front_forwarded_ms", front_mono)):
                try:
                    span.set(k, round((now - float(at)) * 1e3, 3))
                except (TypeError, ValueError):
                    pass
        text = raw.decode("utf-8") if raw else "{}"
        inner = tracer().start_span("query run", "internal", parent=span) if span is not None else None
        try:
            q = json.loads(text)
            res = a.query(q, prefix, s, sort_keys) if isinstance(q, dict) else None
            res = s.query(text, prefix, sort_keys) if res is None else res
        except ValueError as ex:
            if inner is not None:
                inner.end()
            if span is not None:
                span.end()
            return 400, str(ex).encode(), []
        if inner is not None:
            inner.end()
        body = res if isinstance(res, bytes) else res.encode()
        s.debit(s.query_ru(len(body)) - s.query_ru(0))  # result size part: owed after the fact
        if span is None:
            return 200, body, []
        span.set("bytes", len(body))
        span.end()
        return 200, body, [("x-tt-handler-end-mono", f"{time.monotonic():.6f}")]

    def accel(self, account: str, db: str, coll: str) -> CollectionAccelerator:
        key = (account, db, coll)
        a = self.accels.get(key)
        if a is None:
            a = self.accels[key] = CollectionAccelerator(self.accel_mode, self.accel_min_docs, self.mirror_paths)
        return a

    def broker(self, ns: str):
        b = self.brokers.get(ns)
        if b is None:
            b = self.brokers[ns] = self.N.Broker(self._path("servicebus", ns + ".log"), self.fsync)
            if self.front is not None:
                self.front.attach_broker(ns, b)
        return b

    def prewarm_accelerator(self) -> None:
        try:
            CollectionAccelerator(self.accel_mode, self.accel_min_docs).kernels()
        except Exception as e:
            log.warning("GPU query accelerator unavailable: %s", e)

    def _load_vaults(self) -> None:
        if self.data_dir is None:
            return
        f = self.data_dir / "keyvault.json"
        if f.exists():
            self.vaults = json.loads(f.read_text())
        ob = self.data_dir / "sendgrid-outbox.jsonl"
        if ob.exists():
            self.outbox = [json.loads(x) for x in ob.read_text().splitlines() if x.strip()]

    def _save_vaults(self) -> None:
        if self.data_dir is None:
            return
        tmp = self.data_dir / "keyvault.json.tmp"
        tmp.write_text(json.dumps(self.vaults))
        os.replace(tmp, self.data_dir / "keyvault.json")

    # -- auth ------------------------------------------------------------------
    def authorize(self, req: Request, action: str, scope: str) -> None:
        ident = req.headers.get("x-tt-identity")
        key = req.headers.get("x-tt-key")
        if not self.policy.check(action, scope, ident, key):
            raise HTTPError(403, detail=f"{ident or 'anonymous'} is not authorized to perform {action} on {scope}")

    # -- app -------------------------------------------------------------------
    def build_app(self) -> WebApp:
        app = WebApp("backing-services")
        self._cosmos_routes(app)
        self._servicebus_routes(app)
        self._storage_routes(app)
        self._keyvault_routes(app)
        self._sendgrid_routes(app)
        self._admin_routes(app)
        return app

    # ---------------------------------------------------------------- cosmos
    def _cosmos_routes(self, app: WebApp) -> None:
        base = "/cosmos/{account}/{db}/{coll}"

        def st(req: Request, action: str):
            p = req.path_params
            self.authorize(req, action, f"cosmos/{p['account']}")
            return self.store(p["account"], p["db"], p["coll"])

        def acc(req: Request) -> CollectionAccelerator:
            p = req.path_params
            return self.accel(p["account"], p["db"], p["coll"])

        def throttled(req: Request, s, ru: float, kind: int = 1) -> Response | None:
            """Provisioned-throughput admission (DocStore.charge, shared with the native front):
            a 429 reserves the caller's slot -- bound to the request: method + target, plus the
            body of a query or a bulk / transactional write -- and hands out its ticket
            (x-tt-ru-ticket).  ``kind``: 0 read, 1 write, 2 query, 3 delete."""
            bind = f"{req.method} {req.target}"
            if kind == 2 or req.method == "POST":
                bind += "\xff" + req.body.decode("utf-8", "replace")
            wait_ms, ticket = s.charge(ru, int(req.headers.get("x-tt-ru-ticket") or 0), bind, kind)
            if not wait_ms:
                return None
            r = problem(429, detail="Request rate is large: the container's provisioned throughput is exhausted")
            r.headers += [("x-ms-retry-after-ms", str(wait_ms)), ("Retry-After", str((wait_ms + 999) // 1000))]
            if ticket:
                r.headers.append(("x-tt-ru-ticket", str(ticket)))
            return r

        async def put_doc(req: Request) -> Response:
            s = st(req, "cosmos.write")
            if (t := throttled(req, s, s.write_ru(len(req.body)))) is not None:
                return t
            etag = req.headers.get("if-match") or None
            value = req.body.decode("utf-8")
            ttl = int(req.headers.get("x-tt-ttl-ms", "0") or 0)
            try:
                e = s.set(req.path_params["key"], value, etag, req.headers.get("x-tt-first-write") == "1", ttl)
            except self.N.EtagMismatch as ex:
                return problem(412, detail=str(ex))
            except ValueError as ex:
                return problem(400, detail=str(ex))
            return json_response({"etag": e}, headers=[("ETag", e)])

        async def get_doc(req: Request) -> Response:
            s = st(req, "cosmos.read")
            if (t := throttled(req, s, s.read_ru(0), 0)) is not None:
                return t
            r = s.get(req.path_params["key"])
            if r is None:
                return empty(404)
            return Response(r[0].encode(), 200, [("ETag", r[1])], "application/json")

        async def del_doc(req: Request) -> Response:
            s = st(req, "cosmos.write")
            if (t := throttled(req, s, s.write_ru(0), 3)) is not None:
                return t
            try:
                ok = s.delete(req.path_params["key"], req.headers.get("if-match") or None)
            except self.N.EtagMismatch as ex:
                return problem(412, detail=str(ex))
            return empty(204 if ok else 404)

        async def bulk_get(req: Request) -> Response:
            s = st(req, "cosmos.read")
            keys = (req.json() or {}).get("keys", [])
            if (t := throttled(req, s, s.read_ru(0) * max(1, len(keys)), 0)) is not None:
                return t
            out = []
            for k in keys:
                r = s.get(k)
                out.append({"key": k, "data": json.loads(r[0]), "etag": r[1]} if r else {"key": k})
            return json_response(out)

        async def bulk_set(req: Request) -> Response:
            s = st(req, "cosmos.write")
            items = req.json() or []
            # a value sent as JSON itself (the native data plane's form) is stored as its compact
            # text -- the very bytes of the request, compacted by the native front's own scanner
            # (numbers and escapes as sent); a string value holds JSON text
            texts = self.N.bulk_values(req.body) if len(req.body) else []
            if texts is None or len(texts) != len(items):
                texts = [v if isinstance(v := it.get("value"), str) else _compact_json(v) for it in items]
            if (t := throttled(req, s, sum(s.write_ru(len(v)) for v in texts) or 1)) is not None:
                return t
            out = []
            for it, value in zip(items, texts):
                try:
                    ttl = int(it.get("ttlMs") or 0)
                    e = s.set(it["key"], value, it.get("etag") or None, bool(it.get("firstWrite")), ttl)
                    out.append({"key": it["key"], "etag": e})
                except self.N.EtagMismatch as ex:
                    out.append({"key": it["key"], "error": "etag", "detail": str(ex)})
                except ValueError as ex:
                    out.append({"key": it["key"], "error": "invalid", "detail": str(ex)})
            status = 412 if any(o.get("error") == "etag" for o in out) else (
                400 if any("error" in o for o in out) else 200)
            return json_response(out, status)

        async def query(req: Request) -> Response:
            s = st(req, "cosmos.read")
            # ?project=sortkeys: {"key", "etag", "sort"} per result -- phase one of a
            # cross-partition page (the sidecar fetches the merged page's documents after)
            sort_keys = (req.query_get("project", "") or "").lower() == "sortkeys"
            if (t := throttled(req, s, s.query_ru(0), 2)) is not None:
                return t
            p = req.path_params
            status, body, headers = await asyncio.get_running_loop().run_in_executor(
                self.query_pool, self.run_query, p["account"], p["db"], p["coll"], req.body,
                req.query_get("prefix", "") or "", sort_keys, req.headers.get("traceparent") or "",
                req.headers.get("x-tt-sent-mono") or "", req.headers.get("x-tt-front-mono") or "")
            if status != 200:
                return problem(status, detail=body.decode("utf-8", "replace"))
            return Response(body, 200, headers or None, "application/json")

        async def transaction(req: Request) -> Response:
            s = st(req, "cosmos.write")
            if (t := throttled(req, s, s.write_ru(len(req.body)))) is not None:
                return t
            ops = []
            raw_ops = (req.json() or {}).get("ops", [])
            # each value stored as the request's own compact bytes (numbers and escapes as sent),
            # the same text a save or a bulk save of that value stores
            texts = self.N.tx_values(req.body) if len(req.body) else None
            if texts is None or len(texts) != len(raw_ops):
                texts = [v if isinstance(v := o.get("value"), str) else _compact_json(v) for o in raw_ops]
            for o, text in zip(raw_ops, texts):
                is_del = o.get("op") == "delete"
                ops.append(self.N.TxOp(is_del, o["key"], "" if is_del else text,
                                       o.get("etag") or None, bool(o.get("firstWrite")), int(o.get("ttlMs") or 0)))
            try:
                s.transact(ops)
            except self.N.EtagMismatch as ex:
                return problem(412, detail=str(ex))
            except ValueError as ex:
                return problem(400, detail=str(ex))
            return empty(204)

        async def stats(req: Request) -> Response:
            s = st(req, "cosmos.read")
            d = dict(s.stats())
            d["indexedPaths"] = s.indexed_paths()
            d["throughput"] = dict(s.throughput_stats())
            d["durability"] = {"fsync_mode": self.fsync, "group_commit": s.group_commit(), **dict(s.commit_stats())}
            a = acc(req)
            d["accelerator"] = {"mode": a.mode, "rows": a.index.live_rows() if a.index else 0, **a.stats,
                                "mirror": dict(s.mirror_stats())}
            return json_response(d)

        async def keys(req: Request) -> Response:
            s = st(req, "cosmos.read")
            return json_response(s.keys(req.query_get("prefix", "") or "", int(req.query_get("limit", "0") or 0)))

        app.add_route(base + "/docs/{key}", put_doc, ("PUT",))
        app.add_route(base + "/docs/{key}", get_doc, ("GET",))
        app.add_route(base + "/docs/{key}", del_doc, ("DELETE",))
        app.add_route(base + "/bulkget", bulk_get, ("POST",))
        app.add_route(base + "/bulkset", bulk_set, ("POST",))
        app.add_route(base + "/query", query, ("POST",))
        app.add_route(base + "/transaction", transaction, ("POST",))
        async def set_throughput(req: Request) -> Response:
            """Provision the container's RU/s (Bicep ``autoscaleSettings.maxThroughput`` /
            ``options.throughput``; 0 = unlimited)."""
            s = st(req, "cosmos.write")
            body = req.json() or {}
            s.set_throughput(float(body.get("ruPerSecond") or 0))
            return json_response(dict(s.throughput_stats()))

        app.add_route(base + "/stats", stats, ("GET",))
        app.add_route(base + "/throughput", set_throughput, ("PUT",))
        app.add_route(base + "/keys", keys, ("GET",))

    # ---------------------------------------------------------------- service bus
    def _servicebus_routes(self, app: WebApp) -> None:
        def opts(d: dict[str, Any]):
            return self.N.QueueOptions(int(d.get("lockMs", 60000)), int(d.get("maxDelivery", 10)),
                                       int(d.get("ttlMs", 0)), bool(d.get("deadLetterOnExpiry", False)))

        async def create_topic(req: Request) -> Response:
            p = req.path_params
            self.authorize(req, "sb.manage", f"servicebus/{p['ns']}")
            self.broker(p["ns"]).create_topic(p["topic"])
            return empty(204)

        async def create_sub(req: Request) -> Response:
            p = req.path_params
            self.authorize(req, "sb.manage", f"servicebus/{p['ns']}")
            self.broker(p["ns"]).create_subscription(p["topic"], p["sub"], opts(req.json() or {}))
            return empty(204)

        async def create_queue(req: Request) -> Response:
            p = req.path_params
            self.authorize(req, "sb.manage", f"servicebus/{p['ns']}")
            self.broker(p["ns"]).create_queue(p["queue"], opts(req.json() or {}))
            return empty(204)

        def _notify_topic(ns: str, topic: str) -> None:
            for sub in self.broker(ns).subscriptions(topic):
                self.waiters.notify(f"{ns}|{topic}/subscriptions/{sub}")

        async def publish(req: Request) -> Response:
            p = req.path_params
            self.authorize(req, "sb.send", f"servicebus/{p['ns']}/topics/{p['topic']}")
            h = req.headers
            seq = self.broker(p["ns"]).publish(p["topic"], req.body, h.get("content-type", "application/json"),
                                               h.get("x-tt-props", "{}"), h.get("x-tt-message-id", ""),
                                               int(h.get("x-tt-ttl-ms", "0") or 0), int(h.get("x-tt-delay-ms", "0") or 0))
            _notify_topic(p["ns"], p["topic"])
            return json_response({"seq": seq}, 201)

        async def publish_batch(req: Request) -> Response:
            p = req.path_params
            self.authorize(req, "sb.send", f"servicebus/{p['ns']}/topics/{p['topic']}")
            b = self.broker(p["ns"])
            seqs = []
            for e in req.json() or []:
                seqs.append(b.publish(p["topic"], _decode_body(e), e.get("contentType", "application/json"),
                                      json.dumps(e.get("props") or {}), e.get("id", ""), int(e.get("ttlMs", 0)), 0))
            _notify_topic(p["ns"], p["topic"])
            return json_response({"seqs": seqs}, 201)

        async def send(req: Request) -> Response:
            p = req.path_params
            self.authorize(req, "sb.send", f"servicebus/{p['ns']}/queues/{p['queue']}")
            h = req.headers
            seq = self.broker(p["ns"]).send(p["queue"], req.body, h.get("content-type", "application/json"),
                                            h.get("x-tt-props", "{}"), h.get("x-tt-message-id", ""),
                                            int(h.get("x-tt-ttl-ms", "0") or 0), int(h.get("x-tt-delay-ms", "0") or 0))
            self.waiters.notify(f"{p['ns']}|{p['queue']}")
            return json_response({"seq": seq}, 201)

        async def receive(req: Request) -> Response:
            ns = req.path_params["ns"]
            entity = req.query_get("entity") or ""
            self.authorize(req, "sb.receive", f"servicebus/{ns}/{_entity_scope(entity)}")
            mx = int(req.query_get("max", "1") or 1)
            lock = int(req.query_get("lockMs", "0") or 0)
            wait_s = int(req.query_get("waitMs", "0") or 0) / 1000.0
            b = self.broker(ns)
            key = f"{ns}|{entity}"
            deadline = time.monotonic() + wait_s
            conn = req.state.get("conn")
            while True:
                if conn is not None and conn.closed:
                    return json_response([])  # the receiver is gone: take no messages for it
                msgs = b.receive(entity, mx, lock)
                rem = deadline - time.monotonic()
                if msgs or rem <= 0:
                    break
                await self.waiters.wait(key, min(rem, 0.2))
            out = []
            for m in msgs:
                d = {"lockToken": m.lock_token, "seq": m.seq, "id": m.id, "contentType": m.content_type,
                     "props": json.loads(m.props or "{}"), "deliveryCount": m.delivery_count, "enqueuedMs": m.enqueued_ms}
                d.update(_encode_body(m.body))
                out.append(d)
            return json_response(out)

        async def settle(req: Request) -> Response:
            ns = req.path_params["ns"]
            body = req.json() or {}
            entity = body.get("entity", "")
            self.authorize(req, "sb.receive", f"servicebus/{ns}/{_entity_scope(entity)}")
            b = self.broker(ns)
            res: dict[str, list[bool]] = {}
            res["complete"] = [b.complete(entity, t) for t in body.get("complete", [])]
            res["abandon"] = [b.abandon(entity, a["token"], int(a.get("delayMs", 0))) for a in body.get("abandon", [])]
            res["deadletter"] = [b.dead_letter(entity, d["token"], d.get("reason", "")) for d in body.get("deadletter", [])]
            res["renew"] = [b.renew(entity, r["token"], int(r.get("lockMs", 0))) for r in body.get("renew", [])]
            if body.get("abandon"):
                self.waiters.notify(f"{ns}|{entity}")
            return json_response(res)

        async def counts(req: Request) -> Response:
            ns = req.path_params["ns"]
            entity = req.query_get("entity") or ""
            return json_response(dict(self.broker(ns).counts(entity)))

        async def dead_letters(req: Request) -> Response:
            ns = req.path_params["ns"]
            entity = req.query_get("entity") or ""
            self.authorize(req, "sb.receive", f"servicebus/{ns}/{_entity_scope(entity)}")
            out = []
            for seq, mid, body, reason, dc in self.broker(ns).drain_dead_letters(entity, int(req.query_get("max", "100"))):
                d = {"seq": seq, "id": mid, "reason": reason, "deliveryCount": dc}
                d.update(_encode_body(body))
                out.append(d)
            return json_response(out)

        async def entities(req: Request) -> Response:
            b = self.broker(req.path_params["ns"])
            return json_response({e: dict(b.counts(e)) for e in b.entities()})

        app.add_route("/servicebus/{ns}/topics/{topic}", create_topic, ("PUT",))
        app.add_route("/servicebus/{ns}/topics/{topic}/subscriptions/{sub}", create_sub, ("PUT",))
        app.add_route("/servicebus/{ns}/queues/{queue}", create_queue, ("PUT",))
        app.add_route("/servicebus/{ns}/topics/{topic}/messages", publish, ("POST",))
        app.add_route("/servicebus/{ns}/topics/{topic}/batch", publish_batch, ("POST",))
        app.add_route("/servicebus/{ns}/queues/{queue}/messages", send, ("POST",))
        app.add_route("/servicebus/{ns}/receive", receive, ("POST",))
        app.add_route("/servicebus/{ns}/settle", settle, ("POST",))
        app.add_route("/servicebus/{ns}/counts", counts, ("GET",))
        app.add_route("/servicebus/{ns}/deadletters", dead_letters, ("POST",))
        app.add_route("/servicebus/{ns}/entities", entities, ("GET",))

    # ---------------------------------------------------------------- storage
    def _storage_routes(self, app: WebApp) -> None:
        def qbroker(account: str):
            return self.broker(f"storage-{account}")

        async def put_message(req: Request) -> Response:
            p = req.path_params
            self.authorize(req, "queue.send", f"storage/{p['account']}")
            ttl = int(req.query_get("messagettl", "0") or 0) * 1000
            delay = int(req.query_get("visibilitytimeout", "0") or 0) * 1000
            seq = qbroker(p["account"]).send(p["queue"], req.body, "text/plain", "{}", "", ttl, delay)
            self.waiters.notify(f"storage-{p['account']}|{p['queue']}")
            return json_response({"messageId": str(seq)}, 201)

        async def get_messages(req: Request) -> Response:
            p = req.path_params
            self.authorize(req, "queue.receive", f"storage/{p['account']}")
            mx = int(req.query_get("numofmessages", "1") or 1)
            vis = int(req.query_get("visibilityMs", "30000") or 30000)
            wait_s = int(req.query_get("waitMs", "0") or 0) / 1000.0
            b = qbroker(p["account"])
            key = f"storage-{p['account']}|{p['queue']}"
            deadline = time.monotonic() + wait_s
            while True:
                msgs = b.receive(p["queue"], mx, vis)
                rem = deadline - time.monotonic()
                if msgs or rem <= 0:
                    break
                await self.waiters.wait(key, min(rem, 0.2))
            out = []
            for m in msgs:
                d = {"messageId": str(m.seq), "popReceipt": m.lock_token, "dequeueCount": m.delivery_count,
                     "insertionMs": m.enqueued_ms}
                d.update(_encode_body(m.body))
                out.append(d)
            return json_response(out)

        async def delete_message(req: Request) -> Response:
            p = req.path_params
            self.authorize(req, "queue.receive", f"storage/{p['account']}")
            ok = qbroker(p["account"]).complete(p["queue"], p["receipt"])
            return empty(204 if ok else 404)

        async def update_message(req: Request) -> Response:
            p = req.path_params
            self.authorize(req, "queue.receive", f"storage/{p['account']}")
            delay = int(req.query_get("visibilityMs", "0") or 0)
            ok = qbroker(p["account"]).abandon(p["queue"], p["receipt"], delay)
            self.waiters.notify(f"storage-{p['account']}|{p['queue']}")
            return empty(204 if ok else 404)

        async def queue_count(req: Request) -> Response:
            p = req.path_params
            return json_response(dict(qbroker(p["account"]).counts(p["queue"])))

        # per container, the names of its blobs (built by one scan on first use, then kept by
        # put / delete -- this process is the only writer): a count needs no directory walk.
        # With the native front the set is the front's (it writes blobs too): blob_note / blob_count
        names: dict[tuple[str, str], set[str]] = {}

        def note_blob(p: dict[str, Any], added: bool) -> None:
            name = os.path.normpath(p["name"])
            if self.front is not None:
                self.front.blob_note(_safe(p["account"]), _safe(p["container"]), name, added)
            elif added:
                blob_names(p).add(name)
            else:
                blob_names(p).discard(name)

        def count_blobs(p: dict[str, Any], prefix: str) -> int:
            if self.front is not None:
                return int(self.front.blob_count(_safe(p["account"]), _safe(p["container"]), prefix))
            got = blob_names(p)
            return sum(1 for x in got if x.startswith(prefix)) if prefix else len(got)

        def blob_names(p: dict[str, Any]) -> set[str]:
            k = (_safe(p["account"]), _safe(p["container"]))
            got = names.get(k)
            if got is None:
                root = self.blob_root / k[0] / k[1]
                got = names[k] = set()
                if root.is_dir():
                    for f in root.rglob("*"):
                        if f.is_file() and not f.name.endswith((".meta.json", ".tmp")):
                            got.add(str(f.relative_to(root)))
            return got

        def blob_file(p: dict[str, Any]) -> Path:
            root = (self.blob_root / _safe(p["account"]) / _safe(p["container"])).resolve()
            f = (root / p["name"]).resolve()
            if root not in f.parents:
                raise HTTPError(400, detail="invalid blob name")
            return f

        async def put_blob(req: Request) -> Response:
            p = req.path_params
            self.authorize(req, "blob.write", f"storage/{p['account']}")
            f = blob_file(p)
            f.parent.mkdir(parents=True, exist_ok=True)
            tmp = f.with_name(f.name + ".tmp")
            tmp.write_bytes(req.body)
            os.replace(tmp, f)
            meta = {"contentType": req.headers.get("content-type", "application/octet-stream"),
                    "lastModified": time.time(), "size": len(req.body)}
            f.with_name(f.name + ".meta.json").write_text(json.dumps(meta))
            note_blob(p, True)
            return json_response({"blobURL": f"/storage/{p['account']}/blobs/{p['container']}/{p['name']}"}, 201)

        async def get_blob(req: Request) -> Response:
            p = req.path_params
            self.authorize(req, "blob.read", f"storage/{p['account']}")
            f = blob_file(p)
            if not f.is_file():
                return empty(404)
            ctype = "application/octet-stream"
            mf = f.with_name(f.name + ".meta.json")
            if mf.exists():
                ctype = json.loads(mf.read_text()).get("contentType", ctype)
            return Response(f.read_bytes(), 200, None, ctype)

        async def delete_blob(req: Request) -> Response:
            p = req.path_params
            self.authorize(req, "blob.write", f"storage/{p['account']}")
            f = blob_file(p)
            if not f.is_file():
                return empty(404)
            f.unlink()
            mf = f.with_name(f.name + ".meta.json")
            if mf.exists():
                mf.unlink()
            note_blob(p, False)
            return empty(204)

        async def list_blobs(req: Request) -> Response:
            p = req.path_params
            self.authorize(req, "blob.read", f"storage/{p['account']}")
            root = self.blob_root / _safe(p["account"]) / _safe(p["container"])
            prefix = req.query_get("prefix", "") or ""
            if (req.query_get("count", "") or "").lower() in ("1", "true"):  # {"count": n}, no listing
                return json_response({"count": count_blobs(p, prefix)})
            out = []
            if root.is_dir():
                for f in sorted(root.rglob("*")):
                    if f.is_file() and not f.name.endswith((".meta.json", ".tmp")):
                        name = str(f.relative_to(root))
                        if name.startswith(prefix):
                            out.append({"name": name, "size": f.stat().st_size})
            return json_response(out)

        app.add_route("/storage/{account}/queues/{queue}/messages", put_message, ("POST",))
        app.add_route("/storage/{account}/queues/{queue}/messages", get_messages, ("GET",))
        app.add_route("/storage/{account}/queues/{queue}/messages/{receipt}", delete_message, ("DELETE",))
        app.add_route("/storage/{account}/queues/{queue}/messages/{receipt}", update_message, ("PUT",))
        app.add_route("/storage/{account}/queues/{queue}/count", queue_count, ("GET",))
        app.add_route("/storage/{account}/blobs/{container}", list_blobs, ("GET",))
        app.add_route("/storage/{account}/blobs/{container}/{*name}", put_blob, ("PUT",))
        app.add_route("/storage/{account}/blobs/{container}/{*name}", get_blob, ("GET",))
        app.add_route("/storage/{account}/blobs/{container}/{*name}", delete_blob, ("DELETE",))

    # ---------------------------------------------------------------- key vault
    def _keyvault_routes(self, app: WebApp) -> None:
        async def get_secret(req: Request) -> Response:
            p = req.path_params
            self.authorize(req, "kv.get", f"keyvault/{p['vault']}")
            v = self.vaults.get(p["vault"], {}).get(p["name"])
            if v is None:
                return problem(404, detail=f"secret {p['name']} not found")
            return json_response({"name": p["name"], "value": v})

        async def set_secret(req: Request) -> Response:
            p = req.path_params
            self.authorize(req, "kv.set", f"keyvault/{p['vault']}")
            self.vaults.setdefault(p["vault"], {})[p["name"]] = (req.json() or {}).get("value", "")
            self._save_vaults()
            return empty(204)

        async def list_secrets(req: Request) -> Response:
            p = req.path_params
            self.authorize(req, "kv.get", f"keyvault/{p['vault']}")
            return json_response(sorted(self.vaults.get(p["vault"], {})))

        app.add_route("/keyvault/{vault}/secrets", list_secrets, ("GET",))
        app.add_route("/keyvault/{vault}/secrets/{name}", get_secret, ("GET",))
        app.add_route("/keyvault/{vault}/secrets/{name}", set_secret, ("PUT",))

    # ---------------------------------------------------------------- sendgrid
    def _sendgrid_routes(self, app: WebApp) -> None:
        async def send_mail(req: Request) -> Response:
            auth = req.headers.get("authorization", "")
            expected = self.policy.keys.get("sendgrid")
            if self.policy.mode == "enforce" and expected and auth != f"Bearer {expected}":
                return problem(401, detail="invalid SendGrid API key")
            msg = req.json() or {}
            if not msg.get("personalizations") or not msg.get("from"):
                return problem(400, detail="personalizations and from are required")
            rec = {"ts": time.time(), "message": msg}
            self.outbox.append(rec)
            if self.data_dir is not None:
                with open(self.data_dir / "sendgrid-outbox.jsonl", "a") as f:
                    f.write(json.dumps(rec) + "\n")
            return empty(202)

        async def outbox(req: Request) -> Response:
            return json_response(self.outbox)

        app.add_route("/sendgrid/v3/mail/send", send_mail, ("POST",))
        app.add_route("/sendgrid/outbox", outbox, ("GET",))

    # ---------------------------------------------------------------- admin
    def _admin_routes(self, app: WebApp) -> None:
        async def health(req: Request) -> Response:
            return empty(204)

        async def overview(req: Request) -> Response:
            out: dict[str, Any] = {"cosmos": {}, "servicebus": {}}
            for (a, d, c), s in self.stores.items():
                out["cosmos"][f"{a}/{d}/{c}"] = dict(s.stats())
            for ns, b in self.brokers.items():
                out["servicebus"][ns] = {e: dict(b.counts(e)) for e in b.entities()}
            out["keyvault"] = {v: sorted(s) for v, s in self.vaults.items()}
            out["sendgrid"] = {"sent": len(self.outbox)}
            return json_response(out)

        async def set_policy(req: Request) -> Response:
            self.policy = AccessPolicy.from_dict(req.json())
            self._push_policy()
            return empty(204)

        app.add_route("/admin/health", health, ("GET",))
        app.add_route("/admin/overview", overview, ("GET",))
        app.add_route("/admin/policy", set_policy, ("PUT",))

        async def front_stats(req: Request) -> Response:
            return json_response({"front": "native" if self.front is not None else "python",
                                  "requests": dict(self.front.stats()) if self.front is not None else {}})
        app.add_route("/admin/front", front_stats, ("GET",))


def _entity_scope(entity: str) -> str:
    if "/subscriptions/" in entity:
        return "topics/" + entity.split("/subscriptions/")[0]
    return "queues/" + entity



def _compact_json(v) -> str:
    return json.dumps(v, separators=(",", ":"), ensure_ascii=False)

async def serve_backing(host: str = "127.0.0.1", port: int = 0, data_dir: str | None = None,
                        policy: dict[str, Any] | None = None, ready=None, stop: asyncio.Event | None = None,
                        uds: str | None = None) -> None:
    """``uds``: serve on that Unix socket too (the environment's processes on this host use it:
    ``TT_BACKING_UDS``, sidecar/base.py)."""
    from ..web.server import HttpServer
    # TT_BACKING_FSYNC: 0 = a write is on its way to the device when acknowledged (survives a
    # process crash), 1 = fdatasync per record, 2 = group commit (acknowledged once synced, the
    # writes of a sync period sharing one fdatasync) -- applog.hpp
    svc = BackingServices(data_dir, AccessPolicy.from_dict(policy), fsync=int(os.environ.get("TT_BACKING_FSYNC", "0")))
    app = svc.build_app()
    srv = HttpServer(app, asyncio.get_running_loop())
    front = None
    priv_dir = None
    if os.environ.get("TT_BACKING_FRONT", "native").lower() == "native":
        # hot routes on the native front (own thread, GIL-free); Python serves the rest privately
        priv_dir = tempfile.mkdtemp(prefix="ttbf-")
        await srv.listen_unix(os.path.join(priv_dir, "py.sock"))
        # 4 shards: with 2, the front's loops were the stack's busiest threads (72-78 %) under the
        # headline, and 4 measured +8 % tasks/s (profiles/r4_hot_threads.md)
        threads = int(os.environ.get("TT_BACKING_FRONT_THREADS", "4"))
        front = svc.N.BackingFront(host, port, os.path.join(priv_dir, "py.sock"), threads, uds or "")
        svc.attach_front(front)
        if os.environ.get("TT_BACKING_QUERY_WORKER", "1") != "0":
            front.set_query_fn(svc.run_query)  # scans run on the front's query worker (run_query)
        bound = front.port()
    else:
        bound = await srv.listen_tcp(host, port)
        if uds:
            await srv.listen_unix(uds)
    log.info("backing services listening on %s:%d (data=%s, front=%s)", host, bound, data_dir,
             "native" if front is not None else "python")
    if svc.mirror_paths and svc.accel_mode in ("auto", "gpu"):
        # collections are mirrored from their first write: open the GPU context now, off the
        # event loop, so the first scan-shaped query does not pay the HIP runtime start-up
        svc.query_pool.submit(svc.prewarm_accelerator)
    if ready:
        ready(bound)
    stop = stop or asyncio.Event()
    loop = asyncio.get_running_loop()
    import signal
    for sig in (signal.SIGTERM, signal.SIGINT):
        try:
            loop.add_signal_handler(sig, stop.set)
        except (NotImplementedError, RuntimeError):
            pass
    await stop.wait()
    for a in svc.accels.values():
        a.close()
    if front is not None:
        front.stop()
    await srv.close()
    if priv_dir:
        import shutil
        shutil.rmtree(priv_dir, ignore_errors=True)


def main(argv: list[str] | None = None) -> None:
    ap = argparse.ArgumentParser(description="Backing-services emulator (Cosmos/ServiceBus/Storage/KeyVault/SendGrid)")
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=10000)
    ap.add_argument("--data-dir", default=None)
    ap.add_argument("--policy", default=None, help="JSON file with access policy (mode/keys/roleAssignments)")
    ap.add_argument("--port-file", default=None)
    ap.add_argument("--uds", default=None, help="also serve on this Unix socket (processes on this host)")
    a = ap.parse_args(argv)
    # queries run on worker threads next to the event loop; every native call that releases the
    # GIL (mirror sync, result assembly, device copies) waits for it again, up to the switch
    # interval (5 ms by default) when the loop is busy -- tens of ms per query under write load
    sys.setswitchinterval(0.0002)
    configure_logging("backing-services")
    configure("backing-services")
    policy = json.loads(Path(a.policy).read_text()) if a.policy else None

    def ready(port: int) -> None:
        if a.port_file:
            tmp = a.port_file + ".tmp"
            Path(tmp).write_text(str(port))
            os.replace(tmp, a.port_file)

    gctrace.install("backing-" + os.path.basename(a.port_file or str(a.port)))
    pc = os.environ.get("TT_PC_SAMPLE")  # native PC sampling of this whole process (diagnostics)
    if pc:
        from .. import native
        native.load().pc_sample_start()
    try:
        with maybe_profile(f"backing-{os.path.basename(a.port_file or str(a.port))}"):
            asyncio.run(serve_backing(a.host, a.port, a.data_dir, policy, ready, uds=a.uds))
    except KeyboardInterrupt:
        pass
    finally:
        if pc:
            from .. import native
            native.load().pc_sample_dump("backing")


if __name__ == "__main__":
    main()
