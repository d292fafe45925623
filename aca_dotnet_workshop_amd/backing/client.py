"""Async client for the backing-services emulator (used by sidecar components, the
platform's provisioning step and tests)."""
from __future__ import annotations

import asyncio
import json
import os
from typing import Any
from urllib.parse import quote, urlencode

from ..web.client import ClientResponse, HttpClient


class BackingError(Exception):
    def __init__(self, status: int, body: bytes, what: str) -> None:
        super().__init__(f"{what}: HTTP {status} {body[:200]!r}")
        self.status = status
        self.body = body


class EtagConflict(BackingError):
    pass


def backing_url(environ: dict[str, str] | None = None) -> str:
    env = os.environ if environ is None else environ
    return env.get("TT_BACKING_URL", "http://127.0.0.1:10000").rstrip("/")


def q(s: str) -> str:
    return quote(s, safe="")


class BackingClient:
    def __init__(self, base_url: str | None = None, identity: str | None = None, key: str | None = None,
                 http: HttpClient | None = None) -> None:
        self.base = (base_url or backing_url()).rstrip("/")
        self.identity = identity if identity is not None else os.environ.get("TT_IDENTITY")
        self.key = key
        self.http = http or HttpClient()
        self.throttled_retries = 0

    def _h(self, extra: dict[str, str] | None = None, key: str | None = None) -> list[tuple[str, str]]:
        h = []
        if self.identity:
            h.append(("x-tt-identity", self.identity))
        k = key or self.key
        if k:
            h.append(("x-tt-key", k))
        if extra:
            h.extend(extra.items())
        return h

    # throttled (429) answers are retried after the store's hint, like the Cosmos SDK behind
    # Dapr's state.azure.cosmosdb: at most THROTTLE_RETRIES times / THROTTLE_MAX_WAIT_S in total
    THROTTLE_RETRIES = 9
    THROTTLE_MAX_WAIT_S = 30.0

    async def _req(self, method: str, path: str, body: bytes | None = None, headers: dict[str, str] | None = None,
                   ok: tuple[int, ...] = (200, 201, 202, 204), what: str = "", timeout: float | None = None) -> ClientResponse:
        waited = 0.0
        hdrs = self._h(headers)
        for attempt in range(self.THROTTLE_RETRIES + 1):
            r = await self.http.request(method, self.base + path, headers=hdrs, body=body, timeout=timeout)
            if r.status != 429 or attempt == self.THROTTLE_RETRIES:
                break
            delay = min(max(float(r.headers.get("x-ms-retry-after-ms") or 100) / 1000.0, 0.001), 5.0)
            if waited + delay > self.THROTTLE_MAX_WAIT_S:
                break
            ticket = r.headers.get("x-tt-ru-ticket")  # the slot the store reserved for this retry
            hdrs = [h for h in hdrs if h[0] != "x-tt-ru-ticket"] + ([("x-tt-ru-ticket", ticket)] if ticket else [])
            waited += delay
            self.throttled_retries += 1
            await asyncio.sleep(delay)
        if r.status == 412 or r.status == 409:
            raise EtagConflict(r.status, r.body, what or path)
        if r.status not in ok:
            raise BackingError(r.status, r.body, what or path)
        return r

    # -- cosmos-like document store -----------------------------------------
    def _coll(self, account: str, db: str, coll: str) -> str:
        return f"/cosmos/{q(account)}/{q(db)}/{q(coll)}"

    async def doc_put(self, account: str, db: str, coll: str, key: str, value: str, etag: str | None = None,
                      first_write: bool = False, ttl_ms: int = 0) -> str:
        h = {"Content-Type": "application/json"}
        if etag:
            h["If-Match"] = etag
        if first_write:
            h["x-tt-first-write"] = "1"
        if ttl_ms:
            h["x-tt-ttl-ms"] = str(ttl_ms)
        r = await self._req("PUT", f"{self._coll(account, db, coll)}/docs/{q(key)}", value.encode(), h, what="state save")
        return r.headers.get("etag", "")

    async def doc_get(self, account: str, db: str, coll: str, key: str) -> tuple[bytes, str] | None:
        r = await self._req("GET", f"{self._coll(account, db, coll)}/docs/{q(key)}", ok=(200, 404), what="state get")
        if r.status == 404:
            return None
        return r.body, r.headers.get("etag", "")

    async def doc_delete(self, account: str, db: str, coll: str, key: str, etag: str | None = None) -> bool:
        h = {"If-Match": etag} if etag else None
        r = await self._req("DELETE", f"{self._coll(account, db, coll)}/docs/{q(key)}", None, h, ok=(204, 404),
                            what="state delete")
        return r.status == 204

    async def doc_bulk_get(self, account: str, db: str, coll: str, keys: list[str]) -> list[dict[str, Any]]:
        r = await self._req("POST", f"{self._coll(account, db, coll)}/bulkget", json.dumps({"keys": keys}).encode(),
                            {"Content-Type": "application/json"}, what="state bulk get")
        return r.json()

    async def doc_bulk_set(self, account: str, db: str, coll: str, items: list[dict[str, Any]]) -> list[dict[str, Any]]:
        r = await self._req("POST", f"{self._coll(account, db, coll)}/bulkset", json.dumps(items).encode(),
                            {"Content-Type": "application/json"}, ok=(200,), what="state bulk save")
        return r.json()

    async def doc_query(self, account: str, db: str, coll: str, query: bytes, prefix: str = "") -> bytes:
        path = f"{self._coll(account, db, coll)}/query"
        if prefix:
            path += "?" + urlencode({"prefix": prefix})
        r = await self._req("POST", path, query, {"Content-Type": "application/json"}, what="state query")
        return r.body

    async def doc_transaction(self, account: str, db: str, coll: str, ops: list[dict[str, Any]]) -> None:
        await self._req("POST", f"{self._coll(account, db, coll)}/transaction", json.dumps({"ops": ops}).encode(),
                        {"Content-Type": "application/json"}, what="state transaction")

    async def doc_stats(self, account: str, db: str, coll: str) -> dict[str, Any]:
        return (await self._req("GET", f"{self._coll(account, db, coll)}/stats")).json()

    async def doc_set_throughput(self, account: str, db: str, coll: str, ru_per_s: float) -> dict[str, Any]:
        """Provision a container's RU/s (0 = unlimited)."""
        return (await self._req("PUT", f"{self._coll(account, db, coll)}/throughput",
                                json.dumps({"ruPerSecond": ru_per_s}).encode(),
                                {"Content-Type": "application/json"})).json()

    # -- service bus ----------------------------------------------------------
    async def sb_create_topic(self, ns: str, topic: str) -> None:
        await self._req("PUT", f"/servicebus/{q(ns)}/topics/{q(topic)}")

    async def sb_create_subscription(self, ns: str, topic: str, sub: str, lock_ms: int = 60000,
                                     max_delivery: int = 10, ttl_ms: int = 0) -> None:
        body = json.dumps({"lockMs": lock_ms, "maxDelivery": max_delivery, "ttlMs": ttl_ms}).encode()
        await self._req("PUT", f"/servicebus/{q(ns)}/topics/{q(topic)}/subscriptions/{q(sub)}", body,
                        {"Content-Type": "application/json"})

    async def sb_create_queue(self, ns: str, queue: str, lock_ms: int = 60000, max_delivery: int = 10) -> None:
        body = json.dumps({"lockMs": lock_ms, "maxDelivery": max_delivery}).encode()
        await self._req("PUT", f"/servicebus/{q(ns)}/queues/{q(queue)}", body, {"Content-Type": "application/json"})

    async def sb_publish(self, ns: str, topic: str, body: bytes, content_type: str = "application/json",
                         props: dict[str, Any] | None = None, message_id: str = "", ttl_ms: int = 0) -> int:
        h = {"Content-Type": content_type}
        if props:
            h["x-tt-props"] = json.dumps(props)
        if message_id:
            h["x-tt-message-id"] = message_id
        if ttl_ms:
            h["x-tt-ttl-ms"] = str(ttl_ms)
        r = await self._req("POST", f"/servicebus/{q(ns)}/topics/{q(topic)}/messages", body, h, what="publish")
        return r.json()["seq"]

    async def sb_publish_batch(self, ns: str, topic: str, entries: list[dict[str, Any]]) -> list[int]:
        r = await self._req("POST", f"/servicebus/{q(ns)}/topics/{q(topic)}/batch", json.dumps(entries).encode(),
                            {"Content-Type": "application/json"}, what="publish batch")
        return r.json()["seqs"]

    async def sb_send(self, ns: str, queue: str, body: bytes, content_type: str = "application/json") -> int:
        r = await self._req("POST", f"/servicebus/{q(ns)}/queues/{q(queue)}/messages", body,
                            {"Content-Type": content_type}, what="send")
        return r.json()["seq"]

    async def sb_receive(self, ns: str, entity: str, max_messages: int = 1, lock_ms: int = 0,
                         wait_ms: int = 0) -> list[dict[str, Any]]:
        path = f"/servicebus/{q(ns)}/receive?" + urlencode({"entity": entity, "max": max_messages, "lockMs": lock_ms,
                                                           "waitMs": wait_ms})
        r = await self._req("POST", path, b"", what="receive", timeout=wait_ms / 1000.0 + 30)
        return r.json()

    async def sb_settle(self, ns: str, entity: str, complete: list[str] = (), abandon: list[dict[str, Any]] = (),
                        deadletter: list[dict[str, Any]] = (), renew: list[dict[str, Any]] = ()) -> dict[str, list[bool]]:
        body = {"entity": entity, "complete": list(complete), "abandon": list(abandon),
                "deadletter": list(deadletter), "renew": list(renew)}
        r = await self._req("POST", f"/servicebus/{q(ns)}/settle", json.dumps(body).encode(),
                            {"Content-Type": "application/json"}, what="settle")
        return r.json()

    async def sb_counts(self, ns: str, entity: str) -> dict[str, int]:
        return (await self._req("GET", f"/servicebus/{q(ns)}/counts?" + urlencode({"entity": entity}))).json()

    async def sb_dead_letters(self, ns: str, entity: str, max_messages: int = 100) -> list[dict[str, Any]]:
        path = f"/servicebus/{q(ns)}/deadletters?" + urlencode({"entity": entity, "max": max_messages})
        return (await self._req("POST", path, b"")).json()

    # -- storage queue / blob -------------------------------------------------
    async def queue_put(self, account: str, queue: str, body: bytes, ttl_s: int = 0) -> str:
        path = f"/storage/{q(account)}/queues/{q(queue)}/messages"
        if ttl_s:
            path += f"?messagettl={ttl_s}"
        r = await self._req("POST", path, body, {"Content-Type": "text/plain"}, what="queue put")
        return r.json()["messageId"]

    async def queue_get(self, account: str, queue: str, max_messages: int = 1, visibility_ms: int = 30000,
                        wait_ms: int = 0) -> list[dict[str, Any]]:
        path = f"/storage/{q(account)}/queues/{q(queue)}/messages?" + urlencode(
            {"numofmessages": max_messages, "visibilityMs": visibility_ms, "waitMs": wait_ms})
        return (await self._req("GET", path, timeout=wait_ms / 1000.0 + 30, what="queue get")).json()

    async def queue_delete(self, account: str, queue: str, receipt: str) -> bool:
        r = await self._req("DELETE", f"/storage/{q(account)}/queues/{q(queue)}/messages/{q(receipt)}", ok=(204, 404))
        return r.status == 204

    async def queue_release(self, account: str, queue: str, receipt: str, visibility_ms: int) -> bool:
        r = await self._req("PUT", f"/storage/{q(account)}/queues/{q(queue)}/messages/{q(receipt)}?visibilityMs={visibility_ms}",
                            b"", ok=(204, 404))
        return r.status == 204

    async def queue_count(self, account: str, queue: str) -> dict[str, int]:
        return (await self._req("GET", f"/storage/{q(account)}/queues/{q(queue)}/count")).json()

    async def blob_put(self, account: str, container: str, name: str, data: bytes,
                       content_type: str = "application/octet-stream") -> dict[str, Any]:
        r = await self._req("PUT", f"/storage/{q(account)}/blobs/{q(container)}/{quote(name)}", data,
                            {"Content-Type": content_type}, what="blob put")
        return r.json()

    async def blob_get(self, account: str, container: str, name: str) -> bytes | None:
        r = await self._req("GET", f"/storage/{q(account)}/blobs/{q(container)}/{quote(name)}", ok=(200, 404))
        return None if r.status == 404 else r.body

    async def blob_delete(self, account: str, container: str, name: str) -> bool:
        r = await self._req("DELETE", f"/storage/{q(account)}/blobs/{q(container)}/{quote(name)}", ok=(204, 404))
        return r.status == 204

    async def blob_list(self, account: str, container: str, prefix: str = "") -> list[dict[str, Any]]:
        path = f"/storage/{q(account)}/blobs/{q(container)}"
        if prefix:
            path += "?" + urlencode({"prefix": prefix})
        return (await self._req("GET", path)).json()

    async def blob_count(self, account: str, container: str, prefix: str = "") -> int:
        """How many blobs the container holds (no listing)."""
        args = {"count": "true"} | ({"prefix": prefix} if prefix else {})
        return int((await self._req("GET", f"/storage/{q(account)}/blobs/{q(container)}?" + urlencode(args))).json()["count"])

    # -- key vault ------------------------------------------------------------
    async def kv_get(self, vault: str, name: str) -> str | None:
        r = await self._req("GET", f"/keyvault/{q(vault)}/secrets/{q(name)}", ok=(200, 404))
        return None if r.status == 404 else r.json()["value"]

    async def kv_set(self, vault: str, name: str, value: str) -> None:
        await self._req("PUT", f"/keyvault/{q(vault)}/secrets/{q(name)}", json.dumps({"value": value}).encode(),
                        {"Content-Type": "application/json"})

    async def kv_list(self, vault: str) -> list[str]:
        return (await self._req("GET", f"/keyvault/{q(vault)}/secrets")).json()

    # -- sendgrid -------------------------------------------------------------
    async def sendgrid_send(self, message: dict[str, Any], api_key: str | None = None) -> None:
        h = {"Content-Type": "application/json"}
        if api_key:
            h["Authorization"] = f"Bearer {api_key}"
        await self._req("POST", "/sendgrid/v3/mail/send", json.dumps(message).encode(), h, what="sendgrid send")

    async def sendgrid_outbox(self) -> list[dict[str, Any]]:
        return (await self._req("GET", "/sendgrid/outbox")).json()

    # -- admin ----------------------------------------------------------------
    async def overview(self) -> dict[str, Any]:
        return (await self._req("GET", "/admin/overview")).json()

    async def set_policy(self, policy: dict[str, Any]) -> None:
        await self._req("PUT", "/admin/policy", json.dumps(policy).encode(), {"Content-Type": "application/json"})

    async def healthy(self) -> bool:
        try:
            r = await self.http.request("GET", self.base + "/admin/health", timeout=2.0)
            return r.status == 204
        except OSError:
            return False

    async def close(self) -> None:
        await self.http.close()
