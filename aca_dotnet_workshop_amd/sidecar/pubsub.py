"""Pub/sub components and the competing-consumer delivery engine.

Types:
* ``pubsub.azure.servicebus`` / ``pubsub.azure.servicebus.topics`` -- topic + subscription
  named by ``consumerID`` (default: app-id) in the backing emulator (reference
  components/dapr-pubsub-svcbus.yaml, aca-components/containerapps-pubsub-svcbus.yaml);
* ``pubsub.redis``     -- Redis-Streams-style consumer groups (reference
  components/dapr-pubsub-redis.yaml);
* ``pubsub.in-memory`` -- in-process broker for single-process use and tests.

Delivery engine (``Consumer``): prefetches up to ``maxActiveMessages`` under peek-lock,
runs at most ``maxConcurrentHandlers`` app callbacks at once, renews locks of long
running handlers, and settles outcomes in batches -- ``success`` -> complete,
``retry`` -> abandon (redelivery; MaxDeliveryCount -> DLQ), ``drop`` -> dead-letter (or
forward to the subscription's ``deadLetterTopic``).  Several replicas of one app share a
subscription, which is exactly the KEDA competing-consumer scale-out of the reference
(SURVEY.md §2.10).
"""
from __future__ import annotations

import asyncio
import json
import logging
from typing import Any, Awaitable, Callable

from .. import native
from .base import ComponentBase, redis_namespace, register, servicebus_namespace

log = logging.getLogger("sidecar.pubsub")

SUCCESS, RETRY, DROP = "success", "retry", "drop"


class Transport:
    async def publish(self, topic: str, body: bytes, ctype: str, props: dict[str, Any], ttl_ms: int = 0) -> None: ...
    async def ensure_subscription(self, topic: str, sub: str, lock_ms: int, max_delivery: int) -> None: ...
    async def receive(self, entity: str, n: int, lock_ms: int, wait_ms: int) -> list[dict[str, Any]]: ...
    async def settle(self, entity: str, complete=(), abandon=(), deadletter=(), renew=()) -> None: ...
    async def counts(self, entity: str) -> dict[str, int]: ...


class BackingTransport(Transport):
    def __init__(self, client, ns: str) -> None:
        self.client = client
        self.ns = ns

    async def publish(self, topic, body, ctype, props, ttl_ms=0):
        await self.client.sb_publish(self.ns, topic, body, ctype, props, ttl_ms=ttl_ms)

    async def publish_batch(self, topic, entries):
        await self.client.sb_publish_batch(self.ns, topic, entries)

    async def ensure_subscription(self, topic, sub, lock_ms, max_delivery):
        await self.client.sb_create_subscription(self.ns, topic, sub, lock_ms, max_delivery)

    async def receive(self, entity, n, lock_ms, wait_ms):
        return await self.client.sb_receive(self.ns, entity, n, lock_ms, wait_ms)

    async def settle(self, entity, complete=(), abandon=(), deadletter=(), renew=()):
        await self.client.sb_settle(self.ns, entity, complete, abandon, deadletter, renew)

    async def counts(self, entity):
        return await self.client.sb_counts(self.ns, entity)

    def per_shard(self) -> list["BackingTransport"]:
        """A partitioned namespace (backing/shards.py): one transport per shard, so a consumer
        long-polls its own shard and settles there -- no receive call scans every shard."""
        shards = getattr(self.client, "shards", None)
        if not shards or len(shards) < 2:
            return [self]
        return [BackingTransport(c, self.ns) for c in shards]


class InMemoryTransport(Transport):
    def __init__(self) -> None:
        self.N = native.load()
        self.broker = self.N.Broker()
        self._ev: dict[str, asyncio.Event] = {}

    def _notify(self, entity: str) -> None:
        ev = self._ev.pop(entity, None)
        if ev:
            ev.set()

    async def publish(self, topic, body, ctype, props, ttl_ms=0):
        self.broker.publish(topic, body, ctype, json.dumps(props), "", ttl_ms, 0)
        for s in self.broker.subscriptions(topic):
            self._notify(f"{topic}/subscriptions/{s}")

    async def ensure_subscription(self, topic, sub, lock_ms, max_delivery):
        self.broker.create_subscription(topic, sub, self.N.QueueOptions(lock_ms, max_delivery, 0, False))

    async def receive(self, entity, n, lock_ms, wait_ms):
        loop = asyncio.get_running_loop()
        deadline = loop.time() + wait_ms / 1000.0
        while True:
            msgs = self.broker.receive(entity, n, lock_ms)
            rem = deadline - loop.time()
            if msgs or rem <= 0:
                break
            ev = self._ev.setdefault(entity, asyncio.Event())
            try:
                await asyncio.wait_for(ev.wait(), min(rem, 0.2))
            except asyncio.TimeoutError:
                pass
        return [{"lockToken": m.lock_token, "seq": m.seq, "id": m.id, "body": m.body, "contentType": m.content_type,
                 "props": json.loads(m.props or "{}"), "deliveryCount": m.delivery_count} for m in msgs]

    async def settle(self, entity, complete=(), abandon=(), deadletter=(), renew=()):
        for t in complete:
            self.broker.complete(entity, t)
        for a in abandon:
            self.broker.abandon(entity, a["token"], int(a.get("delayMs", 0)))
        for d in deadletter:
            self.broker.dead_letter(entity, d["token"], d.get("reason", ""))
        for r in renew:
            self.broker.renew(entity, r["token"], int(r.get("lockMs", 0)))
        if abandon:
            self._notify(entity)

    async def counts(self, entity):
        return dict(self.broker.counts(entity))


def message_body(m: dict[str, Any]) -> bytes:
    b = m.get("body")
    if isinstance(b, bytes):
        return b
    if b is not None:
        return b.encode()
    import base64
    return base64.b64decode(m.get("bodyB64", ""))


Handler = Callable[[dict[str, Any]], Awaitable[str]]


class Consumer:
    """Competing consumer on one subscription entity."""

    def __init__(self, transport: Transport, entity: str, handler: Handler, *, max_concurrent: int = 32,
                 prefetch: int = 64, lock_ms: int = 60000, retry_delay_ms: int = 0,
                 on_drop: Callable[[dict[str, Any]], Awaitable[bool]] | None = None, name: str = "") -> None:
        self.t = transport
        self.entity = entity
        self.handler = handler
        self.sem = asyncio.Semaphore(max(1, max_concurrent))
        self.prefetch = max(1, prefetch)
        self.lock_ms = lock_ms
        self.retry_delay_ms = retry_delay_ms
        self.on_drop = on_drop
        self.name = name or entity
        self.inflight: dict[str, dict[str, Any]] = {}
        self._space = asyncio.Event()
        self._space.set()
        self._stopping = False
        self._task: asyncio.Task | None = None
        self._renew_task: asyncio.Task | None = None
        self._pending: dict[str, list[Any]] = {"complete": [], "abandon": [], "deadletter": []}
        self._flush_scheduled = False
        self._handlers: set[asyncio.Task] = set()
        self.stats = {"delivered": 0, "succeeded": 0, "retried": 0, "dropped": 0, "errors": 0}

    def start(self) -> None:
        self._task = asyncio.ensure_future(self._run())
        self._renew_task = asyncio.ensure_future(self._renew_loop())

    async def _run(self) -> None:
        backoff = 0.1
        while not self._stopping:
            room = self.prefetch - len(self.inflight)
            if room <= 0:
                self._space.clear()
                await self._space.wait()
                continue
            try:
                msgs = await self.t.receive(self.entity, min(room, 256), self.lock_ms, 2000)
                backoff = 0.1
            except asyncio.CancelledError:
                raise
            except Exception as e:
                if self._stopping:
                    break
                log.warning("%s: receive failed (%s); retrying in %.1fs", self.name, e, backoff)
                await asyncio.sleep(backoff)
                backoff = min(backoff * 2, 5.0)
                continue
            for m in msgs:
                if self._stopping:
                    self._queue("abandon", {"token": m["lockToken"]})
                    continue
                self.inflight[m["lockToken"]] = m
                t = asyncio.ensure_future(self._handle(m))
                self._handlers.add(t)
                t.add_done_callback(self._handlers.discard)

    async def _handle(self, m: dict[str, Any]) -> None:
        tok = m["lockToken"]
        try:
            async with self.sem:
                self.stats["delivered"] += 1
                try:
                    outcome = await self.handler(m)
                except Exception as e:
                    log.warning("%s: handler raised %r; message will be retried", self.name, e)
                    self.stats["errors"] += 1
                    outcome = RETRY
            if outcome == SUCCESS:
                self.stats["succeeded"] += 1
                self._queue("complete", tok)
            elif outcome == DROP:
                self.stats["dropped"] += 1
                forwarded = False
                if self.on_drop is not None:
                    try:
                        forwarded = await self.on_drop(m)
                    except Exception as e:
                        log.warning("%s: dead-letter forward failed: %r", self.name, e)
                if forwarded:
                    self._queue("complete", tok)
                else:
                    self._queue("deadletter", {"token": tok, "reason": "dropped by application"})
            else:
                self.stats["retried"] += 1
                self._queue("abandon", {"token": tok, "delayMs": self.retry_delay_ms})
        finally:
            self.inflight.pop(tok, None)
            self._space.set()

    def _queue(self, kind: str, item: Any) -> None:
        self._pending[kind].append(item)
        if not self._flush_scheduled:
            self._flush_scheduled = True
            asyncio.get_running_loop().call_soon(lambda: asyncio.ensure_future(self._flush()))

    async def _flush(self) -> None:
        self._flush_scheduled = False
        p = self._pending
        self._pending = {"complete": [], "abandon": [], "deadletter": []}
        if not any(p.values()):
            return
        try:
            await self.t.settle(self.entity, p["complete"], p["abandon"], p["deadletter"])
        except Exception as e:  # message locks will expire and the broker redelivers (at-least-once)
            log.warning("%s: settle failed: %r", self.name, e)

    async def _renew_loop(self) -> None:
        period = max(self.lock_ms / 3000.0, 0.05)
        while not self._stopping:
            await asyncio.sleep(period)
            toks = list(self.inflight)
            if toks:
                try:
                    await self.t.settle(self.entity, renew=[{"token": t, "lockMs": self.lock_ms} for t in toks])
                except Exception as e:
                    log.debug("%s: renew failed: %r", self.name, e)

    async def stop(self, grace: float = 5.0) -> None:
        self._stopping = True
        self._space.set()
        for t in (self._task, self._renew_task):
            if t is not None:
                t.cancel()
        if self._handlers:
            await asyncio.wait(list(self._handlers), timeout=grace)
        await self._flush()


class PubSub(ComponentBase):
    transport: Transport
    default_concurrency = 32

    def consumer_group(self) -> str:
        return self.comp.get("consumerID") or self.ctx.app_id

    def lock_ms(self) -> int:
        return self.comp.get_int("lockDurationInSec", 60) * 1000

    def max_delivery(self) -> int:
        return self.comp.get_int("maxDeliveryCount", 10)

    async def publish(self, topic: str, body: bytes, ctype: str, metadata: dict[str, str]) -> None:
        ttl = int(float(metadata.get("ttlInSeconds", 0) or 0) * 1000)
        props = {k: v for k, v in metadata.items() if k not in ("ttlInSeconds", "rawPayload")}
        await self.transport.publish(topic, body, ctype, props, ttl)

    async def ensure_entity(self, topic: str) -> str:
        """Create the topic subscription for this consumer group (unless entity management is
        disabled or not permitted) and return its entity path."""
        group = self.consumer_group()
        if not self.comp.get_bool("disableEntityManagement"):
            try:
                await self.transport.ensure_subscription(topic, group, self.lock_ms(), self.max_delivery())
            except Exception as e:
                # receive-only identities cannot manage entities; the subscription is expected
                # to be provisioned by the environment (IaC), exactly like Dapr on Azure.
                if getattr(e, "status", None) != 403:
                    raise
                log.info("%s: no permission to manage %s/subscriptions/%s; using the provisioned entity",
                         self.name, topic, group)
        return f"{topic}/subscriptions/{group}"

    def consumer_settings(self) -> dict[str, int]:
        return {"maxConcurrent": self.comp.get_int("maxConcurrentHandlers", self.default_concurrency) or 1 << 20,
                "prefetch": self.comp.get_int("maxActiveMessages", 64), "lockMs": self.lock_ms(),
                "retryDelayMs": self.comp.get_int("retryDelayMs", 0)}

    async def subscribe(self, topic: str, handler: Handler, sub_metadata: dict[str, str],
                        on_drop=None) -> list[Consumer]:
        """The subscription's competing consumers in this replica: one, or one per shard of a
        partitioned namespace with the replica's prefetch and concurrency split over them (the
        native data plane does the same, sidecar/runtime.py ``_subscribe_native``)."""
        entity = await self.ensure_entity(topic)
        cs = self.consumer_settings()
        per = getattr(self.transport, "per_shard", None)
        transports = per() if per is not None else [self.transport]
        n = len(transports)
        out = []
        for i, t in enumerate(transports):
            c = Consumer(t, entity, handler, max_concurrent=max(1, -(-cs["maxConcurrent"] // n)),
                         prefetch=max(1, -(-cs["prefetch"] // n)), lock_ms=cs["lockMs"],
                         retry_delay_ms=cs["retryDelayMs"], on_drop=on_drop,
                         name=f"{self.name}/{topic}" + (f"#{i}" if n > 1 else ""))
            c.start()
            out.append(c)
        return out


@register("pubsub.azure.servicebus", "pubsub.azure.servicebus.topics")
class ServiceBusPubSub(PubSub):
    async def init(self) -> None:
        self.ns, key = servicebus_namespace(self.comp)
        self.transport = BackingTransport(self.ctx.backing(self.comp, key=key), self.ns)


@register("pubsub.redis")
class RedisPubSub(PubSub):
    default_concurrency = 10

    async def init(self) -> None:
        self.ns = redis_namespace(self.comp)
        self.transport = BackingTransport(self.ctx.backing(self.comp, key=self.comp.get("redisPassword") or None),
                                          self.ns)

    def lock_ms(self) -> int:
        from ..utils.cron import parse_duration
        v = self.comp.get("processingTimeout")
        return int(parse_duration(v).total_seconds() * 1000) if v else 60000

    def max_delivery(self) -> int:
        return self.comp.get_int("maxDeliveryCount", 0) or 1 << 30

    def consumer_settings(self) -> dict[str, int]:
        if not self.comp.get("maxConcurrentHandlers") and self.comp.get("concurrency"):
            self.comp.metadata["maxConcurrentHandlers"] = self.comp.get("concurrency")
        return super().consumer_settings()


@register("pubsub.in-memory")
class InMemoryPubSub(PubSub):
    async def init(self) -> None:
        self.transport = InMemoryTransport()
