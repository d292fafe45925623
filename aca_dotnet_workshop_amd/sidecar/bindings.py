"""Binding components (input/output bindings building block).

===============================  =====  ============================================================
type                             dir    reference
===============================  =====  ============================================================
bindings.azure.storagequeues     in/out components/dapr-bindings-in-storagequeue.yaml (queue
                                        ``external-tasks-queue``, ``decodeBase64``, ``route``)
bindings.azure.blobstorage       out    components/dapr-bindings-out-blobstorage.yaml (``create``
                                        with ``blobName`` metadata, ExternalTasksProcessorController.cs:38-43)
bindings.twilio.sendgrid         out    components/dapr-bindings-out-sendgrid.yaml; caller
                                        docs/aca/06-aca-dapr-bindingsapi/TasksNotifierController.cs:50-56
bindings.cron                    in     components/dapr-scheduled-cron.yaml (``5 0 * * *``)
bindings.localstorage            out    self-hosted file binding (no cloud needed)
bindings.http                    out    generic outbound HTTP
===============================  =====  ============================================================

Input bindings call ``deliver(data, metadata) -> bool``; ``True`` acknowledges (queue
message deleted), ``False`` leaves the message to reappear after the visibility timeout
(reference docs/aca/06-aca-dapr-bindingsapi/index.md:54-58).

The cron binding optionally elects a single firing replica per tick
(``singleReplica: "true"``): replicas race to create a lease document with first-write
concurrency in the state backend, resolving the cron-vs-scale-out conflict the reference
leaves open.
"""
from __future__ import annotations

import asyncio
import base64
import json
import logging
import os
import uuid
from datetime import datetime, timezone
from pathlib import Path
from typing import Any, Awaitable, Callable

from ..backing.client import EtagConflict
from ..utils.cron import CronSchedule, parse_duration
from .base import ComponentBase, register
from .components import ComponentError

log = logging.getLogger("sidecar.bindings")

Deliver = Callable[[bytes, dict[str, str]], Awaitable[bool]]


class BindingError(Exception):
    def __init__(self, status: int, msg: str) -> None:
        super().__init__(msg)
        self.status = status


class Binding(ComponentBase):
    is_input = False
    is_output = False
    operations: tuple[str, ...] = ()

    def route(self) -> str:
        return self.comp.get("route") or f"/{self.name}"

    async def start(self, deliver: Deliver) -> None:
        raise BindingError(400, f"binding {self.name} is not an input binding")

    async def invoke(self, operation: str, data: bytes, metadata: dict[str, str]) -> tuple[bytes | None, dict[str, str]]:
        raise BindingError(400, f"binding {self.name} is not an output binding")

    async def close(self) -> None:
        t = getattr(self, "_task", None)
        if t is not None:
            t.cancel()
            try:
                await t
            except (asyncio.CancelledError, Exception):
                pass


def _dur_ms(v: str | None, default_ms: int) -> int:
    if not v:
        return default_ms
    try:
        return int(parse_duration(v).total_seconds() * 1000)
    except ValueError:
        return int(float(v) * 1000)


@register("bindings.azure.storagequeues")
class StorageQueueBinding(Binding):
    is_input = True
    is_output = True
    operations = ("create",)

    async def init(self) -> None:
        self.account = self.comp.get("storageAccount") or self.comp.get("accountName")
        self.queue = self.comp.get("queue") or self.comp.get("queueName")
        if not self.account or not self.queue:
            raise ComponentError(f"{self.name}: storageAccount and queue are required")
        self.client = self.ctx.backing(self.comp, key=self.comp.get("storageAccessKey") or None)
        self.decode = self.comp.get_bool("decodeBase64")
        self.encode = self.comp.get_bool("encodeBase64")
        self.visibility_ms = _dur_ms(self.comp.get("visibilityTimeout"), 30000)
        self.poll_ms = _dur_ms(self.comp.get("pollingInterval"), 10000)
        self.ttl_s = self.comp.get_int("ttlInSeconds", 0)
        self.concurrency = self.comp.get_int("concurrency", 16)

    async def start(self, deliver: Deliver) -> None:
        self._task = asyncio.ensure_future(self._poll(deliver))

    async def _poll(self, deliver: Deliver) -> None:
        """Continuous delivery: a receive asks for as many messages as there are free delivery
        slots (``concurrency``, at most 32 a call) and every message is delivered on its own task
        -- a slot frees the moment its delivery ends and the next receive refills it.  A slow or
        failing delivery holds only its own slot: the rest of the queue keeps flowing (no wait
        for a whole batch).  A failed delivery is not deleted: the message reappears once its
        visibility timeout elapses (docs/aca/06-aca-dapr-bindingsapi/index.md:54-58)."""
        free = asyncio.Semaphore(self.concurrency)
        inflight: set[asyncio.Task] = set()
        backoff = 0.1

        def done(t: asyncio.Task) -> None:
            inflight.discard(t)
            free.release()
        try:
            while True:
                await free.acquire()  # one free slot at least, then every other one free right now
                n = 1
                while n < 32 and not free.locked():
                    await free.acquire()
                    n += 1
                try:
                    msgs = await self.client.queue_get(self.account, self.queue, n, self.visibility_ms,
                                                       wait_ms=min(self.poll_ms, 5000))
                    backoff = 0.1
                except asyncio.CancelledError:
                    raise
                except Exception as e:
                    for _ in range(n):
                        free.release()
                    log.warning("%s: queue poll failed: %r", self.name, e)
                    await asyncio.sleep(backoff)
                    backoff = min(backoff * 2, 5.0)
                    continue
                for _ in range(n - len(msgs)):
                    free.release()
                for m in msgs[:n]:
                    t = asyncio.ensure_future(self._deliver_one(m, deliver))
                    inflight.add(t)
                    t.add_done_callback(done)
        finally:
            for t in list(inflight):
                t.cancel()

    async def _deliver_one(self, m: dict[str, Any], deliver: Deliver) -> None:
        raw = m.get("body", "").encode() if "body" in m else base64.b64decode(m.get("bodyB64", ""))
        if self.decode:
            try:
                raw = base64.b64decode(raw, validate=True)
            except ValueError:
                log.warning("%s: message %s is not valid base64; leaving it in the queue", self.name, m.get("messageId"))
                return
        ok = False
        try:
            ok = await deliver(raw, {"MessageId": str(m.get("messageId")), "DequeueCount": str(m.get("dequeueCount")),
                                     "InsertionTime": str(m.get("insertionMs"))})
        except Exception as e:
            log.warning("%s: delivery failed: %r", self.name, e)
        if ok:
            try:
                await self.client.queue_delete(self.account, self.queue, m["popReceipt"])
            except Exception as e:  # it reappears after its visibility timeout and is delivered again
                log.warning("%s: delete of %s failed: %r", self.name, m.get("messageId"), e)
        # on failure the message reappears once its visibility timeout elapses

    async def invoke(self, operation, data, metadata):
        if operation != "create":
            raise BindingError(400, f"unsupported operation {operation}")
        body = base64.b64encode(data) if self.encode else data
        ttl = int(metadata.get("ttlInSeconds", self.ttl_s) or 0)
        mid = await self.client.queue_put(self.account, self.queue, body, ttl)
        return None, {"messageId": mid}


@register("bindings.azure.blobstorage")
class BlobBinding(Binding):
    is_output = True
    operations = ("create", "get", "delete", "list")

    async def init(self) -> None:
        self.account = self.comp.get("storageAccount") or self.comp.get("accountName")
        self.container = self.comp.get("container") or self.comp.get("containerName")
        if not self.account or not self.container:
            raise ComponentError(f"{self.name}: storageAccount and container are required")
        self.client = self.ctx.backing(self.comp, key=self.comp.get("storageAccessKey") or None)
        self.decode = self.comp.get_bool("decodeBase64")

    async def invoke(self, operation, data, metadata):
        if operation == "create":
            name = metadata.get("blobName") or str(uuid.uuid4())
            payload = base64.b64decode(data) if self.decode else data
            ctype = metadata.get("contentType") or "application/json"
            res = await self.client.blob_put(self.account, self.container, name, payload, ctype)
            return json.dumps({"blobURL": res["blobURL"]}).encode(), {"blobName": name}
        if operation == "get":
            name = metadata.get("blobName")
            if not name:
                raise BindingError(400, "blobName metadata is required")
            body = await self.client.blob_get(self.account, self.container, name)
            if body is None:
                raise BindingError(404, f"blob {name} not found")
            if metadata.get("encodeBase64", "").lower() == "true":
                body = base64.b64encode(body)
            return body, {}
        if operation == "delete":
            name = metadata.get("blobName")
            if not name:
                raise BindingError(400, "blobName metadata is required")
            if not await self.client.blob_delete(self.account, self.container, name):
                raise BindingError(404, f"blob {name} not found")
            return None, {}
        if operation == "list":
            prefix = ""
            if data:
                try:
                    prefix = (json.loads(data) or {}).get("prefix", "")
                except ValueError:
                    prefix = ""
            items = await self.client.blob_list(self.account, self.container, prefix)
            return json.dumps(items).encode(), {"metadata": json.dumps({"numberOfItems": len(items)})}
        raise BindingError(400, f"unsupported operation {operation}")


@register("bindings.twilio.sendgrid")
class SendGridBinding(Binding):
    is_output = True
    operations = ("create",)

    async def init(self) -> None:
        self.client = self.ctx.backing(self.comp)

    async def invoke(self, operation, data, metadata):
        if operation != "create":
            raise BindingError(400, f"unsupported operation {operation}")
        to = metadata.get("emailTo") or self.comp.get("emailTo")
        frm = metadata.get("emailFrom") or self.comp.get("emailFrom")
        if not to or not frm:
            raise BindingError(400, "emailTo and emailFrom are required")
        pers: dict[str, Any] = {"to": [{"email": to, "name": metadata.get("emailToName") or self.comp.get("emailToName") or to}],
                                "subject": metadata.get("subject") or self.comp.get("subject") or ""}
        for k, f in (("emailCc", "cc"), ("emailBcc", "bcc")):
            v = metadata.get(k) or self.comp.get(k)
            if v:
                pers[f] = [{"email": x.strip()} for x in v.split(",") if x.strip()]
        msg = {"personalizations": [pers],
               "from": {"email": frm, "name": metadata.get("emailFromName") or self.comp.get("emailFromName") or frm},
               "content": [{"type": "text/plain", "value": data.decode("utf-8", "replace")}]}
        await self.client.sendgrid_send(msg, self.comp.get("apiKey"))
        return None, {}


@register("bindings.cron")
class CronBinding(Binding):
    is_input = True
    is_output = True
    operations = ("delete",)

    async def init(self) -> None:
        sched = self.comp.get("schedule")
        if not sched:
            raise ComponentError(f"{self.name}: schedule is required")
        self.schedule = CronSchedule.parse(sched)
        self.single = self.comp.get_bool("singleReplica")
        self.fired = 0

    async def start(self, deliver: Deliver) -> None:
        self._task = asyncio.ensure_future(self._loop(deliver))

    async def _claim(self, tick: datetime) -> bool:
        if not self.single:
            return True
        client = self.ctx.backing(self.comp)
        key = f"{self.ctx.app_id}||{self.name}||{tick.isoformat()}"
        try:
            await client.doc_put("tt-leases", "cron", "leases", key, json.dumps({"owner": self.ctx.identity or os.getpid()}),
                                 first_write=True, ttl_ms=24 * 3600 * 1000)
            return True
        except EtagConflict:
            return False

    async def _loop(self, deliver: Deliver) -> None:
        now = datetime.now(timezone.utc)
        while True:
            nxt = self.schedule.next_after(now)
            delay = (nxt - datetime.now(timezone.utc)).total_seconds()
            if delay > 0:
                await asyncio.sleep(delay)
            now = nxt
            try:
                if await self._claim(nxt):
                    self.fired += 1
                    await deliver(b"", {"timeZone": "UTC", "fireTime": nxt.isoformat()})
            except asyncio.CancelledError:
                raise
            except Exception as e:
                log.warning("%s: cron delivery failed: %r", self.name, e)

    async def invoke(self, operation, data, metadata):
        if operation == "delete":
            await self.close()
            return None, {}
        raise BindingError(400, f"unsupported operation {operation}")


@register("bindings.localstorage")
class LocalStorageBinding(Binding):
    is_output = True
    operations = ("create", "get", "delete", "list")

    async def init(self) -> None:
        root = self.comp.get("rootPath")
        if not root:
            raise ComponentError(f"{self.name}: rootPath is required")
        self.root = Path(root).resolve()
        self.root.mkdir(parents=True, exist_ok=True)

    def _file(self, name: str) -> Path:
        f = (self.root / name).resolve()
        if self.root not in f.parents:
            raise BindingError(400, "invalid fileName")
        return f

    async def invoke(self, operation, data, metadata):
        if operation == "create":
            name = metadata.get("fileName") or str(uuid.uuid4())
            f = self._file(name)
            f.parent.mkdir(parents=True, exist_ok=True)
            f.write_bytes(data)
            return json.dumps({"fileName": str(f)}).encode(), {"fileName": name}
        if operation == "get":
            f = self._file(metadata.get("fileName", ""))
            if not f.is_file():
                raise BindingError(404, "file not found")
            return f.read_bytes(), {}
        if operation == "delete":
            f = self._file(metadata.get("fileName", ""))
            if not f.is_file():
                raise BindingError(404, "file not found")
            f.unlink()
            return None, {}
        if operation == "list":
            return json.dumps(sorted(str(p.relative_to(self.root)) for p in self.root.rglob("*") if p.is_file())).encode(), {}
        raise BindingError(400, f"unsupported operation {operation}")


@register("bindings.http")
class HttpBinding(Binding):
    is_output = True
    operations = ("get", "head", "post", "put", "patch", "delete", "options", "trace", "create")

    async def init(self) -> None:
        self.url = (self.comp.get("url") or "").rstrip("/")
        if not self.url:
            raise ComponentError(f"{self.name}: url is required")

    async def invoke(self, operation, data, metadata):
        method = "POST" if operation == "create" else operation.upper()
        path = metadata.get("path", "")
        headers = {k: v for k, v in metadata.items() if k not in ("path",)}
        r = await self.ctx.http.request(method, self.url + ("/" + path.lstrip("/") if path else ""), headers=headers,
                                        body=data or None)
        if r.status >= 400:
            raise BindingError(502, f"received status code {r.status}")
        return r.body, {"statusCode": str(r.status)}
