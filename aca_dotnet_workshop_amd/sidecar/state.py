"""State store components (the state management building block).

Types:
* ``state.azure.cosmosdb`` -- ``url``/``database``/``collection`` (+ ``masterKey`` or the
  app's managed identity), reference components/dapr-statestore-cosmos.yaml:8-16;
* ``state.redis``          -- ``redisHost``/``redisPassword``;
* ``state.in-memory``      -- in-process native engine (no sharing across processes).

All three support ETags, first-write/last-write concurrency, TTL (``ttlInSeconds``),
transactions and the query API.  Keys are prefixed per Dapr convention
(reference docs/aca/04-aca-dapr-stateapi/index.md:413-425): ``<app-id>||<key>`` by
default, overridable with the ``keyPrefix`` metadata (``appid`` | ``name`` | ``none`` |
any constant).
"""
from __future__ import annotations

import asyncio
import json
from dataclasses import dataclass
from typing import Any

from .. import native
from ..backing.client import EtagConflict
from .base import ComponentBase, cosmos_account, redis_namespace, register
from .components import ComponentError


class EtagMismatch(Exception):
    pass


@dataclass
class SetRequest:
    key: str
    value: str  # JSON text
    etag: str | None = None
    first_write: bool = False
    ttl_ms: int = 0


class StateStore(ComponentBase):
    supports_query = True

    async def init(self) -> None:
        kp = (self.comp.get("keyPrefix") or "appid").strip()
        low = kp.lower()
        if low == "appid":
            self.prefix = f"{self.ctx.app_id}||"
        elif low == "name":
            self.prefix = f"{self.name}||"
        elif low == "none":
            self.prefix = ""
        else:
            self.prefix = f"{kp}||"
        await self._init()

    async def _init(self) -> None:
        pass

    def full(self, key: str) -> str:
        if "||" in key and self.prefix == "":
            return key
        return self.prefix + key

    async def get(self, key: str) -> tuple[bytes, str] | None:
        raise NotImplementedError

    async def set_many(self, reqs: list[SetRequest]) -> None:
        raise NotImplementedError

    async def delete(self, key: str, etag: str | None) -> bool:
        raise NotImplementedError

    async def bulk_get(self, keys: list[str]) -> list[dict[str, Any]]:
        out = []
        for k in keys:
            r = await self.get(k)
            out.append({"key": k, "data": json.loads(r[0]), "etag": r[1]} if r else {"key": k})
        return out

    async def transact(self, ops: list[dict[str, Any]]) -> None:
        raise NotImplementedError

    async def query(self, query: bytes) -> bytes:
        raise NotImplementedError


def _tx_ops(store: StateStore, ops: list[dict[str, Any]]) -> list[dict[str, Any]]:
    out = []
    for o in ops:
        op = (o.get("operation") or "").lower()
        req = o.get("request") or {}
        if "key" not in req:
            raise ValueError("transaction operation without key")
        meta = req.get("metadata") or {}
        opts = req.get("options") or {}
        etag = req.get("etag")
        if isinstance(etag, dict):
            etag = etag.get("value")
        entry: dict[str, Any] = {"key": store.full(req["key"]), "etag": etag or None,
                                 "firstWrite": (opts.get("concurrency") == "first-write"),
                                 "ttlMs": int(float(meta.get("ttlInSeconds", 0) or 0) * 1000)}
        if op == "upsert":
            entry["op"] = "upsert"
            entry["value"] = json.dumps(req.get("value"))
        elif op == "delete":
            entry["op"] = "delete"
        else:
            raise ValueError(f"unsupported transaction operation {op!r}")
        out.append(entry)
    return out


@register("state.azure.cosmosdb", "state.redis")
class BackingStateStore(StateStore):
    async def _init(self) -> None:
        if self.comp.type == "state.azure.cosmosdb":
            url = self.comp.get("url")
            if not url:
                raise ComponentError(f"{self.name}: url is required")
            self.account = cosmos_account(url)
            self.db = self.comp.get("database") or "db"
            self.coll = self.comp.get("collection") or "coll"
            key = self.comp.get("masterKey")
        else:
            self.account = redis_namespace(self.comp)
            self.db, self.coll = "0", "kv"
            key = self.comp.get("redisPassword")
        self.client = self.ctx.backing(self.comp, key=key or None)

    async def get(self, key):
        return await self.client.doc_get(self.account, self.db, self.coll, self.full(key))

    async def set_many(self, reqs):
        if len(reqs) == 1:
            r = reqs[0]
            try:
                await self.client.doc_put(self.account, self.db, self.coll, self.full(r.key), r.value, r.etag,
                                          r.first_write, r.ttl_ms)
            except EtagConflict as e:
                raise EtagMismatch(str(e)) from None
            return
        items = [{"key": self.full(r.key), "value": r.value, "etag": r.etag, "firstWrite": r.first_write,
                  "ttlMs": r.ttl_ms} for r in reqs]
        try:
            await self.client.doc_bulk_set(self.account, self.db, self.coll, items)
        except EtagConflict as e:
            raise EtagMismatch(str(e)) from None

    async def delete(self, key, etag):
        try:
            return await self.client.doc_delete(self.account, self.db, self.coll, self.full(key), etag)
        except EtagConflict as e:
            raise EtagMismatch(str(e)) from None

    async def bulk_get(self, keys):
        res = await self.client.doc_bulk_get(self.account, self.db, self.coll, [self.full(k) for k in keys])
        for r, k in zip(res, keys):
            r["key"] = k
        return res

    async def transact(self, ops):
        try:
            await self.client.doc_transaction(self.account, self.db, self.coll, _tx_ops(self, ops))
        except EtagConflict as e:
            raise EtagMismatch(str(e)) from None

    async def query(self, query):
        return await self.client.doc_query(self.account, self.db, self.coll, query, self.prefix)


@register("state.in-memory")
class InMemoryStateStore(StateStore):
    async def _init(self) -> None:
        self.N = native.load()
        self.store = self.N.DocStore()

    async def get(self, key):
        r = self.store.get(self.full(key))
        return None if r is None else (r[0].encode(), r[1])

    async def set_many(self, reqs):
        try:
            if len(reqs) == 1:
                r = reqs[0]
                self.store.set(self.full(r.key), r.value, r.etag, r.first_write, r.ttl_ms)
            else:
                self.store.transact([self.N.TxOp(False, self.full(r.key), r.value, r.etag, r.first_write, r.ttl_ms)
                                     for r in reqs])
        except self.N.EtagMismatch as e:
            raise EtagMismatch(str(e)) from None

    async def delete(self, key, etag):
        try:
            return self.store.delete(self.full(key), etag)
        except self.N.EtagMismatch as e:
            raise EtagMismatch(str(e)) from None

    async def transact(self, ops):
        tx = []
        for e in _tx_ops(self, ops):
            tx.append(self.N.TxOp(e["op"] == "delete", e["key"], e.get("value", ""), e["etag"], e["firstWrite"],
                                  e["ttlMs"]))
        try:
            self.store.transact(tx)
        except self.N.EtagMismatch as e:
            raise EtagMismatch(str(e)) from None

    async def query(self, query):
        return (await asyncio.to_thread(self.store.query, query.decode(), self.prefix)).encode()
