"""A partitioned document store and broker: one backing shard per rank, one client over all.

Cosmos DB spreads a container over physical partitions by the hash of its partition key and
Service Bus spreads a partitioned entity over message brokers; the SDKs route each
point operation to its partition and fan cross-partition queries out, merging the pages
(the reference's state store is ``state.azure.cosmosdb`` with the Dapr key as partition key,
components/dapr-statestore-cosmos.yaml:8-16; the overdue query of
TasksStoreManager.cs:128-140 is cross-partition).  ``ShardedBackingClient`` is that routing
layer over several backing processes -- one per rank of a shared environment, each with its
own GPU column mirror:

* documents live on shard ``fnv1a64(full key) % n`` (the native data plane,
  native/src/dataplane.cpp ``Store::shard_of``, uses the same hash);
* a transaction must stay within one partition (Cosmos transactional batches are scoped to
  one partition key; Dapr's Cosmos store rejects mixed ones) -- 400 otherwise;
* queries run on every shard and the sorted pages are merged; the continuation token
  carries each shard's own offset;
* a message goes to the shard of its ``partitionKey`` (else its id); receivers take from every
  shard, lock tokens carry their shard; counts are summed;
* provisioned throughput is split evenly over the shards, as Cosmos splits RU/s over
  physical partitions;
* everything else (Key Vault, Storage, SendGrid, admin) is the rank's own backing, ``home``.

Configured with ``TT_BACKING_SHARDS_<FAMILY>`` (comma-separated URLs in rank order) for the
``COSMOS`` and ``SERVICEBUS`` families (sidecar/base.py).
"""
from __future__ import annotations

import asyncio
import base64
import functools
import heapq
import itertools
import json
import uuid
from typing import Any

from .client import BackingClient, BackingError

PARTITIONED_FAMILIES = ("COSMOS", "SERVICEBUS")
_FNV_OFFSET, _FNV_PRIME, _MASK = 14695981039346656037, 1099511628211, (1 << 64) - 1


def fnv1a64(data: str | bytes) -> int:
    if isinstance(data, str):
        data = data.encode()
    h = _FNV_OFFSET
    for c in data:
        h = ((h ^ c) * _FNV_PRIME) & _MASK
    return h


def shard_of(key: str | bytes, n: int) -> int:
    return fnv1a64(key) % n if n > 1 else 0


def shard_urls(environ: dict[str, str], family: str) -> list[str]:
    raw = environ.get(f"TT_BACKING_SHARDS_{family}") or ""
    urls = [u.strip().rstrip("/") for u in raw.split(",") if u.strip()]
    return urls if len(urls) > 1 else []


# -- cross-partition query merge --------------------------------------------------------------
def encode_token(offsets: list[int | None]) -> str | None:
    if all(o is None for o in offsets):
        return None
    return "p1." + base64.urlsafe_b64encode(json.dumps(offsets, separators=(",", ":")).encode()).decode().rstrip("=")


def decode_token(token: str | None, n: int) -> list[int | None]:
    if not token:
        return [0] * n
    try:
        if not token.startswith("p1."):
            raise ValueError
        body = token[3:]
        offs = json.loads(base64.urlsafe_b64decode(body + "=" * (-len(body) % 4)))
        if not isinstance(offs, list) or len(offs) != n or not all(o is None or (isinstance(o, int) and o >= 0)
                                                                   for o in offs):
            raise ValueError
        return offs
    except (ValueError, TypeError):
        raise BackingError(400, b"invalid continuation token for a partitioned collection", "state query") from None


def _sort_specs(sort: list[dict[str, Any]]) -> list[tuple[str, int]]:
    return [(s["key"], -1 if str(s.get("order", "ASC")).upper() == "DESC" else 1) for s in sort or []
            if isinstance(s, dict) and "key" in s]


def _sort_values(r: dict, specs: list[tuple[str, int]], get_path, missing) -> tuple:
    """The result's sort-key values, extracted once (a missing path sorts like null, the
    store's order)."""
    out = []
    for key, _ in specs:
        v = get_path(r.get("data"), key)
        out.append(None if v is missing else v)
    return tuple(out)


def _sort_cmp(specs: list[tuple[str, int]]):
    from ..ops.columnar import compare

    def cmp(a: tuple, b: tuple) -> int:  # (values, shard, result)
        for (_, sign), x, y in zip(specs, a[0], b[0]):
            c = compare(x, y)
            if c:
                return c * sign
        return (a[1] > b[1]) - (a[1] < b[1])  # ties: shard order
    return cmp


def _plain_order(streams: list[list[tuple]], nkeys: int) -> bool:
    """Every sort column holds one plain type across the merged results (all strings, or all
    non-boolean numbers): Python's own tuple order is then the store's order."""
    for k in range(nkeys):
        kinds = set()
        for st in streams:
            for vals, _, _ in st:
                v = vals[k]
                kinds.add("s" if type(v) is str else "n" if type(v) in (int, float) else "x")
                if len(kinds) > 1 or "x" in kinds:
                    return False
    return True


def merge_pages(query: dict[str, Any], pages: list[tuple[int, dict[str, Any]] | None],
                offsets: list[int | None]) -> dict[str, Any]:
    """Merge every shard's sorted page: ``pages[i]`` is (shard, response) for the shards still
    holding matches (None for exhausted ones), ``offsets`` their positions before this page."""
    from ..ops.columnar import _MISSING, get_path
    limit = int((query.get("page") or {}).get("limit") or 0)
    specs = _sort_specs(query.get("sort") or [])
    streams = [[(_sort_values(r, specs, get_path, _MISSING) if specs else (), i, r) for r in resp.get("results") or []]
               for i, resp in pages if resp is not None]
    if not specs:
        merged = itertools.chain(*streams)
    elif len({sign for _, sign in specs}) == 1 and _plain_order(streams, len(specs)):
        # one direction over plain values (the overdue sweep's taskCreatedOn strings): the
        # values themselves are the merge key; equal keys keep shard order
        merged = heapq.merge(*streams, key=lambda t: t[0], reverse=specs[0][1] < 0)
    else:
        merged = heapq.merge(*streams, key=functools.cmp_to_key(_sort_cmp(specs)))
    # a k-way PAGED merge: once a shard that has more matches (it sent a token) runs out of this
    # page's entries, its unfetched ones may sort before anything left -- the page ends there
    # (a shard can send a short page: its mirror skipped stale rows)
    by_shard = {i: resp for i, resp in pages if resp is not None}
    left = {i: len(resp.get("results") or []) for i, resp in by_shard.items()}
    more = {i for i, resp in by_shard.items() if resp.get("token")}
    take: list[tuple] = []
    used = [0] * len(offsets)
    if not any(left[i] == 0 for i in more):
        for item in merged:
            take.append(item)
            i = item[1]
            used[i] += 1
            if (limit and len(take) >= limit) or (i in more and used[i] == left[i]):
                break
    new: list[int | None] = []
    for i, off in enumerate(offsets):
        resp = pages[i][1] if off is not None else None
        if resp is None:
            new.append(None)
            continue
        n_i = len(resp.get("results") or [])
        tok = resp.get("token")
        if not tok and used[i] == n_i:
            new.append(None)
        elif used[i] == n_i and str(tok).isdigit():  # a fully used page resumes where the shard said
            new.append(int(tok))
        else:
            new.append(off + used[i])
    out: dict[str, Any] = {"results": [r for _, _, r in take]}
    tok = encode_token(new) if limit else None
    if tok:
        out["token"] = tok
    return out


class ShardedBackingClient:
    """``BackingClient``'s interface over the shards of a partitioned collection/namespace."""

    def __init__(self, urls: list[str], identity: str | None = None, key: str | None = None, http=None,
                 home: str | None = None) -> None:
        from ..web.client import HttpClient
        http = http or HttpClient()  # one connection pool for every shard
        self.shards = [BackingClient(u, identity=identity, key=key, http=http) for u in urls]
        self.bases = [c.base for c in self.shards]
        self.home = BackingClient(home, identity=identity, key=key, http=http) if home else self.shards[0]
        self.base = self.home.base
        self.identity, self.key, self.http = self.home.identity, key, self.home.http
        self._rr = itertools.count()

    def __getattr__(self, name: str):  # non-partitioned services: the rank's own backing
        if name.startswith("__") or name in ("home", "shards"):
            raise AttributeError(name)  # not set yet (construction, copy): no recursion
        return getattr(self.home, name)

    @property
    def n(self) -> int:
        return len(self.shards)

    def _of(self, key: str) -> BackingClient:
        return self.shards[shard_of(key, self.n)]

    @property
    def throttled_retries(self) -> int:
        return sum(c.throttled_retries for c in self.shards)

    # -- documents -------------------------------------------------------------------------
    async def doc_put(self, account, db, coll, key, value, etag=None, first_write=False, ttl_ms=0):
        return await self._of(key).doc_put(account, db, coll, key, value, etag, first_write, ttl_ms)

    async def doc_get(self, account, db, coll, key):
        return await self._of(key).doc_get(account, db, coll, key)

    async def doc_delete(self, account, db, coll, key, etag=None):
        return await self._of(key).doc_delete(account, db, coll, key, etag)

    def _split(self, keys: list[str]) -> dict[int, list[int]]:
        groups: dict[int, list[int]] = {}
        for pos, k in enumerate(keys):
            groups.setdefault(shard_of(k, self.n), []).append(pos)
        return groups

    async def doc_bulk_get(self, account, db, coll, keys):
        groups = self._split(keys)
        res = await asyncio.gather(*(self.shards[s].doc_bulk_get(account, db, coll, [keys[p] for p in pos])
                                     for s, pos in groups.items()))
        out: list[Any] = [None] * len(keys)
        for (s, pos), part in zip(groups.items(), res):
            for p, r in zip(pos, part):
                out[p] = r
        return out

    async def doc_bulk_set(self, account, db, coll, items):
        groups = self._split([it["key"] for it in items])
        res = await asyncio.gather(*(self.shards[s].doc_bulk_set(account, db, coll, [items[p] for p in pos])
                                     for s, pos in groups.items()), return_exceptions=True)
        errs = [r for r in res if isinstance(r, BaseException)]
        if errs:  # every shard has answered; the first failure is the caller's
            raise errs[0]
        out: list[Any] = [None] * len(items)
        for (s, pos), part in zip(groups.items(), res):
            for p, r in zip(pos, part):
                out[p] = r
        return out

    async def doc_transaction(self, account, db, coll, ops):
        parts = {shard_of(o["key"], self.n) for o in ops}
        if len(parts) > 1:
            raise BackingError(400, b"a transaction's operations must share one partition key "
                                    b"(the collection is partitioned)", "state transaction")
        target = self.shards[parts.pop()] if parts else self.home
        return await target.doc_transaction(account, db, coll, ops)

    async def doc_query(self, account, db, coll, query: bytes, prefix: str = "") -> bytes:
        try:
            q = json.loads(query or b"{}")
        except ValueError:
            raise BackingError(400, b"invalid query JSON", "state query") from None
        if not isinstance(q, dict):
            raise BackingError(400, b"query must be a JSON object", "state query")
        page = dict(q.get("page") or {})
        offsets = decode_token(page.get("token"), self.n)

        async def one(i: int):
            if offsets[i] is None:
                return i, None
            sub = dict(q)
            p = {k: v for k, v in page.items() if k != "token"}
            if offsets[i]:
                p["token"] = str(offsets[i])
            sub["page"] = p
            if not p:
                sub.pop("page")
            body = await self.shards[i].doc_query(account, db, coll, json.dumps(sub).encode(), prefix)
            return i, json.loads(body)
        pages = await asyncio.gather(*(one(i) for i in range(self.n)))
        return json.dumps(merge_pages(q, list(pages), offsets), separators=(",", ":")).encode()

    async def doc_stats(self, account, db, coll):
        parts = await asyncio.gather(*(c.doc_stats(account, db, coll) for c in self.shards))
        out: dict[str, Any] = {k: sum(p.get(k, 0) for p in parts) for k, v in parts[0].items()
                               if isinstance(v, (int, float)) and not isinstance(v, bool)}
        out["shards"] = parts
        return out

    async def doc_set_throughput(self, account, db, coll, ru_per_s):
        """Cosmos divides a container's RU/s evenly over its physical partitions."""
        share = float(ru_per_s) / self.n if ru_per_s else 0.0
        parts = await asyncio.gather(*(c.doc_set_throughput(account, db, coll, share) for c in self.shards))
        return {"ruPerSecond": float(ru_per_s or 0), "perShard": share, "shards": parts}

    # -- service bus -----------------------------------------------------------------------
    async def sb_create_topic(self, ns, topic):
        await asyncio.gather(*(c.sb_create_topic(ns, topic) for c in self.shards))

    async def sb_create_subscription(self, ns, topic, sub, lock_ms=60000, max_delivery=10, ttl_ms=0):
        await asyncio.gather(*(c.sb_create_subscription(ns, topic, sub, lock_ms, max_delivery, ttl_ms)
                               for c in self.shards))

    async def sb_create_queue(self, ns, queue, lock_ms=60000, max_delivery=10):
        await asyncio.gather(*(c.sb_create_queue(ns, queue, lock_ms, max_delivery) for c in self.shards))

    async def sb_publish(self, ns, topic, body, content_type="application/json", props=None, message_id="",
                         ttl_ms=0):
        pk = str((props or {}).get("partitionKey") or message_id or uuid.uuid4().hex)
        return await self._of(pk).sb_publish(ns, topic, body, content_type, props, message_id, ttl_ms)

    async def sb_publish_batch(self, ns, topic, entries):
        keys = [str((e.get("metadata") or {}).get("partitionKey") or e.get("entryId") or uuid.uuid4().hex)
                for e in entries]
        groups = self._split(keys)
        res = await asyncio.gather(*(self.shards[s].sb_publish_batch(ns, topic, [entries[p] for p in pos])
                                     for s, pos in groups.items()))
        out: list[Any] = [None] * len(entries)
        for (s, pos), part in zip(groups.items(), res):
            for p, r in zip(pos, part):
                out[p] = r
        return out

    async def sb_send(self, ns, queue, body, content_type="application/json"):
        return await self.shards[next(self._rr) % self.n].sb_send(ns, queue, body, content_type)

    @staticmethod
    def _tag(i: int, msgs: list[dict[str, Any]]) -> list[dict[str, Any]]:
        for m in msgs:
            if "lockToken" in m:
                m["lockToken"] = f"{i}:{m['lockToken']}"
        return msgs

    async def sb_receive(self, ns, entity, max_messages=1, lock_ms=0, wait_ms=0):
        """Every shard in turn without waiting; when all are empty, a bounded long poll on the
        next shard in rotation (so no shard's messages wait longer than ~200 ms)."""
        start = next(self._rr)
        out: list[dict[str, Any]] = []
        for k in range(self.n):
            i = (start + k) % self.n
            got = await self.shards[i].sb_receive(ns, entity, max_messages - len(out), lock_ms, 0)
            out += self._tag(i, got)
            if len(out) >= max_messages:
                return out
        if out or not wait_ms:
            return out
        i = start % self.n
        return self._tag(i, await self.shards[i].sb_receive(ns, entity, max_messages, lock_ms, min(wait_ms, 200)))

    async def sb_settle(self, ns, entity, complete=(), abandon=(), deadletter=(), renew=()):
        def split(tok: str) -> tuple[int, str]:
            i, _, t = str(tok).partition(":")
            return int(i), t
        plan: dict[int, dict[str, list]] = {}
        where: dict[str, list[tuple[int, int]]] = {k: [] for k in ("complete", "abandon", "deadletter", "renew")}
        for kind, items in (("complete", complete), ("abandon", abandon), ("deadletter", deadletter),
                            ("renew", renew)):
            for it in items:
                if kind == "complete":
                    i, t = split(it)
                    entry: Any = t
                else:
                    i, t = split(it["token"])
                    entry = dict(it, token=t)
                lst = plan.setdefault(i, {k: [] for k in where})[kind]
                where[kind].append((i, len(lst)))
                lst.append(entry)
        res = dict(zip(plan, await asyncio.gather(*(self.shards[i].sb_settle(ns, entity, **p)
                                                    for i, p in plan.items()))))
        return {kind: [res[i][kind][j] for i, j in where[kind]] for kind in where}

    async def sb_counts(self, ns, entity):
        parts = await asyncio.gather(*(c.sb_counts(ns, entity) for c in self.shards))
        return {k: sum(p.get(k, 0) for p in parts) for k in parts[0]}

    async def sb_dead_letters(self, ns, entity, max_messages=100):
        parts = await asyncio.gather(*(c.sb_dead_letters(ns, entity, max_messages) for c in self.shards))
        return [m for p in parts for m in p][:max_messages]

    async def healthy(self) -> bool:
        return all(await asyncio.gather(*(c.healthy() for c in self.shards)))

    async def close(self) -> None:
        await self.shards[0].http.close()
        if self.home.http is not self.shards[0].http:
            await self.home.http.close()
