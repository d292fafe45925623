"""Query planner + columnar accelerator attached to a document-store collection.

Planner: a filter the native engine can answer from its hash indexes (every AND branch has
an EQ/IN leaf; every OR branch is indexable) stays native -- O(matches).  Anything that
needs a collection scan (ranges, NEQ, OR over non-equality leaves, no filter with a sort)
runs on the collection's ``ColumnarIndex``: on the GPU (``ops/hip/query_scan.hip``) when a
HIP device is present, else the NumPy executor of the same compiled program.

Mode (``TT_QUERY_ACCEL``): ``off`` | ``cpu`` | ``gpu`` | ``auto`` (default: GPU if
available, else CPU) and size threshold ``TT_QUERY_ACCEL_MIN_DOCS`` (default 20000).
The index mirrors every write (upsert/delete/transaction); collections that use TTL fall
back to the native engine (expiry is evaluated there).
"""
from __future__ import annotations

import json
import logging
import os
from typing import Any

from ..ops.columnar import ColumnarIndex, Unsupported, filter_paths

log = logging.getLogger("backing.accel")
PREFIX_PATH = "\x00keyprefix"


def indexable(f: Any) -> bool:
    """Mirror of the native engine's ``candidates()``: can hash indexes answer this?"""
    if not f:
        return False
    if not isinstance(f, dict) or len(f) != 1:
        return False
    (op, arg), = f.items()
    op = op.upper()
    if op in ("EQ", "IN"):
        # equality on booleans / null is not selective: the hash bucket is a large share of
        # the collection, so a columnar scan beats probing it
        vals = list(arg.values())[0] if isinstance(arg, dict) and arg else None
        vals = vals if isinstance(vals, list) else [vals]
        return not all(v is None or isinstance(v, bool) for v in vals)
    if op == "AND":
        return any(indexable(x) for x in arg or [])
    if op == "OR":
        return bool(arg) and all(indexable(x) for x in arg)
    return False


class CollectionAccelerator:
    def __init__(self, mode: str, min_docs: int) -> None:
        self.mode = mode
        self.min_docs = min_docs
        self.index: ColumnarIndex | None = None
        self.disabled = mode == "off"
        self.stats = {"native": 0, "gpu": 0, "cpu": 0, "fallback": 0}
        self._kernels = None
        self.before_build = None  # hook: route the collection's writes through on_put/on_delete

    # -- write mirroring ------------------------------------------------------
    def on_put(self, key: str, value: str, ttl_ms: int = 0) -> None:
        if ttl_ms:
            self.disabled = True
            self.index = None
            return
        if self.index is not None:
            try:
                self.index.upsert(key, _with_prefix(key, json.loads(value)))
            except ValueError:
                self.index.delete(key)

    def on_delete(self, key: str) -> None:
        if self.index is not None:
            self.index.delete(key)

    # -- querying ---------------------------------------------------------------
    def kernels(self):
        if self._kernels is None and self.mode in ("auto", "gpu"):
            try:
                from ..ops.gpu import GpuKernels
                self._kernels = GpuKernels()
            except Exception as e:
                if self.mode == "gpu":
                    raise
                log.info("GPU query path unavailable (%s); using the CPU columnar executor", e)
                self.mode = "cpu"
        return self._kernels

    def should_accelerate(self, q: dict[str, Any], store) -> bool:
        if self.disabled:
            return False
        flt = q.get("filter")
        if indexable(flt):
            return False
        if not flt and not q.get("sort"):
            return False
        return self.index is not None or len(store) >= self.min_docs

    def build(self, store, paths: list[str] = ()) -> None:
        if self.before_build is not None:
            self.before_build()
        # native bulk encode (DocStore.encode_columns, one thread per column) of every column the
        # triggering query needs: no per-document Python objects
        ix = ColumnarIndex.from_source(lambda ps: store.encode_columns("", ps), [PREFIX_PATH, *paths])
        self.index = ix
        log.info("built columnar index over %d documents", ix.live_rows())

    def query(self, q: dict[str, Any], prefix: str, store) -> str | None:
        """JSON result text, or None to let the native engine answer."""
        if not self.should_accelerate(q, store):
            self.stats["native"] += 1
            return None
        if self.index is None:
            self.build(store, filter_paths(q.get("filter")) + [s["key"] for s in q.get("sort") or []
                                                               if isinstance(s, dict) and "key" in s])
        flt = q.get("filter") or {}
        if prefix:
            flt = {"AND": [{"EQ": {PREFIX_PATH: prefix}}, flt]} if flt else {"EQ": {PREFIX_PATH: prefix}}
        qq = dict(q)
        qq["filter"] = flt
        k = self.kernels()
        try:
            keys, token = self.index.query(qq, k)
        except Unsupported:
            self.stats["fallback"] += 1
            return None
        self.stats["gpu" if k is not None else "cpu"] += 1
        parts = []
        for key in keys:
            got = store.get(key)
            if got is None:
                continue
            parts.append('{"key":' + json.dumps(key[len(prefix):]) + ',"data":' + got[0] + ',"etag":"' + got[1] + '"}')
        out = '{"results":[' + ",".join(parts) + "]"
        if token:
            out += ',"token":"' + token + '"'
        return out + "}"


def _with_prefix(key: str, doc: Any) -> Any:
    """Attach the key's ``<app-id>||`` prefix as a hidden column value."""
    i = key.find("||")
    pfx = key[:i + 2] if i >= 0 else ""
    if isinstance(doc, dict):
        d = dict(doc)
        d[PREFIX_PATH] = pfx
        return d
    return {PREFIX_PATH: pfx, "\x00value": doc}


def accelerator_from_env() -> tuple[str, int]:
    return os.environ.get("TT_QUERY_ACCEL", "auto").lower(), int(os.environ.get("TT_QUERY_ACCEL_MIN_DOCS", "20000"))
