"""Query planner + columnar accelerator attached to a document-store collection.

Planner: a filter the native engine can answer from its hash indexes (every AND branch has
an EQ/IN leaf; every OR branch is indexable) stays native -- O(matches).  Anything that
needs a collection scan (ranges, NEQ, OR over non-equality leaves, no filter with a sort)
runs on the collection's ``ColumnarIndex``: on the GPU (``ops/hip/query_scan.hip``) when a
HIP device is present, else the NumPy executor of the same compiled program.

The index is fed by the document store's own column mirror (``DocStore.mirror_*``,
native/src/docstore.hpp): every write -- from the GIL-free native HTTP front or from
Python -- appends its row in C++ under the store lock, and a query first pulls only what
changed since the previous one.  Turning the accelerator on therefore never moves a
collection's writes off the native path.  Collections that use TTL are not mirrored
(expiry is evaluated by the native engine) and fall back to it.

``query`` blocks (mirror build / sync, kernel launches, result assembly): the backing
server calls it from a worker thread, never on its event loop.

Between queries a background thread keeps the mirror warm (``TT_QUERY_MIRROR_SYNC_MS``,
default 100; 0 = off): it pulls the rows written since the last sync, uploads them to the
device and refreshes the zone maps of the sorts already served, so a query under a heavy write
stream (the overdue sweep next to 40 k creates/s) syncs ~100 ms of writes instead of a second's.

Mode (``TT_QUERY_ACCEL``): ``off`` | ``cpu`` | ``gpu`` | ``auto`` (default: GPU if
available, else CPU); size threshold ``TT_QUERY_ACCEL_MIN_DOCS`` (default 20000);
``TT_QUERY_MIRROR_PATHS`` (comma separated): paths mirrored from a collection's first write,
so the first scan-shaped query finds the mirror already built (Cosmos "indexing policy").
"""
from __future__ import annotations

import json
import logging
import os
import threading
import time
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


_STALL = {"file": None, "min_s": None}


def _stall_note(what: str, secs: float, **phases: float) -> None:
    """``TT_STALL_LOG`` diagnostics: one JSON line for a query or background sync slower than
    ``TT_STALL_MS`` (default 100) ms, with its phases -- both hold the collection lock."""
    if _STALL["min_s"] is None:
        path = os.environ.get("TT_STALL_LOG")
        _STALL["file"] = open(path, "a", buffering=1) if path else None
        _STALL["min_s"] = float(os.environ.get("TT_STALL_MS", "100") or 100) / 1e3
    if _STALL["file"] is None or secs <= _STALL["min_s"]:
        return
    _STALL["file"].write(json.dumps({"what": what, "ms": round(secs * 1e3, 2), **{k: round(v, 2) for k, v in phases.items()},
                                     "pid": os.getpid(), "wall": round(time.time(), 4)}) + "\n")


class CollectionAccelerator:
    def __init__(self, mode: str, min_docs: int, preload: list[str] | None = None) -> None:
        self.mode = mode
        self.min_docs = min_docs
        self.preload = [p for p in (preload or []) if p]
        self.index: ColumnarIndex | None = None
        self.disabled = mode == "off"
        self.stats = {"native": 0, "gpu": 0, "cpu": 0, "fallback": 0, "skipped_rows": 0}
        self._kernels = None
        self.lock = threading.Lock()  # one query / sync at a time per collection
        self._bg: threading.Thread | None = None
        self._bg_stop = threading.Event()
        # 40 ms: a query then finds at most ~40 ms of writes to sync, rank and upload itself
        self.sync_interval = max(0.0, float(os.environ.get("TT_QUERY_MIRROR_SYNC_MS", "40")) / 1000.0)

    def attach(self, store) -> None:
        """New collection: start mirroring the configured paths from its first write."""
        if self.preload and not self.disabled:
            if not store.mirror_enable([PREFIX_PATH, *self.preload]):
                self.disabled = True

    # -- querying ---------------------------------------------------------------
    def kernels(self):
        if self._kernels is None and self.mode in ("auto", "gpu"):
            try:
                from ..ops.gpu import GpuKernels
                from ..parallel import hold_affinity
                with hold_affinity():  # the runtime's threads stay on this process's CPUs
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
        # the store encodes every column the triggering query needs (one thread per column)
        # and from then on appends a row per write itself
        self.index = ColumnarIndex.from_native(store, [PREFIX_PATH, *self.preload, *paths])
        log.info("columnar mirror over %d documents", self.index.live_rows())
        if self.sync_interval > 0 and self._bg is None:
            self._bg = threading.Thread(target=self._warm_loop, name="tt-mirror-sync", daemon=True)
            self._bg.start()

    def _warm_loop(self) -> None:
        while not self._bg_stop.wait(self.sync_interval):
            with self.lock:
                if self.index is None or self.disabled:
                    return
                t0 = time.perf_counter()
                t1 = t0
                try:
                    self.index.sync()
                    t1 = time.perf_counter()
                    k = self._kernels
                    if k is not None:
                        self.index.warm(k)
                except Unsupported:
                    self.disabled, self.index = True, None
                    return
                except Exception:  # a failed warm-up only leaves the work to the next query
                    log.exception("background mirror sync failed")
                t2 = time.perf_counter()
                self.stats["bg_syncs"] = self.stats.get("bg_syncs", 0) + 1
                self.stats["bg_sync_ms"] = round(self.stats.get("bg_sync_ms", 0.0) + (t2 - t0) * 1e3, 3)
                self.stats["bg_sync_max_ms"] = round(max(self.stats.get("bg_sync_max_ms", 0.0), (t2 - t0) * 1e3), 3)
                _stall_note("mirror-bg-sync", t2 - t0, sync_ms=(t1 - t0) * 1e3, warm_ms=(t2 - t1) * 1e3)

    def close(self, timeout: float = 10.0) -> None:
        """Stop the background sync and wait for it: no sync may still be inside the native
        store or the HIP kernels when the caller tears those down."""
        self._bg_stop.set()
        bg = self._bg
        if bg is not None and bg is not threading.current_thread():
            bg.join(timeout)
        with self.lock:  # a query's own sync finishes before close returns
            pass

    def query(self, q: dict[str, Any], prefix: str, store, sort_keys: bool = False) -> bytes | None:
        """JSON result text (UTF-8 bytes, as the store built it: the page goes out without a
        decode/encode round trip), or None to let the native engine answer.  Blocking.
        ``sort_keys``: the results as sort-keys projections (``{"key", "etag", "sort"}``, the
        first phase of a cross-partition page)."""
        if not self.should_accelerate(q, store):
            self.stats["native"] += 1
            return None
        t_wait = time.perf_counter()
        with self.lock:
            t0 = time.perf_counter()
            try:
                if self.index is None:
                    self.build(store, filter_paths(q.get("filter")) + [s["key"] for s in q.get("sort") or []
                                                                       if isinstance(s, dict) and "key" in s])
                else:
                    self.index.sync()
            except Unsupported as e:
                log.info("columnar accelerator off for this collection: %s", e)
                self.disabled, self.index = True, None
                self.stats["fallback"] += 1
                return None
            t1 = time.perf_counter()
            flt = q.get("filter") or {}
            if prefix:
                flt = {"AND": [{"EQ": {PREFIX_PATH: prefix}}, flt]} if flt else {"EQ": {PREFIX_PATH: prefix}}
            qq = dict(q)
            qq["filter"] = flt
            k = self.kernels()
            # the row numbers are only meaningful in the mirror generation they were selected
            # from: a write that compacts the mirror between the sync and the lookup (the native
            # front writes without the GIL) renumbers them -- re-sync and select again
            t_sel = t_res = 0.0
            for attempt in range(3):
                ta = time.perf_counter()
                try:
                    rows, token = self.index.query_rows(qq, k)
                except Unsupported:
                    self.stats["fallback"] += 1
                    return None
                tb = time.perf_counter()
                res = store.mirror_results(rows, prefix, token or "", gen=self.index.generation,
                                           sort_paths=[sp["key"] for sp in q.get("sort") or []
                                                       if isinstance(sp, dict) and "key" in sp] if sort_keys else None)
                t_sel, t_res = t_sel + tb - ta, t_res + time.perf_counter() - tb
                # a page that lost rows to writes since the sync (killed rows are skipped) and has
                # more matches behind it is selected again on a fresh sync: a short page with a
                # continuation would let a cross-partition merge run past this shard's order
                if res is not None and (not res[1] or not token or attempt == 2):
                    break
                key = "stale_retries" if res is None else "short_page_retries"
                self.stats[key] = self.stats.get(key, 0) + 1
                try:
                    self.index.sync()
                except Unsupported:
                    self.disabled, self.index = True, None
                    self.stats["fallback"] += 1
                    return None
            else:  # compacting faster than we can select: the native engine answers
                self.stats["fallback"] += 1
                return None
            self.stats["gpu" if k is not None else "cpu"] += 1
            out, skipped = res
            self.stats["skipped_rows"] += skipped
            t2 = time.perf_counter()
            # where an accelerated query spends its time (summed; stats route reports them)
            for key, v in (("lock_wait_ms", t0 - t_wait), ("sync_ms", t1 - t0), ("select_and_results_ms", t2 - t1),
                           ("select_ms", t_sel), ("results_ms", t_res)):
                self.stats[key] = round(self.stats.get(key, 0.0) + v * 1e3, 3)
            _stall_note("accel-query", t2 - t_wait, lock_wait_ms=(t0 - t_wait) * 1e3, sync_ms=(t1 - t0) * 1e3,
                        select_ms=t_sel * 1e3, results_ms=t_res * 1e3)
            for key, v in self.index.timing.items():  # the paged device path's own breakdown
                self.stats[key] = round(v, 3)
            return out


def accelerator_from_env() -> tuple[str, int]:
    return os.environ.get("TT_QUERY_ACCEL", "auto").lower(), int(os.environ.get("TT_QUERY_ACCEL_MIN_DOCS", "20000"))


def mirror_paths_from_env() -> list[str]:
    return [p.strip() for p in os.environ.get("TT_QUERY_MIRROR_PATHS", "").split(",") if p.strip()]
