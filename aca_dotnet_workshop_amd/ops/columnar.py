"""Columnar, dictionary-encoded mirror of a state-store collection + the query compiler.

Why: the reference's queries (``EQ taskCreatedBy``, ``EQ taskDueDate`` then in-app
filtering, Services/TasksStoreManager.cs:54-69, 104-139) are whole-collection scans in
Cosmos; equality is served by the native store's hash indexes, but range/NEQ/OR filters,
the corrected overdue sweep (``taskDueDate < today AND NOT isCompleted AND NOT isOverDue``)
and dashboard aggregates (open tasks per assignee) are O(collection).  Those run here,
on the GPU when one is present (``ops/hip/query_scan.hip``), with a NumPy executor of the
*same* compiled program as the CPU path and as the correctness oracle.

Encoding: each indexed JSON path is an int32 column of dictionary ids (-1 = path missing).
Equality and ordering semantics are evaluated on the host against the (small) dictionary,
exactly mirroring the native engine's ``compare`` (type order null < bool < number < string;
numbers by value; ranges only between like types), producing one bitmap per leaf.
"""
from __future__ import annotations

import functools
import itertools
import json
import operator
import os
import time
from dataclasses import dataclass
from typing import Any, Iterable

import numpy as np

OP_LEAF, OP_AND, OP_OR, OP_NOT, OP_TRUE, OP_EQ, OP_RANGE = 1, 2, 3, 4, 5, 6, 7
TILE = 8192           # rows per kernel tile (ops/hip/query_scan.hip kTileRows)
MAX_DEPTH = 8         # device stack depth (16-bit masks in a 128-bit register)
_TYPE_ORDER = {type(None): 0, bool: 1, int: 2, float: 2, str: 3, list: 4, dict: 5}


@functools.lru_cache(maxsize=1)
def cpu_share() -> int:
    """CPUs this process may use: the cgroup quota (``cpu.max``) when set, else its affinity
    (read once per process)."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            return max(1, int(quota) // int(period))
    except (OSError, ValueError):
        pass
    return max(1, len(os.sched_getaffinity(0)))


class Unsupported(Exception):
    """Filter cannot run on the columnar engine (caller falls back to the native store)."""


def vkey(v: Any) -> str:
    """Canonical dictionary key with the native engine's equality semantics."""
    if v is None:
        return "n"
    if isinstance(v, bool):
        return "b1" if v else "b0"
    if isinstance(v, (int, float)):
        return "d" + repr(float(v) + 0.0)  # + 0.0 folds -0.0 into 0.0 (IEEE equality)
    if isinstance(v, str):
        return "s" + v
    return "j" + json.dumps(_norm(v), separators=(",", ":"))


def _norm(v: Any) -> Any:
    if isinstance(v, bool) or v is None or isinstance(v, str):
        return v
    if isinstance(v, (int, float)):
        return float(v) + 0.0
    if isinstance(v, list):
        return [_norm(x) for x in v]
    if isinstance(v, dict):
        return {k: _norm(x) for k, x in v.items()}
    return v


def type_rank(v: Any) -> int:
    return _TYPE_ORDER.get(type(v), 6)


def compare(a: Any, b: Any) -> int:
    ta, tb = type_rank(a), type_rank(b)
    if ta != tb:
        return -1 if ta < tb else 1
    if ta == 0:
        return 0
    if ta in (1, 2, 3):
        return (a > b) - (a < b)
    if ta == 4:
        for x, y in zip(a, b):
            c = compare(x, y)
            if c:
                return c
        return (len(a) > len(b)) - (len(a) < len(b))
    sa, sb = json.dumps(a, separators=(",", ":")), json.dumps(b, separators=(",", ":"))
    return (sa > sb) - (sa < sb)


_MISSING = object()


def get_path(doc: Any, path: str) -> Any:
    cur = doc
    for seg in path.split("."):
        if isinstance(cur, dict):
            if seg in cur:
                cur = cur[seg]
            else:
                low = seg.lower()
                for k, v in cur.items():
                    if k.lower() == low:
                        cur = v
                        break
                else:
                    return _MISSING
        elif isinstance(cur, list) and seg.isdigit():
            i = int(seg)
            if i >= len(cur):
                return _MISSING
            cur = cur[i]
        else:
            return _MISSING
    return cur


def filter_paths(f: Any) -> list[str]:
    """Every document path a filter references (so all columns are encoded in one pass)."""
    out: list[str] = []
    if isinstance(f, dict) and len(f) == 1:
        (op, arg), = f.items()
        if op.upper() in ("AND", "OR") and isinstance(arg, list):
            for x in arg:
                out += filter_paths(x)
        elif isinstance(arg, dict) and len(arg) == 1:
            out.append(next(iter(arg)))
    return out


def rank_interval(c: "Column", sat: np.ndarray) -> tuple[int, int] | None:
    """A range predicate's satisfying dictionary ids as a half-open interval of sort ranks, when
    they are exactly the ids whose rank falls in it (values of one JSON type are contiguous in
    the sort order, so GT/GTE/LT/LTE always are)."""
    if sat.size == 0:
        return None
    ranks = c.ranks()
    if not sat.any():
        return (1, 1)  # empty interval: no row satisfies
    r = ranks[sat]
    lo, hi = int(r.min()), int(r.max()) + 1
    inside = (ranks >= lo) & (ranks < hi)
    if not np.array_equal(inside, sat):
        return None
    return lo, hi


class KeyTable:
    """Row -> document key.  Bulk-loaded keys stay in one UTF-8 blob with offsets (decoded on
    access, so a 10 M-row index holds no 10 M Python strings); appended keys go to a list."""

    def __init__(self, blob: bytes = b"", offsets: np.ndarray | None = None) -> None:
        self.blob = blob
        self.off = offsets if offsets is not None else np.zeros(1, dtype=np.int64)
        self.base = len(self.off) - 1
        self.extra: list[str] = []

    def __len__(self) -> int:
        return self.base + len(self.extra)

    def __getitem__(self, i: int) -> str:
        if i < self.base:
            return self.blob[self.off[i]:self.off[i + 1]].decode()
        return self.extra[i - self.base]

    def append(self, key: str) -> None:
        self.extra.append(key)

    def __iter__(self):
        for i in range(len(self)):
            yield self[i]


_RANK_EPOCHS = itertools.count(1)


_starts_with_quote = operator.methodcaller("startswith", '"')

_NATIVE = []  # [module or None], resolved on first use


def _native_module():
    """The native extension for ``StrRanker`` (None where it cannot load, or with
    ``TT_NATIVE_RANKS=0``: the numpy ranks then answer)."""
    if not _NATIVE:
        mod = None
        if os.environ.get("TT_NATIVE_RANKS", "1") != "0":
            try:
                from ..native import load
                mod = load()
                if not hasattr(mod, "StrRanker"):
                    mod = None
            except Exception:  # no compiler / stale build: the numpy path is complete on its own
                mod = None
        _NATIVE.append(mod)
    return _NATIVE[0]


class Column:
    def __init__(self, path: str) -> None:
        self.path = path
        self._ids: dict[str, int] = {}
        self._ids_n = 0  # values[:_ids_n] are in _ids (bulk-appended strings are keyed lazily)
        self.values: list[Any] = []
        self._num_cache: np.ndarray | None = None
        self._rank_cache: np.ndarray | None = None
        self.rank_version = 0  # bumps whenever a new value may shift the sort ranks
        # which ids' ranks each recomputation changed: (recomputation number, first id whose rank
        # moved); consumers that keep a copy of the ranks (the device sort plan) re-copy only
        # ids >= that bound (the newest ids, for timestamps written roughly in order)
        self.rank_seq = next(_RANK_EPOCHS)
        self._rank_log: list[tuple[int, int]] = []
        self._rank_lo = 0
        # every value a str without a trailing NUL (numpy's fixed-width strings drop those):
        # the ranks are then positions in the sorted dictionary (_string_ranks)
        self.str_only = True
        self._str_sorted = None
        self._nr = None       # native/src/strrank.hpp StrRanker (the string-only ranks)
        self._nr_buf = None   # its rank buffer (int64, capacity-doubled, owned here)

    @property
    def ids(self) -> dict[str, int]:
        """vkey -> dictionary id.  Strings appended in bulk by ``encode_json_many`` are keyed on
        first use: a column only ordered or range-filtered (timestamps) never pays for it."""
        n = len(self.values)
        if self._ids_n < n:
            self._ids.update(zip([vkey(v) for v in self.values[self._ids_n:]], range(self._ids_n, n)))
            self._ids_n = n
        return self._ids

    @ids.setter
    def ids(self, d: dict[str, int]) -> None:
        self._ids, self._ids_n = d, len(self.values)

    def encode(self, v: Any) -> int:
        if v is _MISSING:
            return -1
        k = vkey(v)
        ids = self.ids
        i = ids.get(k)
        if i is None:
            i = ids[k] = len(self.values)
            self.values.append(v)
            self._ids_n += 1
            if type(v) is not str or v.endswith("\x00"):
                self.str_only = False
            self._num_cache = None
            self._rank_cache = None
            self.rank_version += 1
        return i

    def encode_json_many(self, texts: list[str], all_strings: bool | None = None) -> np.ndarray:
        """Dictionary ids of JSON value texts (the native mirror's new dictionary entries).
        Strings -- timestamps, names, e-mails, the values a growing collection adds on every
        write -- are decoded in one ``json.loads`` and appended in bulk: the native dictionary
        holds each string once (strings compare by value there, as here), so none is already
        here and no per-value ``vkey`` or dictionary probe is needed."""
        if all_strings is None:  # the mirror says; other callers have it checked (a C-level loop)
            all_strings = all(map(_starts_with_quote, texts))
        if texts and all_strings:
            joined = ",".join(texts)
            strs = json.loads("[" + joined + "]")
            base = len(self.values)
            self.values.extend(strs)  # keyed lazily (``ids``)
            if self.str_only and "\\u0000" in joined and any(x.endswith("\x00") for x in strs):
                self.str_only = False
            self._num_cache = None
            self._rank_cache = None
            self.rank_version += 1
            return np.arange(base, base + len(strs), dtype=np.int32)
        return np.fromiter((self.encode(json.loads(t)) for t in texts), dtype=np.int32, count=len(texts))

    def lookup(self, v: Any) -> int:
        return self.ids.get(vkey(v), -2)

    def satisfying(self, op: str, val: Any) -> np.ndarray:
        """Boolean array over the dictionary: which ids satisfy ``<value> op val``."""
        n = len(self.values)
        out = np.zeros(n, dtype=bool)
        if op == "IN":
            for x in val:
                i = self.lookup(x)
                if i >= 0:
                    out[i] = True
            return out
        tv = type_rank(val)
        if tv == 2:  # numeric fast path (vectorised)
            if self._num_cache is None:
                self._num_cache = np.array([float(x) if type_rank(x) == 2 else np.nan for x in self.values],
                                           dtype=np.float64)
            arr = self._num_cache
            with np.errstate(invalid="ignore"):
                res = {"GT": arr > val, "GTE": arr >= val, "LT": arr < val, "LTE": arr <= val}[op]
            return res & ~np.isnan(arr)
        for i, x in enumerate(self.values):
            if type_rank(x) != tv:
                continue
            c = compare(x, val)
            out[i] = {"GT": c > 0, "GTE": c >= 0, "LT": c < 0, "LTE": c <= 0}[op]
        return out

    def missing_rank(self) -> int:
        """A missing path sorts like JSON null (the native engine compares it as null)."""
        if self.str_only:
            return 0  # no null in a string-only dictionary (and no need to key it)
        i = self.ids.get("n")
        return int(self.ranks()[i]) if i is not None else 0

    def ranks(self) -> np.ndarray:
        """Sort rank of every dictionary id (ties share a rank, ranks start at 1)."""
        if self._rank_cache is None:
            self._rank_lo = 0
            self._rank_cache = self._string_ranks() if self._all_strings() else self._general_ranks()
            self.rank_seq = next(_RANK_EPOCHS)
            self._rank_log.append((self.rank_seq, self._rank_lo))
            if len(self._rank_log) > 64:
                del self._rank_log[0]
        return self._rank_cache

    def rank_changes_since(self, seq: int) -> int | None:
        """The first id whose rank may differ from the ranks of recomputation ``seq`` (the
        dictionary size when none moved); None when ``seq`` is too old to tell."""
        self.ranks()
        if seq == self.rank_seq:
            return len(self.values)
        if not any(s == seq for s, _ in self._rank_log):
            return None
        return min([lo for s, lo in self._rank_log if s > seq] or [len(self.values)])

    def _all_strings(self) -> bool:
        if not self.str_only:
            self._str_sorted = None
            self._nr = self._nr_buf = None
        return self.str_only

    def _string_ranks(self) -> np.ndarray:
        r = self._string_ranks_native()
        return r if r is not None else self._string_ranks_numpy()

    def _string_ranks_native(self) -> np.ndarray | None:
        """``_string_ranks`` in C++ (``native/src/strrank.hpp``): the new values are read from
        the dictionary list as UTF-8 (no numpy string array), sorted alone and merged into the
        tail of the order; the ranks land in a buffer owned here, so earlier views stay valid.
        None without the native module (the numpy path then answers)."""
        mod = _native_module()
        if mod is None:
            return None
        n = len(self.values)
        nr = self._nr
        if nr is None or nr.size > n:  # first use, or the dictionary was replaced
            nr, self._nr_buf = mod.StrRanker(), None
        buf = self._nr_buf
        if buf is None or buf.size < n:
            grown = np.empty(max(1024, 2 * n), dtype=np.int64)
            if buf is not None:
                grown[:nr.size] = buf[:nr.size]
            buf = grown
        try:
            lo = nr.extend(self.values, buf)
        except (TypeError, ValueError):  # not a list of values as expected: the numpy path
            lo = -1
        if lo < 0:  # a value UTF-8 cannot carry (a lone surrogate): the numpy path orders it
            self._nr = self._nr_buf = None
            return None
        self._nr, self._nr_buf = nr, buf
        self._rank_lo = int(lo)
        return buf[:n]

    def _string_ranks_numpy(self) -> np.ndarray:
        """A dictionary of strings only (timestamps, e-mails, names): distinct values never tie
        and Python's string order is ``compare``'s, so the ranks are positions in the sorted
        dictionary.  Kept incrementally: values appended since the last call are sorted alone
        and merged in (``searchsorted`` + ``insert``), an O(dictionary) vector pass instead of a
        comparison sort of the whole dictionary per new value -- the overdue sweep orders by
        ``taskCreatedOn``, whose dictionary grows with every created task.  When every new value
        sorts after the old ones (timestamps of new writes) the sorted copy and the ranks grow
        in place, in capacity-doubling buffers: O(new values), not O(dictionary)."""
        n = len(self.values)
        prev = self._str_sorted
        if prev is None or prev[1] > n:
            arr = np.array(self.values, dtype=str) if n else np.zeros(0, dtype="<U1")
            order = np.argsort(arr, kind="stable")
            r = np.empty(n, dtype=np.int64)
            r[order] = np.arange(1, n + 1)
            self._str_sorted = (arr[order], n, r, order.astype(np.int64))
            self._rank_lo = 0
            return r[:n]
        srt, m, old_r, ids = prev  # sorted values, count, rank per id, id per sorted position
        if m == n:
            self._rank_lo = n
            return old_r[:n]
        new = np.array(self.values[m:], dtype=str)
        k = new.size
        if k < 2 or bool(np.all(new[1:] >= new[:-1])):  # written in order (timestamps): no sort
            norder = np.arange(k, dtype=np.int64)
            new_sorted = new
        else:
            norder = np.argsort(new, kind="stable")
            new_sorted = new[norder]
        # insertion point of the smallest new value: only the old values from there on move
        pos0 = m if m == 0 or new_sorted[0] > srt[m - 1] else int(np.searchsorted(srt[:m], new_sorted[0]))
        if new_sorted.dtype.itemsize <= srt.dtype.itemsize and m - pos0 <= 4 * k + 65536:
            # new values land in (or just before) the tail of the order -- new timestamps,
            # written a little out of order by concurrent writers: re-sort only that tail with
            # them, in capacity-doubling buffers; O(tail + new), not O(dictionary)
            if srt.size < n:  # grow the buffers (doubling): amortised O(1) per appended value
                cap = max(n, 2 * srt.size, 1024)
                srt2 = np.empty(cap, dtype=srt.dtype)
                srt2[:m] = srt[:m]
                r2 = np.empty(cap, dtype=np.int64)
                r2[:m] = old_r[:m]
                i2 = np.empty(cap, dtype=np.int64)
                i2[:m] = ids[:m]
                srt, old_r, ids = srt2, r2, i2
            tail_ids = ids[pos0:m].copy()
            if pos0 == m:
                srt[m:n] = new_sorted
                ids[m:n] = m + norder
            else:
                # merge two sorted runs (the old tail, the new values) without a comparison
                # sort: each new value lands after the old ones equal to it (a stable sort of
                # old-then-new would do the same)
                tail = srt[pos0:m].copy()
                ins = np.searchsorted(tail, new_sorted, side="right")
                at_new = ins + np.arange(k)                                  # merged positions of new values
                at_old = np.arange(tail.size) + np.searchsorted(ins, np.arange(tail.size), side="right")
                seg_v = np.empty(tail.size + k, dtype=srt.dtype)
                seg_i = np.empty(tail.size + k, dtype=np.int64)
                seg_v[at_old], seg_v[at_new] = tail, new_sorted
                seg_i[at_old], seg_i[at_new] = tail_ids, m + norder
                srt[pos0:n] = seg_v
                ids[pos0:n] = seg_i
            old_r[ids[pos0:n]] = np.arange(pos0 + 1, n + 1)
            self._str_sorted = (srt, n, old_r, ids)
            self._rank_lo = int(min(int(tail_ids.min()), m)) if tail_ids.size else m
            return old_r[:n]
        srt = srt[:m]
        old_r = old_r[:m]
        ids = ids[:m]
        width = max(srt.dtype.itemsize, new.dtype.itemsize) // 4
        srt = srt.astype(f"<U{max(width, 1)}", copy=False)
        new_sorted = new_sorted.astype(srt.dtype, copy=False)
        pos = np.searchsorted(srt, new_sorted)            # insertion points in the old order
        before = np.searchsorted(pos, old_r - 1, side="right")  # new values ahead of each old one
        r = np.empty(n, dtype=np.int64)
        r[:m] = old_r + before
        r[m + norder] = pos + np.arange(new.size) + 1
        # the old values at or after the first insertion point moved up: the first id among
        # them bounds what changed (new timestamps arriving a little out of order: recent ids)
        moved = ids[int(pos[0]):]
        self._rank_lo = int(min(int(moved.min()), m)) if moved.size else m
        self._str_sorted = (np.insert(srt, pos, new_sorted), n, r, np.insert(ids, pos, m + norder))
        return r

    def _general_ranks(self) -> np.ndarray:
        import functools
        order = sorted(range(len(self.values)), key=functools.cmp_to_key(lambda a, b: compare(self.values[a], self.values[b])))
        r = np.empty(len(order), dtype=np.int64)
        rank = 0
        for pos, i in enumerate(order):
            if pos and compare(self.values[order[pos - 1]], self.values[i]) != 0:
                rank += 1
            r[i] = rank + 1  # 0 reserved for missing (sorts like null, first)
        return r


@dataclass
class Program:
    code: np.ndarray      # [L, 4] int32
    bitmaps: np.ndarray   # int32 words (uint32 bit patterns)
    columns: list[int]


class ColumnarIndex:
    def __init__(self, paths: Iterable[str] = (), capacity: int = TILE) -> None:
        self.columns: list[Column] = []
        self.col_of: dict[str, int] = {}
        self.cap = max(TILE, (capacity + TILE - 1) // TILE * TILE)
        self.ids = np.full((0, self.cap), -1, dtype=np.int32)
        self.live = np.zeros(self.cap, dtype=np.int32)
        self.seq = np.zeros(self.cap, dtype=np.int64)
        self._next_seq = 0
        self.keys: KeyTable | list[str] = []
        self._row_of: dict[str, int] | None = {}
        self.docs: list[Any] | None = []  # None when columns come from `source` (bulk-encoded)
        self.source = None  # callable(paths) -> (keys, seqs, [(values_json, ids)]) for re-encoding
        self.native = None  # DocStore whose column mirror feeds this index (from_native)
        self._dead = 0      # tombstoned rows since the last compaction (upsert/delete path)
        self.n = 0
        self.version = 0
        self._dev = None  # device mirror state
        # compiled programs / device ordering plans, keyed by the query and the dictionaries'
        # state (append-only dictionaries: sizes + rank versions identify their contents)
        self._prog_cache: dict[Any, Program] = {}
        self._plan_cache: dict[Any, Any] = {}
        self._dict_gen = 0  # bumps when the dictionaries are rebuilt (re-encode from `source`)
        self._tomb_dirty = False   # liveness changed for rows that are already on the device
        self._full_dirty = True    # layout changed (compaction / new column / growth)
        # zone maps of the paged device path, per sort spec (page_gpu): per tile the row with the
        # smallest ordering key, re-computed for the tiles whose rows changed
        self._zones: dict[Any, dict] = {}
        self.timing: dict[str, float] = {}  # where the paged device path spends its time (summed)
        self._plan_tm: dict[str, float] | None = None  # set while page_gpu plans (sub-step times)
        for p in paths:
            self.add_column(p)

    # -- bulk load ------------------------------------------------------------
    @classmethod
    def from_source(cls, source, paths: Iterable[str]) -> "ColumnarIndex":
        """Index built from a native bulk encoder (``DocStore.encode_columns``): no per-document
        Python objects are kept; a column added later re-encodes from ``source``."""
        ix = cls()
        ix.source = source
        ix.docs = None
        ix._load(list(dict.fromkeys(paths)))
        return ix

    def _load(self, paths: list[str]) -> None:
        keys, seqs, cols = self.source(paths)
        n = len(seqs)
        cap = max(TILE, (n + TILE - 1) // TILE * TILE)
        self.cap = cap
        self.columns, self.col_of = [], {}
        self._dict_gen += 1
        self.ids = np.full((len(paths), cap), -1, dtype=np.int32)
        for i, (path, (values, ids)) in enumerate(zip(paths, cols)):
            c = Column(path)
            remap = np.empty(len(values), dtype=np.int32)
            for j, text in enumerate(values):  # dictionary built by Python's own equality (vkey)
                remap[j] = c.encode(json.loads(text))
            ids = np.asarray(ids, dtype=np.int32)
            self.ids[i, :n] = np.where(ids >= 0, remap[np.maximum(ids, 0)] if remap.size else -1, -1)
            self.columns.append(c)
            self.col_of[path] = i
        self.live = np.zeros(cap, dtype=np.int32)
        self.live[:n] = 1
        self.seq = np.zeros(cap, dtype=np.int64)
        self.seq[:n] = seqs
        self._next_seq = int(seqs.max()) if n else 0
        if isinstance(keys, tuple):  # (blob, offsets) from DocStore.encode_columns
            self.keys = KeyTable(keys[0], np.asarray(keys[1], dtype=np.int64))
        else:
            self.keys = list(keys)
        self._row_of = None  # built on the first write (read-only use never needs it)
        self.n = n
        self.version += 1
        self._full_dirty = True
        self._tomb_dirty = False
        self._zones_reset()

    # -- native mirror (DocStore column mirror, native/src/docstore.hpp) ---------------
    @classmethod
    def from_native(cls, store, paths: Iterable[str]) -> "ColumnarIndex":
        """Index fed by the document store's own column mirror: the store appends a row per
        write in C++ (the native HTTP front never hands writes to Python), and ``sync`` pulls
        only what changed since the last sync (new rows, new dictionary values, killed rows).
        Rows map back to documents through ``store.mirror_results``."""
        ix = cls()
        ix.native = store
        ix.docs = None
        ix._ncur = (0, 0, 0)  # (generation, rows seen, kill-log position)
        # per column: native dictionary id -> this index's id, in a capacity-doubled buffer
        # (``_remap_n`` entries used): a sync appends the new values' ids in place instead of
        # copying the whole map (taskCreatedOn's grows by one per write)
        ix._remap: list[np.ndarray] = []
        ix._remap_n: list[int] = []
        if not store.mirror_enable(list(dict.fromkeys(paths))):
            raise Unsupported("collection cannot be mirrored (TTL writes)")
        ix.sync()
        return ix

    def sync(self) -> bool:
        """Apply the native mirror's changes; returns True when anything changed."""
        gen, rows, kc = self._ncur
        d = self.native.mirror_delta(gen, rows, kc, list(self._remap_n))
        if d["disabled"] or not d["on"]:
            raise Unsupported("collection mirror disabled (TTL writes)")
        lo, hi = int(d["from"]), int(d["n"])
        changed = d["full"] or hi > lo or d["kills"].size > 0
        if d["full"]:
            self.columns, self.col_of, self._remap, self._remap_n = [], {}, [], []
            for path, *_ in d["columns"]:
                self.col_of[path] = len(self.columns)
                self.columns.append(Column(path))
                self._remap.append(np.zeros(0, dtype=np.int32))
                self._remap_n.append(0)
            self.cap = max(TILE, (hi + TILE - 1) // TILE * TILE)
            self.ids = np.full((len(self.columns), self.cap), -1, dtype=np.int32)
            self.live = np.zeros(self.cap, dtype=np.int32)
            self.seq = np.zeros(self.cap, dtype=np.int64)
            self.n, self._next_seq = 0, 0
            self._dict_gen += 1
            self._full_dirty = True
            self.keys = []
        assert lo == self.n, (lo, self.n)
        self._grow(hi)
        for c, (path, dict_from, values, ids, all_str) in enumerate(d["columns"]):
            col = self.columns[c]
            if values:  # new dictionary values, mapped onto Python's equality (vkey)
                add = col.encode_json_many(values, all_str)
                need = dict_from + add.size
                buf = self._remap[c]
                if buf.size < need:
                    grown = np.empty(max(need, 2 * buf.size, 1024), dtype=np.int32)
                    grown[:dict_from] = buf[:dict_from]
                    buf = self._remap[c] = grown
                buf[dict_from:need] = add
                self._remap_n[c] = need
            rm = self._remap[c][:self._remap_n[c]]
            if hi > lo:
                self.ids[c, lo:hi] = np.where(ids >= 0, rm[np.maximum(ids, 0)] if rm.size else -1, -1)
        if hi > lo:
            self.seq[lo:hi] = d["seqs"]
            self.live[lo:hi] = d["live"]
            self._next_seq = max(self._next_seq, int(d["seqs"].max()))
            self._zones_touch(np.arange(lo // TILE, (hi - 1) // TILE + 1))
        if d["kills"].size:
            self.live[d["kills"].astype(np.int64)] = 0
            self._tomb_dirty = True
            self._zones_touch(np.unique(d["kills"].astype(np.int64) // TILE))
        if d["full"]:
            self._zones_reset()
        self.n = hi
        self._ncur = (int(d["gen"]), hi, int(d["kill_cursor"]))
        if changed:
            self.version += 1
        return bool(changed)

    @property
    def generation(self) -> int:
        """Mirror generation the row numbers belong to (``DocStore.mirror_results`` checks it)."""
        return int(self._ncur[0]) if getattr(self, "native", None) is not None else 0

    @property
    def row_of(self) -> dict[str, int]:
        if self._row_of is None:
            self._row_of = {self.keys[r]: r for r in np.nonzero(self.live[:self.n])[0].tolist()}
        return self._row_of

    def ensure_columns(self, paths: Iterable[str]) -> None:
        """Add every missing column at once (one re-encode for a source-backed index)."""
        missing = [p for p in dict.fromkeys(paths) if p not in self.col_of]
        if not missing:
            return
        if getattr(self, "native", None) is not None:
            if not self.native.mirror_enable([c.path for c in self.columns] + missing):
                raise Unsupported("collection mirror disabled (TTL writes)")
            self.sync()  # a new column is a new mirror generation: full reload
        elif self.docs is None:
            self._load([c.path for c in self.columns] + missing)
        else:
            for p in missing:
                self.add_column(p)

    # -- zone maps (paged device path) ---------------------------------------------------
    def _zones_touch(self, tiles) -> None:
        for z in self._zones.values():
            if not z["all"]:
                z["dirty"].update(int(t) for t in tiles)

    def _zones_reset(self) -> None:
        for z in self._zones.values():
            z["all"], z["dirty"] = True, set()

    # -- maintenance ----------------------------------------------------------
    def add_column(self, path: str) -> int:
        if path in self.col_of:
            return self.col_of[path]
        if self.docs is None:
            self.ensure_columns([path])
            return self.col_of[path]
        c = Column(path)
        idx = len(self.columns)
        self.columns.append(c)
        self.col_of[path] = idx
        col = np.full((1, self.cap), -1, dtype=np.int32)
        for r in range(self.n):
            if self.live[r]:
                col[0, r] = c.encode(get_path(self.docs[r], path))
        self.ids = np.concatenate([self.ids, col], axis=0)
        self.version += 1
        self._full_dirty = True
        return idx

    def _grow(self, need: int) -> None:
        if need <= self.cap:
            return
        cap = self.cap
        while cap < need:
            cap *= 2
        ids = np.full((len(self.columns), cap), -1, dtype=np.int32)
        ids[:, :self.n] = self.ids[:, :self.n]
        live = np.zeros(cap, dtype=np.int32)
        live[:self.n] = self.live[:self.n]
        seq = np.zeros(cap, dtype=np.int64)
        seq[:self.n] = self.seq[:self.n]
        self.ids, self.live, self.seq, self.cap = ids, live, seq, cap
        self._full_dirty = True

    def upsert(self, key: str, doc: Any) -> None:
        old = self.row_of.get(key)
        if old is not None:
            self.live[old] = 0
            if self.docs is not None:
                self.docs[old] = None
            self._tomb_dirty = True
            self._dead += 1
            seq = int(self.seq[old])  # an update keeps the key's original position (native engine semantics)
        else:
            self._next_seq += 1
            seq = self._next_seq
        self._grow(self.n + 1)
        r = self.n
        self.seq[r] = seq
        for i, c in enumerate(self.columns):
            self.ids[i, r] = c.encode(get_path(doc, c.path))
        self.live[r] = 1
        self.keys.append(key)
        if self.docs is not None:
            self.docs.append(doc)
        self.row_of[key] = r
        self.n += 1
        self.version += 1
        self._zones_touch([r // TILE] if old is None else [r // TILE, old // TILE])
        self._maybe_compact()

    def delete(self, key: str) -> None:
        r = self.row_of.pop(key, None)
        if r is not None:
            self.live[r] = 0
            if self.docs is not None:
                self.docs[r] = None
            self._tomb_dirty = True
            self._dead += 1
            self.version += 1
            self._zones_touch([r // TILE])
        self._maybe_compact()

    def _maybe_compact(self) -> None:
        """Keep the index proportional to the live documents, not to the number of writes."""
        if self._dead > TILE and self._dead * 2 > self.n:
            self.compact()

    def bulk_load(self, items: Iterable[tuple[str, Any]]) -> None:
        for k, d in items:
            self.upsert(k, d)

    def live_rows(self) -> int:
        return int(np.count_nonzero(self.live[:self.n]))

    def compact(self) -> None:
        """Drop tombstones (rows are renumbered in order)."""
        keep = np.nonzero(self.live[:self.n])[0]
        self.ids[:, :len(keep)] = self.ids[:, keep]
        self.ids[:, len(keep):] = -1
        self.seq[:len(keep)] = self.seq[keep]
        self.live[:] = 0
        self.live[:len(keep)] = 1
        self.keys = [self.keys[i] for i in keep.tolist()]
        if self.docs is not None:
            self.docs = [self.docs[i] for i in keep]
        self._row_of = {k: i for i, k in enumerate(self.keys)}
        self.n = len(keep)
        self._dead = 0
        self.version += 1
        self._full_dirty = True
        self._zones_reset()

    # -- compilation ---------------------------------------------------------
    def _dict_state(self) -> tuple:
        return (self._dict_gen,) + tuple((len(c.values), c.rank_version) for c in self.columns)

    def compile_cached(self, flt: Any) -> Program:
        """``compile`` memoised per filter and the dictionary state of the columns it reads
        (queries repeat: the cron sweep, the same creator's list page) -- not of every column:
        the sort key's dictionary (``taskCreatedOn``, one value per write) grows between any two
        sweeps and would otherwise recompile, and re-upload, the same program every time.
        Bounded, oldest entries dropped."""
        fj = json.dumps(flt, sort_keys=True, default=str)
        cols = [self.col_of.get(p) for p in filter_paths(flt)]
        if any(c is None for c in cols):  # compile adds the column: key on everything this once
            state = self._dict_state()
        else:
            state = (self._dict_gen,) + tuple((c, len(self.columns[c].values), self.columns[c].rank_version)
                                              for c in sorted(set(cols)))
        key = (fj, state)
        prog = self._prog_cache.get(key)
        if prog is None:
            prog = self.compile(flt)
            if len(self._prog_cache) >= 128:
                self._prog_cache.pop(next(iter(self._prog_cache)))
            self._prog_cache[key] = prog
        return prog

    def compile(self, flt: Any) -> Program:
        code: list[list[int]] = []
        words: list[np.ndarray] = []
        nwords = [0]
        used: list[int] = []
        depth = [0, 0]

        def push() -> None:
            depth[0] += 1
            depth[1] = max(depth[1], depth[0])

        def leaf_bitmap(col: int, sat: np.ndarray) -> None:
            nbits = len(sat)
            padded = np.zeros(((nbits + 31) // 32) * 32, dtype=bool)
            padded[:nbits] = sat
            w = np.packbits(padded, bitorder="little").view("<u4").astype(np.uint32)
            if w.size == 0:
                w = np.zeros(1, dtype=np.uint32)
            code.append([OP_LEAF, col, nwords[0], nbits])
            words.append(w)
            nwords[0] += w.size
            push()

        def emit(f: Any) -> None:
            if not isinstance(f, dict) or len(f) != 1:
                raise Unsupported("filter node must be a single-operator object")
            (op, arg), = f.items()
            op = op.upper()
            if op in ("AND", "OR"):
                if not isinstance(arg, list) or not arg:
                    raise Unsupported(f"{op} expects a non-empty array")
                for x in arg:
                    emit(x)
                n = len(arg)
                if n > 1:
                    code.append([OP_AND if op == "AND" else OP_OR, n, 0, 0])
                    depth[0] -= n - 1
                return
            if not isinstance(arg, dict) or len(arg) != 1:
                raise Unsupported(f"{op} expects {{path: value}}")
            (path, val), = arg.items()
            col = self.col_of.get(path)
            if col is None:
                col = self.add_column(path)
            used.append(col)
            c = self.columns[col]
            if op in ("EQ", "NEQ"):
                if isinstance(val, (list, dict)):
                    raise Unsupported("structured equality")
                code.append([OP_EQ, col, c.lookup(val), 0])
                push()
                if op == "NEQ":
                    code.append([OP_NOT, 0, 0, 0])
            elif op == "IN":
                if not isinstance(val, list):
                    raise Unsupported("IN expects a list")
                leaf_bitmap(col, c.satisfying("IN", val))
            elif op in ("GT", "GTE", "LT", "LTE"):
                sat = c.satisfying(op, val)
                rng = rank_interval(c, sat)
                if rng is None:
                    leaf_bitmap(col, sat)
                else:  # one integer compare per row on the rank-encoded column
                    code.append([OP_RANGE, col, rng[0], rng[1]])
                    push()
            else:
                raise Unsupported(f"operator {op}")

        if not flt:
            code.append([OP_TRUE, 0, 0, 0])
            push()
        else:
            emit(flt)
        if depth[1] > MAX_DEPTH:
            raise Unsupported("filter nesting too deep for the device stack")
        bitmaps = np.concatenate(words) if words else np.zeros(1, dtype=np.uint32)
        return Program(np.asarray(code, dtype=np.int32), bitmaps.view(np.int32), sorted(set(used)))

    # -- execution -------------------------------------------------------------
    def select_numpy(self, prog: Program) -> np.ndarray:
        """Reference executor: identical semantics to the HIP kernel."""
        n = self.n
        stack: list[np.ndarray] = []
        bm = prog.bitmaps.view(np.uint32)
        for op, a, b, c in prog.code.tolist():
            if op == OP_EQ:
                stack.append(self.ids[a, :n] == b)
            elif op == OP_RANGE:
                v = self.ids[a, :n]
                ranks = self.columns[a].ranks()
                r = np.where(v >= 0, ranks[np.maximum(v, 0)] if ranks.size else -1, -1)
                stack.append((r >= b) & (r < c))
            elif op == OP_LEAF:
                v = self.ids[a, :n]
                ok = (v >= 0) & (v < c)
                vv = np.where(ok, v, 0)
                bits = (bm[b + (vv >> 5)] >> (vv & 31).astype(np.uint32)) & 1
                stack.append(ok & (bits == 1))
            elif op in (OP_AND, OP_OR):
                xs = stack[-a:]
                del stack[-a:]
                r = xs[0].copy()
                for x in xs[1:]:
                    r = (r & x) if op == OP_AND else (r | x)
                stack.append(r)
            elif op == OP_NOT:
                stack[-1] = ~stack[-1]
            else:
                stack.append(np.ones(n, dtype=bool))
        sel = stack[-1] & (self.live[:n] != 0)
        return np.nonzero(sel)[0].astype(np.int32)

    def select_native(self, prog: Program, threads: int | None = None, simd: bool = True) -> np.ndarray:
        """The program on the host's CPU share (``native/src/cpuscan.hpp``): every core, SIMD
        compares, over the same narrow codes / rank copies / liveness bits the GPU kernels read
        -- the fair CPU baseline for ``select_gpu`` and the executor without a GPU.  Same result
        as ``select_numpy`` (the reference)."""
        from ..native import load
        hm = self._host_mirror(prog)
        code = prog.code
        rng = code[:, 0] == OP_RANGE
        if rng.any():  # range leaves read the rank-encoded copy of their column
            code = code.copy()
            code[rng, 1] = [hm["rank_slot"][c] for c in prog.code[rng, 1].tolist()]
        return load().scan_select(hm["cols"], hm["live"], self.n, np.ascontiguousarray(code, dtype=np.int32),
                                  prog.bitmaps.view(np.uint32), threads or cpu_share(), simd)

    def _host_mirror(self, prog: Program) -> dict:
        """Host copies of the columns in the device layout (narrow codes, rank-encoded copies for
        the program's range leaves, 1-bit liveness), rebuilt when the index changed."""
        key = (self.version, self.n, self.cap, self._dict_state())
        hm = getattr(self, "_host", None)
        if hm is None or hm["key"] != key:
            widths = [self.width_for(len(c.values)) for c in self.columns]
            hm = self._host = {"key": key, "widths": widths, "ranks": {},
                               "cols": [(np.ascontiguousarray(self._narrow(i, 0, self.cap, w)).view(np.uint8), w)
                                        for i, w in enumerate(widths)],
                               "live": np.ascontiguousarray(self._live_words(0, self.cap // 16)).view(np.uint16)}
        rank_cols = sorted(set(prog.code[prog.code[:, 0] == OP_RANGE, 1].tolist()))
        slots = {}
        cols = list(hm["cols"][:len(self.columns)])
        for col in rank_cols:
            r = hm["ranks"].get(col)
            if r is None:
                w = max(1, hm["widths"][col])
                table = self.columns[col].ranks()
                v = self.ids[col, :self.cap]
                rk = np.where(v >= 0, table[np.maximum(v, 0)] if table.size else -1, -1)
                dt = np.uint8 if w == 1 else np.uint16 if w == 2 else np.int32
                rk = np.where(rk < 0, np.iinfo(dt).max if w < 4 else -1, rk).astype(dt)
                r = hm["ranks"][col] = (np.ascontiguousarray(rk).view(np.uint8), w)
            slots[col] = len(cols)
            cols.append(r)
        return {"cols": cols, "live": hm["live"], "rank_slot": slots}

    # device mirror -------------------------------------------------------------
    @staticmethod
    def width_for(dict_size: int) -> int:
        """Code width of a column whose dictionary has ``dict_size`` ids (all-ones = missing):
        0 = 2 bits per row (<= 3 ids: booleans, with or without null), else bytes per row."""
        return 0 if dict_size <= 3 else 1 if dict_size <= 254 else 2 if dict_size <= 65534 else 4

    @staticmethod
    def col_bytes(rows: int, width: int) -> int:
        return rows // 4 if width == 0 else rows * width

    def _narrow(self, col: int, lo: int, hi: int, width: int) -> np.ndarray:
        """Codes of rows [lo, hi) in the device layout (width 0: ``lo``/``hi`` multiples of 4,
        four rows per byte, row r in bits 2(r mod 4))."""
        v = self.ids[col, lo:hi]
        if width == 4:
            return v
        if width == 0:
            c = np.where(v < 0, 3, v).astype(np.uint8).reshape(-1, 4)
            return c[:, 0] | (c[:, 1] << 2) | (c[:, 2] << 4) | (c[:, 3] << 6)
        dt = np.uint8 if width == 1 else np.uint16
        return np.where(v < 0, np.iinfo(dt).max, v).astype(dt)

    def _device_codes(self, col: int, width: int) -> np.ndarray:
        """The whole column in the device layout; 2-bit columns get 16 bytes of padding (the
        reads past the end of a partial group stay inside the buffer)."""
        v = self._narrow(col, 0, self.cap, width)
        if width == 0:
            v = np.concatenate([v, np.zeros(16, dtype=np.uint8)])
        return np.ascontiguousarray(v)

    def _live_words(self, lo_word: int, hi_word: int) -> np.ndarray:
        bits = self.live[lo_word * 16:hi_word * 16].astype(np.uint8)
        return np.packbits(bits, bitorder="little").view("<u2").view(np.int16)

    def to_device(self, kernels, rank_cols=()):
        """Sync the device mirror.  Columns are append-only between compactions, so only rows
        added since the last sync are uploaded; tombstones re-upload the 1-bit liveness mask
        (N/8 bytes); a column whose dictionary outgrows its width is re-encoded."""
        torch = kernels.torch
        dev = kernels.device
        st = self._dev
        widths = [self.width_for(len(c.values)) for c in self.columns]
        nwords = self.cap // 16
        if st is None or self._full_dirty or st["cap"] != self.cap or len(st["cols"]) != len(self.columns):
            if self._full_dirty:
                self._zones_reset()
            cols = [torch.from_numpy(self._device_codes(i, w)).to(dev) for i, w in enumerate(widths)]
            live = torch.from_numpy(self._live_words(0, nwords)).to(dev)
            seq = torch.from_numpy(self.seq[:self.cap].astype(np.int32)).to(dev)  # uint32 on device
            st = self._dev = {"cols": cols, "widths": widths, "live": live, "synced": self.n, "cap": self.cap,
                              "seq": seq}
        else:
            lo, hi = st["synced"], self.n
            # the appended rows of every column, the sequence and the liveness words go up in
            # one scatter launch (GpuKernels.upload), not one copy each
            segs = []
            for i, w in enumerate(widths):
                if w != st["widths"][i]:
                    st["cols"][i] = torch.from_numpy(self._device_codes(i, w)).to(dev)
                    st["widths"][i] = w
                elif hi > lo and w == 0:  # whole bytes of 4 rows: re-pack the edge bytes
                    a, b = lo // 4, (hi + 3) // 4
                    segs.append((st["cols"][i].data_ptr() + a, self._narrow(i, 4 * a, 4 * b, 0)))
                elif hi > lo:
                    segs.append((st["cols"][i].data_ptr() + lo * w, self._narrow(i, lo, hi, w)))
            if hi > lo:
                segs.append((st["seq"].data_ptr() + 4 * lo, self.seq[lo:hi].astype(np.int32)))
            if self._tomb_dirty:
                segs.append((st["live"].data_ptr(), self._live_words(0, nwords)))
            elif hi > lo:
                w0, w1 = lo // 16, (hi + 15) // 16
                segs.append((st["live"].data_ptr() + 2 * w0, self._live_words(w0, w1)))
            kernels.upload(segs)
            st["synced"] = hi
        self._full_dirty = False
        self._tomb_dirty = False
        rows = [[c.data_ptr(), w] for c, w in zip(st["cols"], st["widths"])]
        if rank_cols:
            # rank-encoded copies of the columns that range leaves read (appended to the table)
            ranks = st.setdefault("ranks", {})
            slot = {}
            for col in sorted(set(rank_cols)):
                self._sync_rank_column(kernels, st, ranks, col)
                slot[col] = len(rows)
                rows.append([ranks[col]["t"].data_ptr(), ranks[col]["w"]])
            st["rank_slot"] = slot
        # the descriptor table only changes with the device buffers: no upload per query
        st["table_widths"] = np.array([w for _, w in rows], dtype=np.int64)
        tkey = tuple(tuple(r) for r in rows)
        tables = st.setdefault("tables", {})
        t = tables.get(tkey)
        if t is None:
            if len(tables) >= 16:
                tables.clear()
            t = tables[tkey] = torch.from_numpy(np.array(rows, dtype=np.int64).reshape(-1, 2)).to(dev)
        st["table"] = t
        return st

    def _sync_rank_column(self, kernels, st, ranks, col: int) -> None:
        torch = kernels.torch
        c = self.columns[col]
        w = max(1, st["widths"][col])  # ranks run 1..n and need a distinct missing code: >= 1 byte
        cur = ranks.get(col)
        full = cur is None or cur["w"] != w or cur["ver"] != c.rank_version
        lo = 0 if full else cur["synced"]
        if not full and lo >= self.n:
            return
        segs = []  # the rank table and the source descriptor: one scatter launch, no copies
        if full:
            dt = {1: torch.uint8, 2: torch.int16, 4: torch.int32}[w]
            prev = cur
            # re-encoded from row 0 into the same buffer when it still fits: its address is in
            # the column descriptor table, which then needs no new upload
            keep = prev is not None and prev["w"] == w and prev["t"].numel() == self.cap
            cur = ranks[col] = {"t": prev["t"] if keep else torch.empty(self.cap, dtype=dt, device=kernels.device),
                                "w": w, "ver": c.rank_version, "table": None, "synced": 0}
            table = c.ranks().astype(np.int32) if c.values else np.zeros(1, dtype=np.int32)
            # a new dictionary value re-ranks the column (every new due date does): the table's
            # device buffer is kept across versions and grown by doubling
            buf = prev.get("table_buf") if prev is not None else None
            if buf is None or buf.numel() < table.size:
                buf = torch.empty(max(1024, 1 << (table.size - 1).bit_length()), dtype=torch.int32,
                                  device=kernels.device)
            cur["table_buf"], cur["table"] = buf, buf[:table.size]
            segs.append((buf.data_ptr(), table))
            if prev is not None and "src" in prev:
                cur["src"], cur["src_key"] = prev["src"], prev["src_key"]
        key = (st["cols"][col].data_ptr(), st["widths"][col])
        if cur.get("src_key") != key:  # the source column's descriptor: uploaded when it changes
            if "src" not in cur:
                cur["src"] = torch.empty((1, 2), dtype=torch.int64, device=kernels.device)
            segs.append((cur["src"].data_ptr(), np.array([list(key)], dtype=np.int64)))
            cur["src_key"] = key
        kernels.upload(segs)
        kernels.rank_encode(cur["src"], cur["table"], lo, self.n, cur["t"], w)
        cur["synced"] = self.n

    def device_program(self, prog: Program, kernels):
        """Sync the device mirror for ``prog`` and return (state, program, bitmaps) ready for
        ``GpuKernels.select`` (range leaves remapped to their rank-encoded columns)."""
        leaf = (prog.code[:, 0] == OP_LEAF) | (prog.code[:, 0] == OP_EQ) | (prog.code[:, 0] == OP_RANGE)
        if leaf.any() and int(prog.code[leaf, 1].max()) >= len(self.columns):
            raise ValueError("program references a column outside the index")
        rng = prog.code[:, 0] == OP_RANGE
        self._warm_rank_cols = prog.code[rng, 1].tolist()
        st = self.to_device(kernels, self._warm_rank_cols)
        slots = tuple(sorted(st.get("rank_slot", {}).items())) if rng.any() else ()
        cached = getattr(prog, "_dev", None)
        if cached is not None and cached[0] == (slots, str(kernels.device)):
            return st, cached[1], cached[2]
        code_np = prog.code
        if rng.any():  # range leaves read the rank-encoded copy of their column
            code_np = prog.code.copy()
            code_np[rng, 1] = [st["rank_slot"][c] for c in prog.code[rng, 1].tolist()]
        code = kernels.torch.from_numpy(code_np).to(kernels.device)
        bitmaps = kernels.torch.from_numpy(prog.bitmaps).to(kernels.device)
        prog._dev = ((slots, str(kernels.device)), code, bitmaps)  # reused while the program is
        return st, code, bitmaps

    def select_gpu(self, prog: Program, kernels, return_mask: bool = False, on_device: bool = False):
        st, code, bitmaps = self.device_program(prog, kernels)
        res = kernels.select(st["table"], st["live"], self.cap, self.n, code, bitmaps, return_mask=return_mask)
        if return_mask or on_device:
            return res
        return res.cpu().numpy()

    def group_count_gpu(self, prog: Program, group_path: str, kernels) -> dict[str, int]:
        g = self.add_column(group_path)
        _, mask = self.select_gpu(prog, kernels, return_mask=True)
        col = self.columns[g]
        if mask is None or not col.values:
            return {}
        counts = kernels.group_count(self._dev["table"], g, mask, self.n, len(col.values)).cpu().numpy()
        return {json.dumps(col.values[i]): int(x) for i, x in enumerate(counts) if x}

    def group_count_numpy(self, prog: Program, group_path: str) -> dict[str, int]:
        g = self.add_column(group_path)
        rows = self.select_numpy(prog)
        col = self.columns[g]
        ids = self.ids[g, rows]
        ids = ids[ids >= 0]
        cnt = np.bincount(ids, minlength=len(col.values))
        return {json.dumps(col.values[i]): int(x) for i, x in enumerate(cnt) if x}

    # -- full query --------------------------------------------------------------
    def order(self, rows: np.ndarray, sort: list[dict[str, Any]] | None, k: int | None = None) -> np.ndarray:
        """``rows`` in result order; with ``k``, only the first ``k`` of that order (a page: one
        partition of the packed keys, then a sort of those ``k``, instead of a full sort)."""
        if rows.size == 0:
            return rows
        plan = self.sort_specs(sort)
        if plan is not None:  # packed keys (the ones the GPU path sorts; unique: seq is the tail)
            keys = self.sort_keys_numpy(rows, plan)
            if k is not None and 0 < k < rows.size:
                part = np.argpartition(keys, k - 1)[:k]
                return rows[part[np.argsort(keys[part])]]
            return rows[np.argsort(keys, kind="stable")]
        out = self.order_lexsort(rows, sort)
        return out[:k] if k else out

    def order_lexsort(self, rows: np.ndarray, sort: list[dict[str, Any]] | None) -> np.ndarray:
        """Reference ordering: insertion order, then a stable lexsort on the sort keys' ranks."""
        if rows.size == 0:
            return rows
        rows = rows[np.argsort(self.seq[rows], kind="stable")]  # insertion order, then stable sort keys
        if not sort:
            return rows
        keys = []
        for s in reversed(sort):  # np.lexsort: last key is primary
            col = self.add_column(s["key"])
            ranks = self.columns[col].ranks()
            ids = self.ids[col, rows]
            miss = self.columns[col].missing_rank()
            r = np.where(ids >= 0, ranks[np.maximum(ids, 0)] if ranks.size else miss, miss)
            if str(s.get("order", "ASC")).upper() == "DESC":
                r = -r
            keys.append(r)
        return rows[np.lexsort(keys)]

    def sort_specs(self, sort: list[dict[str, Any]] | None) -> tuple[np.ndarray, np.ndarray, int] | None:
        """Device ordering plan: (specs int32 [nkeys, 8], concatenated rank tables, seq bits), or
        None when the packed key would not fit 63 bits (the host path orders instead)."""
        seq_bits = max(1, int(self._next_seq).bit_length())  # every seq is <= the last one handed out
        specs, tables, off, total = [], [], 0, seq_bits
        for s in sort or []:
            col = self.add_column(s["key"])
            c = self.columns[col]
            ranks = c.ranks().astype(np.int32) if c.values else np.zeros(0, dtype=np.int32)
            miss = c.missing_rank()
            max_rank = int(max(int(ranks.max(initial=0)), miss))
            bits = max(1, max_rank.bit_length())
            total += bits
            desc = 1 if str(s.get("order", "ASC")).upper() == "DESC" else 0
            specs.append([col, off, ranks.size, bits, desc, miss, max_rank, 0])
            tables.append(ranks)
            off += ranks.size
        if total > 63:
            return None
        spec_arr = np.array(specs, dtype=np.int32).reshape(-1, 8)
        rank_arr = np.concatenate(tables) if tables else np.zeros(1, dtype=np.int32)
        return spec_arr, (rank_arr if rank_arr.size else np.zeros(1, dtype=np.int32)), seq_bits

    def sort_keys_numpy(self, rows: np.ndarray, plan) -> np.ndarray:
        """Host reference of ``hip/sort_keys.hip``: the packed ordering key of every row."""
        specs, ranks, seq_bits = plan
        k = np.zeros(rows.size, dtype=np.int64)
        for col, off, nranks, bits, desc, miss, max_rank, _ in specs.tolist():
            ids = self.ids[col, rows]
            ok = (ids >= 0) & (ids < nranks)
            r = np.full(rows.size, miss, dtype=np.int64)
            r[ok] = ranks[off + ids[ok]]
            if desc:
                r = max_rank - r
            k = (k << bits) | r
        return (k << seq_bits) | self.seq[rows]

    def _device_sort_plan(self, sort, kernels):
        """(specs, rank tables, seq bits, key bits) on the device and the host plan of the same
        packed key, kept per sort spec; None when the device cannot order by it (too many keys,
        a key over 63 bits, a sequence over 32 bits).

        The rank tables live in one buffer, one capacity-doubled region per sort key, on the
        device and (for ``sort_keys_numpy``) on the host.  Only the ids whose rank is new or moved
        since the last query are copied (``Column.rank_changes_since``): for the timestamps of
        new writes, which arrive nearly in order, those are the newest ids -- O(new values) per
        query instead of re-uploading the whole table (``taskCreatedOn`` has one value per
        task)."""
        if len(sort or []) > kernels.max_sort_keys:
            return None
        tm = self._plan_tm  # page_gpu's timing dict while it plans (None for the background warm)
        c0 = time.thread_time()
        cols = [self.add_column(srt["key"]) for srt in sort or []]
        seq_bits = max(1, int(self._next_seq).bit_length())
        if seq_bits > 32:
            return None  # the device keeps a 32-bit insertion sequence
        torch = kernels.torch
        pkey = (json.dumps(sort, sort_keys=True, default=str), str(kernels.device), self._dict_gen)
        ent = self._plan_cache.get(pkey)
        tables, specs_rows, total = [], [], seq_bits
        for srt, col in zip(sort or [], cols):
            c = self.columns[col]
            r = c.ranks() if c.values else np.zeros(0, dtype=np.int64)
            miss = c.missing_rank()
            max_rank = len(c.values) if c.str_only else int(r.max(initial=0))
            max_rank = max(max_rank, miss)
            bits = max(1, max_rank.bit_length())
            total += bits
            desc = 1 if str(srt.get("order", "ASC")).upper() == "DESC" else 0
            tables.append((r, c))
            specs_rows.append([col, 0, r.size, bits, desc, miss, max_rank, 0])
        if total > 63:
            return None
        los = [None] * len(tables) if ent is None else \
            [c.rank_changes_since(sq) for (_, c), sq in zip(tables, ent["seqs"])]
        rebuild = ent is None or any(lo is None for lo in los) or \
            any(r.size > cap for (r, _), cap in zip(tables, ent["caps"]))
        c1 = time.thread_time()
        if tm is not None:
            tm["plan_ranks_ms"] = tm.get("plan_ranks_ms", 0.0) + (c1 - c0) * 1e3
            tm["plan_rebuilds"] = tm.get("plan_rebuilds", 0) + int(rebuild)
        if rebuild:
            caps = [max(1024, 1 << max(0, int(r.size * 1.25) + 1).bit_length()) for r, _ in tables]
            offs = np.concatenate([[0], np.cumsum(caps)[:-1]]).astype(np.int64) if caps else np.zeros(0, np.int64)
            host = np.zeros(max(1, int(sum(caps))), dtype=np.int32)
            for (r, _), off in zip(tables, offs):
                host[off:off + r.size] = r
            ent = {"caps": caps, "offs": offs, "seqs": [c.rank_seq for _, c in tables],
                   "host": host, "dev": torch.from_numpy(host).to(kernels.device), "specs": None,
                   "specs_dev": torch.empty((len(specs_rows), 8), dtype=torch.int32, device=kernels.device)}
            if len(self._plan_cache) >= 64:
                self._plan_cache.pop(next(iter(self._plan_cache)))
            self._plan_cache[pkey] = ent
        segs = []  # rank tails and the spec rows: one scatter launch (ops/gpu.py upload)
        if not rebuild:
            for i, ((r, c), lo) in enumerate(zip(tables, los)):
                off = int(ent["offs"][i])
                if r.size > lo:  # the ids whose rank is new or moved (the newest ones)
                    tail = r[lo:].astype(np.int32)
                    ent["host"][off + lo:off + r.size] = tail
                    segs.append((ent["dev"].data_ptr() + 4 * (off + lo), tail))
                ent["seqs"][i] = c.rank_seq
        for row, off in zip(specs_rows, ent["offs"]):
            row[1] = int(off)
        specs = np.array(specs_rows, dtype=np.int32).reshape(-1, 8)
        if ent["specs"] is None or not np.array_equal(specs, ent["specs"]):
            # the spec rows change with every new dictionary value (row[2] is the table's size):
            # they ride the same launch into a buffer allocated once per plan
            ent["specs"] = specs
            segs.append((ent["specs_dev"].data_ptr(), specs))
        c2 = time.thread_time()
        kernels.upload(segs)
        if tm is not None:
            c3 = time.thread_time()
            tm["plan_tails_ms"] = tm.get("plan_tails_ms", 0.0) + (c2 - c1) * 1e3
            tm["plan_upload_ms"] = tm.get("plan_upload_ms", 0.0) + (c3 - c2) * 1e3
            tm["plan_tail_rows"] = tm.get("plan_tail_rows", 0) + sum(int(t.size) for _, t in segs)
        key_bits = seq_bits + int(specs[:, 3].sum()) if specs.size else seq_bits
        return ent["specs_dev"], ent["dev"], seq_bits, key_bits, (specs, ent["host"], seq_bits)

    def order_gpu(self, rows, sort, kernels, k: int | None = None):
        """Order a device selection on the GPU (``hip/sort_keys.hip`` + radix sort / top-k);
        returns device rows, or None when the host path must order."""
        hit = self._device_sort_plan(sort, kernels)
        if hit is None:
            return None
        specs_t, ranks_t, seq_bits, key_bits, _ = hit
        st = self.to_device(kernels)  # sort keys may have added columns
        return kernels.order(st["table"], rows, specs_t, ranks_t, st["seq"], seq_bits, k, key_bits)

    def _zone_refresh(self, z: dict, kernels, st: dict, specs_t, ranks_t, seq_bits: int) -> None:
        """Recompute the zone argmin of the tiles that changed since the last refresh."""
        ntiles = (self.n + TILE - 1) // TILE
        if z["zarg"].size < ntiles:  # new tiles: not computed yet
            z["dirty"].update(range(z["zarg"].size, ntiles))
            z["zarg"] = np.concatenate([z["zarg"], np.full(ntiles - z["zarg"].size, -1, dtype=np.int32)])
        z["zarg"] = z["zarg"][:ntiles]
        todo = np.arange(ntiles, dtype=np.int32) if z["all"] else \
            np.fromiter((t for t in z["dirty"] if t < ntiles), dtype=np.int32)
        if todo.size:
            z["zarg"][todo] = kernels.zone_argmin(st["table"], st["live"], self.n, specs_t, ranks_t, st["seq"],
                                                  seq_bits, todo)
        z["all"], z["dirty"] = False, set()

    def warm(self, kernels) -> None:
        """Bring the device mirror up to the host index between queries: upload the rows
        synced since the last query (with the rank-encoded columns the last queries read) and
        refresh the zone maps of the sorts already served, so a query finds little to do.
        Called by the accelerator's background sync (backing/accel.py) under its lock."""
        st = self.to_device(kernels, getattr(self, "_warm_rank_cols", ()))
        for z in list(self._zones.values()):
            if z["all"] or z["dirty"] or z["zarg"].size < (self.n + TILE - 1) // TILE:
                hit = self._device_sort_plan(z["sort"], kernels)
                if hit is not None:
                    self._zone_refresh(z, kernels, st, hit[0], hit[1], hit[2])

    def page_gpu(self, prog: Program, sort, kernels, offset: int, limit: int):
        """A page [offset, offset + limit) of an ordered query without scanning the collection
        (``hip/page_topk.hip``): zone maps pick the tiles that can hold the page, only those are
        evaluated, one workgroup orders the candidates.  Returns (rows, token) or None when the
        page does not fit the device top-k (the caller takes the full path)."""
        k_total = offset + limit
        if limit <= 0 or k_total > kernels.page_cap:
            return None
        tm = self.timing
        t0, c0 = time.perf_counter(), time.thread_time()
        self._plan_tm = tm
        try:
            hit = self._device_sort_plan(sort, kernels)
        finally:
            self._plan_tm = None
        if hit is None:
            return None
        specs_t, ranks_t, seq_bits, _, plan = hit
        t1 = time.perf_counter()
        st, code, bitmaps = self.device_program(prog, kernels)
        t2, c2 = time.perf_counter(), time.thread_time()
        tm["page_plan_ms"] = tm.get("page_plan_ms", 0.0) + (t1 - t0) * 1e3
        tm["page_program_ms"] = tm.get("page_program_ms", 0.0) + (t2 - t1) * 1e3
        # this thread's CPU time in plan + program: the wall time above less the waits (GIL,
        # other threads on the core)
        tm["page_host_cpu_ms"] = tm.get("page_host_cpu_ms", 0.0) + (c2 - c0) * 1e3
        ntiles = (self.n + TILE - 1) // TILE
        if ntiles == 0:
            return np.zeros(0, dtype=np.int32), None
        zkey = json.dumps(sort, sort_keys=True, default=str)
        z = self._zones.get(zkey)
        if z is None:
            z = self._zones[zkey] = {"zarg": np.zeros(0, dtype=np.int32), "dirty": set(), "all": True, "density": {},
                                     "sort": sort}
        self._zone_refresh(z, kernels, st, specs_t, ranks_t, seq_bits)
        t3 = time.perf_counter()
        tm["page_zones_ms"] = tm.get("page_zones_ms", 0.0) + (t3 - t2) * 1e3
        zarg = z["zarg"]
        valid = zarg >= 0
        nvalid = int(valid.sum())
        if nvalid == 0:
            return np.zeros(0, dtype=np.int32), None
        top = np.iinfo(np.uint64).max
        keys = np.full(ntiles, top, dtype=np.uint64)
        keys[valid] = self.sort_keys_numpy(zarg[valid], plan).astype(np.uint64)
        pkey = (prog.code.tobytes(), prog.bitmaps.tobytes())
        dens = z["density"].get(pkey, 0.25)  # candidates per row of a chosen tile, from the last page
        b = min(nvalid, max(1, int(np.ceil(1.5 * k_total / max(dens * TILE, 1.0)))))
        if z.setdefault("short", {}).get(pkey):
            # the last page of this filter held every match in the collection (fewer than the
            # page): start from every tile instead of growing towards it one launch at a time
            b = nvalid
        lo_b, hi_b = 0, None  # largest tile count seen short of k candidates / smallest that overflowed
        launches = 0
        for _ in range(24):
            if b >= nvalid:
                chosen, bound = np.nonzero(valid)[0].astype(np.int32), top
            else:
                part = np.argpartition(keys, b)
                chosen, bound = part[:b].astype(np.int32), int(keys[part[b]])
            rows, total, complete = kernels.page(st["table"], st["live"], self.n, code, bitmaps, specs_t, ranks_t,
                                                 st["seq"], seq_bits, chosen, k_total, offset, bound)
            launches += 1
            if complete:
                break
            if total > kernels.page_cap:  # more candidates than one workgroup sorts: fewer tiles
                hi_b = b
            else:
                lo_b = b
            if hi_b is None:
                b = min(nvalid, b * 4)
            elif hi_b - lo_b <= 1:
                return None  # no tile count gives k candidates the LDS sort holds
            else:
                b = (lo_b + hi_b) // 2
        else:
            return None
        if len(chosen):
            z["density"][pkey] = max(total / (len(chosen) * TILE), 1e-4)
            if len(z["density"]) > 64:
                z["density"].pop(next(iter(z["density"])))
        z["short"][pkey] = bound == top and total < k_total
        if len(z["short"]) > 64:
            z["short"].pop(next(iter(z["short"])))
        t4 = time.perf_counter()
        tm["page_kernels_ms"] = tm.get("page_kernels_ms", 0.0) + (t4 - t3) * 1e3
        tm["page_launches"] = tm.get("page_launches", 0) + launches
        if total > k_total:
            more = True
        elif bound == top:
            more = False
        else:  # the page used every candidate: are there matches in the tiles left out?
            more = int(self.select_gpu(prog, kernels, on_device=True).numel()) > k_total
            tm["page_more_ms"] = tm.get("page_more_ms", 0.0) + (time.perf_counter() - t4) * 1e3
        return rows, (str(k_total) if more else None)

    def query(self, q: dict[str, Any], kernels=None) -> tuple[list[str], str | None]:
        """Returns (keys in result order for the requested page, continuation token)."""
        rows, token = self.query_rows(q, kernels)
        return [self.keys[i] for i in rows.tolist()], token

    def query_rows(self, q: dict[str, Any], kernels=None) -> tuple[np.ndarray, str | None]:
        """(rows in result order for the requested page, continuation token)."""
        sort = q.get("sort")
        # every referenced column first: one re-encode (source-backed) and one device upload
        self.ensure_columns(filter_paths(q.get("filter")) + [s["key"] for s in sort or []
                                                             if isinstance(s, dict) and "key" in s])
        prog = self.compile_cached(q.get("filter") or {})
        page = q.get("page") or {}
        limit = int(page.get("limit") or 0)
        offset = int(page.get("token") or 0)
        rows = None
        if kernels is not None and limit:
            paged = self.page_gpu(prog, sort, kernels, offset, limit)
            if paged is not None:
                return paged
        if kernels is not None:
            dev_rows = self.select_gpu(prog, kernels, on_device=True)
            total = int(dev_rows.numel())
            ordered = self.order_gpu(dev_rows, sort, kernels, offset + limit if limit else None)
            if ordered is not None:
                end = min(total, offset + limit) if limit else total
                sel = ordered[offset:end].cpu().numpy()
                if kernels.check_sort():
                    token = str(end) if limit and end < total else None
                    return sel.astype(np.int32, copy=False), token
                # a look-back timed out in the device sort: this query orders on the host
            rows = dev_rows.cpu().numpy()
        if rows is None:  # no GPU: every core of the CPU share over the same narrow codes
            try:
                rows = self.select_native(prog)
            except ImportError:
                rows = self.select_numpy(prog)
        total = rows.size
        rows = self.order(rows, sort, offset + limit if limit else None)
        end = min(total, offset + limit) if limit else total
        sel = rows[offset:end]
        token = str(end) if limit and end < total else None
        return sel.astype(np.int32, copy=False), token
