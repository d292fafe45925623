#!/usr/bin/env python3
"""GPU columnar query microbenchmark (state-store scan accelerator, ops/hip/query_scan.hip).

Builds a synthetic task collection of ``--rows`` documents (dictionary-encoded columns for
``taskCreatedBy``, ``taskDueDate``, ``isCompleted``, ``isOverDue``, ``priority``) directly
in columnar form, then times the corrected overdue sweep

    taskDueDate < today AND isCompleted == false AND isOverDue == false

(scan + order-preserving compaction) on the GPU and, as the host baseline, the same compiled
program over the same narrow codes on every core of the process's CPU share
(``ColumnarIndex.select_native``, AVX-512); ``--cpu`` adds the single-threaded NumPy reference.
Reports rows scanned per second and effective HBM GB/s.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=100_000_000)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--cpu", action="store_true", help="also time the NumPy executor (slow at 1e8 rows)")
    ap.add_argument("--no-cpu-native", action="store_true",
                    help="skip the multi-threaded native CPU executor (the fair host baseline)")
    ap.add_argument("--query", action="store_true", help="also time the whole paged query path (ColumnarIndex.query)")
    ap.add_argument("--page", action="store_true",
                    help="also time the paged sweep query: ORDER BY taskCreatedOn (clustered by insertion) LIMIT 1000 "
                         "through the zone-map page path (hip/page_topk.hip)")
    ap.add_argument("--sorted", action="store_true",
                    help="also time ORDER BY taskDueDate DESC: top-100 page and full ordering (tt_sort_keys + sort)")
    a = ap.parse_args()

    import numpy as np
    import torch

    from aca_dotnet_workshop_amd.ops.columnar import TILE, Column, ColumnarIndex
    from aca_dotnet_workshop_amd.ops.gpu import GpuKernels

    n = a.rows
    rng = np.random.default_rng(0)
    ix = ColumnarIndex(capacity=n)
    specs = {"taskCreatedBy": [f"user{i}@bench" for i in range(10_000)],
             "taskDueDate": [f"2024-{m:02d}-{d:02d}T00:00:00" for m in range(1, 13) for d in range(1, 29)],
             "isCompleted": [False, True], "isOverDue": [False, True], "priority": list(range(5))}
    probs = {"isCompleted": [0.7, 0.3], "isOverDue": [0.9, 0.1]}
    cols = []
    for path, values in specs.items():
        c = Column(path)
        for v in values:
            c.encode(v)
        ix.columns.append(c)
        ix.col_of[path] = len(ix.columns) - 1
        p = probs.get(path)
        cols.append(rng.choice(len(values), size=n, p=p).astype(np.int32))
    ix.ids = np.full((len(cols), ix.cap), -1, dtype=np.int32)
    for i, c in enumerate(cols):
        ix.ids[i, :n] = c
    ix.live[:n] = 1
    ix.seq[:n] = np.arange(1, n + 1)
    ix._next_seq = n
    ix.n = n
    ix.keys = []  # not needed for the scan benchmark
    ix.version += 1
    ix._full_dirty = True

    k = GpuKernels("cuda:0")
    flt = {"AND": [{"LT": {"taskDueDate": "2024-07-01T00:00:00"}}, {"EQ": {"isCompleted": False}},
                   {"EQ": {"isOverDue": False}}]}
    prog = ix.compile(flt)
    st, code, bm = ix.device_program(prog, k)  # includes rank-encoding range-leaf columns

    def timed(**kw):
        for _ in range(a.warmup):
            res = k.select(st["table"], st["live"], ix.cap, n, code, bm, **kw)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            res = k.select(st["table"], st["live"], ix.cap, n, code, bm, **kw)
        torch.cuda.synchronize()
        return res, (time.perf_counter() - t0) / a.iters

    out, dt = timed()
    selected = int(out.numel())
    # bytes: referenced columns at their narrow widths + liveness bit + mask write & read + output indices
    # bytes per row of the columns the scan reads (2-bit codes: width 0 = 1/4 byte; range leaves
    # read their rank-encoded copy, at least one byte)
    rank_cols = set(prog.code[prog.code[:, 0] == 7, 1].tolist())
    widths = sum((max(1, st["widths"][c]) if c in rank_cols else (st["widths"][c] or 0.25)) for c in prog.columns)
    nbytes = n * widths + n // 8 + 2 * n // 8 + selected * 4
    res = {"metric": "overdue_sweep_rows_per_sec", "value": round(n / dt, 1), "unit": "rows/s", "rows": n,
           "selected": selected, "ms_per_query": round(dt * 1e3, 4), "effective_GBps": round(nbytes / dt / 1e9, 1),
           "device": torch.cuda.get_device_name(0), "tile_rows": TILE,
           "eval_groups": 2, "column_bytes_per_row": widths,
           "range_leaves": int((prog.code[:, 0] == 7).sum())}
    if a.page:
        # creation timestamps: one per 64 rows, rising with the row (rows are appended as tasks
        # are created), 1.56 M distinct values at 1e8 rows -- a 4-byte dictionary column
        c = Column("taskCreatedOn")
        ndist = (n + 63) // 64
        t_enc = time.perf_counter()
        for i in range(ndist):
            c.encode(f"2025-{1 + i // 2_678_400 % 12:02d}-{1 + i // 86_400 % 28:02d}T{i // 3600 % 24:02d}:"
                     f"{i // 60 % 60:02d}:{i % 60:02d}.{i % 7}Z")
        ix.columns.append(c)
        ix.col_of["taskCreatedOn"] = len(ix.columns) - 1
        ids = np.full((1, ix.cap), -1, dtype=np.int32)
        ids[0, :n] = np.arange(n, dtype=np.int64) // 64
        ix.ids = np.concatenate([ix.ids, ids])
        ix.version += 1
        ix._full_dirty = True
        ix.seq[:n] = np.arange(1, n + 1)
        sort = [{"key": "taskCreatedOn", "order": "ASC"}]
        q = {"filter": flt, "sort": sort, "page": {"limit": 1000}}
        c.ranks()
        res["page_setup_s"] = round(time.perf_counter() - t_enc, 2)
        t0 = time.perf_counter()
        rows, token = ix.query_rows(q, k)  # first page: uploads the column, builds every tile's zone argmin
        torch.cuda.synchronize()
        res["page_first_ms"] = round((time.perf_counter() - t0) * 1e3, 3)
        calls = {"pages": 0, "tiles": 0}
        real_page = k.page

        def counted(*args, **kw):
            calls["pages"] += 1
            calls["tiles"] += len(args[9])
            return real_page(*args, **kw)
        k.page = counted
        it = max(5, a.iters)
        t0 = time.perf_counter()
        for _ in range(it):
            rows, token = ix.query_rows(q, k)
        res["page1000_ms"] = round((time.perf_counter() - t0) / it * 1e3, 4)
        k.page = real_page
        res["page_kernel_calls_per_query"] = calls["pages"] / it
        res["page_tiles_per_query"] = calls["tiles"] / it
        # the page equals the host ordering of the full selection (first 1000)
        sel = out.cpu().numpy()
        plan = ix.sort_specs(sort)
        want = sel[np.argsort(ix.sort_keys_numpy(sel, plan), kind="stable")[:1000]]
        res["page_match"] = bool(np.array_equal(rows, want)) and token == "1000"
    if a.sorted:
        ix.seq[:n] = rng.permutation(n) + 1  # updates move rows: result order != row order
        ix._full_dirty = True
        sort = [{"key": "taskDueDate", "order": "DESC"}]
        st = ix.to_device(k)
        # the device ordering: tt_sort_keys + the repo's onesweep LSD radix sort of (key, row) pairs
        # over the used key bits (hip/radix_pairs.hip), or radix select + sort for the top 100
        for label, kk in (("top100", 100), ("full", None)):
            for _ in range(2):
                ix.order_gpu(out, sort, k, kk)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            it = max(1, a.iters // 4)
            for _ in range(it):
                ordered = ix.order_gpu(out, sort, k, kk)
            torch.cuda.synchronize()
            res[f"order_{label}_ms"] = round((time.perf_counter() - t0) / it * 1e3, 3)
        res["ordered_rows"] = int(ordered.numel())
        # the device order equals the host's stable ordering of the same selection, entirely
        sel = out.cpu().numpy()
        plan = ix.sort_specs(sort)
        host_keys = ix.sort_keys_numpy(sel, plan)
        host_order = sel[np.argsort(host_keys, kind="stable")]
        res["order_match"] = bool(np.array_equal(host_order, ordered.cpu().numpy()))
        k.check_sort()
    if a.query:
        # the whole state-query path the backing planner runs: filter + ORDER BY + first page
        # (ColumnarIndex.query: select, device ordering/top-k, page copy, keys)
        class _Keys:  # row -> key without materialising 1e8 strings
            def __getitem__(self, i):
                return f"task-{i}"
        ix.keys = _Keys()
        ix.seq[:n] = rng.permutation(n) + 1
        ix._full_dirty = True
        q = {"filter": flt, "sort": [{"key": "taskDueDate", "order": "DESC"}], "page": {"limit": 100}}
        for _ in range(3):
            ix.query(q, k)
        stages = {"select": 0.0, "order": 0.0, "page": 0.0}
        it = max(5, a.iters)
        t0 = time.perf_counter()
        for _ in range(it):
            keys, token = ix.query(q, k)
        res["query_page100_ms"] = round((time.perf_counter() - t0) / it * 1e3, 4)
        # stage breakdown (synchronised after each stage)
        for _ in range(it):
            t = time.perf_counter()
            dev_rows = ix.select_gpu(ix.compile_cached(flt), k, on_device=True)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            ordered = ix.order_gpu(dev_rows, q["sort"], k, 100)
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            page = ordered[:100].cpu().numpy()
            t3 = time.perf_counter()
            stages["select"] += t1 - t
            stages["order"] += t2 - t1
            stages["page"] += t3 - t2
        res["query_stages_ms"] = {k2: round(v / it * 1e3, 4) for k2, v in stages.items()}
        res["query_page_rows"] = len(keys)
    if not a.no_cpu_native:
        # the fair host baseline: the same program over the same narrow codes, every core of this
        # process's CPU share, AVX-512 compares (native/src/cpuscan.hpp)
        from aca_dotnet_workshop_amd.ops.columnar import cpu_share
        threads = cpu_share()
        ref = ix.select_native(prog, threads)  # builds the host mirror (narrow copies, rank column)
        res["cpu_native_matches"] = bool(np.array_equal(ref, out.cpu().numpy()))
        for label, th in (("cpu_native_ms", threads), ("cpu_native_1thread_ms", 1)):
            it = max(3, a.iters // (4 if th == 1 else 1))
            t0 = time.perf_counter()
            for _ in range(it):
                ix.select_native(prog, th)
            res[label] = round((time.perf_counter() - t0) / it * 1e3, 3)
        res["cpu_threads"] = threads
        res["gpu_speedup_vs_cpu_native"] = round(res["cpu_native_ms"] / res["ms_per_query"], 1)
    if a.cpu:
        t0 = time.perf_counter()
        ref = ix.select_numpy(prog)
        res["numpy_ms"] = round((time.perf_counter() - t0) * 1e3, 2)
        res["match"] = bool(np.array_equal(ref, out.cpu().numpy()))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
