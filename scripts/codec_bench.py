"""Host cost of the overdue sweep's codec passes, per step, over one page of tasks in the
layouts the services exchange (the backing's compact query answer, the API's page, the
markoverdue chunks), through the native module's bindings -- the same functions the app host
and the sidecar run.

    python scripts/codec_bench.py [--tasks 1100] [--chunk 256] [--reps 50]

Prints one JSON line: milliseconds per call of each step (best of ``--reps``).
"""
from __future__ import annotations

import argparse
import json
import sys
import time
import uuid
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from aca_dotnet_workshop_amd import native  # noqa: E402


def _varint(n: int) -> bytes:
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        out.append(b | (0x80 if n else 0))
        if not n:
            return bytes(out)


def _len_field(f: int, v: bytes) -> bytes:
    return _varint(f << 3 | 2) + _varint(len(v)) + v


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--tasks", type=int, default=1100)
    ap.add_argument("--chunk", type=int, default=256)
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    N = native.load()
    sep = (",", ":")
    docs = []
    for i in range(a.tasks):
        d = {"taskId": str(uuid.UUID(int=i + 1)), "taskName": f"Task {i} created by the load",
             "taskCreatedBy": "load@example.com",
             "taskCreatedOn": f"2026-10-17T10:{i // 60 % 60:02d}:{i % 60:02d}.{i % 1000000:06d}0",
             "taskDueDate": "2026-10-16T00:00:00", "taskAssignedTo": "someone@example.com",
             "isCompleted": False, "isOverDue": False}
        docs.append((d["taskId"], json.dumps(d, separators=sep), str(i + 1)))
    query_json = ('{"results":[' + ",".join(f'{{"key":"{k}","data":{v},"etag":"{e}"}}' for k, v, e in docs)
                  + '],"token":""}').encode()
    out: dict[str, float] = {}

    def bench(name: str, f):
        r = f()
        best = 1e9
        for _ in range(a.reps):
            t = time.perf_counter()
            f()
            best = min(best, time.perf_counter() - t)
        out[name] = round(best * 1e3, 3)
        return r

    # the GET hop: sidecar (JSON -> pb), app host (pb -> JSON -> the API's page), processor filter
    pb = bench("sidecar_query_json_to_pb", lambda: N.dapr_pb_query_from_json(query_json))
    assert pb is not None
    js = bench("app_query_pb_to_json", lambda: N.dapr_pb_query_json(pb))
    page = bench("app_query_tasks", lambda: N.tasks_from_query(js, True, False))[1]
    fused = bench("app_query_pb_tasks_one_pass", lambda: N.tasks_from_query_pb(pb, True, False))
    assert fused is not None and fused[1] == page
    run_day = "2026-10-18"
    parts = bench("processor_filter_chunks", lambda: N.tasks_overdue_filter_chunks(page, run_day, a.chunk))[2]
    # the markoverdue hop, one chunk: binder, bulk get, conditional mark, save
    chunk = parts[0]
    bench("app_markoverdue_binder_chunk", lambda: N.tasks_mark_overdue(chunk))
    assert N.tasks_mark_overdue_ids(chunk) is not None
    bench("app_markoverdue_ids_one_pass_chunk", lambda: N.tasks_mark_overdue_ids(chunk))
    n = min(a.chunk, len(docs))
    keys = [k for k, _, _ in docs[:n]]
    bench("app_get_bulk_pb_chunk", lambda: N.dapr_pb_get_bulk_state("statestore", keys, 10))
    bulk_pb = b"".join(_len_field(1, _len_field(1, k.encode()) + _len_field(2, v.encode()) + _len_field(3, e.encode()))
                       for k, v, e in docs[:n])
    bulk_js = bench("app_bulk_pb_to_json_chunk", lambda: N.dapr_pb_bulk_state_json(bulk_pb))
    cm = bench("app_conditional_mark_chunk", lambda: N.tasks_conditional_mark(bulk_js))
    save_body = [x for x in cm if isinstance(x, bytes)][0]
    save_pb = bench("app_save_state_bulk_pb_chunk", lambda: N.dapr_pb_save_state_bulk("statestore", save_body))
    fm = bench("app_conditional_mark_pb_one_pass_chunk", lambda: N.tasks_conditional_mark_pb(bulk_pb, "statestore"))
    assert fm is not None and fm[0] == save_pb
    chain_get = sum(out[k] for k in ("sidecar_query_json_to_pb", "app_query_pb_to_json", "app_query_tasks",
                                     "processor_filter_chunks"))
    one_pass_get = sum(out[k] for k in ("sidecar_query_json_to_pb", "app_query_pb_tasks_one_pass",
                                        "processor_filter_chunks"))
    chain_chunk = sum(out[k] for k in ("app_markoverdue_binder_chunk", "app_get_bulk_pb_chunk",
                                       "app_bulk_pb_to_json_chunk", "app_conditional_mark_chunk",
                                       "app_save_state_bulk_pb_chunk"))
    one_pass_chunk = sum(out[k] for k in ("app_markoverdue_ids_one_pass_chunk", "app_get_bulk_pb_chunk",
                                          "app_conditional_mark_pb_one_pass_chunk"))
    print(json.dumps({"tasks": a.tasks, "chunk": n, "query_bytes": len(query_json), "page_bytes": len(page),
                      "ms": out, "get_hop_ms": {"chain": round(chain_get, 3), "one_pass": round(one_pass_get, 3)},
                      "mark_chunk_ms": {"chain": round(chain_chunk, 3), "one_pass": round(one_pass_chunk, 3)}}))


if __name__ == "__main__":
    main()
