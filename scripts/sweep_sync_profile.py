"""Host-side cost of one overdue sweep against a collection that grows under load
(VERDICT r2 #4): the columnar mirror sync (pulling the rows written since the last sweep),
the ordered page selection and the result assembly, timed separately and profiled.

    python scripts/sweep_sync_profile.py [--base 400000] [--per-sweep 40000] [--sweeps 5] [--profile]

CPU executor by default (the same host work the GPU path does around its kernels); ``--gpu``
uses the HIP kernels when a device is present.  Prints one JSON line.
"""
from __future__ import annotations

import argparse
import cProfile
import io
import json
import pstats
import sys
import time
import uuid
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from aca_dotnet_workshop_amd import native  # noqa: E402
from aca_dotnet_workshop_amd.backing.accel import PREFIX_PATH, CollectionAccelerator  # noqa: E402

PATHS = ["taskDueDate", "isCompleted", "isOverDue", "taskCreatedOn"]
PREFIX = "tasksmanager-backend-api||"


def task(i: int, due_past: bool) -> str:
    ts = f"2026-10-{1 + i // 2_000_000 % 28:02d}T{i // 3_600_000 % 24:02d}:{i // 60_000 % 60:02d}:{i // 1000 % 60:02d}.{i % 1000:03d}"
    due = "2020-01-01T00:00:00" if due_past else "2030-01-01T00:00:00"
    return json.dumps({"taskId": str(uuid.UUID(int=i)), "taskName": f"Task {i}", "taskCreatedBy": "load@example.com",
                       "taskCreatedOn": ts, "taskDueDate": due, "taskAssignedTo": "a@example.com",
                       "isCompleted": False, "isOverDue": False})


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--base", type=int, default=400_000)
    ap.add_argument("--per-sweep", type=int, default=40_000)
    ap.add_argument("--sweeps", type=int, default=5)
    ap.add_argument("--past-due-every", type=int, default=64)
    ap.add_argument("--page", type=int, default=1000)
    ap.add_argument("--gpu", action="store_true")
    ap.add_argument("--profile", action="store_true")
    a = ap.parse_args()
    N = native.load()
    store = N.DocStore()
    acc = CollectionAccelerator("gpu" if a.gpu else "cpu", 0, PATHS)
    acc.attach(store)
    i = 0

    def write(n: int) -> None:
        nonlocal i
        for _ in range(n):
            store.set(f"{PREFIX}{uuid.UUID(int=i)}", task(i, i % a.past_due_every == 0))
            i += 1
    write(a.base)
    q = {"filter": {"AND": [{"LT": {"taskDueDate": "2026-10-17T00:00:00"}}, {"EQ": {"isCompleted": False}},
                            {"EQ": {"isOverDue": False}}]},
         "sort": [{"key": "taskCreatedOn", "order": "ASC"}], "page": {"limit": a.page}}
    acc.query(q, PREFIX, store)  # builds the mirror index
    prof = cProfile.Profile() if a.profile else None
    sweeps = []
    for _ in range(a.sweeps):
        write(a.per_sweep)
        for k in ("sync_ms", "select_and_results_ms"):
            acc.stats[k] = 0.0
        marked = 0
        t0 = time.perf_counter()
        if prof:
            prof.enable()
        while True:  # one sweep: pages until the store has no more open past-due tasks
            text = acc.query(q, PREFIX, store)
            res = json.loads(text)
            for r in res["results"]:
                d = r["data"]
                d["isOverDue"] = True
                store.set(f"{PREFIX}{r['key']}", json.dumps(d))
            marked += len(res["results"])
            if not res.get("token"):
                break
        if prof:
            prof.disable()
        sweeps.append({"ms": round((time.perf_counter() - t0) * 1e3, 2), "marked": marked,
                       "sync_ms": acc.stats["sync_ms"], "select_and_results_ms": acc.stats["select_and_results_ms"]})
    out = {"rows": len(store), "per_sweep_new_rows": a.per_sweep, "mode": acc.mode, "sweeps": sweeps}
    print(json.dumps(out))
    if prof:
        s = io.StringIO()
        pstats.Stats(prof, stream=s).sort_stats("cumulative").print_stats(25)
        print(s.getvalue(), file=sys.stderr)


if __name__ == "__main__":
    main()
