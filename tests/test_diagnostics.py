"""Stall diagnostics (docs/appendix/01-run-debug.md): the accelerator's slow query / mirror sync
notes under TT_STALL_LOG and the GC pause log's survivor types."""
import gc
import json

from aca_dotnet_workshop_amd.backing import accel
from aca_dotnet_workshop_amd.telemetry import profiler


def test_accel_stall_note_writes_phases_over_threshold(tmp_path, monkeypatch):
    log = tmp_path / "stall.jsonl"
    monkeypatch.setenv("TT_STALL_LOG", str(log))
    monkeypatch.setenv("TT_STALL_MS", "15")
    monkeypatch.setattr(accel, "_STALL", {"file": None, "min_s": None})
    accel._stall_note("accel-query", 0.010, sync_ms=1.0)  # under the threshold: nothing
    accel._stall_note("mirror-bg-sync", 0.046, sync_ms=45.02, warm_ms=1.65)
    accel._STALL["file"].flush()
    rows = [json.loads(x) for x in log.read_text().splitlines()]
    assert len(rows) == 1
    r = rows[0]
    assert r["what"] == "mirror-bg-sync" and r["ms"] == 46.0 and r["sync_ms"] == 45.02 and r["warm_ms"] == 1.65
    assert r["pid"] > 0 and r["wall"] > 0


def test_gc_log_reports_full_collections_with_survivor_types(tmp_path):
    log = tmp_path / "gc.jsonl"
    before = list(gc.callbacks)
    profiler._install_gc_log("unit", str(log), threshold_s=0.0)
    try:
        keep = [{"i": i} for i in range(1000)]  # survivors of the collection below
        gc.collect()
    finally:
        gc.callbacks[:] = before
    rows = [json.loads(x) for x in log.read_text().splitlines()]
    full = [r for r in rows if r["gen"] == 2]
    assert full and full[-1]["proc"] == "unit" and full[-1]["objects"] >= len(keep)
    assert isinstance(full[-1]["top"], list) and any(t == "dict" for t, _ in full[-1]["top"])
    assert "frozen" in full[-1]


def test_native_loop_busy_notes(tmp_path, monkeypatch):
    """A native event loop attached to its GapTracer reports iterations busier than TT_STALL_MS
    (here 1 µs: every iteration that handled a request) as loop-busy lines."""
    import asyncio
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).parent))
    from test_dataplane import Env
    from helpers import run
    log = tmp_path / "stall.jsonl"
    monkeypatch.setenv("TT_STALL_LOG", str(log))
    monkeypatch.setenv("TT_STALL_MS", "0.001")

    async def main():
        async with Env("native", tmp_path) as e:
            st = f"{e.base['app-a']}/v1.0/state/statestore"
            for i in range(20):
                assert (await e.http.post(st, json_body=[{"key": f"k{i}", "value": i}])).status == 204
            await asyncio.sleep(0.05)
    run(main())
    rows = [json.loads(x) for x in log.read_text().splitlines() if '"loop-busy"' in x]
    assert rows and all(r["who"] == "dataplane" and r["ms"] > 0 and r["events"] >= 0 for r in rows)
