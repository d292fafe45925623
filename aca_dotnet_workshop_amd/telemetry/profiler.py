"""Opt-in CPU profiler for every long-running process of the stack.

``TT_PROFILE_DIR=/path`` makes each process (sidecars, apps, backing services) run under
``cProfile`` and write ``<dir>/<name>-<pid>.prof`` when it exits (SIGTERM included), so a
bench run can be broken down per process::

    TT_PROFILE_DIR=/tmp/prof python bench.py --steps 10
    python -m aca_dotnet_workshop_amd.telemetry.profiler /tmp/prof   # top functions per file

(The reference relies on Application Insights' profiler; SURVEY.md §5 "Tracing / profiling".)
"""
from __future__ import annotations

import contextlib
import os
import signal
import sys
from typing import Iterator


def _install_gc_log(name: str, path: str, threshold_s: float = 0.02) -> None:
    """``TT_GC_LOG=<file>``: append one JSON line per garbage-collector pause longer than 20 ms
    (stall diagnostics: a gen-2 collection stops every Python thread of the process)."""
    import gc
    import json
    import time
    start = [0.0]
    out = open(path, "a", buffering=1)

    def cb(phase: str, info: dict) -> None:
        if phase == "start":
            start[0] = time.perf_counter()
            return
        d = time.perf_counter() - start[0]
        if d > threshold_s:
            gen = info["generation"]
            objs = gc.get_objects(gen)
            top = None
            if gen == 2:  # what the full collection had to scan: the survivors' commonest types
                counts: dict[str, int] = {}
                for o in objs:
                    t = type(o).__name__
                    counts[t] = counts.get(t, 0) + 1
                top = sorted(counts.items(), key=lambda kv: -kv[1])[:10]
            out.write(json.dumps({"what": "gc-pause", "proc": name, "pid": os.getpid(), "gen": gen,
                                  "ms": round(d * 1e3, 2), "collected": info["collected"], "objects": len(objs),
                                  "frozen": gc.get_freeze_count(), "top": top,
                                  "wall": round(time.time(), 4)}) + "\n")
            del objs
    gc.callbacks.append(cb)


@contextlib.contextmanager
def maybe_profile(name: str) -> Iterator[None]:
    gc_log = os.environ.get("TT_GC_LOG")
    if gc_log:
        _install_gc_log(name, gc_log)
    out_dir = os.environ.get("TT_PROFILE_DIR")
    if not out_dir:
        yield
        return
    import cProfile

    os.makedirs(out_dir, exist_ok=True)
    prof = cProfile.Profile()
    path = os.path.join(out_dir, f"{name.replace('/', '_')}-{os.getpid()}.prof")
    # asyncio.run installs its own SIGINT handling; SIGTERM must unwind the stack so we dump.
    prev = signal.getsignal(signal.SIGTERM)
    if prev in (signal.SIG_DFL, None):
        signal.signal(signal.SIGTERM, lambda *_: (_ for _ in ()).throw(KeyboardInterrupt()))
    prof.enable()
    try:
        yield
    finally:
        prof.disable()
        prof.dump_stats(path)


def summarize(paths: list[str], top: int = 25, sort: str = "tottime") -> str:
    import io
    import pstats

    buf = io.StringIO()
    for p in paths:
        buf.write(f"==== {os.path.basename(p)}\n")
        st = pstats.Stats(p, stream=buf)
        st.sort_stats(sort).print_stats(top)
    return buf.getvalue()


def main(argv: list[str] | None = None) -> int:
    import argparse
    import glob

    ap = argparse.ArgumentParser(description="summarize TT_PROFILE_DIR dumps")
    ap.add_argument("dir")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--sort", default="tottime")
    ap.add_argument("--match", default="")
    a = ap.parse_args(argv)
    files = sorted(f for f in glob.glob(os.path.join(a.dir, "*.prof")) if a.match in os.path.basename(f))
    sys.stdout.write(summarize(files, a.top, a.sort))
    return 0


if __name__ == "__main__":
    sys.exit(main())
