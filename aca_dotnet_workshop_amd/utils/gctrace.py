"""Collection pauses of one Python process (diagnostics).

With ``TT_GC_TRACE=<dir>`` set, every collection of the cyclic GC that takes at least
``TT_GC_TRACE_MS`` (default 1) milliseconds appends one line to ``<dir>/gc-<name>-<pid>.tsv``:

    wall time at its start (s)   generation   pause (ms)   objects collected

A native event loop that needs the GIL (a query worker, a log sink, a Python route) waits out
such a pause; lining the file up with a benchmark's step times says whether a slow step was one.
"""
from __future__ import annotations

import gc
import os
import time

_state: dict = {}


def install(name: str, environ: dict[str, str] | None = None) -> str | None:
    """Start tracing this process's collections when the environment asks for it; returns the
    file written, or None."""
    env = os.environ if environ is None else environ
    d = env.get("TT_GC_TRACE")
    if not d or _state:
        return None
    os.makedirs(d, exist_ok=True)
    path = os.path.join(d, f"gc-{name}-{os.getpid()}.tsv")
    f = open(path, "a", buffering=1)
    thr = float(env.get("TT_GC_TRACE_MS", "1")) / 1e3
    _state.update(f=f, thr=thr, t0=0.0, w0=0.0)

    def cb(phase: str, info: dict) -> None:
        if phase == "start":
            _state["t0"] = time.perf_counter()
            _state["w0"] = time.time()
            return
        dt = time.perf_counter() - _state["t0"]
        if dt >= _state["thr"]:
            _state["f"].write(f"{_state['w0']:.6f}\t{info.get('generation', -1)}\t{dt * 1e3:.3f}\t"
                              f"{info.get('collected', 0)}\n")

    gc.callbacks.append(cb)
    return path
