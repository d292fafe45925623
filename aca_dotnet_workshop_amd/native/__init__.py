"""Native (C++) engines: document store and message broker.

The extension is built in-tree on first import if missing or stale (a few seconds with
g++); there is deliberately no pure-Python fallback -- the backing services run on the
native engines or not at all.
"""
from __future__ import annotations

import importlib
import threading

_lock = threading.Lock()
_mod = None


def load():
    global _mod
    if _mod is not None:
        return _mod
    with _lock:
        if _mod is None:
            from .build import build_native
            build_native()
            _mod = importlib.import_module(f"{__name__}._ttnative")
    return _mod


def __getattr__(name: str):
    if name in ("DocStore", "Broker", "QueueOptions", "TxOp", "EtagMismatch", "Received"):
        return getattr(load(), name)
    raise AttributeError(name)
