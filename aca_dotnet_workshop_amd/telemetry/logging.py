"""Structured logging (``ILogger<T>`` + console -> Log Analytics equivalent).

Every record carries the role name and, when inside a request, the W3C trace/span ids so
logs join traces (App Insights "Transaction Search").  Levels follow the reference's
``Logging:LogLevel`` section (``Default: Information``, ``Microsoft.AspNetCore: Warning``,
reference Backend.Api/appsettings.json:2-8).  Records are also appended as JSON lines to
``$TT_TELEMETRY_DIR/logs-<role>-<pid>.jsonl`` when the platform provides a telemetry dir.
"""
from __future__ import annotations

import json
import logging
import os
import sys
import time
from typing import Any

from .tracing import current_span

_LEVELS = {"trace": 5, "debug": logging.DEBUG, "information": logging.INFO, "info": logging.INFO,
           "warning": logging.WARNING, "warn": logging.WARNING, "error": logging.ERROR,
           "critical": logging.CRITICAL, "none": logging.CRITICAL + 10}


class _Ctx(logging.Filter):
    def __init__(self, role: str) -> None:
        super().__init__()
        self.role = role

    def filter(self, record: logging.LogRecord) -> bool:
        record.role = self.role
        s = current_span()
        record.trace_id = s.trace_id if s else ""
        record.span_id = s.span_id if s else ""
        return True


class JsonFormatter(logging.Formatter):
    def format(self, record: logging.LogRecord) -> str:
        rec: dict[str, Any] = {"ts": round(record.created, 6), "level": record.levelname, "role": getattr(record, "role", ""),
                               "category": record.name, "message": record.getMessage()}
        if getattr(record, "trace_id", ""):
            rec["traceId"] = record.trace_id
            rec["spanId"] = record.span_id
        if record.exc_info:
            rec["exception"] = self.formatException(record.exc_info)
        return json.dumps(rec, separators=(",", ":"))


class ConsoleFormatter(logging.Formatter):
    def format(self, record: logging.LogRecord) -> str:
        t = time.strftime("%H:%M:%S", time.localtime(record.created))
        base = f"{t} {record.levelname[:4].lower()}: {getattr(record, 'role', '')} {record.name}: {record.getMessage()}"
        if record.exc_info:
            base += "\n" + self.formatException(record.exc_info)
        return base


def configure_logging(role: str, config: Any = None, json_console: bool | None = None) -> None:
    root = logging.getLogger()
    for h in list(root.handlers):
        if getattr(h, "_tt", False):
            root.removeHandler(h)
    ctx = _Ctx(role)
    default = "information"
    if config is not None:
        default = str(config.get("Logging:LogLevel:Default", default))
    root.setLevel(_LEVELS.get(default.lower(), logging.INFO))
    if config is not None:
        for k, v in config.section("Logging:LogLevel").items():
            if k.lower() != "default" and isinstance(v, (str, int)):
                cat = {"Microsoft.AspNetCore": "web"}.get(k, k)
                logging.getLogger(cat).setLevel(_LEVELS.get(str(v).lower(), logging.INFO))
    if json_console is None:
        json_console = os.environ.get("TT_LOG_FORMAT", "console") == "json"
    h = logging.StreamHandler(sys.stderr)
    h.setFormatter(JsonFormatter() if json_console else ConsoleFormatter())
    h.addFilter(ctx)
    h._tt = True  # type: ignore[attr-defined]
    root.addHandler(h)
    d = os.environ.get("TT_TELEMETRY_DIR")
    if d:
        os.makedirs(d, exist_ok=True)
        fh = logging.FileHandler(os.path.join(d, f"logs-{role}-{os.getpid()}.jsonl"))
        fh.setFormatter(JsonFormatter())
        fh.addFilter(ctx)
        fh._tt = True  # type: ignore[attr-defined]
        root.addHandler(fh)
