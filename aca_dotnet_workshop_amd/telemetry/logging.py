"""Structured logging (``ILogger<T>`` + console -> Log Analytics equivalent).

Every record carries the role name and, when inside a request, the W3C trace/span ids so
logs join traces (App Insights "Transaction Search").  Levels follow the reference's
``Logging:LogLevel`` section (``Default: Information``, ``Microsoft.AspNetCore: Warning``,
reference Backend.Api/appsettings.json:2-8).  Records are also appended as JSON lines to
``$TT_TELEMETRY_DIR/logs-<role>-<pid>-<YYYYMMDD>.jsonl`` when the platform provides a telemetry dir
(the Log Analytics workspace of the environment); ``TT_LOG_CONSOLE=0`` keeps them off the
console (the platform then ships only the JSON stream).

Hot path.  The reference logs three Information lines per created task
(TasksStoreManager.cs:34,153; TasksNotifierController.cs:27).  The standard ``logging``
pipeline costs ~20 us per record here (LogRecord construction, caller lookup, handler
locks, a flush per line), so loggers are switched to ``FastLogger``: while only this
module's sinks are installed, ``info()`` & co. format the line directly (JSON via the C
string encoder) into a buffered sink flushed every ``FLUSH_S`` / 64 KiB -- the equivalent of
.NET's source-generated ``LoggerMessage`` + batched console/OTLP exporters.  Any foreign
handler (pytest's ``caplog``, a user's handler), ``exc_info`` or ``extra`` takes the
standard path, so behaviour is unchanged for them.
"""
from __future__ import annotations

import atexit
import logging
import os
import sys
import threading
import time
from json.encoder import encode_basestring
from typing import Any

from .tracing import current_span

_LEVELS = {"trace": 5, "debug": logging.DEBUG, "information": logging.INFO, "info": logging.INFO,
           "warning": logging.WARNING, "warn": logging.WARNING, "error": logging.ERROR,
           "critical": logging.CRITICAL, "none": logging.CRITICAL + 10}
# .NET level names in the JSON stream (Log Analytics "SeverityLevel" vocabulary)
_NET_LEVEL = {logging.DEBUG: "Debug", logging.INFO: "Information", logging.WARNING: "Warning",
              logging.ERROR: "Error", logging.CRITICAL: "Critical", 5: "Trace"}
FLUSH_S = 0.2


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


def json_line(ts: float, level: int, role_json: str, category: str, message: str, trace_id: str = "",
              span_id: str = "", exception: str | None = None) -> str:
    out = ('{"ts":%.6f,"level":"%s","role":%s,"category":%s,"message":%s'
           % (ts, _NET_LEVEL.get(level, logging.getLevelName(level)), role_json, encode_basestring(category),
              encode_basestring(message)))
    if trace_id:
        out += ',"traceId":"%s","spanId":"%s"' % (trace_id, span_id)
    if exception:
        out += ',"exception":' + encode_basestring(exception)
    return out + "}\n"


class JsonFormatter(logging.Formatter):
    def format(self, record: logging.LogRecord) -> str:
        exc = self.formatException(record.exc_info) if record.exc_info else None
        return json_line(record.created, record.levelno, encode_basestring(getattr(record, "role", "")), record.name,
                         record.getMessage(), getattr(record, "trace_id", ""), getattr(record, "span_id", ""),
                         exc)[:-1]


class ConsoleFormatter(logging.Formatter):
    def format(self, record: logging.LogRecord) -> str:
        t = time.strftime("%H:%M:%S", time.localtime(record.created))
        base = f"{t} {record.levelname[:4].lower()}: {getattr(record, 'role', '')} {record.name}: {record.getMessage()}"
        if record.exc_info:
            base += "\n" + self.formatException(record.exc_info)
        return base


class BufferedSink(logging.Handler):
    """Line sink with batched writes (``FLUSH_S`` / 64 KiB, and at exit).  Also a regular
    ``logging.Handler`` for records that take the standard path."""

    def __init__(self, stream, json_lines: bool, role: str, buffered: bool) -> None:
        super().__init__()
        self.stream = stream
        self.json_lines = json_lines
        self.role = role
        self.role_json = encode_basestring(role)
        self.buffered = buffered
        self.setFormatter(JsonFormatter() if json_lines else ConsoleFormatter())
        self._buf: list[str] = []
        self._size = 0
        self._mu = threading.Lock()
        self._sec = -1
        self._hms = ""
        self._prefix: dict[tuple[int, str], str] = {}
        if buffered:
            _Flusher.add(self)

    def line_prefix(self, level: int, name: str) -> str:
        """'{"level":..,"role":..,"category":..' of this JSON sink's lines for (level, logger)."""
        pre = self._prefix.get((level, name))
        if pre is None:
            pre = self._prefix[(level, name)] = '{"level":"%s","role":%s,"category":%s' % (
                _NET_LEVEL.get(level, logging.getLevelName(level)), self.role_json, encode_basestring(name))
        return pre

    # fast path (FastLogger)
    def write_fast(self, level: int, name: str, message: str, trace_id: str, span_id: str) -> None:
        now = time.time()
        if self.json_lines:
            pre = self._prefix.get((level, name))
            if pre is None:  # '{"level":..,"role":..,"category":..' per (level, logger)
                pre = self.line_prefix(level, name)
            if trace_id:
                line = '%s,"ts":%.6f,"message":%s,"traceId":"%s","spanId":"%s"}\n' % (
                    pre, now, encode_basestring(message), trace_id, span_id)
            else:
                line = '%s,"ts":%.6f,"message":%s}\n' % (pre, now, encode_basestring(message))
        else:
            sec = int(now)
            if sec != self._sec:
                self._sec, self._hms = sec, time.strftime("%H:%M:%S", time.localtime(now))
            line = f"{self._hms} {_NET_LEVEL.get(level, 'info')[:4].lower()}: {self.role} {name}: {message}\n"
        self._put(line)

    def write_fast_many(self, level: int, name: str, messages: list[str], trace_id: str, span_id: str) -> None:
        """``write_fast`` for a run of records emitted back to back (one timestamp for the run)."""
        now = time.time()
        if self.json_lines:
            pre = self._prefix.get((level, name))
            if pre is None:
                pre = self._prefix[(level, name)] = '{"level":"%s","role":%s,"category":%s' % (
                    _NET_LEVEL.get(level, logging.getLevelName(level)), self.role_json, encode_basestring(name))
            head = '%s,"ts":%.6f,"message":' % (pre, now)
            tail = ',"traceId":"%s","spanId":"%s"}\n' % (trace_id, span_id) if trace_id else "}\n"
            lines = [head + encode_basestring(m) + tail for m in messages]
        else:
            sec = int(now)
            if sec != self._sec:
                self._sec, self._hms = sec, time.strftime("%H:%M:%S", time.localtime(now))
            head = f"{self._hms} {_NET_LEVEL.get(level, 'info')[:4].lower()}: {self.role} {name}: "
            lines = [head + m + "\n" for m in messages]
        if not self.buffered:
            self._put("".join(lines))
            return
        self._buf.extend(lines)
        self._size += sum(map(len, lines))
        if self._size >= 65536:
            self.flush()

    def _put(self, line: str) -> None:
        if not self.buffered:
            try:
                self.stream.write(line)
                self.stream.flush()
            except (OSError, ValueError):
                pass
            return
        self._buf.append(line)
        self._size += len(line)
        if self._size >= 65536:
            self.flush()

    # standard path
    def emit(self, record: logging.LogRecord) -> None:
        try:
            self._put(self.format(record) + "\n")
        except Exception:
            self.handleError(record)

    def flush(self) -> None:
        if not self._buf:
            return
        with self._mu:
            buf, self._buf, self._size = self._buf, [], 0
            try:
                self.stream.write("".join(buf))
                self.stream.flush()
            except (OSError, ValueError):
                pass

    def close(self) -> None:
        self.flush()
        _Flusher.remove(self)
        super().close()


class _Flusher:
    """One daemon thread per process flushing buffered sinks every ``FLUSH_S``."""
    sinks: list[BufferedSink] = []
    thread: threading.Thread | None = None

    @classmethod
    def add(cls, sink: BufferedSink) -> None:
        cls.sinks.append(sink)
        if cls.thread is None:
            cls.thread = threading.Thread(target=cls._run, name="tt-log-flush", daemon=True)
            cls.thread.start()
            atexit.register(cls.flush_all)

    @classmethod
    def remove(cls, sink: BufferedSink) -> None:
        if sink in cls.sinks:
            cls.sinks.remove(sink)

    @classmethod
    def flush_all(cls) -> None:
        for s in list(cls.sinks):
            s.flush()

    @classmethod
    def _run(cls) -> None:
        while True:
            time.sleep(FLUSH_S)
            cls.flush_all()


class _State:
    sinks: tuple[BufferedSink, ...] = ()
    root_handlers: int = -1  # handler count of the root logger when only our sinks are installed


class FastLogger(logging.Logger):
    """``logging.Logger`` whose level methods bypass ``LogRecord`` while only this module's
    sinks are installed (see module docstring)."""

    def _fast(self, level: int, msg: Any, args: tuple, kw: dict) -> bool:
        if kw or self.handlers or len(_root.handlers) != _State.root_handlers or not self.propagate:
            return False
        if self.isEnabledFor(level):
            message = (msg % args) if args else str(msg)
            s = current_span()
            tid, sid = (s.trace_id, s.span_id) if s is not None else ("", "")
            for sink in _State.sinks:
                if level >= sink.level:
                    sink.write_fast(level, self.name, message, tid, sid)
        return True

    def log_ids(self, level: int, message: str, trace_id: str, span_id: str) -> None:
        """One record with the trace context given (a record made outside this thread's request
        context: a native route's log line, web/native_host.py)."""
        if not self.isEnabledFor(level):
            return
        if not (self.handlers or len(_root.handlers) != _State.root_handlers or not self.propagate):
            for sink in _State.sinks:
                if level >= sink.level:
                    sink.write_fast(level, self.name, message, trace_id, span_id)
            return
        from . import tracing  # the standard path: handlers read the context from the current span
        tok = tracing._current.set(tracing.Span(tracing.tracer(), "", "server", trace_id, span_id, None, False, None))
        try:
            logging.Logger.log(self, level, message)
        finally:
            tracing._current.reset(tok)

    def info_each(self, msg: str, args_seq) -> None:
        """One Information record per argument tuple -- the same lines as ``info(msg, *args)``
        in a loop (e.g. one per task of a bulk operation), formatted as one batch."""
        if self.handlers or len(_root.handlers) != _State.root_handlers or not self.propagate:
            for args in args_seq:
                super().info(msg, *args)
            return
        if not self.isEnabledFor(logging.INFO):
            return
        messages = [msg % args for args in args_seq]
        s = current_span()
        tid, sid = (s.trace_id, s.span_id) if s is not None else ("", "")
        for sink in _State.sinks:
            if logging.INFO >= sink.level:
                sink.write_fast_many(logging.INFO, self.name, messages, tid, sid)

    def debug(self, msg, *args, **kw):
        if not self._fast(logging.DEBUG, msg, args, kw):
            super().debug(msg, *args, **kw)

    def info(self, msg, *args, **kw):
        if not self._fast(logging.INFO, msg, args, kw):
            super().info(msg, *args, **kw)

    def warning(self, msg, *args, **kw):
        if not self._fast(logging.WARNING, msg, args, kw):
            super().warning(msg, *args, **kw)

    def error(self, msg, *args, **kw):
        if not self._fast(logging.ERROR, msg, args, kw):
            super().error(msg, *args, **kw)


_root = logging.getLogger()


def _adopt_fast_loggers() -> None:
    logging.setLoggerClass(FastLogger)
    for lg in list(logging.Logger.manager.loggerDict.values()):
        if type(lg) is logging.Logger:  # created before us: same layout, switch behaviour
            lg.__class__ = FastLogger


def configure_logging(role: str, config: Any = None, json_console: bool | None = None) -> None:
    root = logging.getLogger()
    for h in list(root.handlers):
        if getattr(h, "_tt", False):
            root.removeHandler(h)
            h.close()
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
    sinks: list[BufferedSink] = []
    if os.environ.get("TT_LOG_CONSOLE", "1") != "0":
        h = BufferedSink(sys.stderr, json_console, role, buffered=False)
        sinks.append(h)
    d = os.environ.get("TT_TELEMETRY_DIR")
    if d:
        os.makedirs(d, exist_ok=True)
        from .retention import DailyFile
        sinks.append(BufferedSink(DailyFile(d, f"logs-{role}-{os.getpid()}"), True, role, buffered=True))
    for h in sinks:
        h.addFilter(ctx)
        h._tt = True  # type: ignore[attr-defined]
        root.addHandler(h)
    _State.sinks = tuple(sinks)
    # fast path only while the root logger's handlers are exactly these sinks
    _State.root_handlers = len(root.handlers) if all(getattr(h, "_tt", False) for h in root.handlers) else -1
    _adopt_fast_loggers()


def native_line_sink(name: str, level: int = logging.INFO) -> "BufferedSink | None":
    """The one JSON sink a record of logger ``name`` at ``level`` goes to when the fast path
    writes it, or None (another configuration: format the record in Python).  A native route
    (web/native_host.py) then hands over the finished line."""
    sinks = _State.sinks
    if len(sinks) != 1 or not sinks[0].json_lines or level < sinks[0].level:
        return None
    lg = logging.getLogger(name)
    if not isinstance(lg, FastLogger) or lg.handlers or len(_root.handlers) != _State.root_handlers \
            or not lg.propagate or not lg.isEnabledFor(level):
        return None
    return sinks[0]


def native_line_prefix(name: str, level: int = logging.INFO) -> str:
    """The line prefix (``{"level":..,"role":..,"category":..``) ``native_line_sink``'s sink
    writes for ``name``, or "" when records of ``name`` are not written by the fast path."""
    sink = native_line_sink(name, level)
    return sink.line_prefix(level, name) if sink is not None else ""


def info_each(logger: logging.Logger, msg: str, args_seq) -> None:
    """``logger.info(msg, *args)`` for every tuple of ``args_seq``: batched on a ``FastLogger``,
    a plain loop on any other logger."""
    if isinstance(logger, FastLogger):
        logger.info_each(msg, args_seq)
    else:
        for args in args_seq:
            logger.info(msg, *args)


def flush_logs() -> None:
    _Flusher.flush_all()
