"""Wire-format helpers that reproduce System.Text.Json's defaults for the types the
reference's DTOs use (reference: TasksTracker.TasksManager.Backend.Api/Models/TaskModel.cs:3-13).

* ``DateTime`` is written as ISO-8601 with trailing-zero-trimmed fraction and a ``Z``
  suffix only for UTC-kind values.  A date picked in the UI (``type=date``,
  reference Pages/Tasks/Create.cshtml:22) is an *unspecified-kind* midnight value and
  serialises as ``"2024-05-01T00:00:00"`` -- the exact string the overdue query
  compares against (reference Services/TasksStoreManager.cs:104-128).
* ``Guid`` is lowercase hyphenated; ``Guid.Empty`` is the default.
* Property names are camelCase on output and matched case-insensitively on input
  (ASP.NET ``JsonSerializerDefaults.Web``).

Python ``datetime`` carries microseconds (6 digits); .NET ticks carry 7.  Parsing
accepts up to 7 fraction digits (the 7th is truncated), formatting emits at most 6.
"""
from __future__ import annotations

import re
import uuid
from datetime import date, datetime, timedelta, timezone
from typing import Any

DOTNET_MIN = datetime(1, 1, 1)
GUID_EMPTY = uuid.UUID(int=0)

_ISO_RE = re.compile(
    r"^(\d{4})-(\d{2})-(\d{2})"
    r"(?:[T ](\d{2}):(\d{2})(?::(\d{2})(?:[.,](\d{1,9}))?)?)?"
    r"(Z|z|[+-]\d{2}:?\d{2})?$"
)


def parse_datetime(value: Any) -> datetime:
    """Parse the ISO-8601 forms System.Text.Json accepts into a ``datetime``.

    ``Z`` / offsets produce an aware UTC value (``DateTimeKind.Utc``); no suffix
    produces a naive value (``DateTimeKind.Unspecified``).
    """
    if isinstance(value, datetime):
        return value
    if isinstance(value, date):
        return datetime(value.year, value.month, value.day)
    if not isinstance(value, str):
        raise ValueError(f"cannot convert {type(value).__name__} to DateTime")
    m = _ISO_RE.match(value.strip())
    if not m:
        raise ValueError(f"invalid DateTime string: {value!r}")
    y, mo, d, hh, mm, ss, frac, tz = m.groups()
    micro = 0
    if frac:
        micro = int((frac + "000000")[:6])
    dt = datetime(int(y), int(mo), int(d), int(hh or 0), int(mm or 0), int(ss or 0), micro)
    if tz:
        if tz in ("Z", "z"):
            return dt.replace(tzinfo=timezone.utc)
        sign = 1 if tz[0] == "+" else -1
        digits = tz[1:].replace(":", "")
        off = timedelta(hours=int(digits[:2]), minutes=int(digits[2:4]))
        return (dt - sign * off).replace(tzinfo=timezone.utc)
    return dt


def format_datetime(dt: datetime) -> str:
    """Format like System.Text.Json (round-trip "O" with trimmed fraction)."""
    s = f"{dt.year:04d}-{dt.month:02d}-{dt.day:02d}T{dt.hour:02d}:{dt.minute:02d}:{dt.second:02d}"
    if dt.microsecond:
        s += "." + f"{dt.microsecond:06d}".rstrip("0")
    if dt.tzinfo is not None:
        off = dt.utcoffset() or timedelta(0)
        if off == timedelta(0):
            s += "Z"
        else:
            total = int(off.total_seconds() // 60)
            sign = "+" if total >= 0 else "-"
            total = abs(total)
            s += f"{sign}{total // 60:02d}:{total % 60:02d}"
    return s


def format_roundtrip(dt: datetime) -> str:
    """.NET's round-trip ``"O"`` form: always seven fractional digits (microsecond precision
    here, the tick digit 0).  The store holds ``TaskCreatedOn`` this way, so the string order it
    sorts by equals the DateTime order (System.Text.Json's trimmed fraction does not sort:
    ``...:42Z`` > ``...:42.1Z``); every reader parses both forms."""
    s = f"{dt.year:04d}-{dt.month:02d}-{dt.day:02d}T{dt.hour:02d}:{dt.minute:02d}:{dt.second:02d}.{dt.microsecond:06d}0"
    if dt.tzinfo is not None:
        off = dt.utcoffset() or timedelta(0)
        if off == timedelta(0):
            s += "Z"
        else:
            total = int(off.total_seconds() // 60)
            sign = "+" if total >= 0 else "-"
            total = abs(total)
            s += f"{sign}{total // 60:02d}:{total % 60:02d}"
    return s


def format_fixed(dt: datetime, fmt: str = "yyyy-MM-ddTHH:mm:ss") -> str:
    """Port of the custom ``DateTimeConverter`` write path
    (reference Utilities/DateTimeConverter.cs:26-29) for the formats the reference uses."""
    table = {
        "yyyy": f"{dt.year:04d}", "MM": f"{dt.month:02d}", "dd": f"{dt.day:02d}",
        "HH": f"{dt.hour:02d}", "mm": f"{dt.minute:02d}", "ss": f"{dt.second:02d}",
    }
    out, i = [], 0
    while i < len(fmt):
        for tok in ("yyyy", "MM", "dd", "HH", "mm", "ss"):
            if fmt.startswith(tok, i):
                out.append(table[tok])
                i += len(tok)
                break
        else:
            out.append(fmt[i])
            i += 1
    return "".join(out)


def parse_fixed(value: str | None, fmt: str = "yyyy-MM-ddTHH:mm:ss") -> datetime:
    """``DateTime.ParseExact`` for the converter formats; ``None`` raises like the
    reference (Utilities/DateTimeConverter.cs:15-24)."""
    if value is None:
        raise ValueError("Date string from reader is null.")
    pyfmt = (fmt.replace("yyyy", "%Y").replace("MM", "%m").replace("dd", "%d")
                .replace("HH", "%H").replace("mm", "%M").replace("ss", "%S"))
    return datetime.strptime(value, pyfmt)


def naive_utc(dt: datetime) -> datetime:
    """Comparison key: .NET compares DateTime ticks ignoring Kind."""
    if dt.tzinfo is not None:
        return dt.astimezone(timezone.utc).replace(tzinfo=None)
    return dt


def utcnow() -> datetime:
    return datetime.now(timezone.utc)


def today() -> datetime:
    """``DateTime.Today`` (local midnight, unspecified kind); containers run in UTC."""
    n = datetime.now()
    return datetime(n.year, n.month, n.day)


def parse_guid(value: Any) -> uuid.UUID:
    if isinstance(value, uuid.UUID):
        return value
    if not isinstance(value, str):
        raise ValueError("invalid Guid")
    return uuid.UUID(value.strip().strip("{}"))


_GUID_RE = re.compile(r"^\{?[0-9a-fA-F]{8}-?[0-9a-fA-F]{4}-?[0-9a-fA-F]{4}-?[0-9a-fA-F]{4}-?[0-9a-fA-F]{12}\}?$")


def is_guid(value: str) -> bool:
    return bool(_GUID_RE.match(value))
