"""Task DTOs shared by the three services.

Reference parity:
* ``TaskModel`` / ``TaskAddModel`` / ``TaskUpdateModel`` -- Backend.Api/Models/TaskModel.cs:3-29,
  the processor's copy Processor.Backend.Svc/Models/TaskModel.cs:3-13 and the UI copy with
  ``[Required]``/``[Display]`` annotations Frontend.Ui/Pages/Tasks/Models/TasksModel.cs:6-49.

One definition serves all three (the reference triplicates it).  UI-only metadata
(display names, required flags) lives in ``FIELD_DISPLAY`` / ``REQUIRED_FIELDS`` and is
enforced by the frontend's form binder, not by the API -- exactly like the reference,
whose API models carry no validation attributes.
"""
from __future__ import annotations

import json
import uuid
from datetime import datetime
from typing import Annotated, Any, ClassVar

from pydantic import BaseModel, BeforeValidator, ConfigDict, PlainSerializer, model_validator
from pydantic.alias_generators import to_camel

from .dotnet import DOTNET_MIN, GUID_EMPTY, format_datetime, format_roundtrip, parse_datetime, parse_guid

DotNetDateTime = Annotated[
    datetime,
    BeforeValidator(parse_datetime),
    PlainSerializer(format_datetime, return_type=str, when_used="json"),
]
Guid = Annotated[
    uuid.UUID,
    BeforeValidator(parse_guid),
    PlainSerializer(lambda u: str(u), return_type=str, when_used="json"),
]


class WireModel(BaseModel):
    """Base: camelCase on the wire, case-insensitive property matching on input,
    unknown properties ignored (ASP.NET model binding drops extras, which is how the
    processor's full ``TaskModel`` binds to the API's ``TaskAddModel``,
    reference ExternalTasksProcessorController.cs:33 vs TasksController.cs:34-46)."""

    model_config = ConfigDict(alias_generator=to_camel, populate_by_name=True, extra="ignore",
                              validate_assignment=False)
    _lower_aliases: ClassVar[dict[str, str]] = {}
    _aliases: ClassVar[frozenset[str]] = frozenset()

    def __init_subclass__(cls, **kw: Any) -> None:
        super().__init_subclass__(**kw)
        cls._lower_aliases = {}
        cls._aliases = frozenset()

    @classmethod
    def __pydantic_init_subclass__(cls, **kw: Any) -> None:
        super().__pydantic_init_subclass__(**kw)
        cls._lower_aliases = {
            (f.alias or name).lower(): (f.alias or name) for name, f in cls.model_fields.items()
        }
        # keys that need no remapping: the camelCase aliases and the Python field names
        cls._aliases = frozenset(cls._lower_aliases.values()) | frozenset(cls.model_fields)

    @model_validator(mode="before")
    @classmethod
    def _case_insensitive(cls, data: Any) -> Any:
        if isinstance(data, dict):
            if cls._aliases.issuperset(data):  # canonical camelCase or field names (the common case)
                return data
            la = cls._lower_aliases
            out = {}
            for k, v in data.items():
                if isinstance(k, str):
                    a = la.get(k.lower())
                    if a is not None:
                        out[a] = v
                        continue
                out[k] = v
            return out
        return data

    def to_wire(self) -> dict[str, Any]:
        return self.model_dump(mode="json", by_alias=True)

    def to_json(self) -> str:
        return self.model_dump_json(by_alias=True)

    @classmethod
    def from_wire(cls, data: Any):
        if isinstance(data, (bytes, bytearray, str)):
            data = json.loads(data)
        return cls.model_validate(data)


class TaskModel(WireModel):
    task_id: Guid = GUID_EMPTY
    task_name: str = ""
    task_created_by: str = ""
    task_created_on: DotNetDateTime = DOTNET_MIN
    task_due_date: DotNetDateTime = DOTNET_MIN
    task_assigned_to: str = ""
    is_completed: bool = False
    is_over_due: bool = False


    def to_store_json(self) -> str:
        """The document the store holds (and the tasksaved event carries): the wire JSON with
        ``taskCreatedOn`` in the round-trip form (``format_roundtrip``), whose string order is the
        DateTime order -- the ORDER BY the overdue sweep pages by (TasksStoreManager.cs:136)."""
        s = self.to_json()
        c = self.task_created_on
        return s.replace(f'"taskCreatedOn":"{format_datetime(c)}"', f'"taskCreatedOn":"{format_roundtrip(c)}"', 1)


class TaskAddModel(WireModel):
    task_name: str = ""
    task_created_by: str = ""
    task_due_date: DotNetDateTime = DOTNET_MIN
    task_assigned_to: str = ""


class TaskUpdateModel(WireModel):
    task_id: Guid = GUID_EMPTY
    task_name: str = ""
    task_due_date: DotNetDateTime = DOTNET_MIN
    task_assigned_to: str = ""


# UI annotations (reference Frontend.Ui/Pages/Tasks/Models/TasksModel.cs:20-48)
FIELD_DISPLAY = {
    "taskName": "Task Name",
    "taskDueDate": "Task DueDate",
    "taskAssignedTo": "Assigned To",
}
REQUIRED_FIELDS = ("taskName", "taskDueDate", "taskAssignedTo")


_native_codec: Any = None


def create_task_wire(body: bytes) -> tuple[str, str, str, bytes, bytes] | None:
    """Bind a ``TaskAddModel`` body and build the new ``TaskModel`` in one native pass
    (``native/src/taskcodec.hpp``): ``(taskId, taskName, taskAssignedTo, TaskModel JSON,
    state-save body)``, byte-identical to binding with ``TaskAddModel`` and serialising
    ``TaskModel(task_id=uuid4(), task_created_on=utcnow(), ...)``.  ``None`` when the body is
    outside the codec's envelope (unusual property casing, offsets, invalid values, ...) or the
    native module is absent: the caller binds it with pydantic, which decides those cases."""
    global _native_codec
    if _native_codec is None:
        try:
            from ..native import load
            _native_codec = load().task_create
        except Exception:  # no native module in this process: the pydantic binder serves
            _native_codec = False
    return _native_codec(body) if _native_codec else None


def task_model_name(body: bytes) -> str | None:
    """``taskName`` of a ``TaskModel`` JSON body when it binds within the native codec's envelope
    (``native/src/taskcodec.hpp``), else ``None`` (bind with ``TaskModel``)."""
    global _native_name
    if _native_name is None:
        try:
            from ..native import load
            _native_name = load().task_model_name
        except Exception:
            _native_name = False
    return _native_name(body) if _native_name else None


_native_name: Any = None
_native_lists: Any = None


def _lists():
    global _native_lists
    if _native_lists is None:
        try:
            from ..native import load
            n = load()
            _native_lists = (n.tasks_mark_overdue, n.tasks_overdue_filter, n.tasks_conditional_mark)
        except Exception:
            _native_lists = False
    return _native_lists


def mark_overdue_wire(body: bytes) -> tuple[list[str], bytes] | None:
    """``POST markoverdue`` body -> (task ids, the state API's bulk-save body with every task
    ``isOverDue = true``), each TaskModel written like ``to_wire()``; ``None``: bind with
    ``[TaskModel]`` (``native/src/taskcodec.hpp``)."""
    fns = _lists()
    return fns[0](body) if fns else None


def conditional_mark_wire(got: bytes) -> tuple[list[str], bytes, int] | None:
    """The state API's bulk-get answer for a markoverdue page (``[{"key", "data", "etag"}]``) ->
    (ids to mark, a bulk-save body setting ``isOverDue`` on the STORED task where it is still
    open and not yet overdue, each item ETag-guarded with first-write concurrency, the number
    skipped: completed, already overdue or deleted).  Native (``taskcodec.hpp
    conditional_mark``) or this module's Python twin, which also takes the documents the native
    codec turns down (a null string, a duplicate key, an unusual date form); a stored document
    that does not bind as a TaskModel at all is skipped, so the rest of the page is still marked
    and later sweeps do not fail on it forever.  ``None``: the answer is not a bulk-get array."""
    fns = _lists()
    if fns:
        made = fns[2](got)
        if made is not None:
            return made
    try:
        rows = json.loads(got)
    except ValueError:
        return None
    if not isinstance(rows, list):
        return None
    ids, items, skipped = [], [], 0
    for r in rows:
        data = r.get("data") if isinstance(r, dict) else None
        if data is None:
            skipped += 1
            continue
        try:
            t = TaskModel.model_validate(data)
        except ValueError:  # pydantic's ValidationError: not a task -- leave it as stored
            skipped += 1
            continue
        if t.is_completed or t.is_over_due:
            skipped += 1
            continue
        t.is_over_due = True
        item: dict[str, Any] = {"key": r["key"], "value": json.loads(t.to_store_json()),
                                "options": {"concurrency": "first-write"}}
        if r.get("etag"):
            item["etag"] = r["etag"]
        items.append(item)
        ids.append(str(t.task_id))
    return ids, json.dumps(items, separators=(",", ":")).encode(), skipped


def tasks_from_query_wire(body: bytes, by_created: bool = False,
                          descending: bool = False) -> tuple[int, bytes, bool] | None:
    """State-query response -> (tasks, TaskModel JSON array of the results with data, whether the
    response carries a continuation token), each task written like ``to_wire()``; in result
    order, or with ``by_created`` ordered by ``TaskCreatedOn`` as a DateTime (ascending, stable:
    the reference's ``OrderBy``, TasksStoreManager.cs:136; ``descending``: newest first, stable,
    its ``OrderByDescending``, :66).  ``None``: bind with ``TaskModel``."""
    global _native_query
    if _native_query is None:
        try:
            from ..native import load
            _native_query = load().tasks_from_query
        except Exception:
            _native_query = False
    return _native_query(body, by_created, descending) if _native_query else None


_native_query: Any = None


def overdue_filter_wire(body: bytes, run_day: str) -> tuple[int, int, bytes] | None:
    """The cron job's filter over an overdue page: (tasks on the page, tasks due before
    ``run_day`` (YYYY-MM-DD, UTC), those tasks as a TaskModel JSON array); ``None``: bind with
    ``TaskModel`` and filter in Python."""
    fns = _lists()
    return fns[1](body, run_day) if fns else None


def overdue_filter_chunks(body: bytes, run_day: str, chunk: int) -> tuple[int, int, list[bytes]] | None:
    """``overdue_filter_wire`` with the kept tasks cut into TaskModel JSON arrays of at most
    ``chunk`` tasks (the processor's concurrent markoverdue calls), in one native pass;
    ``None``: as for ``overdue_filter_wire``."""
    try:
        from ..native import load
        fn = load().tasks_overdue_filter_chunks
    except Exception:
        fn = None
    if fn is not None and chunk > 0:
        return fn(body, run_day, chunk)
    got = overdue_filter_wire(body, run_day)
    if got is None or chunk <= 0:
        return None
    n_page, n_kept, kept = got
    parts = json_array_chunks(kept, chunk) if n_kept else []
    return None if parts is None else (n_page, n_kept, parts)


def tasks_to_json(tasks: list[TaskModel]) -> bytes:
    return ("[" + ",".join(t.to_json() for t in tasks) + "]").encode()


def tasks_from_json(data: Any) -> list[TaskModel]:
    if isinstance(data, (bytes, bytearray, str)):
        data = json.loads(data) if data else []
    return [TaskModel.model_validate(d) for d in (data or [])]


def json_array_chunks(body: bytes, n: int) -> list[bytes] | None:
    """A JSON array's items re-grouped into arrays of at most ``n`` (raw slices: the items'
    bytes are not re-encoded), or None when ``body`` is not a valid JSON array."""
    try:
        from ..native import load
        fn = load().json_array_chunks
    except Exception:
        fn = None
    if fn is not None:
        return fn(body, n)
    try:
        items = json.loads(body)
    except ValueError:
        return None
    if not isinstance(items, list) or n < 1:
        return None
    return [json.dumps(items[i:i + n], separators=(",", ":"), ensure_ascii=False).encode()
            for i in range(0, len(items), n)]
