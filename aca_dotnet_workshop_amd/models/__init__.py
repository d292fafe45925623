"""Data contracts (the reference's ``Models/`` folders)."""
from .dotnet import (DOTNET_MIN, GUID_EMPTY, format_datetime, format_fixed, format_roundtrip, naive_utc,
                     parse_datetime, parse_fixed, parse_guid, today, utcnow)
from .task import (FIELD_DISPLAY, REQUIRED_FIELDS, TaskAddModel, TaskModel, TaskUpdateModel,
                   WireModel, conditional_mark_wire, create_task_wire, json_array_chunks, mark_overdue_wire, overdue_filter_chunks, overdue_filter_wire, task_model_name,
                   tasks_from_json, tasks_from_query_wire, tasks_to_json)

__all__ = [
    "DOTNET_MIN", "GUID_EMPTY", "format_datetime", "format_fixed", "format_roundtrip", "naive_utc", "parse_datetime",
    "parse_fixed", "parse_guid", "today", "utcnow", "FIELD_DISPLAY", "REQUIRED_FIELDS",
    "TaskAddModel", "TaskModel", "TaskUpdateModel", "WireModel", "conditional_mark_wire", "create_task_wire", "json_array_chunks", "mark_overdue_wire", "overdue_filter_chunks", "overdue_filter_wire", "task_model_name",
    "tasks_from_json", "tasks_from_query_wire",
    "tasks_to_json",
]
