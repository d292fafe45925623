"""Tasks/Index's table rows without a TaskModel per task (the read path).

The row markup has ONE definition, the ``task_row`` macro in ``templates/_task_row.html``
(reference Pages/Tasks/Index.cshtml:24-40).  At startup ``RowRenderer`` renders that macro with
sentinel values -- once for each combination of the two checkboxes -- and splits the output
into literal fragments and field slots.  A page then fills the slots straight from the API's
JSON (``GET api/tasks``: TaskModel JSON, newest first) with the same HTML escaping Jinja
applies, instead of binding a pydantic model per task and interpreting the template per row
(~13 + ~19 us per task, profiles/r5_read_path.md).

Equality with the template is by construction and checked: the renderer compiles itself
against the macro and then renders a probe list of awkward tasks both ways; any difference and
the fast path stays off (``RowRenderer.ok``).  A task whose fields are outside the plain shape
(an id not in canonical form, a due date with an offset, a non-boolean flag) makes ``render``
return None, and the page binds TaskModels as before.
"""
from __future__ import annotations

import logging
import re
from datetime import datetime
from types import SimpleNamespace
from typing import Any

from markupsafe import Markup

log = logging.getLogger("Frontend.Rows")

_S = {"task_id": "zqTIDqz", "task_name": "zqTNAMEqz", "task_assigned_to": "zqTASSIGNEDqz"}
_S_DATE = datetime(1901, 12, 31)  # formats as the sentinel text "31-12-1901"
_S_DATE_TEXT = "31-12-1901"
_GUID = re.compile(r"^[0-9a-f]{8}-[0-9a-f]{4}-[0-9a-f]{4}-[0-9a-f]{4}-[0-9a-f]{12}$")
# .NET DateTime text in UTC or unspecified kind: the calendar day is the text's own
_DAY = re.compile(r"^(\d{4})-(\d{2})-(\d{2})T\d{2}:\d{2}:\d{2}(?:\.\d{1,7})?Z?$")


def _esc(s: str) -> str:
    """Jinja's autoescape (markupsafe.escape) for text: & < > ' " -- the self-check holds the two
    equal."""
    if "&" in s or "<" in s or ">" in s or "'" in s or '"' in s:
        return s.replace("&", "&amp;").replace(">", "&gt;").replace("<", "&lt;").replace("'", "&#39;") \
            .replace('"', "&#34;")
    return s


class RowRenderer:
    def __init__(self, env) -> None:
        self.macro = env.get_template("_task_row.html").module.task_row
        self.plans: dict[tuple[bool, bool], list[str | None]] = {}
        self.formats: dict[tuple[bool, bool], str] = {}  # the plans as str.format templates
        self.ok = False
        try:
            for done in (False, True):
                for over in (False, True):
                    plan = self.plans[(done, over)] = self._compile(done, over)
                    self.formats[(done, over)] = "".join(
                        p.replace("{", "{{").replace("}", "}}") if i % 2 == 0 else "{" + p + "}"
                        for i, p in enumerate(plan))
            self.ok = self._selfcheck()
        except Exception as e:  # a template this compiler does not understand: the slow path
            log.warning("Tasks/Index row fast path off: %r", e)
        if not self.ok:
            log.warning("Tasks/Index row fast path off: it does not reproduce the task_row macro")

    def _compile(self, done: bool, over: bool) -> list[str | None]:
        """Literal fragments interleaved with slot names (the odd items)."""
        probe = SimpleNamespace(task_id=_S["task_id"], task_name=_S["task_name"], task_due_date=_S_DATE,
                                task_assigned_to=_S["task_assigned_to"], is_completed=done, is_over_due=over)
        html = str(self.macro(probe))
        names = {v: k for k, v in _S.items()}
        names[_S_DATE_TEXT] = "due"
        parts = re.split("(" + "|".join(map(re.escape, names)) + ")", html)
        return [p if i % 2 == 0 else names[p] for i, p in enumerate(parts)]

    @staticmethod
    def _fields(d: Any) -> dict[str, str] | None:
        if not isinstance(d, dict):
            return None
        tid, name, who, due = d.get("taskId"), d.get("taskName"), d.get("taskAssignedTo"), d.get("taskDueDate")
        if not (isinstance(tid, str) and _GUID.match(tid) and isinstance(name, str) and isinstance(who, str)
                and isinstance(due, str) and type(d.get("isCompleted")) is bool and type(d.get("isOverDue")) is bool):
            return None
        m = _DAY.match(due)
        if m is None:
            return None
        return {"task_id": tid, "task_name": _esc(name), "task_assigned_to": _esc(who),
                "due": f"{m.group(3)}-{m.group(2)}-{m.group(1)}"}

    def render(self, items: Any) -> Markup | None:
        """The rows of ``items`` (the API's TaskModel JSON, parsed), or None: bind TaskModels."""
        if not self.ok or not isinstance(items, list):
            return None
        out: list[str] = []
        fmt = self.formats
        for d in items:
            f = self._fields(d)
            if f is None:
                return None
            out.append(fmt[(d["isCompleted"], d["isOverDue"])].format_map(f))
        return Markup("".join(out))

    def page_pieces(self, env, name: str, **ctx: Any) -> list[str] | None:
        """The page ``name`` rendered around the list as pieces for the app host's native route
        (apphost.hpp ``Pieces``): [literal, slot, literal, ...] with the slots ``created_by``,
        ``af_token`` and ``rows`` -- the same render call the page makes, with sentinels in
        those places.  None when a sentinel does not come through exactly once."""
        sent = {"created_by": "zqCREATEDBYqz", "af_token": "zqAFTOKENqz", "rows": "zqROWSqz"}
        html = env.get_template(name).render(created_by=sent["created_by"], af_token=sent["af_token"],
                                             rows_html=Markup(sent["rows"]), **ctx)
        names = {v: k for k, v in sent.items()}
        parts = re.split("(" + "|".join(map(re.escape, names)) + ")", html)
        slots = [names[p] for p in parts[1::2]]
        if sorted(slots) != sorted(sent):
            return None
        return [p if i % 2 == 0 else names[p] for i, p in enumerate(parts)]

    @staticmethod
    def edit_page_pieces(env, name: str, **ctx: Any) -> list[str] | None:
        """The Edit page as pieces for the app host's native route (apphost.hpp ``edit_page``):
        the render call ``edit_get`` makes, with sentinels for the antiforgery token and the
        task's id, name, assignee and due date; None when a sentinel does not come through intact
        (the template escapes or cuts it)."""
        sent = {"af_token": "zqAFTOKENqz", "task_id": "zqTIDqz", "task_name": "zqTNAMEqz",
                "task_assigned_to": "zqTASSIGNEDqz", "due": "zqDUEqz"}
        values = {"taskId": sent["task_id"], "taskName": sent["task_name"], "taskAssignedTo": sent["task_assigned_to"],
                  "taskDueDate": sent["due"]}
        html = env.get_template(name).render(af_token=sent["af_token"], values=values, **ctx)
        names = {v: k for k, v in sent.items()}
        parts = re.split("(" + "|".join(map(re.escape, names)) + ")", html)
        slots = [names[p] for p in parts[1::2]]
        if set(slots) != set(sent):
            return None
        return [p if i % 2 == 0 else names[p] for i, p in enumerate(parts)]

    @staticmethod
    def edit_values(d: Any) -> dict[str, str] | None:
        """``edit_get``'s values straight from the API's TaskModel JSON when it is in the plain
        shape the native route fills (the due date's calendar day from the text), else None."""
        if not isinstance(d, dict):
            return None
        tid, name, who, due = d.get("taskId"), d.get("taskName"), d.get("taskAssignedTo"), d.get("taskDueDate")
        if not (isinstance(tid, str) and _GUID.match(tid) and isinstance(name, str) and isinstance(who, str)
                and isinstance(due, str) and _DAY.match(due)):
            return None
        return {"taskId": tid, "taskName": name, "taskAssignedTo": who, "taskDueDate": due[:10]}

    def row_pieces(self) -> dict[str, list[str]] | None:
        """The compiled rows for the native route: ``row_<c><o>`` (c, o: ``f`` / ``t`` for
        isCompleted / isOverDue) -> pieces with the slots task_id, task_name, task_assigned_to, due."""
        if not self.ok:
            return None
        return {f"row_{'t' if c else 'f'}{'t' if o else 'f'}": self.plans[(c, o)] for c in (False, True)
                for o in (False, True)}

    def _selfcheck(self) -> bool:
        from ...models import TaskModel
        probe = [{"taskId": "0f8fad5b-d9cb-469f-a165-70867728950e", "taskName": 'a <b> & "c" \'d\' é 😀',
                  "taskCreatedBy": "x@y", "taskCreatedOn": "2026-01-02T03:04:05.1234567Z",
                  "taskDueDate": "2026-02-03T00:00:00", "taskAssignedTo": "<script>x@y</script>",
                  "isCompleted": c, "isOverDue": o}
                 for c in (False, True) for o in (False, True)]
        probe.append({**probe[0], "taskDueDate": "1999-12-31T23:59:59.5Z", "taskName": ""})
        fast = self.render_unchecked(probe)
        slow = "".join(str(self.macro(TaskModel.model_validate(d))) for d in probe)
        return fast == slow

    def render_unchecked(self, items: list) -> str | None:
        ok, self.ok = self.ok, True
        try:
            r = self.render(items)
            return None if r is None else str(r)
        finally:
            self.ok = ok
