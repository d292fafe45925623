"""Task manager port and its two adapters.

* ``TasksManager``       -- the ``ITasksManager`` port, 8 operations
  (reference Backend.Api/Services/ITasksManager.cs:5-15).
* ``FakeTasksManager``   -- in-memory list seeded with 10 tasks for
  ``tjoudeh@bitoftech.net`` (reference Services/FakeTasksManager.cs:10-25).
* ``TasksStoreManager``  -- sidecar-backed: state store ``statestore``, query API and
  ``tasksavedtopic`` publication (reference Services/TasksStoreManager.cs:1-158).

Deliberate deviations from the reference's latent bugs, all covered by
tests/test_backend_api.py:
* #1  the fake implements ``mark_overdue_tasks`` (the reference throws NotImplementedException);
* #2  the fake's "yesterday" query compares calendar dates, filters open tasks and orders
      ascending, matching the store semantics (the reference compares exact timestamps);
* #3  ``update_task`` checks for a missing task *before* dereferencing it;
* #4  ``delete_task`` reports a missing task (404) instead of always succeeding;
* #5  query filters are built as JSON objects, not by string concatenation;
* #11 asyncio single-threaded execution makes the fake's list race-free;
* #12 read-modify-write operations use ETag first-write concurrency with bounded retry
      instead of last-writer-wins -- markoverdue included: it re-reads the page's tasks and
      marks only those still open, each save guarded by the ETag it read, so a completion that
      lands between the sweep's query and its save is never reverted (the reference saves the
      processor's copy, TasksStoreManager.cs:141-149).
Everything else (status codes, orderings, the ``yyyy-MM-ddTHH:mm:ss`` due-date equality
trap of #7, publish-on-create and publish-on-assignee-change) is kept.
"""
from __future__ import annotations

import abc
import json
import logging
import random
import uuid
from datetime import datetime, timedelta

from ...models import (TaskModel, conditional_mark_wire, create_task_wire, format_fixed, mark_overdue_wire, naive_utc,
                       tasks_from_query_wire, today, utcnow)
from ...sdk.client import InvocationError, RawJson, SidecarClient
from ...telemetry.logging import info_each

log = logging.getLogger("TasksManager")

# The create flow's log templates (TasksStoreManager.cs:34, :153): the Python manager logs with
# them and the app host's native route (apphost.hpp api_create) is handed the same text -- one
# definition, so the native lines follow any edit here
LOG_SAVE_NEW = "Save a new task with name: '%s' to state store"
LOG_PUBLISH = "Publish Task Saved event for task with Id: '%s' and Name: '%s' for Assignee: '%s'"
LOG_OVERDUE_PAGE = "Getting open tasks due before: '%s' (page of %d)"
LOG_MARK_OVERDUE = "Mark task with Id: '%s' as OverDue task"
LOG_GET = "Getting task with Id: '%s'"
LOG_COMPLETE = "Mark task with Id: '%s' as completed"
LOG_UPDATE = "Update task with Id: '%s'"
LOG_DELETE = "Delete task with Id: '%s'"

_codecs: dict = {}


def _codec(name: str):
    """A task codec of the native module (taskcodec.hpp via module.cpp), or None without it."""
    if name not in _codecs:
        try:
            from ...native import load
            _codecs[name] = getattr(load(), name)
        except Exception:
            _codecs[name] = None
    return _codecs[name]


def _complete(t: TaskModel) -> None:
    t.is_completed = True

STORE_NAME = "statestore"
PUBSUB_NAME = "dapr-pubsub-servicebus"
TOPIC_NAME = "tasksavedtopic"
SEED_CREATOR = "tjoudeh@bitoftech.net"


class TasksManager(abc.ABC):
    @abc.abstractmethod
    async def get_tasks_by_creator(self, created_by: str) -> list[TaskModel]: ...

    @abc.abstractmethod
    async def get_task_by_id(self, task_id: uuid.UUID) -> TaskModel | None: ...

    @abc.abstractmethod
    async def create_new_task(self, task_name: str, created_by: str, assigned_to: str, due_date: datetime) -> uuid.UUID: ...

    @abc.abstractmethod
    async def update_task(self, task_id: uuid.UUID, task_name: str, assigned_to: str, due_date: datetime) -> bool: ...

    @abc.abstractmethod
    async def mark_task_completed(self, task_id: uuid.UUID) -> bool: ...

    @abc.abstractmethod
    async def delete_task(self, task_id: uuid.UUID) -> bool: ...

    @abc.abstractmethod
    async def mark_overdue_tasks(self, tasks: list[TaskModel]) -> None: ...

    @abc.abstractmethod
    async def get_yesterdays_due_tasks(self, limit: int | None = None) -> list[TaskModel]: ...


def _created_key(t: TaskModel) -> datetime:
    return naive_utc(t.task_created_on)


class FakeTasksManager(TasksManager):
    def __init__(self, seed: bool = True, rng: random.Random | None = None) -> None:
        self._tasks: list[TaskModel] = []
        self._by_id: dict[uuid.UUID, TaskModel] = {}
        rnd = rng or random.Random()
        if seed:
            now = utcnow()
            for i in range(10):
                self._add(TaskModel(task_id=uuid.uuid4(), task_name=f"Task number: {i}", task_created_by=SEED_CREATOR,
                                    task_created_on=now + timedelta(minutes=i), task_due_date=now + timedelta(days=i),
                                    task_assigned_to=f"assignee{rnd.randrange(50)}@mail.com"))

    def _add(self, t: TaskModel) -> None:
        self._tasks.append(t)
        self._by_id[t.task_id] = t

    async def create_new_task(self, task_name, created_by, assigned_to, due_date) -> uuid.UUID:
        t = TaskModel(task_id=uuid.uuid4(), task_name=task_name, task_created_by=created_by, task_created_on=utcnow(),
                      task_due_date=due_date, task_assigned_to=assigned_to)
        self._add(t)
        return t.task_id

    async def delete_task(self, task_id) -> bool:
        t = self._by_id.pop(task_id, None)
        if t is None:
            return False
        self._tasks.remove(t)
        return True

    async def get_task_by_id(self, task_id) -> TaskModel | None:
        return self._by_id.get(task_id)

    async def get_tasks_by_creator(self, created_by) -> list[TaskModel]:
        if not created_by:
            return []
        return sorted((t for t in self._tasks if t.task_created_by == created_by), key=_created_key, reverse=True)

    async def mark_task_completed(self, task_id) -> bool:
        t = self._by_id.get(task_id)
        if t is None:
            return False
        t.is_completed = True
        return True

    async def update_task(self, task_id, task_name, assigned_to, due_date) -> bool:
        t = self._by_id.get(task_id)
        if t is None:
            return False
        t.task_name, t.task_assigned_to, t.task_due_date = task_name, assigned_to, due_date
        return True

    async def mark_overdue_tasks(self, tasks) -> None:
        for incoming in tasks:
            t = self._by_id.get(incoming.task_id)
            if t is not None:
                t.is_over_due = True

    async def get_yesterdays_due_tasks(self, limit: int | None = None) -> list[TaskModel]:
        y = (today() - timedelta(days=1)).date()
        return sorted((t for t in self._tasks if naive_utc(t.task_due_date).date() == y
                       and not t.is_completed and not t.is_over_due), key=_created_key)


class ConcurrencyConflict(Exception):
    pass


class TasksStoreManager(TasksManager):
    """Sidecar-backed manager; ``client`` is the ``DaprClient`` equivalent."""

    def __init__(self, client: SidecarClient, store: str = STORE_NAME, pubsub: str = PUBSUB_NAME,
                 topic: str = TOPIC_NAME, max_retries: int = 5, overdue_query: str = "equality",
                 overdue_page: int = 1000) -> None:
        self.client = client
        self.store = store
        self.pubsub = pubsub
        self.topic = topic
        self.max_retries = max_retries
        if overdue_query not in ("equality", "range"):
            raise ValueError(f"OverdueTasks:Query must be 'equality' or 'range', not {overdue_query!r}")
        self.overdue_query = overdue_query
        self.overdue_page = overdue_page

    @classmethod
    def from_config(cls, client: SidecarClient, config) -> "TasksStoreManager":
        """``TasksManager:*`` names and the ``OverdueTasks:*`` sweep settings from configuration."""
        return cls(client, store=config.get_str("TasksManager:StateStoreName", STORE_NAME),
                   pubsub=config.get_str("TasksManager:PubSubName", PUBSUB_NAME),
                   topic=config.get_str("TasksManager:TopicName", TOPIC_NAME),
                   overdue_query=(config.get_str("OverdueTasks:Query") or "equality").lower(),
                   overdue_page=config.get_int("OverdueTasks:PageSize", 1000))

    async def create_new_task(self, task_name, created_by, assigned_to, due_date) -> uuid.UUID:
        t = TaskModel(task_id=uuid.uuid4(), task_name=task_name, task_created_by=created_by, task_created_on=utcnow(),
                      task_due_date=due_date, task_assigned_to=assigned_to)
        log.info(LOG_SAVE_NEW, t.task_name)
        payload = RawJson(t.to_store_json())  # serialised once for the save and the event
        await self.client.save_state(self.store, str(t.task_id), payload)
        await self._publish_task_saved(t, payload)
        return t.task_id

    async def create_new_task_from_body(self, body: bytes) -> str | None:
        """``create_new_task`` straight from the request body: binding, the new TaskModel and its
        JSON come from the native codec in one pass (``models.create_task_wire``); the same log
        lines, state save and event follow.  ``None``: the body needs the general binder."""
        made = create_task_wire(body)
        if made is None:
            return None
        tid, name, assignee, task_json, state_body = made
        log.info(LOG_SAVE_NEW, name)
        # the state API's body as is (HTTP) or as a SaveStateRequest of the same items (gRPC)
        await self.client.save_state_body(self.store, state_body)
        log.info(LOG_PUBLISH, tid, name, assignee)
        await self.client.publish_event(self.pubsub, self.topic, task_json, content_type="application/json")
        return tid

    def _native_endpoint(self) -> dict | None:
        ep_of = getattr(self.client, "native_endpoint", None)
        return ep_of() if ep_of is not None else None

    def _native_calls(self, ep: dict, **targets: tuple[str, str]) -> tuple[dict, dict]:
        """The route settings and the ``what`` map of a native route's sidecar calls.
        ``targets``: step -> (HTTP API path, gRPC method).  Over gRPC (the reference's
        ``DaprClient`` transport for state and publish) the targets are the RPCs' paths, the
        route writes the request messages (it gets the component names) and a failed call raises
        what ``GrpcSidecarClient`` raises (its ``what`` is the RPC); over HTTP the API paths and
        ``SidecarClient``'s messages."""
        from ...sdk import proto as P
        cfg = {"sidecar": ep["sidecar"], "token": ep["token"], "timeout": ep["timeout"]}
        grpc = ep.get("protocol") == "grpc"
        what: dict[str, str] = {}
        http_what = {"save": f"save state {self.store}", "publish": f"publish {self.pubsub}/{self.topic}",
                     "query": f"query state {self.store}", "bulk": f"bulk get {self.store}",
                     "get": f"get state {self.store}", "delete": f"delete state {self.store}"}
        for step, (path, rpc) in targets.items():
            cfg[f"{step}_target"] = P.method_path(rpc) if grpc else ep["prefix"] + path
            what[step] = rpc if grpc else http_what[step]
        if grpc:
            cfg.update({"protocol": "grpc", "store": self.store, "pubsub": self.pubsub, "topic": self.topic})
            what["protocol"] = "grpc"
        return cfg, what

    def native_create_route(self) -> dict | None:
        """``create_new_task_from_body`` as a native route of the app host (apphost.hpp
        ``api_create``: codec, "Save a new task" log line, state save, "Publish Task Saved"
        log line, publish, 201) over the client's protocol, or None when this client cannot take
        one (asyncio I/O).  ``what``: the SDK's error messages for the two calls, raised when a
        call fails."""
        ep = self._native_endpoint()
        if ep is None or (ep.get("protocol") != "grpc" and getattr(self.client, "save_state_body", None) is None):
            return None
        cfg, what = self._native_calls(ep, save=(f"/v1.0/state/{self.store}", "SaveState"),
                                       publish=(f"/v1.0/publish/{self.pubsub}/{self.topic}", "PublishEvent"))
        cfg.update({"log_category": log.name,
                    # the lines create_new_task_from_body logs, with the codec's fields in order
                    "log_save": LOG_SAVE_NEW, "log_save_args": "name",
                    "log_publish": LOG_PUBLISH, "log_publish_args": "id,name,assigned_to"})
        return {"kind": "api_create", "method": "POST", "path": "/api/tasks", "route": "/api/tasks",
                "cfg": cfg, "what": what}

    async def delete_task(self, task_id) -> bool:
        log.info(LOG_DELETE, task_id)
        raw_get = getattr(self.client, "get_state_raw", None)
        if raw_get is not None:  # only the ETag is needed: no decode
            data, etag = await raw_get(self.store, str(task_id))
        else:
            data, etag = await self.client.get_state_and_etag(self.store, str(task_id))
        if data is None:
            return False
        try:
            await self.client.delete_state(self.store, str(task_id), etag=etag)
        except InvocationError as e:
            if e.status not in (409, 412):  # concurrently deleted/changed -> already gone is fine
                raise
        return True

    async def get_task_by_id(self, task_id) -> TaskModel | None:
        log.info(LOG_GET, task_id)
        data = await self.client.get_state(self.store, str(task_id))
        return TaskModel.model_validate(data) if data is not None else None

    async def get_tasks_by_creator(self, created_by) -> list[TaskModel]:
        if not created_by:
            return []
        resp = await self.client.query_state(self.store, self._by_creator_query(created_by))
        tasks = [TaskModel.model_validate(r.data) for r in resp.results if r.data is not None]
        tasks.sort(key=_created_key, reverse=True)
        return tasks

    def _by_creator_query(self, created_by: str) -> dict:
        return {"filter": {"EQ": {"taskCreatedBy": created_by}}}

    def native_list_route(self) -> dict | None:
        """``tasks_by_creator_json`` as a native route of the app host (apphost.hpp ``api_list``):
        the same query text -- this manager's, split around the JSON-encoded creator -- through
        the same sidecar, the same codec; None when this client cannot take one."""
        ep = self._native_endpoint()
        if ep is None or getattr(self.client, "query_state_raw", None) is None:
            return None
        mark = "zqCREATORqz"
        text = json.dumps(self._by_creator_query(mark))  # query_state_raw's encoding of the dict
        at = text.find(json.dumps(mark))
        if at < 0 or text.count(mark) != 1:
            return None
        cfg, what = self._native_calls(ep, query=(f"/v1.0-alpha1/state/{self.store}/query", "QueryStateAlpha1"))
        cfg.update({"query_prefix": text[:at], "query_suffix": text[at + len(json.dumps(mark)):]})
        return {"kind": "api_list", "method": "GET", "path": "/api/tasks", "route": "/api/tasks", "cfg": cfg,
                "what": what}

    async def tasks_by_creator_json(self, created_by: str) -> bytes | None:
        """``get_tasks_by_creator`` as the response body: the query's results turned into the
        TaskModel JSON array newest first in one native pass (``tasks_from_query_wire``, the
        reference's ``OrderByDescending(o => o.TaskCreatedOn)``, TasksStoreManager.cs:54-69) --
        no TaskModel per task.  ``None``: a response outside the codec's envelope (the caller
        binds the TaskModels), or no raw query on this client."""
        raw_query = getattr(self.client, "query_state_raw", None)
        if raw_query is None:
            return None
        if not created_by:
            return b"[]"
        raw = await raw_query(self.store, self._by_creator_query(created_by))
        made = tasks_from_query_wire(raw, by_created=True, descending=True)
        return made[1] if made is not None else None

    async def get_task_json(self, task_id: uuid.UUID) -> bytes | None | bool:
        """``get_task_by_id`` as the response body: the stored document turned into the TaskModel
        JSON in one native pass (``taskcodec.hpp task_json``).  None: no such task; False: a
        document outside the codec's envelope, or no raw read on this client (bind a TaskModel)."""
        raw_get = getattr(self.client, "get_state_raw", None)
        codec = _codec("task_json")
        if raw_get is None or codec is None:
            return False
        log.info(LOG_GET, task_id)
        raw, _ = await raw_get(self.store, str(task_id))
        if raw is None:
            return None
        made = codec(raw)
        return made if made is not None else TaskModel.model_validate(json.loads(raw)).to_json().encode()

    @staticmethod
    def _rmw_body(key: str, etag: str | None, value: bytes) -> bytes:
        """The ETag-guarded save of a read-modify-write, as ``SidecarClient.save_state(..., etag,
        concurrency="first-write")`` writes it (the app host's routes send these bytes too)."""
        item: dict = {"key": key}
        if etag is not None:
            item["etag"] = etag
        item["options"] = {"concurrency": "first-write"}
        return ("[" + json.dumps(item, separators=(",", ":"))[:-1] + ',"value":').encode() + value + b"}]"

    async def _edit(self, task_id: uuid.UUID, complete: bool, update: tuple | None):
        """The read-modify-write through the native codec (``taskcodec.hpp edit_task``): the
        stored document read with its ETag, edited, saved back guarded by that ETag (first-write),
        re-read and re-applied on a conflict.  (document written, stored assignee); None: no such
        task; False: the codec or this client cannot take it (the TaskModel path)."""
        raw_get = getattr(self.client, "get_state_raw", None)
        save_body = getattr(self.client, "save_state_body", None)
        edit = _codec("task_edit")
        if raw_get is None or save_body is None or edit is None:
            return False
        key = str(task_id)
        for _ in range(self.max_retries):
            raw, etag = await raw_get(self.store, key)
            if raw is None:
                return None
            made = edit(raw, complete, update)
            if made is None:
                return False
            doc, _tid, old = made
            try:
                await save_body(self.store, self._rmw_body(key, etag, doc))
                return doc, old
            except InvocationError as e:
                if e.status in (409, 412):
                    continue  # lost a race: re-read and re-apply
                raise
        raise ConcurrencyConflict(f"task {task_id} kept changing under concurrent writers")

    async def mark_task_completed_fast(self, task_id: uuid.UUID) -> bool | None:
        """``mark_task_completed`` through the native codec; None: take the TaskModel path."""
        if _codec("task_edit") is None or getattr(self.client, "get_state_raw", None) is None:
            return None
        log.info(LOG_COMPLETE, task_id)
        res = await self._edit(task_id, True, None)
        if res is False:
            return (await self._read_modify_write(task_id, _complete)) is not None
        return res is not None

    async def update_task_from_body(self, task_id: uuid.UUID, body: bytes) -> bool | None:
        """``update_task`` straight from the request body: TaskUpdateModel bound by the native
        binder, the read-modify-write through the codec, the assignee-change publish
        (TasksStoreManager.cs:95-98) with the document written.  None: the body needs the
        general binder (or no native codec / raw client calls)."""
        bind = _codec("task_update_bind")
        if bind is None or _codec("task_edit") is None or getattr(self.client, "get_state_raw", None) is None:
            return None
        upd = bind(body)
        if upd is None:
            return None
        log.info(LOG_UPDATE, task_id)
        res = await self._edit(task_id, False, upd)
        if res is False:  # a stored document outside the codec's envelope: the TaskModel path
            from ...models.dotnet import parse_datetime
            name, who, due = upd
            return await self._update(task_id, name, who, parse_datetime(due))
        if res is None:
            return False
        doc, old = res
        if upd[1].lower() != old.lower():
            log.info(LOG_PUBLISH, task_id, upd[0], upd[1])
            await self.client.publish_event(self.pubsub, self.topic, doc, content_type="application/json")
        return True

    async def _read_modify_write(self, task_id: uuid.UUID, mutate) -> TaskModel | None:
        for _ in range(self.max_retries):
            data, etag = await self.client.get_state_and_etag(self.store, str(task_id))
            if data is None:
                return None
            t = TaskModel.model_validate(data)
            before = t.model_copy()
            mutate(t)
            try:
                await self.client.save_state(self.store, str(t.task_id), RawJson(t.to_store_json()), etag=etag,
                                             concurrency="first-write")
                return before, t  # type: ignore[return-value]
            except InvocationError as e:
                if e.status in (409, 412):
                    continue  # lost a race: re-read and re-apply
                raise
        raise ConcurrencyConflict(f"task {task_id} kept changing under concurrent writers")

    async def mark_task_completed(self, task_id) -> bool:
        log.info(LOG_COMPLETE, task_id)
        return (await self._read_modify_write(task_id, _complete)) is not None

    async def update_task(self, task_id, task_name, assigned_to, due_date) -> bool:
        log.info(LOG_UPDATE, task_id)
        return await self._update(task_id, task_name, assigned_to, due_date)

    async def _update(self, task_id, task_name, assigned_to, due_date) -> bool:
        def m(t: TaskModel) -> None:
            t.task_name, t.task_assigned_to, t.task_due_date = task_name, assigned_to, due_date
        res = await self._read_modify_write(task_id, m)
        if res is None:
            return False
        before, after = res
        if after.task_assigned_to.lower() != before.task_assigned_to.lower():
            await self._publish_task_saved(after)
        return True

    async def get_yesterdays_due_tasks(self, limit: int | None = None) -> list[TaskModel]:
        if self.overdue_query == "range":
            return await self._open_tasks_due_before_today(limit)
        yesterday = today() - timedelta(days=1)
        json_date = format_fixed(yesterday, "yyyy-MM-ddTHH:mm:ss")
        log.info("Getting overdue tasks for yesterday date: '%s'", json_date)
        q = {"filter": {"EQ": {"taskDueDate": json_date}}}
        resp = await self.client.query_state(self.store, q)
        tasks = [TaskModel.model_validate(r.data) for r in resp.results if r.data is not None]
        tasks = [t for t in tasks if not t.is_completed and not t.is_over_due]
        tasks.sort(key=_created_key)
        return tasks

    async def overdue_page_json(self, limit: int | None = None) -> tuple[bytes, bool] | None:
        """``get_yesterdays_due_tasks`` as the response body, for the range sweep: the query
        results turned into the TaskModel JSON array in one native pass, ordered by
        ``TaskCreatedOn`` (``models.tasks_from_query_wire``), plus whether the store has more
        matches than this page (its continuation token).  ``None``: equality mode, or a response
        outside the codec's envelope -- the caller binds the TaskModels."""
        raw_query = getattr(self.client, "query_state_raw", None)
        if self.overdue_query != "range" or raw_query is None:
            return None
        q, midnight, page = self._range_query(limit)
        log.info(LOG_OVERDUE_PAGE, midnight, page)
        raw = await raw_query(self.store, q)
        made = tasks_from_query_wire(raw, by_created=True)
        if made is not None:
            return made[1], made[2]
        doc = json.loads(raw) if raw else {}
        tasks = [TaskModel.model_validate(r["data"]) for r in doc.get("results") or [] if r.get("data") is not None]
        tasks.sort(key=_created_key)
        return ("[" + ",".join(t.to_json() for t in tasks) + "]").encode(), bool(doc.get("token"))

    def native_overdue_route(self) -> dict | None:
        """``overdue_page_json`` as a native route of the app host (apphost.hpp ``api_overdue``):
        this manager's range query and log line as templates over the two values that change --
        the local midnight and the page size -- the same codec, the more-results flag; None
        outside range mode or when this client cannot take one."""
        ep = self._native_endpoint()
        if self.overdue_query != "range" or ep is None or getattr(self.client, "query_state_raw", None) is None:
            return None
        mid, page = "zqMIDNIGHTqz", 987654321
        q, _, _ = self._range_query(page, midnight=mid)
        text = json.dumps(q).replace("%", "%%")  # query_state_raw's encoding of the dict
        jm, jp = json.dumps(mid), str(page)
        if text.count(jm) != 1 or text.count(jp) != 1:
            return None
        args = "midnight,page" if text.find(jm) < text.find(jp) else "page,midnight"
        text = text.replace(jm, '"%s"').replace(jp, "%s")
        # the log line fills midnight then page (%d of an int prints as %s of it)
        log_tpl = LOG_OVERDUE_PAGE
        if log_tpl.count("%s") != 1 or log_tpl.count("%d") != 1 or log_tpl.find("%s") > log_tpl.find("%d"):
            return None
        cfg, what = self._native_calls(ep, query=(f"/v1.0-alpha1/state/{self.store}/query", "QueryStateAlpha1"))
        cfg.update({"query": text, "query_args": args, "page_default": self.overdue_page,
                    "log_category": log.name, "log_overdue": log_tpl.replace("%d", "%s"),
                    "log_overdue_args": "midnight,page"})
        return {"kind": "api_overdue", "method": "GET", "path": "/api/overduetasks", "route": "/api/overduetasks",
                "cfg": cfg, "what": what}

    def native_task_routes(self) -> list[dict]:
        """The single-task routes on the app host's I/O thread (apphost.hpp ``api_task``): GET /
        PUT / PUT markcomplete / DELETE ``api/tasks/{id}`` -- this manager's codec passes
        (``get_task_json``, ``update_task_from_body``, ``mark_task_completed_fast``,
        ``delete_task``), log lines, ETag-guarded saves and the assignee-change publish, over the
        client's protocol.  Empty when this client cannot take them.  A ``what`` holding
        ``{key}`` is filled with the request's task id (the HTTP SDK's messages name the key)."""
        ep = self._native_endpoint()
        if ep is None or getattr(self.client, "get_state_raw", None) is None or _codec("task_edit") is None:
            return []
        routes = []
        for kind, method, path, log_op, missing in (("api_get", "GET", "/api/tasks/{id}", LOG_GET, 404),
                                                    ("api_update", "PUT", "/api/tasks/{id}", LOG_UPDATE, 400),
                                                    ("api_complete", "PUT", "/api/tasks/{id}/markcomplete", LOG_COMPLETE, 400),
                                                    ("api_delete", "DELETE", "/api/tasks/{id}", LOG_DELETE, 404)):
            cfg, what = self._native_calls(ep, get=(f"/v1.0/state/{self.store}/", "GetState"),
                                           save=(f"/v1.0/state/{self.store}", "SaveState"),
                                           publish=(f"/v1.0/publish/{self.pubsub}/{self.topic}", "PublishEvent"),
                                           delete=(f"/v1.0/state/{self.store}/", "DeleteState"))
            if ep.get("protocol") != "grpc":  # the HTTP SDK's messages name the key
                what.update({"get": f"get state {self.store}/{{key}}", "delete": f"delete state {self.store}/{{key}}"})
            cfg.update({"store": self.store, "log_category": log.name, "log_op": log_op, "log_op_args": "id",
                        "max_retries": self.max_retries, "missing": missing, "log_publish": LOG_PUBLISH,
                        "log_publish_args": "id,name,assigned_to"})
            route = path.replace("{id}", "{taskId}")
            routes.append({"kind": kind, "method": method, "path": path, "route": route, "cfg": cfg, "what": what})
        return routes

    def native_markoverdue_route(self) -> dict | None:
        """``mark_overdue_from_body`` as a native route of the app host (apphost.hpp
        ``api_markoverdue``): the native binder's ids, then this manager's conditional mark pass --
        bulk get, codec, a log line per marked task, ETag-guarded bulk save, re-read on a conflict
        up to ``max_retries`` passes -- over the client's protocol; None when this client cannot
        take one."""
        ep = self._native_endpoint()
        if ep is None or getattr(self.client, "get_bulk_state_raw", None) is None:
            return None
        cfg, what = self._native_calls(ep, bulk=(f"/v1.0/state/{self.store}/bulk", "GetBulkState"),
                                       save=(f"/v1.0/state/{self.store}", "SaveState"))
        if ep.get("protocol") != "grpc":
            what["bulk"] = f"bulk get {self.store}"
        cfg.update({"store": self.store, "log_category": log.name, "log_mark": LOG_MARK_OVERDUE, "log_mark_args": "id",
                    "max_retries": self.max_retries, "parallelism": 10})
        return {"kind": "api_markoverdue", "method": "POST", "path": "/api/overduetasks/markoverdue",
                "route": "/api/overduetasks/markoverdue", "cfg": cfg, "what": what}

    def _range_query(self, limit: int | None, midnight: str | None = None) -> tuple[dict, str, int]:
        """The open tasks due before today's midnight, oldest first: ``ORDER BY taskCreatedOn``
        in the store picks the page (reference ``.OrderBy(o => o.TaskCreatedOn)``,
        TasksStoreManager.cs:136) -- the stored round-trip strings sort as DateTimes; the page is
        re-ordered by the DateTime value on the way out all the same (documents written by other
        clients may carry System.Text.Json's trimmed fraction, see ``tasks_from_query_wire``)."""
        midnight = format_fixed(today(), "yyyy-MM-ddTHH:mm:ss") if midnight is None else midnight
        page = limit if limit and limit > 0 else self.overdue_page
        q = {"filter": {"AND": [{"LT": {"taskDueDate": midnight}}, {"EQ": {"isCompleted": False}},
                                {"EQ": {"isOverDue": False}}]},
             "sort": [{"key": "taskCreatedOn", "order": "ASC"}],
             "page": {"limit": page}}
        return q, midnight, page

    async def _open_tasks_due_before_today(self, limit: int | None) -> list[TaskModel]:
        """``OverdueTasks:Query=range`` (SURVEY.md §2.12 #7 fixed): every open task due before
        today, whatever its time of day and however many daily runs were missed, filtered by
        the store rather than in the app -- a range leaf plus two boolean leaves, which the
        backing planner runs as a gfx950 columnar scan.  The store orders by the stored
        ``taskCreatedOn`` (round-trip form, ``TaskModel.to_store_json``), which is the DateTime
        order of the reference's ``OrderBy``.  One page (oldest first) per call: the
        processor marks a page overdue and asks again, and marked tasks drop out of the filter."""
        q, midnight, page = self._range_query(limit)
        log.info(LOG_OVERDUE_PAGE, midnight, page)
        resp = await self.client.query_state(self.store, q)
        tasks = [TaskModel.model_validate(r.data) for r in resp.results if r.data is not None]
        tasks.sort(key=_created_key)
        return tasks

    async def mark_overdue_from_body(self, body: bytes) -> bool:
        """``mark_overdue_tasks`` straight from the request body: the ids come from the native
        binder (``models.mark_overdue_wire``), then the conditional mark.  False: the body needs
        the general binder (or the client has no raw bulk calls)."""
        if getattr(self.client, "save_state_body", None) is None or \
                getattr(self.client, "get_bulk_state_raw", None) is None:
            return False
        made = mark_overdue_wire(body)
        if made is None:
            return False
        await self._mark_conditionally(made[0])
        return True

    async def mark_overdue_tasks(self, tasks) -> None:
        await self._mark_conditionally([str(t.task_id) for t in tasks])

    async def _mark_conditionally(self, ids: list[str]) -> None:
        """Bulk read-modify-write of ``isOverDue``: read the tasks with their
        ETags, set the flag on the STORED copy of every task still open and not yet overdue, save
        each guarded by its ETag (first-write).  A conflict (a task changed in between: a
        completion, an edit) re-reads the tasks of that pass and re-applies; the tasks the save
        did write are overdue by then and drop out."""
        pending = list(dict.fromkeys(ids))
        raw_get = getattr(self.client, "get_bulk_state_raw", None)
        save_body = getattr(self.client, "save_state_body", None)
        for _ in range(self.max_retries):
            if not pending:
                return
            if raw_get is not None:
                got = await raw_get(self.store, pending)
            else:  # gRPC: bulk get as state items
                got = json.dumps([{"key": x.key, "data": x.data, "etag": x.etag}
                                  for x in await self.client.get_bulk_state(self.store, pending)]).encode()
            made = conditional_mark_wire(got)
            if made is None:
                raise ValueError("the task collection holds documents outside the TaskModel shape")
            marked, bulk, _skipped = made
            info_each(log, LOG_MARK_OVERDUE, [(tid,) for tid in marked])
            if not marked:
                return
            try:
                if save_body is not None:
                    await save_body(self.store, bulk)
                else:
                    await self.client.save_bulk_state(self.store, json.loads(bulk))
                return
            except InvocationError as e:
                if e.status not in (409, 412):
                    raise
                pending = marked  # lost a race on some of them: re-read and re-apply
        raise ConcurrencyConflict(f"{len(pending)} overdue tasks kept changing under concurrent writers")

    async def _publish_task_saved(self, t: TaskModel, payload: RawJson | None = None) -> None:
        log.info(LOG_PUBLISH, t.task_id, t.task_name, t.task_assigned_to)
        await self.client.publish_event(self.pubsub, self.topic,
                                        payload if payload is not None else RawJson(t.to_store_json()))
