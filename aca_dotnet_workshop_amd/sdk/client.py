"""Application-side client for the sidecar -- the ``Dapr.Client.DaprClient`` equivalent.

Every call the reference makes through ``DaprClient`` has a method here (SURVEY.md §2.10
call-site table):

=====================  ===================================================  =========================
reference call         reference site                                        here
=====================  ===================================================  =========================
InvokeMethodAsync      Frontend Pages/Tasks/Index.cshtml.cs:48 (+5 more)      ``invoke_method``
SaveStateAsync         Backend.Api Services/TasksStoreManager.cs:35,78,94     ``save_state``
GetStateAsync          TasksStoreManager.cs:50,74,87                          ``get_state``
DeleteStateAsync       TasksStoreManager.cs:43                                ``delete_state``
QueryStateAsync        TasksStoreManager.cs:61,130                            ``query_state``
PublishEventAsync      TasksStoreManager.cs:155                               ``publish_event``
InvokeBindingAsync     Processor ExternalTasksProcessorController.cs:43       ``invoke_binding``
=====================  ===================================================  =========================

The sidecar is reached over a Unix domain socket when ``TT_SIDECAR_UDS`` is set (the
platform does this for co-located app/sidecar pairs), else over
``DAPR_HTTP_ENDPOINT`` / ``http://127.0.0.1:$DAPR_HTTP_PORT`` (default 3500), matching
the reference's port plan (.vscode/tasks.json:126-165).
"""
from __future__ import annotations

import asyncio
import base64
import json
import os
from dataclasses import dataclass, field
from typing import Any
from urllib.parse import quote, urlencode

from ..telemetry import tracing
from ..web.client import ClientResponse, HttpClient


class InvocationError(Exception):
    """Non-success response from a sidecar call (``InvocationException`` / ``DaprException``)."""

    def __init__(self, status: int, body: bytes, what: str) -> None:
        super().__init__(f"{what} failed with HTTP {status}: {body[:300]!r}")
        self.status = status
        self.body = body


@dataclass
class StateItem:
    key: str
    data: Any
    etag: str | None = None


@dataclass
class QueryResponse:
    results: list[StateItem] = field(default_factory=list)
    token: str | None = None
    metadata: dict[str, str] = field(default_factory=dict)


class RawJson(str):
    """A value that is already JSON text (e.g. ``TaskModel.to_json()``): sent verbatim, so a
    model serialised once can be saved and published without re-encoding."""


class RawJsonBytes(bytes):
    """JSON text already encoded as UTF-8 (e.g. a page a native codec produced): sent verbatim
    as ``application/json`` without a decode/encode round trip."""


def _value_json(v: Any) -> str:
    if isinstance(v, RawJson):
        return v
    return json.dumps(to_jsonable(v), separators=(",", ":"))


def _encode(data: Any) -> tuple[bytes, str]:
    if data is None:
        return b"", "application/json"
    if isinstance(data, RawJson):
        return data.encode(), "application/json"
    if isinstance(data, RawJsonBytes):
        return bytes(data), "application/json"
    if isinstance(data, (bytes, bytearray)):
        return bytes(data), "application/octet-stream"
    if isinstance(data, str):
        return json.dumps(data).encode(), "application/json"
    return json.dumps(to_jsonable(data), separators=(",", ":")).encode(), "application/json"


def to_jsonable(data: Any) -> Any:
    if hasattr(data, "to_wire"):
        return data.to_wire()
    if isinstance(data, list):
        return [to_jsonable(x) for x in data]
    if isinstance(data, tuple):
        return [to_jsonable(x) for x in data]
    if isinstance(data, dict):
        return {k: to_jsonable(v) for k, v in data.items()}
    if hasattr(data, "isoformat"):
        from ..models.dotnet import format_datetime
        return format_datetime(data)
    if hasattr(data, "hex") and data.__class__.__name__ == "UUID":
        return str(data)
    return data


def sidecar_base_url(environ: dict[str, str] | None = None) -> str:
    env = os.environ if environ is None else environ
    uds = env.get("TT_SIDECAR_UDS")
    if uds:
        return f"unix:{uds}:"
    ep = env.get("DAPR_HTTP_ENDPOINT")
    if ep:
        return ep.rstrip("/")
    return f"http://127.0.0.1:{env.get('DAPR_HTTP_PORT', '3500')}"


class SidecarClient:
    def __init__(self, base_url: str | None = None, api_token: str | None = None,
                 http: HttpClient | None = None, timeout: float = 60.0) -> None:
        self.base = base_url or sidecar_base_url()
        if http is None:
            from ..web import native_host
            http = native_host.NativeHttpClient(timeout=timeout) if native_host.enabled(part="client") else HttpClient(timeout=timeout)
        self.http = http
        self.api_token = api_token if api_token is not None else os.environ.get("DAPR_API_TOKEN")
        # the native host takes requests to a pre-split endpoint (no URL parsing per call)
        self._at = None
        if hasattr(http, "request_at"):
            from ..web.client import parse_endpoint
            key, prefix = parse_endpoint(self.base + "/")
            if key[0] in ("unix", "tcp"):
                self._at, self._key, self._prefix = http.request_at, key, prefix.rstrip("/")

    def native_endpoint(self) -> dict[str, str] | None:
        """Where a native route (web/native_host.py ``native_route``) reaches this sidecar the
        way this client does: the app host's endpoint, the path prefix, the API token and the
        timeout; None when this client does not run on the native host."""
        if self._at is None:
            return None
        key = self._key
        ep = f"unix:{key[1]}" if key[0] == "unix" else f"tcp:{key[1]}:{key[2]}"
        return {"sidecar": ep, "prefix": self._prefix, "token": self.api_token or "",
                "timeout": repr(float(getattr(self.http, "timeout", 60.0)))}

    # -- plumbing -------------------------------------------------------------
    def _headers(self, ctype: str | None = None, extra: dict[str, str] | None = None) -> list[tuple[str, str]]:
        h: list[tuple[str, str]] = []
        tp = tracing.current_traceparent()
        if tp:
            h.append(("traceparent", tp))
        if self.api_token:
            h.append(("dapr-api-token", self.api_token))
        if ctype:
            h.append(("Content-Type", ctype))
        if extra:
            h.extend(extra.items())
        return h

    async def _call(self, method: str, path: str, body: bytes = b"", ctype: str | None = None,
                    extra: dict[str, str] | None = None, span_name: str | None = None) -> ClientResponse:
        parent = tracing.current_span()
        if parent is not None and not parent.sampled and self._at is not None:
            # inside an unsampled trace nothing is recorded: propagate the context, skip the span
            h = [("traceparent", parent.traceparent)]
            if self.api_token:
                h.append(("dapr-api-token", self.api_token))
            if ctype:
                h.append(("Content-Type", ctype))
            if extra:
                h.extend(extra.items())
            return await self._at(self._key, method, self._prefix + path, h, body)
        tr = tracing.tracer()
        span = tr.start_span(span_name or method, "client")
        if span.sampled and not span_name:
            span.name = f"{method} {path}"
        try:
            resp = await self.http.request(method, self.base + path, headers=self._headers(ctype, extra), body=body)
            span.set("http.status", resp.status)
            if resp.status >= 400:
                span.status = "error"
            return resp
        except BaseException as e:
            span.fail(e)
            raise
        finally:
            span.end()

    async def wait_for_sidecar(self, timeout: float = 30.0) -> None:
        deadline = asyncio.get_running_loop().time() + timeout
        while True:
            try:
                r = await self.http.request("GET", self.base + "/v1.0/healthz/outbound", timeout=2.0)
                if r.status < 300:
                    return
            except (OSError, asyncio.TimeoutError):
                pass
            if asyncio.get_running_loop().time() > deadline:
                raise TimeoutError("sidecar not ready")
            await asyncio.sleep(0.05)

    # -- service invocation ---------------------------------------------------
    async def invoke_method_raw(self, method: str, app_id: str, path: str, data: Any = None,
                                headers: dict[str, str] | None = None) -> ClientResponse:
        body, ctype = _encode(data) if data is not None else (b"", None)
        p = path.lstrip("/")
        return await self._call(method.upper(), f"/v1.0/invoke/{app_id}/method/{p}", body, ctype, headers,
                                span_name=f"invoke {app_id} {method.upper()} /{p.split('?')[0]}")

    async def invoke_method(self, method: str, app_id: str, path: str, data: Any = None,
                            headers: dict[str, str] | None = None) -> Any:
        """Invoke and return the parsed JSON response (``None`` for an empty body);
        raises ``InvocationError`` on non-2xx like the .NET SDK."""
        r = await self.invoke_method_raw(method, app_id, path, data, headers)
        if r.status >= 300:
            raise InvocationError(r.status, r.body, f"invoke {app_id}/{path}")
        if not r.body:
            return None
        ctype = r.headers.get("content-type", "")
        if "json" in ctype or not ctype:
            try:
                return json.loads(r.body)
            except ValueError:
                return r.body.decode()
        return r.body.decode() if ctype.startswith("text/") else r.body

    # -- state ------------------------------------------------------------------
    async def save_state(self, store: str, key: str, value: Any, etag: str | None = None,
                         metadata: dict[str, str] | None = None, concurrency: str | None = None,
                         consistency: str | None = None) -> None:
        item: dict[str, Any] = {"key": key}
        if etag is not None:
            item["etag"] = etag
        if metadata:
            item["metadata"] = metadata
        opts = {k: v for k, v in (("concurrency", concurrency), ("consistency", consistency)) if v}
        if opts:
            item["options"] = opts
        # splice the value's JSON in (a RawJson value is not re-encoded)
        body = "[" + json.dumps(item, separators=(",", ":"))[:-1] + ',"value":' + _value_json(value) + "}]"
        await self._save_body(store, body.encode())

    async def save_bulk_state(self, store: str, items: list[dict[str, Any]]) -> None:
        await self._save_body(store, json.dumps(items, separators=(",", ":")).encode())

    async def save_state_body(self, store: str, body: bytes) -> None:
        """Save with a request body already in the state API's form (``[{"key", "value", ...}]``)."""
        r = await self._call("POST", f"/v1.0/state/{store}", body, "application/json", span_name=f"state save {store}")
        if r.status >= 300:
            raise InvocationError(r.status, r.body, f"save state {store}")

    async def _save_body(self, store: str, body: bytes) -> None:
        r = await self._call("POST", f"/v1.0/state/{store}", body, "application/json", span_name=f"state save {store}")
        if r.status >= 300:
            raise InvocationError(r.status, r.body, f"save state {store}")

    async def get_state_and_etag(self, store: str, key: str) -> tuple[Any, str | None]:
        r = await self._call("GET", f"/v1.0/state/{store}/{quote(key, safe='')}", span_name=f"state get {store}")
        if r.status == 204 or (r.status == 200 and not r.body):
            return None, None
        if r.status >= 300:
            raise InvocationError(r.status, r.body, f"get state {store}/{key}")
        return json.loads(r.body), r.headers.get("etag")

    async def get_state(self, store: str, key: str) -> Any:
        return (await self.get_state_and_etag(store, key))[0]

    async def get_state_raw(self, store: str, key: str) -> tuple[bytes | None, str | None]:
        """``get_state_and_etag`` without decoding: (the stored JSON text or None, its ETag)."""
        r = await self._call("GET", f"/v1.0/state/{store}/{quote(key, safe='')}", span_name=f"state get {store}")
        if r.status == 204 or (r.status == 200 and not r.body):
            return None, None
        if r.status >= 300:
            raise InvocationError(r.status, r.body, f"get state {store}/{key}")
        return r.body, r.headers.get("etag")

    async def get_bulk_state(self, store: str, keys: list[str], parallelism: int = 10) -> list[StateItem]:
        return [StateItem(x["key"], x.get("data"), x.get("etag"))
                for x in json.loads(await self.get_bulk_state_raw(store, keys, parallelism))]

    async def get_bulk_state_raw(self, store: str, keys: list[str], parallelism: int = 10) -> bytes:
        """The bulk-get answer as the sidecar sent it (``[{"key", "data", "etag"}]``)."""
        body = json.dumps({"keys": keys, "parallelism": parallelism}, separators=(",", ":")).encode()
        r = await self._call("POST", f"/v1.0/state/{store}/bulk", body, "application/json",
                             span_name=f"state bulkget {store}")
        if r.status >= 300:
            raise InvocationError(r.status, r.body, f"bulk get {store}")
        return r.body

    async def delete_state(self, store: str, key: str, etag: str | None = None) -> None:
        extra = {"If-Match": etag} if etag else None
        r = await self._call("DELETE", f"/v1.0/state/{store}/{quote(key, safe='')}", extra=extra,
                             span_name=f"state delete {store}")
        if r.status >= 300:
            raise InvocationError(r.status, r.body, f"delete state {store}/{key}")

    async def execute_state_transaction(self, store: str, operations: list[dict[str, Any]],
                                        metadata: dict[str, str] | None = None) -> None:
        payload: dict[str, Any] = {"operations": to_jsonable(operations)}
        if metadata:
            payload["metadata"] = metadata
        r = await self._call("POST", f"/v1.0/state/{store}/transaction", json.dumps(payload).encode(),
                             "application/json", span_name=f"state transaction {store}")
        if r.status >= 300:
            raise InvocationError(r.status, r.body, f"transaction {store}")

    async def query_state_raw(self, store: str, query: dict[str, Any] | str,
                              metadata: dict[str, str] | None = None) -> bytes:
        """The state-query API's response body as is (``{"results": [...], "token": ...}``)."""
        body = query.encode() if isinstance(query, str) else json.dumps(query).encode()
        path = f"/v1.0-alpha1/state/{store}/query"
        if metadata:
            path += "?" + urlencode({f"metadata.{k}": v for k, v in metadata.items()})
        r = await self._call("POST", path, body, "application/json", span_name=f"state query {store}")
        if r.status >= 300:
            raise InvocationError(r.status, r.body, f"query state {store}")
        return r.body

    async def query_state(self, store: str, query: dict[str, Any] | str,
                          metadata: dict[str, str] | None = None) -> QueryResponse:
        raw = await self.query_state_raw(store, query, metadata)
        js = json.loads(raw) if raw else {}
        items = [StateItem(x.get("key"), x.get("data"), x.get("etag")) for x in js.get("results") or []]
        return QueryResponse(items, js.get("token"), js.get("metadata") or {})

    # -- pub/sub ----------------------------------------------------------------
    async def publish_event(self, pubsub: str, topic: str, data: Any, content_type: str | None = None,
                            metadata: dict[str, str] | None = None) -> None:
        body, ctype = _encode(data)
        path = f"/v1.0/publish/{pubsub}/{topic}"
        if metadata:
            path += "?" + urlencode({f"metadata.{k}": v for k, v in metadata.items()})
        r = await self._call("POST", path, body, content_type or ctype, span_name=f"publish {pubsub}/{topic}")
        if r.status >= 300:
            raise InvocationError(r.status, r.body, f"publish {pubsub}/{topic}")

    async def publish_events(self, pubsub: str, topic: str, events: list[Any]) -> dict[str, Any]:
        entries = []
        for i, e in enumerate(events):
            entries.append({"entryId": str(i), "event": to_jsonable(e), "contentType": "application/json"})
        r = await self._call("POST", f"/v1.0-alpha1/publish/bulk/{pubsub}/{topic}", json.dumps(entries).encode(),
                             "application/json", span_name=f"publish-bulk {pubsub}/{topic}")
        if r.status >= 300:
            raise InvocationError(r.status, r.body, f"bulk publish {pubsub}/{topic}")
        return r.json() or {"failedEntries": []}

    # -- bindings ---------------------------------------------------------------
    async def invoke_binding(self, name: str, operation: str, data: Any = None,
                             metadata: dict[str, str] | None = None) -> Any:
        payload = {"data": to_jsonable(data), "operation": operation}
        if metadata:
            payload["metadata"] = dict(metadata)
        r = await self._call("POST", f"/v1.0/bindings/{name}", json.dumps(payload).encode(), "application/json",
                             span_name=f"binding {name} {operation}")
        if r.status >= 300:
            raise InvocationError(r.status, r.body, f"binding {name}/{operation}")
        if not r.body:
            return None
        try:
            return json.loads(r.body)
        except ValueError:
            return r.body

    # -- secrets ----------------------------------------------------------------
    async def get_secret(self, store: str, key: str, metadata: dict[str, str] | None = None) -> dict[str, str]:
        path = f"/v1.0/secrets/{store}/{quote(key, safe='')}"
        if metadata:
            path += "?" + urlencode({f"metadata.{k}": v for k, v in metadata.items()})
        r = await self._call("GET", path, span_name=f"secret get {store}")
        if r.status >= 300:
            raise InvocationError(r.status, r.body, f"get secret {store}/{key}")
        return r.json()

    async def get_bulk_secret(self, store: str) -> dict[str, dict[str, str]]:
        r = await self._call("GET", f"/v1.0/secrets/{store}/bulk", span_name=f"secret bulk {store}")
        if r.status >= 300:
            raise InvocationError(r.status, r.body, f"bulk secret {store}")
        return r.json()

    # -- metadata / lifecycle --------------------------------------------------
    async def get_metadata(self) -> dict[str, Any]:
        r = await self._call("GET", "/v1.0/metadata")
        return r.json()

    async def set_metadata(self, key: str, value: str) -> None:
        r = await self._call("PUT", f"/v1.0/metadata/{quote(key, safe='')}", value.encode(), "text/plain")
        if r.status >= 300:
            raise InvocationError(r.status, r.body, f"set metadata {key}")

    async def shutdown_sidecar(self) -> None:
        await self._call("POST", "/v1.0/shutdown")

    async def close(self) -> None:
        await self.http.close()


DaprClient = SidecarClient  # familiar alias for users coming from the reference


def client_from_config(config=None, environ: dict[str, str] | None = None):
    """The sidecar client a service should use: HTTP by default, gRPC when
    ``Dapr:ApiProtocol`` (or ``DAPR_API_PROTOCOL``) is ``grpc`` -- the transport the reference's
    .NET ``DaprClient`` uses for state / pub/sub / bindings."""
    env = os.environ if environ is None else environ
    proto = (config.get_str("Dapr:ApiProtocol") if config is not None else None) or env.get("DAPR_API_PROTOCOL", "http")
    if proto.lower() == "grpc":
        from .grpc_client import GrpcSidecarClient, sidecar_grpc_target
        return GrpcSidecarClient(sidecar_grpc_target(env))
    return SidecarClient(sidecar_base_url(env))


def b64(data: bytes) -> str:
    return base64.b64encode(data).decode()


def native_route_failure(req: Any, what: dict[str, str], key: str | None = None) -> BaseException | None:
    """The error a native route handed over (``fail <step> <status> <base64 body>`` or ``err
    <step> <errno>`` in ``req.state["tt_native"]``, set by web/native_host.py only) as the
    exception this SDK raises for that call (``what``: the step's InvocationError message), or
    None for an ordinary request."""
    note = req.state.get("tt_native")
    if not note or note == "sample":
        return None
    parts = note.split(" ")
    if key is not None and len(parts) >= 2 and "{key}" in what.get(parts[1], ""):
        what = {**what, parts[1]: what[parts[1]].replace("{key}", key)}
    if len(parts) >= 3 and parts[1] in what and parts[1] != "protocol":
        if parts[0] == "fail":
            import base64
            body = base64.b64decode(parts[3]) if len(parts) > 3 else b""
            return InvocationError(int(parts[2]), body, what[parts[1]])
        if parts[0] == "err":
            from ..web.native_host import _client_error
            err = int(parts[2])
            exc = _client_error(err, os.strerror(err))
            if what.get("protocol") == "grpc":  # GrpcSidecarClient's answer to a transport error
                if isinstance(exc, asyncio.TimeoutError):
                    return InvocationError(504, b"Deadline Exceeded", what[parts[1]])
                return InvocationError(503, f"sidecar unreachable: {exc}".encode(), what[parts[1]])
            return exc
    return RuntimeError(f"malformed native route hand-over: {note[:80]!r}")
