"""gRPC flavour of the sidecar client -- ``DaprClient`` as the reference's .NET SDK builds it.

``Dapr.Client.DaprClient`` sends ``SaveStateAsync`` / ``GetStateAsync`` / ``DeleteStateAsync`` /
``QueryStateAsync`` / ``PublishEventAsync`` / ``InvokeBindingAsync`` over the sidecar's gRPC
port (``DAPR_GRPC_PORT``; reference Backend.Api Services/TasksStoreManager.cs:35-156,
Processor ExternalTasksProcessorController.cs:43).  ``GrpcSidecarClient`` has the same method
surface as the HTTP ``SidecarClient`` so a service picks its transport by configuration
(``Dapr:ApiProtocol`` = ``http`` | ``grpc``) without code changes; errors surface as the same
``InvocationError`` (its ``status`` is the HTTP status the sidecar reported, or the closest
HTTP equivalent of the gRPC code).
"""
from __future__ import annotations

import asyncio
import json
import os
from typing import Any

import grpc

from ..telemetry import tracing
from ..web.client import ClientResponse
from ..web.http import Headers
from . import proto as P
from .client import InvocationError, QueryResponse, RawJson, StateItem, _encode, _value_json, to_jsonable

_HTTP_OF = {grpc.StatusCode.INVALID_ARGUMENT: 400, grpc.StatusCode.UNAUTHENTICATED: 401,
            grpc.StatusCode.PERMISSION_DENIED: 403, grpc.StatusCode.NOT_FOUND: 404, grpc.StatusCode.ABORTED: 409,
            grpc.StatusCode.RESOURCE_EXHAUSTED: 429, grpc.StatusCode.UNIMPLEMENTED: 501,
            grpc.StatusCode.UNAVAILABLE: 503, grpc.StatusCode.DEADLINE_EXCEEDED: 504}
_CONCURRENCY = {"first-write": 1, "last-write": 2}
_CONSISTENCY = {"eventual": 1, "strong": 2}


def sidecar_grpc_target(environ: dict[str, str] | None = None) -> str:
    """``DAPR_GRPC_ENDPOINT``, else the co-located sidecar's gRPC Unix socket
    (``TT_SIDECAR_GRPC_UDS``, set by the sidecar runner next to ``TT_SIDECAR_UDS``), else
    ``127.0.0.1:$DAPR_GRPC_PORT``."""
    env = os.environ if environ is None else environ
    ep = env.get("DAPR_GRPC_ENDPOINT")
    if ep:
        return ep.replace("http://", "").replace("https://", "").rstrip("/")
    uds = env.get("TT_SIDECAR_GRPC_UDS")
    if uds:
        return f"unix:{uds}"
    return f"127.0.0.1:{env.get('DAPR_GRPC_PORT', '50001')}"


def _native():
    from ..native import load
    return load()


def query_response_json(raw: bytes) -> bytes:
    """A serialized ``QueryStateResponse`` as the HTTP state-query API's JSON answer
    (``{"results":[{"key","data","etag"}],"token"}``, the layout the task codec reads and the
    app host's gRPC routes build: daprpb.hpp ``query_response_json``)."""
    made = _native().dapr_pb_query_json(raw)
    if made is not None:
        return made
    r = P.rt("QueryStateResponse").FromString(raw)
    parts = []
    for i in r.results:
        parts.append('{"key":%s,"data":%s,"etag":%s}' % (json.dumps(i.key), i.data.decode() if i.data else "null",
                                                        json.dumps(i.etag)))
    out = '{"results":[' + ",".join(parts) + "]"
    if r.token:
        out += ',"token":' + json.dumps(r.token)
    return (out + "}").encode()


def _loads(b: bytes) -> Any:
    if not b:
        return None
    try:
        return json.loads(b)
    except ValueError:
        return b.decode("utf-8", "replace")


def _varint(n: int) -> bytes:
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _ld(field: int, data: bytes) -> bytes:
    """One length-delimited protobuf field (strings, bytes, sub-messages)."""
    return _varint((field << 3) | 2) + _varint(len(data)) + data


def encode_save_state(store: str, key: str, value_json: bytes) -> bytes:
    """``SaveStateRequest{store_name, states: [StateItem{key, value}]}`` without message objects
    (the common save: no ETag, metadata or options)."""
    return _ld(1, store.encode()) + _ld(2, _ld(1, key.encode()) + _ld(2, value_json))


def encode_publish_event(pubsub: str, topic: str, data: bytes, content_type: str) -> bytes:
    """``PublishEventRequest{pubsub_name, topic, data, data_content_type}`` (no metadata)."""
    return _ld(1, pubsub.encode()) + _ld(2, topic.encode()) + _ld(3, data) + _ld(4, content_type.encode())


class _NativeRpcError(Exception):
    """A non-OK gRPC status from the native transport (shape of ``grpc.aio.AioRpcError``)."""

    def __init__(self, code: grpc.StatusCode, details: str, trailing: list[tuple[str, str]]) -> None:
        super().__init__(details)
        self._code, self._details, self._trailing = code, details, trailing

    def code(self) -> grpc.StatusCode:
        return self._code

    def details(self) -> str:
        return self._details

    def trailing_metadata(self):
        return self._trailing


_STATUS_OF = {c.value[0]: c for c in grpc.StatusCode}


class _NativeChannel:
    """Unary calls over the native app host's HTTP/2 client (native/src/h2.hpp GrpcClient): the
    app process's gRPC to its sidecar leaves Python as one batched hand-off per loop iteration,
    like the HTTP client's requests -- no grpcio completion-queue threads in the way."""

    def __init__(self, target: str) -> None:
        from ..web import native_host
        self.endpoint = target if target.startswith("unix:") else f"tcp:{target}"
        self._native = native_host.NativeHttpClient()

    def unary_unary(self, path: str, request_serializer, response_deserializer):
        async def call(req, metadata=None, timeout=None):
            host = self._native._native()
            try:
                r = await host.grpc_call(self.endpoint, path, list(metadata or ()), request_serializer(req),
                                         timeout or 0.0)
            except OSError as e:
                raise _NativeRpcError(grpc.StatusCode.UNAVAILABLE, f"sidecar unreachable: {e}", []) from None
            except asyncio.TimeoutError:
                raise _NativeRpcError(grpc.StatusCode.DEADLINE_EXCEEDED, "Deadline Exceeded", []) from None
            if r.status != 0:
                md = [(k, v) for k, v in r.headers.items() if isinstance(v, str)]
                raise _NativeRpcError(_STATUS_OF.get(r.status, grpc.StatusCode.UNKNOWN),
                                      r.headers.get("grpc-message", ""), md)
            return response_deserializer(r.body)
        return call

    async def channel_ready(self) -> None:
        host = self._native._native()
        req_cls, resp_cls = P.rpc_types("GetMetadata")
        deadline = asyncio.get_running_loop().time() + 30
        while True:  # the sidecar's gRPC port may not be listening yet
            try:
                await host.grpc_call(self.endpoint, P.method_path("GetMetadata"), [], req_cls().SerializeToString(), 5.0)
                return
            except OSError:
                if asyncio.get_running_loop().time() > deadline:
                    raise
                await asyncio.sleep(0.05)

    async def close(self) -> None:
        await self._native.close()


class GrpcSidecarClient:
    def __init__(self, target: str | None = None, api_token: str | None = None, timeout: float = 60.0,
                 transport: str | None = None) -> None:
        self.target = target or sidecar_grpc_target()
        self.api_token = api_token if api_token is not None else os.environ.get("DAPR_API_TOKEN")
        self.timeout = timeout
        if transport is None:  # the native app host's HTTP/2 client when the app runs on it
            from ..web import native_host
            transport = "native" if native_host.enabled(part="client") else "grpcio"
        self.transport = transport
        self._channel: Any = None
        self._stubs: dict[str, Any] = {}

    def native_endpoint(self) -> dict[str, str] | None:
        """Where a native route of the app host reaches this sidecar's gRPC port the way this
        client does (SidecarClient.native_endpoint's shape, ``protocol`` = ``grpc``); None on
        the grpcio transport."""
        if self.transport != "native":
            return None
        ep = self.target if self.target.startswith("unix:") else f"tcp:{self.target}"
        return {"sidecar": ep, "prefix": "", "token": self.api_token or "", "timeout": repr(float(self.timeout)),
                "protocol": "grpc"}

    def _new_channel(self):
        return _NativeChannel(self.target) if self.transport == "native" else grpc.aio.insecure_channel(self.target)

    # -- plumbing -------------------------------------------------------------
    def _stub(self, rpc: str):
        st = self._stubs.get(rpc)
        if st is None:
            if self._channel is None:
                self._channel = self._new_channel()
            req_cls, resp_cls = P.rpc_types(rpc)
            st = self._channel.unary_unary(P.method_path(rpc), request_serializer=req_cls.SerializeToString,
                                           response_deserializer=resp_cls.FromString)
            self._stubs[rpc] = st
        return st

    def _metadata(self) -> list[tuple[str, str]]:
        md = []
        tp = tracing.current_traceparent()
        if tp:
            md.append(("traceparent", tp))
        if self.api_token:
            md.append(("dapr-api-token", self.api_token))
        return md

    async def _call_encoded(self, rpc: str, payload: bytes, span_name: str) -> bytes:
        """A unary call whose request is already serialized; returns the serialized response
        (SaveState, PublishEvent: ``Empty``).  On the native transport inside an unsampled trace
        it goes straight to the app host's HTTP/2 client, without a span."""
        parent = tracing.current_span()
        if self.transport == "native" and parent is not None and not parent.sampled:
            if self._channel is None:
                self._channel = self._new_channel()
            md = [("traceparent", parent.traceparent)]
            if self.api_token:
                md.append(("dapr-api-token", self.api_token))
            try:
                r = await self._channel._native._native().grpc_call(self._channel.endpoint, P.method_path(rpc), md,
                                                                     payload, self.timeout)
            except OSError as e:
                raise InvocationError(503, f"sidecar unreachable: {e}".encode(), rpc) from None
            except asyncio.TimeoutError:
                raise InvocationError(504, b"Deadline Exceeded", rpc) from None
            if r.status != 0:
                status = _HTTP_OF.get(_STATUS_OF.get(r.status, grpc.StatusCode.UNKNOWN), 500)
                if "dapr-http-status" in r.headers:
                    status = int(r.headers["dapr-http-status"])
                raise InvocationError(status, r.headers.get("grpc-message", "").encode(), rpc)
            return r.body
        req_cls, _ = P.rpc_types(rpc)
        return (await self._call(rpc, req_cls.FromString(payload), span_name)).SerializeToString()

    async def _call(self, rpc: str, req, span_name: str):
        span = tracing.tracer().start_span(span_name, "client")
        span.set("rpc.system", "grpc")
        try:
            return await self._stub(rpc)(req, metadata=self._metadata(), timeout=self.timeout)
        except (grpc.aio.AioRpcError, _NativeRpcError) as e:
            span.fail(e)
            status = _HTTP_OF.get(e.code(), 500)
            for k, v in e.trailing_metadata() or ():
                if k == "dapr-http-status":
                    status = int(v)
            raise InvocationError(status, (e.details() or "").encode(), f"{rpc}") from None
        except BaseException as e:
            span.fail(e)
            raise
        finally:
            span.end()

    async def wait_for_sidecar(self, timeout: float = 30.0) -> None:
        if self._channel is None:
            self._channel = self._new_channel()
        await asyncio.wait_for(self._channel.channel_ready(), timeout)

    # -- service invocation ---------------------------------------------------
    async def invoke_method_raw(self, method: str, app_id: str, path: str, data: Any = None,
                                headers: dict[str, str] | None = None) -> ClientResponse:
        path, _, qs = path.lstrip("/").partition("?")
        req = P.rt("InvokeServiceRequest")(id=app_id)
        req.message.method = path
        req.message.http_extension.verb = P.verb_number(method)
        req.message.http_extension.querystring = qs
        if data is not None:
            body, ctype = _encode(data)
            req.message.data.value = body
            req.message.content_type = ctype
        try:
            r = await self._call("InvokeService", req, f"invoke {app_id} {method.upper()} /{path}")
        except InvocationError as e:
            return ClientResponse(e.status, Headers(), e.body)
        h = Headers()
        if r.content_type:
            h["content-type"] = r.content_type
        return ClientResponse(200, h, r.data.value)

    async def invoke_method(self, method: str, app_id: str, path: str, data: Any = None,
                            headers: dict[str, str] | None = None) -> Any:
        r = await self.invoke_method_raw(method, app_id, path, data, headers)
        if r.status >= 300:
            raise InvocationError(r.status, r.body, f"invoke {app_id}/{path}")
        return _loads(r.body)

    # -- state ------------------------------------------------------------------
    @staticmethod
    def _item(msg, key: str, value: Any, etag: str | None, metadata: dict[str, str] | None,
              concurrency: str | None, consistency: str | None) -> None:
        msg.key = key
        msg.value = _value_json(value).encode()
        if etag is not None:
            msg.etag.value = etag
        for k, v in (metadata or {}).items():
            msg.metadata[k] = str(v)
        if concurrency:
            msg.options.concurrency = _CONCURRENCY[concurrency]
        if consistency:
            msg.options.consistency = _CONSISTENCY[consistency]

    async def save_state(self, store: str, key: str, value: Any, etag: str | None = None,
                         metadata: dict[str, str] | None = None, concurrency: str | None = None,
                         consistency: str | None = None) -> None:
        if etag is None and not metadata and not concurrency and not consistency:
            await self._call_encoded("SaveState", encode_save_state(store, key, _value_json(value).encode()),
                                     f"state save {store}")
            return
        req = P.rt("SaveStateRequest")(store_name=store)
        self._item(req.states.add(), key, value, etag, metadata, concurrency, consistency)
        await self._call("SaveState", req, f"state save {store}")

    async def save_bulk_state(self, store: str, items: list[dict[str, Any]]) -> None:
        req = P.rt("SaveStateRequest")(store_name=store)
        for it in items:
            opts = it.get("options") or {}
            etag = it.get("etag")
            self._item(req.states.add(), it["key"], it.get("value"), etag.get("value") if isinstance(etag, dict) else etag,
                       it.get("metadata"), opts.get("concurrency"), opts.get("consistency"))
        await self._call("SaveState", req, f"state save {store}")

    async def get_state_and_etag(self, store: str, key: str) -> tuple[Any, str | None]:
        r = await self._call("GetState", P.rt("GetStateRequest")(store_name=store, key=key), f"state get {store}")
        if not r.data:
            return None, None
        return json.loads(r.data), r.etag or None

    async def get_state(self, store: str, key: str) -> Any:
        return (await self.get_state_and_etag(store, key))[0]

    async def get_state_raw(self, store: str, key: str) -> tuple[bytes | None, str | None]:
        """``get_state_and_etag`` without decoding the value: (its JSON text or None, its ETag)."""
        raw = await self._call_encoded("GetState", P.rt("GetStateRequest")(store_name=store, key=key).SerializeToString(),
                                       f"state get {store}")
        r = P.rt("GetStateResponse").FromString(raw)
        return (r.data, r.etag or None) if r.data else (None, None)

    async def get_bulk_state(self, store: str, keys: list[str], parallelism: int = 10) -> list[StateItem]:
        r = await self._call("GetBulkState", P.rt("GetBulkStateRequest")(store_name=store, keys=keys,
                                                                         parallelism=parallelism),
                             f"state bulkget {store}")
        return [StateItem(i.key, _loads(i.data), i.etag or None) for i in r.items]

    async def delete_state(self, store: str, key: str, etag: str | None = None) -> None:
        req = P.rt("DeleteStateRequest")(store_name=store, key=key)
        if etag:
            req.etag.value = etag
        await self._call("DeleteState", req, f"state delete {store}")

    async def execute_state_transaction(self, store: str, operations: list[dict[str, Any]],
                                        metadata: dict[str, str] | None = None) -> None:
        req = P.rt("ExecuteStateTransactionRequest")(storeName=store)
        for op in operations:
            o = req.operations.add(operationType=op.get("operation", ""))
            r = op.get("request") or {}
            opts = r.get("options") or {}
            etag = r.get("etag")
            o.request.key = r.get("key", "")
            if op.get("operation", "").lower() == "upsert":
                o.request.value = _value_json(to_jsonable(r.get("value"))).encode()
            if etag:
                o.request.etag.value = etag.get("value") if isinstance(etag, dict) else etag
            for k, v in (r.get("metadata") or {}).items():
                o.request.metadata[k] = str(v)
            if opts.get("concurrency"):
                o.request.options.concurrency = _CONCURRENCY[opts["concurrency"]]
        for k, v in (metadata or {}).items():
            req.metadata[k] = str(v)
        await self._call("ExecuteStateTransaction", req, f"state transaction {store}")

    async def query_state(self, store: str, query: dict[str, Any] | str,
                          metadata: dict[str, str] | None = None) -> QueryResponse:
        q = query if isinstance(query, str) else json.dumps(query)
        req = P.rt("QueryStateRequest")(store_name=store, query=q, metadata=metadata or {})
        r = await self._call("QueryStateAlpha1", req, f"state query {store}")
        return QueryResponse([StateItem(i.key, _loads(i.data), i.etag or None) for i in r.results], r.token or None,
                             dict(r.metadata))

    async def save_state_body(self, store: str, body: bytes) -> None:
        """Save with a body in the state HTTP API's form (``[{"key", "value", "etag", "options"}]``,
        what the task codecs write) as one SaveStateRequest (daprpb.hpp ``save_state_bulk``: each
        value's JSON text as is) -- the bytes the app host's native routes send."""
        msg = _native().dapr_pb_save_state_bulk(store, bytes(body))
        if msg is None:
            await self.save_bulk_state(store, json.loads(body))
            return
        await self._call_encoded("SaveState", msg, f"state save {store}")

    async def get_bulk_state_raw(self, store: str, keys: list[str], parallelism: int = 10) -> bytes:
        """``get_bulk_state``'s answer as the HTTP bulk-get API's JSON (``[{"key","data","etag"} |
        {"key"}]``), the text the markoverdue codec reads whichever protocol carried it."""
        raw = await self._call_encoded("GetBulkState", _native().dapr_pb_get_bulk_state(store, list(keys), parallelism),
                                       f"state bulkget {store}")
        made = _native().dapr_pb_bulk_state_json(raw)
        if made is not None:
            return made
        r = P.rt("GetBulkStateResponse").FromString(raw)
        return json.dumps([{"key": i.key, "data": _loads(i.data), "etag": i.etag} if i.data and i.data != b"null"
                           else {"key": i.key} for i in r.items], separators=(",", ":")).encode()

    async def query_state_raw(self, store: str, query: dict[str, Any] | str,
                              metadata: dict[str, str] | None = None) -> bytes:
        """``query_state``'s answer as the HTTP API's JSON text (``query_response_json``): the
        managers' one-pass codecs read it whichever protocol carried it."""
        q = query if isinstance(query, str) else json.dumps(query)
        req = P.rt("QueryStateRequest")(store_name=store, query=q, metadata=metadata or {})
        raw = await self._call_encoded("QueryStateAlpha1", req.SerializeToString(), f"state query {store}")
        return query_response_json(raw)

    # -- pub/sub ----------------------------------------------------------------
    async def publish_event(self, pubsub: str, topic: str, data: Any, content_type: str | None = None,
                            metadata: dict[str, str] | None = None) -> None:
        body, ctype = _encode(data)
        if not metadata:
            await self._call_encoded("PublishEvent", encode_publish_event(pubsub, topic, body, content_type or ctype),
                                     f"publish {pubsub}/{topic}")
            return
        req = P.rt("PublishEventRequest")(pubsub_name=pubsub, topic=topic, data=body,
                                          data_content_type=content_type or ctype, metadata=metadata or {})
        await self._call("PublishEvent", req, f"publish {pubsub}/{topic}")

    async def publish_events(self, pubsub: str, topic: str, events: list[Any]) -> dict[str, Any]:
        req = P.rt("BulkPublishRequest")(pubsub_name=pubsub, topic=topic)
        for i, e in enumerate(events):
            body, ctype = _encode(e)
            req.entries.add(entry_id=str(i), event=body, content_type=ctype)
        r = await self._call("BulkPublishEventAlpha1", req, f"publish-bulk {pubsub}/{topic}")
        return {"failedEntries": [{"entryId": f.entry_id, "error": f.error} for f in r.failedEntries]}

    # -- bindings ---------------------------------------------------------------
    async def invoke_binding(self, name: str, operation: str, data: Any = None,
                             metadata: dict[str, str] | None = None) -> Any:
        body = b"" if data is None else (data.encode() if isinstance(data, str) and not isinstance(data, RawJson)
                                         else _encode(data)[0])
        req = P.rt("InvokeBindingRequest")(name=name, operation=operation, data=body,
                                           metadata={k: str(v) for k, v in (metadata or {}).items()})
        r = await self._call("InvokeBinding", req, f"binding {name} {operation}")
        if not r.data:
            return None
        try:
            return json.loads(r.data)
        except ValueError:
            return r.data

    # -- secrets ----------------------------------------------------------------
    async def get_secret(self, store: str, key: str, metadata: dict[str, str] | None = None) -> dict[str, str]:
        r = await self._call("GetSecret", P.rt("GetSecretRequest")(store_name=store, key=key, metadata=metadata or {}),
                             f"secret get {store}")
        return dict(r.data)

    async def get_bulk_secret(self, store: str) -> dict[str, dict[str, str]]:
        r = await self._call("GetBulkSecret", P.rt("GetBulkSecretRequest")(store_name=store), f"secret bulk {store}")
        return {k: dict(v.secrets) for k, v in r.data.items()}

    # -- metadata / lifecycle --------------------------------------------------
    async def get_metadata(self) -> dict[str, Any]:
        r = await self._call("GetMetadata", P.rt("GetMetadataRequest")(), "metadata")
        return {"id": r.id, "runtimeVersion": r.runtime_version,
                "components": [{"name": c.name, "type": c.type, "version": c.version,
                                "capabilities": list(c.capabilities)} for c in r.registered_components],
                "subscriptions": [{"pubsubname": s.pubsub_name, "topic": s.topic,
                                   "rules": [{"path": x.path} for x in s.rules.rules],
                                   "deadLetterTopic": s.dead_letter_topic} for s in r.subscriptions],
                "extended": dict(r.extended_metadata)}

    async def set_metadata(self, key: str, value: str) -> None:
        await self._call("SetMetadata", P.rt("SetMetadataRequest")(key=key, value=value), "metadata set")

    async def shutdown_sidecar(self) -> None:
        await self._call("Shutdown", P.rt("ShutdownRequest")(), "shutdown")

    async def close(self) -> None:
        if self._channel is not None:
            await self._channel.close()
            self._channel = None
            self._stubs.clear()
