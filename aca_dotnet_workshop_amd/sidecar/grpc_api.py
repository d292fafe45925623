"""The sidecar's gRPC API (``dapr.proto.runtime.v1.Dapr``), next to its HTTP API.

The reference's ``DaprClient`` reaches ``daprd`` over gRPC for ``SaveStateAsync``,
``GetStateAsync``, ``DeleteStateAsync``, ``QueryStateAsync``, ``PublishEventAsync`` and
``InvokeBindingAsync`` (Backend.Api Services/TasksStoreManager.cs:35-156, Processor
ExternalTasksProcessorController.cs:43), on the gRPC ports of the reference's launch plan
(.vscode/tasks.json:126-165: 50001/50002/50003).  This server exposes those RPCs (and the rest of
the building-block surface: bulk state, transactions, bulk publish, secrets, metadata, service
invocation, shutdown) on ``--dapr-grpc-port``.

Design: every RPC is translated into the equivalent HTTP API request and run through the
sidecar's own API pipeline in-process (no socket hop) -- the same middleware (API token,
tracing span, API logging) and the same handlers -- so both protocols share one implementation
and cannot drift.  HTTP status codes of errors map onto gRPC status codes the way ``daprd`` does
(400 -> INVALID_ARGUMENT, 404 -> NOT_FOUND, 409 -> ABORTED, 401 -> UNAUTHENTICATED, ...); the
JSON error body becomes the status details.
"""
from __future__ import annotations

import base64
import json
import logging
from typing import Any, Awaitable, Callable
from urllib.parse import quote, urlencode

import grpc

from ..sdk import proto as P
from ..web.http import Headers, Request, Response

log = logging.getLogger("sidecar.grpc")

_CODES = {400: grpc.StatusCode.INVALID_ARGUMENT, 401: grpc.StatusCode.UNAUTHENTICATED,
          403: grpc.StatusCode.PERMISSION_DENIED, 404: grpc.StatusCode.NOT_FOUND, 405: grpc.StatusCode.UNIMPLEMENTED,
          409: grpc.StatusCode.ABORTED, 429: grpc.StatusCode.RESOURCE_EXHAUSTED, 500: grpc.StatusCode.INTERNAL,
          501: grpc.StatusCode.UNIMPLEMENTED, 502: grpc.StatusCode.UNAVAILABLE, 503: grpc.StatusCode.UNAVAILABLE,
          504: grpc.StatusCode.DEADLINE_EXCEEDED}

_CONCURRENCY = {1: "first-write", 2: "last-write"}
_CONSISTENCY = {1: "eventual", 2: "strong"}


def grpc_code(status: int) -> grpc.StatusCode:
    return _CODES.get(status, grpc.StatusCode.UNKNOWN if status >= 400 else grpc.StatusCode.OK)


def _json_or_text(raw: bytes, ctype: str = "") -> Any:
    """A value carried as bytes on the gRPC side, as the HTTP API's JSON body expects it:
    JSON text is embedded as JSON, anything else as a string."""
    if not raw:
        return None
    if "json" in ctype or not ctype:
        try:
            return json.loads(raw)
        except ValueError:
            pass
    try:
        return raw.decode("utf-8")
    except UnicodeDecodeError:
        return base64.b64encode(raw).decode()


def _dumps(v: Any) -> bytes:
    if v is None:
        return b""
    return json.dumps(v, separators=(",", ":")).encode()


def _meta_qs(meta) -> str:
    return urlencode({f"metadata.{k}": v for k, v in dict(meta).items()}) if meta else ""


def _state_item_json(item) -> dict[str, Any]:
    d: dict[str, Any] = {"key": item.key, "value": _json_or_text(item.value)}
    if item.HasField("etag"):
        d["etag"] = item.etag.value
    if item.metadata:
        d["metadata"] = dict(item.metadata)
    if item.HasField("options"):
        opts = {}
        if item.options.concurrency in _CONCURRENCY:
            opts["concurrency"] = _CONCURRENCY[item.options.concurrency]
        if item.options.consistency in _CONSISTENCY:
            opts["consistency"] = _CONSISTENCY[item.options.consistency]
        if opts:
            d["options"] = opts
    return d


def _percent(msg: str) -> str:
    """grpc-message encoding: bytes outside printable ASCII and '%' as %XX."""
    return "".join(chr(b) if 0x20 <= b <= 0x7e and b != 0x25 else f"%{b:02X}" for b in msg.encode("utf-8"))


def _grpc_reply(code: int, message: str, trailing=()) -> Response:
    h = [("content-type", "application/grpc+proto"), ("grpc-status", str(code)), ("grpc-message", _percent(message))]
    h += [(k, v) for k, v in trailing or ()]
    return Response(b"", 200, h)


class _Abort(Exception):
    def __init__(self, code: grpc.StatusCode, details: str, trailing) -> None:
        super().__init__(details)
        self.code, self.details, self.trailing = code, details, trailing


class _BridgeContext:
    """The slice of ``grpc.aio.ServicerContext`` the handlers use, over a bridged HTTP request."""

    def __init__(self, req: Request) -> None:
        self._md = [(k, v) for k, v in req.headers.items()
                    if k not in ("content-type", "content-length", "host") and isinstance(v, str)]

    def invocation_metadata(self):
        return self._md

    def peer(self) -> str:
        return "native-dataplane"

    async def abort(self, code, details="", trailing_metadata=()):
        raise _Abort(code, details, trailing_metadata)


class DaprGrpcServer:
    """gRPC front of one sidecar; ``api`` is the sidecar's HTTP API ``WebApp``."""

    def __init__(self, sidecar, api: Callable[[Request], Awaitable[Response]]) -> None:
        self.sc = sidecar
        self.api = api
        self.server: grpc.aio.Server | None = None
        self.bound_port: int | None = None

    # -------------------------------------------------------------- plumbing
    async def _http(self, ctx: grpc.aio.ServicerContext, method: str, target: str, body: bytes = b"",
                    ctype: str | None = None, extra: list[tuple[str, str]] | None = None) -> Response:
        h = Headers()
        for k, v in ctx.invocation_metadata() or ():
            k = k.lower()
            if k in ("dapr-api-token", "traceparent", "tracestate") or k.startswith("dapr-"):
                h[k] = v if isinstance(v, str) else v.decode("latin-1")
        if ctype:
            h["content-type"] = ctype
        for k, v in extra or ():
            h[k.lower()] = v
        h["content-length"] = str(len(body))
        req = Request(method, target, h, body, client=("grpc", ctx.peer()))
        return await self.api(req)

    @staticmethod
    async def _fail(ctx: grpc.aio.ServicerContext, r: Response, what: str) -> None:
        try:
            js = json.loads(r.body) if r.body else {}
            msg = f"{js.get('errorCode', '')}: {js.get('message', js)}" if isinstance(js, dict) else str(js)
        except ValueError:
            msg = r.body[:500].decode("utf-8", "replace")
        await ctx.abort(grpc_code(r.status), f"{what}: {msg}",
                        trailing_metadata=(("dapr-http-status", str(r.status)),))

    async def _ok(self, ctx, r: Response, what: str) -> Response:
        if r.status >= 300:
            await self._fail(ctx, r, what)
        return r

    # -------------------------------------------------------------- state
    async def GetState(self, req, ctx):
        qs = _meta_qs(req.metadata)
        r = await self._ok(ctx, await self._http(ctx, "GET", f"/v1.0/state/{quote(req.store_name, safe='')}/"
                                                 f"{quote(req.key, safe='')}" + (f"?{qs}" if qs else "")),
                           "GetState")
        out = P.rt("GetStateResponse")()
        if r.status == 200:
            out.data = r.body
            out.etag = r.header("etag") or ""
        return out

    async def GetBulkState(self, req, ctx):
        body = _dumps({"keys": list(req.keys), "parallelism": req.parallelism or 10})
        r = await self._ok(ctx, await self._http(ctx, "POST", f"/v1.0/state/{quote(req.store_name, safe='')}/bulk",
                                                 body, "application/json"), "GetBulkState")
        out = P.rt("GetBulkStateResponse")()
        for it in r.json() or []:
            out.items.add(key=it.get("key", ""), data=_dumps(it.get("data")), etag=it.get("etag") or "",
                          error=it.get("error") or "")
        return out

    async def SaveState(self, req, ctx):
        body = _dumps([_state_item_json(s) for s in req.states])
        await self._ok(ctx, await self._http(ctx, "POST", f"/v1.0/state/{quote(req.store_name, safe='')}", body,
                                             "application/json"), "SaveState")
        return P.message(".google.protobuf.Empty")()

    async def DeleteState(self, req, ctx):
        extra = [("if-match", req.etag.value)] if req.HasField("etag") and req.etag.value else None
        await self._ok(ctx, await self._http(ctx, "DELETE", f"/v1.0/state/{quote(req.store_name, safe='')}/"
                                             f"{quote(req.key, safe='')}", extra=extra), "DeleteState")
        return P.message(".google.protobuf.Empty")()

    async def DeleteBulkState(self, req, ctx):
        ops = [{"operation": "delete", "request": _state_item_json(s)} for s in req.states]
        await self._ok(ctx, await self._http(ctx, "POST", f"/v1.0/state/{quote(req.store_name, safe='')}/transaction",
                                             _dumps({"operations": ops}), "application/json"), "DeleteBulkState")
        return P.message(".google.protobuf.Empty")()

    async def ExecuteStateTransaction(self, req, ctx):
        ops = [{"operation": o.operationType, "request": _state_item_json(o.request)} for o in req.operations]
        payload: dict[str, Any] = {"operations": ops}
        if req.metadata:
            payload["metadata"] = dict(req.metadata)
        await self._ok(ctx, await self._http(ctx, "POST", f"/v1.0/state/{quote(req.storeName, safe='')}/transaction",
                                             _dumps(payload), "application/json"), "ExecuteStateTransaction")
        return P.message(".google.protobuf.Empty")()

    async def QueryStateAlpha1(self, req, ctx):
        qs = _meta_qs(req.metadata)
        r = await self._ok(ctx, await self._http(ctx, "POST", f"/v1.0-alpha1/state/{quote(req.store_name, safe='')}"
                                                 "/query" + (f"?{qs}" if qs else ""), req.query.encode(),
                                                 "application/json"), "QueryStateAlpha1")
        js = r.json() or {}
        out = P.rt("QueryStateResponse")(token=js.get("token") or "")
        for it in js.get("results") or []:
            out.results.add(key=it.get("key", ""), data=_dumps(it.get("data")), etag=it.get("etag") or "",
                             error=it.get("error") or "")
        for k, v in (js.get("metadata") or {}).items():
            out.metadata[k] = str(v)
        return out

    # -------------------------------------------------------------- pub/sub
    async def PublishEvent(self, req, ctx):
        qs = _meta_qs(req.metadata)
        target = f"/v1.0/publish/{quote(req.pubsub_name, safe='')}/{quote(req.topic, safe='/')}" + (f"?{qs}" if qs else "")
        await self._ok(ctx, await self._http(ctx, "POST", target, req.data, req.data_content_type or "application/json"),
                       "PublishEvent")
        return P.message(".google.protobuf.Empty")()

    async def BulkPublishEventAlpha1(self, req, ctx):
        entries = []
        for e in req.entries:
            ct = e.content_type or "application/json"
            entries.append({"entryId": e.entry_id, "event": _json_or_text(e.event, ct), "contentType": ct,
                            "metadata": dict(e.metadata)})
        r = await self._http(ctx, "POST", f"/v1.0-alpha1/publish/bulk/{quote(req.pubsub_name, safe='')}/"
                             f"{quote(req.topic, safe='/')}", _dumps(entries), "application/json")
        out = P.rt("BulkPublishResponse")()
        if r.status >= 300:
            js = r.json() if r.body else {}
            if not isinstance(js, dict) or "failedEntries" not in js:
                await self._fail(ctx, r, "BulkPublishEventAlpha1")
            for f in js["failedEntries"]:
                out.failedEntries.add(entry_id=str(f.get("entryId", "")), error=str(f.get("error", "")))
        return out

    # -------------------------------------------------------------- bindings
    async def InvokeBinding(self, req, ctx):
        payload: dict[str, Any] = {"data": _json_or_text(req.data), "operation": req.operation}
        if req.metadata:
            payload["metadata"] = dict(req.metadata)
        r = await self._ok(ctx, await self._http(ctx, "POST", f"/v1.0/bindings/{quote(req.name, safe='')}",
                                                 _dumps(payload), "application/json"), "InvokeBinding")
        out = P.rt("InvokeBindingResponse")(data=r.body)
        for k, v in r.headers:
            if k.lower().startswith("metadata."):
                out.metadata[k[9:]] = v
        return out

    # -------------------------------------------------------------- secrets
    async def GetSecret(self, req, ctx):
        qs = _meta_qs(req.metadata)
        r = await self._ok(ctx, await self._http(ctx, "GET", f"/v1.0/secrets/{quote(req.store_name, safe='')}/"
                                                 f"{quote(req.key, safe='')}" + (f"?{qs}" if qs else "")), "GetSecret")
        out = P.rt("GetSecretResponse")()
        for k, v in (r.json() or {}).items():
            out.data[k] = str(v)
        return out

    async def GetBulkSecret(self, req, ctx):
        r = await self._ok(ctx, await self._http(ctx, "GET", f"/v1.0/secrets/{quote(req.store_name, safe='')}/bulk"),
                           "GetBulkSecret")
        out = P.rt("GetBulkSecretResponse")()
        for name, kv in (r.json() or {}).items():
            for k, v in (kv or {}).items():
                out.data[name].secrets[k] = str(v)
        return out

    # -------------------------------------------------------------- invoke
    async def InvokeService(self, req, ctx):
        m = req.message
        verb = P.verb_name(m.http_extension.verb) if m.HasField("http_extension") else "NONE"
        method = "POST" if verb == "NONE" else verb
        qs = m.http_extension.querystring if m.HasField("http_extension") else ""
        target = f"/v1.0/invoke/{quote(req.id, safe='')}/method/{m.method.lstrip('/')}" + (f"?{qs}" if qs else "")
        r = await self._http(ctx, method, target, m.data.value if m.HasField("data") else b"",
                             m.content_type or ("application/json" if m.HasField("data") else None))
        if r.status >= 300:
            await self._fail(ctx, r, f"InvokeService {req.id}/{m.method}")
        out = P.common("InvokeResponse")(content_type=r.header("content-type") or "")
        out.data.value = r.body
        return out

    # -------------------------------------------------------------- runtime
    async def GetMetadata(self, req, ctx):
        r = await self._ok(ctx, await self._http(ctx, "GET", "/v1.0/metadata"), "GetMetadata")
        js = r.json() or {}
        out = P.rt("GetMetadataResponse")(id=js.get("id", ""), runtime_version=js.get("runtimeVersion", ""))
        for c in js.get("components") or []:
            out.registered_components.add(name=c.get("name", ""), type=c.get("type", ""),
                                          version=c.get("version", ""), capabilities=c.get("capabilities") or [])
        for s in js.get("subscriptions") or []:
            sub = out.subscriptions.add(pubsub_name=s.get("pubsubname", ""), topic=s.get("topic", ""),
                                        dead_letter_topic=s.get("deadLetterTopic", ""))
            for rule in s.get("rules") or []:
                sub.rules.rules.add(match=rule.get("match", ""), path=rule.get("path", ""))
        for k, v in (js.get("extended") or {}).items():
            out.extended_metadata[k] = v if isinstance(v, str) else json.dumps(v, separators=(",", ":"))
        acp = js.get("appConnectionProperties") or {}
        out.app_connection_properties.port = int(acp.get("port") or 0)
        out.app_connection_properties.protocol = acp.get("protocol") or ""
        return out

    async def SetMetadata(self, req, ctx):
        await self._ok(ctx, await self._http(ctx, "PUT", f"/v1.0/metadata/{quote(req.key, safe='')}",
                                             req.value.encode(), "text/plain"), "SetMetadata")
        return P.message(".google.protobuf.Empty")()

    async def Shutdown(self, req, ctx):
        await self._ok(ctx, await self._http(ctx, "POST", "/v1.0/shutdown"), "Shutdown")
        return P.message(".google.protobuf.Empty")()

    # -------------------------------------------------------------- native data plane bridge
    async def dispatch_raw(self, req: Request) -> Response:
        """``POST /_tt/grpc/{Method}`` on the control plane's private socket: the native data
        plane (native/src/h2.hpp + dataplane.cpp) serves the gRPC port and decodes the hot RPCs
        itself; any other RPC arrives here as its serialized request message plus the call
        metadata as headers, runs through the same handler as above, and goes back as the
        serialized response with ``grpc-status`` / ``grpc-message`` (percent-encoded) headers."""
        rpc = req.path_params["method"]
        if rpc not in P.RPCS:
            return _grpc_reply(12, f"unknown method {rpc}")
        req_cls, _ = P.rpc_types(rpc)
        try:
            msg = req_cls.FromString(req.body)
        except Exception as e:  # noqa: BLE001 - protobuf raises DecodeError and friends
            return _grpc_reply(3, f"{rpc}: malformed request message: {e}")
        ctx = _BridgeContext(req)
        try:
            out = await getattr(self, rpc)(msg, ctx)
        except _Abort as a:
            return _grpc_reply(a.code.value[0], a.details, a.trailing)
        return Response(out.SerializeToString(), 200,
                        [("content-type", "application/grpc+proto"), ("grpc-status", "0")])

    # -------------------------------------------------------------- server
    def handler(self) -> grpc.GenericRpcHandler:
        methods = {}
        for rpc in P.RPCS:
            req_cls, resp_cls = P.rpc_types(rpc)
            methods[rpc] = grpc.unary_unary_rpc_method_handler(
                getattr(self, rpc), request_deserializer=req_cls.FromString,
                response_serializer=resp_cls.SerializeToString)
        return grpc.method_handlers_generic_handler(P.SERVICE, methods)

    async def start(self, port: int, host: str = "127.0.0.1", uds: str | None = None) -> int:
        self.server = grpc.aio.server(options=[("grpc.so_reuseport", 0)])
        self.server.add_generic_rpc_handlers((self.handler(),))
        self.bound_port = self.server.add_insecure_port(f"{host}:{port}")
        if uds:
            self.server.add_insecure_port(f"unix:{uds}")
        await self.server.start()
        return self.bound_port

    async def stop(self, grace: float = 1.0) -> None:
        if self.server is not None:
            await self.server.stop(grace)
            self.server = None
