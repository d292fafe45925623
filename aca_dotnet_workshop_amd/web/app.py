"""Minimal web application framework -- the ASP.NET Core controller/Razor-Pages host
equivalent.

Features used by the services (with the reference behaviour they mirror):
* attribute-style routing with typed parameters ``{taskId:guid}`` and case-insensitive
  literal segments (ASP.NET routing, which is why ``/externaltasksprocessor/process``
  reaches ``[Route("ExternalTasksProcessor")]``, reference
  components/dapr-bindings-in-storagequeue.yaml:17-18);
* 404 for no route, 405 for wrong verb;
* middleware pipeline (tracing, CloudEvents unwrap, exception handler);
* return-value conversion: ``Response`` | pydantic model | list/dict -> JSON | ``None`` -> 200;
* OpenAPI document generation from route metadata (``MapOpenApi``, reference
  Backend.Api/Program.cs:16,21-24);
* static files (``MapStaticAssets``, reference Frontend.Ui/Program.cs:45-47);
* startup / shutdown hooks and a ``services`` dict used as the DI container.
"""
from __future__ import annotations

import asyncio
import inspect
import logging
import mimetypes
import os
import uuid
from pathlib import Path
from urllib.parse import unquote
from typing import Any, Awaitable, Callable

from ..models.dotnet import is_guid
from .http import HTTPError, Request, Response, json_response, problem

log = logging.getLogger("web.app")

Endpoint = Callable[[Request], Awaitable[Any]]
Middleware = Callable[[Request, Callable[[Request], Awaitable[Response]]], Awaitable[Response]]


def _conv_guid(s: str) -> uuid.UUID:
    if not is_guid(s):
        raise ValueError
    return uuid.UUID(s.strip("{}"))


_CONVERTERS: dict[str, Callable[[str], Any]] = {
    "guid": _conv_guid,
    "int": int,
    "long": int,
    "str": str,
    "string": str,
    "bool": lambda s: {"true": True, "false": False}[s.lower()],
}


class Route:
    __slots__ = ("methods", "template", "segments", "endpoint", "name", "meta", "catch_all")

    def __init__(self, methods: set[str], template: str, endpoint: Endpoint, name: str | None = None,
                 meta: dict[str, Any] | None = None) -> None:
        self.methods = methods
        self.template = "/" + template.strip("/")
        self.endpoint = endpoint
        self.name = name or getattr(endpoint, "__name__", "route")
        self.meta = meta or {}
        self.segments: list[tuple[str, Any]] = []
        self.catch_all: str | None = None
        for seg in self.template.strip("/").split("/") if self.template != "/" else []:
            if seg.startswith("{") and seg.endswith("}"):
                inner = seg[1:-1]
                if inner.startswith("*"):
                    self.catch_all = inner.lstrip("*")
                    break
                pname, _, conv = inner.partition(":")
                optional = pname.endswith("?")
                pname = pname.rstrip("?")
                self.segments.append(("param", (pname, _CONVERTERS[conv.rstrip("?")] if conv else str, optional)))
            else:
                self.segments.append(("lit", seg.lower()))

    def match(self, parts: list[str]) -> dict[str, Any] | None:
        segs = self.segments
        if self.catch_all is None:
            if len(parts) > len(segs):
                return None
        elif len(parts) < len(segs):
            return None
        params: dict[str, Any] = {}
        for i, (kind, val) in enumerate(segs):
            if i >= len(parts):
                if kind == "param" and val[2]:
                    params[val[0]] = None
                    continue
                return None
            p = parts[i]
            if kind == "lit":
                if p.lower() != val:
                    return None
            else:
                try:
                    params[val[0]] = val[1](p)
                except (ValueError, KeyError):
                    return None
        if self.catch_all is not None:
            params[self.catch_all] = "/".join(parts[len(segs):])
        return params


class WebApp:
    def __init__(self, name: str = "app", config: Any = None) -> None:
        self.name = name
        self.config = config
        self.routes: list[Route] = []
        self.middlewares: list[Middleware] = []
        self.services: dict[str, Any] = {}
        self.on_startup: list[Callable[[], Awaitable[None]]] = []
        self.on_shutdown: list[Callable[[], Awaitable[None]]] = []
        self.static_dirs: list[tuple[str, Path]] = []
        self.openapi_info: dict[str, Any] = {"title": name, "version": "1.0"}
        self._pipeline: Callable[[Request], Awaitable[Response]] | None = None
        self._route_cache: dict[str, list[Route]] = {}
        self._exact: dict[tuple[str, str], Route] = {}  # (method, raw path) -> literal route

    # -- registration ---------------------------------------------------------
    def route(self, template: str, methods: list[str] | tuple[str, ...] = ("GET",), name: str | None = None,
              **meta: Any) -> Callable[[Endpoint], Endpoint]:
        def deco(fn: Endpoint) -> Endpoint:
            self.add_route(template, fn, methods, name, **meta)
            return fn
        return deco

    def add_route(self, template: str, fn: Endpoint, methods: list[str] | tuple[str, ...] = ("GET",),
                  name: str | None = None, **meta: Any) -> Route:
        r = Route({m.upper() for m in methods}, template, fn, name, meta)
        self.routes.append(r)
        self._pipeline = None
        self._route_cache.clear()
        self._exact.clear()
        return r

    def _candidates(self, first: str) -> list[Route]:
        """Routes that can match a path whose first segment is ``first`` (registration order)."""
        c = self._route_cache.get(first)
        if c is None:
            c = [r for r in self.routes
                 if not r.segments or r.segments[0][0] == "param" or r.segments[0][1] == first]
            self._route_cache[first] = c
        return c

    def get(self, template: str, **meta: Any):
        return self.route(template, ("GET", "HEAD"), **meta)

    def post(self, template: str, **meta: Any):
        return self.route(template, ("POST",), **meta)

    def put(self, template: str, **meta: Any):
        return self.route(template, ("PUT",), **meta)

    def delete(self, template: str, **meta: Any):
        return self.route(template, ("DELETE",), **meta)

    def use(self, mw: Middleware) -> Middleware:
        self.middlewares.append(mw)
        self._pipeline = None
        return mw

    def mount_static(self, prefix: str, directory: str | os.PathLike) -> None:
        self.static_dirs.append(("/" + prefix.strip("/"), Path(directory)))

    # -- dispatch ---------------------------------------------------------------
    def match(self, method: str, path: str) -> tuple[Route | None, dict[str, Any], bool]:
        """``path`` is the raw (still percent-encoded) path; segments are decoded after
        splitting so an encoded ``%2F`` stays inside its segment."""
        hit = self._exact.get((method, path))
        if hit is not None:  # a literal route this exact request line resolved to before
            return hit, {}, True
        parts = [unquote(p) if "%" in p else p for p in path.split("/") if p]
        path_matched = False
        for r in self._candidates(parts[0].lower() if parts else ""):
            params = r.match(parts)
            if params is None:
                continue
            if method in r.methods or (method == "HEAD" and "GET" in r.methods):
                if r.catch_all is None and all(k == "lit" for k, _ in r.segments) and len(self._exact) < 256:
                    self._exact[(method, path)] = r
                return r, params, True
            path_matched = True
        return None, {}, path_matched

    async def _dispatch(self, req: Request) -> Response:
        route, params, path_matched = self.match(req.method, req.raw_path)
        if route is None:
            if req.method in ("GET", "HEAD") and self.static_dirs:
                resp = self._static(req.path)
                if resp is not None:
                    return resp
            if path_matched:
                return problem(405)
            return problem(404)
        req.path_params = params
        req.route = route
        result = await route.endpoint(req)
        return to_response(result)

    def _static(self, path: str) -> Response | None:
        for prefix, root in self.static_dirs:
            if prefix != "/" and not (path == prefix or path.startswith(prefix + "/")):
                continue
            rel = path[len(prefix):].lstrip("/") if prefix != "/" else path.lstrip("/")
            if not rel:
                continue
            f = (root / rel).resolve()
            try:
                f.relative_to(root.resolve())
            except ValueError:
                return problem(404)
            if f.is_file():
                ctype = mimetypes.guess_type(str(f))[0] or "application/octet-stream"
                return Response(f.read_bytes(), 200, [("Cache-Control", "max-age=3600")], ctype)
        return None

    def build(self) -> Callable[[Request], Awaitable[Response]]:
        handler: Callable[[Request], Awaitable[Response]] = self._dispatch
        for mw in reversed(self.middlewares):
            handler = _bind(mw, handler)
        app = self

        async def entry(req: Request) -> Response:
            req.app = app
            try:
                return await handler(req)
            except HTTPError as e:
                r = e.detail if isinstance(e.detail, Response) else problem(e.status, detail=e.detail)
                r.headers.extend(e.headers)
                return r
            except Exception as e:  # ASP.NET's exception handler middleware
                log.exception("unhandled exception in %s %s", req.method, req.path)
                detail = f"{type(e).__name__}: {e}" if app.is_development else None
                return problem(500, detail=detail, trace_id=req.state.get("trace_id"))
        return entry

    def __call__(self, req: Request) -> Awaitable[Response]:
        """The pipeline's coroutine for ``req`` (no extra await layer per request)."""
        if self._pipeline is None:
            self._pipeline = self.build()
        return self._pipeline(req)

    @property
    def is_development(self) -> bool:
        env = None
        if self.config is not None:
            env = self.config.get("Environment")
        return (env or "Production").lower() == "development"

    async def startup(self) -> None:
        for fn in self.on_startup:
            await fn()

    async def shutdown(self) -> None:
        for fn in self.on_shutdown:
            try:
                await fn()
            except Exception:
                log.exception("shutdown hook failed")

    # -- OpenAPI ----------------------------------------------------------------
    def openapi(self) -> dict[str, Any]:
        paths: dict[str, Any] = {}
        schemas: dict[str, Any] = {}
        for r in self.routes:
            if r.meta.get("include_in_schema") is False:
                continue
            tmpl = r.template
            params = []
            for kind, val in r.segments:
                if kind == "param":
                    fmt = {"_conv_guid": "uuid", "int": "int32"}.get(getattr(val[1], "__name__", ""), None)
                    sch: dict[str, Any] = {"type": "string"} if fmt != "int32" else {"type": "integer"}
                    if fmt:
                        sch["format"] = fmt
                    params.append({"name": val[0], "in": "path", "required": not val[2], "schema": sch})
            for q in r.meta.get("query", []):
                params.append({"name": q, "in": "query", "schema": {"type": "string"}})
            tmpl_clean = "/".join(s.split(":")[0] + ("}" if ":" in s else "") for s in tmpl.split("/"))
            for m in sorted(r.methods - {"HEAD"}):
                op: dict[str, Any] = {"operationId": r.name, "tags": [r.meta.get("tag", self.name)]}
                if params:
                    op["parameters"] = params
                body = r.meta.get("body")
                if body is not None:
                    op["requestBody"] = {"content": {"application/json": {"schema": _schema_ref(body, schemas)}},
                                         "required": True}
                responses: dict[str, Any] = {}
                for status, model in r.meta.get("responses", {200: None}).items():
                    entry: dict[str, Any] = {"description": _status_desc(status)}
                    if model is not None:
                        entry["content"] = {"application/json": {"schema": _schema_ref(model, schemas)}}
                    responses[str(status)] = entry
                op["responses"] = responses
                paths.setdefault(tmpl_clean, {})[m.lower()] = op
        return {"openapi": "3.0.1", "info": self.openapi_info, "paths": paths,
                "components": {"schemas": schemas}}


def _status_desc(status: int) -> str:
    from .http import reason
    return reason(int(status))


def _schema_ref(model: Any, schemas: dict[str, Any]) -> dict[str, Any]:
    if isinstance(model, list):
        return {"type": "array", "items": _schema_ref(model[0], schemas)}
    name = model.__name__
    if name not in schemas:
        js = model.model_json_schema(by_alias=True, ref_template="#/components/schemas/{model}",
                                     mode="serialization")
        js.pop("title", None)
        schemas[name] = js
    return {"$ref": f"#/components/schemas/{name}"}


class _Bound:
    """``mw`` with its ``next`` bound: calling it returns ``mw``'s own coroutine, so a middleware
    adds one frame to a request's await chain, not two."""
    __slots__ = ("mw", "nxt")

    def __init__(self, mw: Middleware, nxt: Callable[[Request], Awaitable[Response]]) -> None:
        self.mw, self.nxt = mw, nxt

    def __call__(self, req: Request) -> Awaitable[Response]:
        return self.mw(req, self.nxt)


def _bind(mw: Middleware, nxt: Callable[[Request], Awaitable[Response]]) -> Callable[[Request], Awaitable[Response]]:
    return _Bound(mw, nxt)


def to_response(result: Any) -> Response:
    if isinstance(result, Response):
        return result
    if result is None:
        return Response(b"", 200)
    if isinstance(result, (bytes, bytearray)):
        return Response(bytes(result), 200, None, "application/octet-stream")
    if isinstance(result, str):
        return Response(result.encode(), 200, None, "text/plain; charset=utf-8")
    if isinstance(result, list) and result and hasattr(result[0], "model_dump_json"):
        body = ("[" + ",".join(x.model_dump_json(by_alias=True) for x in result) + "]").encode()
        return Response(body, 200, None, "application/json; charset=utf-8")
    return json_response(result)


async def read_model(req: Request, model: Any) -> Any:
    """``[FromBody]`` binding: 415 for non-JSON, 400 with validation errors (the
    ``[ApiController]`` automatic 400 response)."""
    from pydantic import ValidationError
    ctype = req.content_type
    if req.body and ctype and "json" not in ctype:
        raise HTTPError(415)
    try:
        data = req.json()
    except ValueError as e:
        raise HTTPError(400, detail=f"invalid JSON: {e}")
    try:
        if isinstance(model, list):
            if not isinstance(data, list):
                raise HTTPError(400, detail="expected a JSON array")
            return [model[0].model_validate(x) for x in data]
        if data is None:
            raise HTTPError(400, detail="A non-empty request body is required.")
        return model.model_validate(data)
    except ValidationError as e:
        raise HTTPError(400, detail=e.errors(include_url=False, include_context=False))


def endpoint_accepts_request(fn: Callable) -> bool:
    return len(inspect.signature(fn).parameters) >= 1


async def run_app(app: WebApp, host: str = "127.0.0.1", port: int = 0, uds: str | None = None,
                  ready: Callable[[int], None] | None = None, stop: asyncio.Event | None = None) -> None:
    """Serve ``app`` until ``stop`` is set (or forever)."""
    from .server import HttpServer
    srv = HttpServer(app, asyncio.get_running_loop())
    await app.startup()
    bound = await srv.listen_tcp(host, port) if port is not None and port >= 0 else 0
    if uds:
        await srv.listen_unix(uds)
    if ready:
        ready(bound)
    try:
        if stop is None:
            await asyncio.Event().wait()
        else:
            await stop.wait()
    finally:
        await srv.close()
        await app.shutdown()
