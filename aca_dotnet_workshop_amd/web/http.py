"""Request / Response primitives shared by the server, the app framework and the client."""
from __future__ import annotations

import json
from http import HTTPStatus
from typing import Any, Iterable
from urllib.parse import parse_qsl, quote, unquote

_REASONS = {s.value: s.phrase for s in HTTPStatus}


def reason(status: int) -> str:
    return _REASONS.get(status, "Unknown")


class Headers(dict):
    """Lower-cased header map.  Repeated headers are comma-joined, except
    ``set-cookie`` which keeps a list (``getlist``)."""

    def getlist(self, key: str) -> list[str]:
        v = self.get(key.lower())
        if v is None:
            return []
        return v if isinstance(v, list) else [v]


class HTTPError(Exception):
    def __init__(self, status: int, detail: Any = None, headers: Iterable[tuple[str, str]] = ()) -> None:
        super().__init__(f"{status} {reason(status)}")
        self.status = status
        self.detail = detail
        self.headers = list(headers)


class Request:
    __slots__ = ("method", "target", "path", "raw_path", "query_string", "headers", "body", "client",
                 "path_params", "state", "_query", "_cookies", "version", "app", "route")

    def __init__(self, method: str, target: str, headers: Headers, body: bytes = b"",
                 client: Any = None, version: str = "HTTP/1.1") -> None:
        self.method = method
        self.target = target
        q = target.find("?")
        if q >= 0:
            self.raw_path = target[:q]
            self.query_string = target[q + 1:]
        else:
            self.raw_path = target
            self.query_string = ""
        self.path = unquote(self.raw_path) if "%" in self.raw_path else self.raw_path
        self.headers = headers
        self.body = body
        self.client = client
        self.version = version
        self.path_params: dict[str, Any] = {}
        self.state: dict[str, Any] = {}
        self._query: dict[str, str] | None = None
        self._cookies: dict[str, str] | None = None
        self.app = None
        self.route = None

    # -- accessors ------------------------------------------------------------
    @property
    def query(self) -> dict[str, str]:
        """Query parameters; first value wins; lookups should use ``query_get`` for
        ASP.NET-style case-insensitive binding."""
        if self._query is None:
            self._query = {}
            for k, v in parse_qsl(self.query_string, keep_blank_values=True):
                self._query.setdefault(k, v)
        return self._query

    def query_get(self, name: str, default: str | None = None) -> str | None:
        q = self.query
        if name in q:
            return q[name]
        low = name.lower()
        for k, v in q.items():
            if k.lower() == low:
                return v
        return default

    @property
    def cookies(self) -> dict[str, str]:
        if self._cookies is None:
            self._cookies = {}
            raw = self.headers.get("cookie")
            if raw:
                for part in raw.split(";"):
                    k, sep, v = part.strip().partition("=")
                    if sep:
                        self._cookies[k] = unquote(v)
        return self._cookies

    def json(self) -> Any:
        if not self.body:
            return None
        cached = self.state.get("json")  # set by middleware that already parsed the body
        if cached is not None and cached[0] is self.body:
            return cached[1]
        return json.loads(self.body)

    def form(self) -> dict[str, str]:
        """``application/x-www-form-urlencoded`` body (the only encoding our forms use)."""
        out: dict[str, str] = {}
        for k, v in parse_qsl(self.body.decode("utf-8", "replace"), keep_blank_values=True):
            out.setdefault(k, v)
        return out

    @property
    def content_type(self) -> str:
        return self.headers.get("content-type", "").split(";")[0].strip().lower()


class Response:
    __slots__ = ("status", "headers", "body")

    def __init__(self, body: bytes | str = b"", status: int = 200,
                 headers: list[tuple[str, str]] | None = None, content_type: str | None = None) -> None:
        if isinstance(body, str):
            body = body.encode()
        self.body = body
        self.status = status
        self.headers = headers if headers is not None else []
        if content_type:
            self.headers.append(("Content-Type", content_type))

    def header(self, name: str) -> str | None:
        low = name.lower()
        for k, v in self.headers:
            if k.lower() == low:
                return v
        return None

    def set_cookie(self, name: str, value: str, path: str = "/", httponly: bool = False,
                   max_age: int | None = None, samesite: str | None = "lax") -> None:
        parts = [f"{name}={quote(value, safe='@.-_')}", f"path={path}"]
        if max_age is not None:
            parts.append(f"max-age={max_age}")
        if samesite:
            parts.append(f"samesite={samesite}")
        if httponly:
            parts.append("httponly")
        self.headers.append(("Set-Cookie", "; ".join(parts)))

    def json(self) -> Any:
        return json.loads(self.body) if self.body else None


def json_response(obj: Any, status: int = 200, headers: list[tuple[str, str]] | None = None) -> Response:
    if hasattr(obj, "model_dump_json"):
        body = obj.model_dump_json(by_alias=True).encode()
    else:
        body = json.dumps(obj, separators=(",", ":"), default=_json_default).encode()
    return Response(body, status, headers, "application/json; charset=utf-8")


def _json_default(o: Any) -> Any:
    if hasattr(o, "model_dump"):
        return o.model_dump(mode="json", by_alias=True)
    if hasattr(o, "isoformat"):
        from ..models.dotnet import format_datetime
        return format_datetime(o)
    return str(o)


def text_response(text: str, status: int = 200) -> Response:
    return Response(text.encode(), status, None, "text/plain; charset=utf-8")


def html_response(html: str, status: int = 200) -> Response:
    return Response(html.encode(), status, None, "text/html; charset=utf-8")


def redirect(location: str, status: int = 302) -> Response:
    return Response(b"", status, [("Location", location)])


def empty(status: int = 204) -> Response:
    return Response(b"", status)


def problem(status: int, title: str | None = None, detail: Any = None, trace_id: str | None = None) -> Response:
    """RFC 7807 problem details, ASP.NET's ``ProblemDetails`` shape."""
    body: dict[str, Any] = {"type": f"https://tools.ietf.org/html/rfc9110#section-15.{status // 100}",
                            "title": title or reason(status), "status": status}
    if detail is not None:
        body["detail"] = detail
    if trace_id:
        body["traceId"] = trace_id
    return Response(json.dumps(body).encode(), status, None, "application/problem+json; charset=utf-8")


def encode_response(resp: Response, keep_alive: bool, head: bool = False) -> bytes:
    status = resp.status
    lines = [f"HTTP/1.1 {status} {reason(status)}"]
    has_len = False
    for k, v in resp.headers:
        if k.lower() == "content-length":
            has_len = True
        lines.append(f"{k}: {v}")
    body = resp.body
    if not has_len and not (100 <= status < 200 or status == 304):
        lines.append(f"Content-Length: {len(body)}")
    if not keep_alive:
        lines.append("Connection: close")
    head_bytes = ("\r\n".join(lines) + "\r\n\r\n").encode("latin-1")
    if head or status in (204, 304):
        return head_bytes
    return head_bytes + body
