"""App-side integration helpers -- the ``Dapr.AspNetCore`` equivalents.

* ``topic(pubsub, topic)``       -- ``[Topic("pubsub","topic")]`` attribute
  (reference Processor Controllers/TasksNotifierController.cs:23-24; stackable).
* ``map_subscribe_handler(app)`` -- ``app.MapSubscribeHandler()`` serving ``GET /dapr/subscribe``
  built from the ``topic`` decorations (reference Processor/Program.cs:33).
* ``cloud_events_middleware()``  -- ``app.UseCloudEvents()``: unwraps a CloudEvents 1.0
  envelope so handlers bind the ``data`` payload (reference Processor/Program.cs:29).
"""
from __future__ import annotations

import base64
import json
from typing import Any, Callable

from ..web.app import WebApp
from ..web.http import Request, Response, json_response

TOPIC_ATTR = "__tt_topics__"


def topic(pubsub: str, name: str, dead_letter_topic: str | None = None,
          metadata: dict[str, str] | None = None, match: str | None = None, priority: int | None = None) -> Callable:
    """Mark an endpoint as a subscriber; apply *before* (i.e. below) the route decorator
    or above it -- either order works because subscription discovery reads the attribute
    off the endpoint function."""
    def deco(fn: Callable) -> Callable:
        subs = list(getattr(fn, TOPIC_ATTR, []))
        subs.append({"pubsubname": pubsub, "topic": name, "deadLetterTopic": dead_letter_topic,
                     "metadata": metadata or {}, "match": match, "priority": priority})
        setattr(fn, TOPIC_ATTR, subs)
        return fn
    return deco


def subscriptions(app: WebApp) -> list[dict[str, Any]]:
    out: list[dict[str, Any]] = []
    for r in app.routes:
        for t in getattr(r.endpoint, TOPIC_ATTR, []):
            entry: dict[str, Any] = {"pubsubname": t["pubsubname"], "topic": t["topic"],
                                     "route": r.template.lstrip("/")}
            if t.get("deadLetterTopic"):
                entry["deadLetterTopic"] = t["deadLetterTopic"]
            if t.get("metadata"):
                entry["metadata"] = t["metadata"]
            if t.get("match"):
                entry["routes"] = {"rules": [{"match": t["match"], "path": r.template.lstrip("/")}]}
            out.append(entry)
    return out


def map_subscribe_handler(app: WebApp) -> None:
    async def dapr_subscribe(req: Request) -> Response:
        return json_response(subscriptions(app))
    app.add_route("/dapr/subscribe", dapr_subscribe, ("GET",), name="dapr_subscribe", include_in_schema=False)


def _native_unwrap():
    try:
        from ..native import load
        return load().cloudevent_unwrap
    except Exception:  # no native module in this process: the Python unwrapper serves
        return None


def cloud_events_middleware():
    native = _native_unwrap()

    async def mw(req: Request, nxt) -> Response:
        if req.content_type == "application/cloudevents+json" and req.body:
            # one native pass (native/src/taskcodec.hpp) for the common envelope: JSON data
            # re-serialised compactly, attributes as a dict; anything else is unwrapped below
            u = native(req.body) if native is not None else None
            if u is not None:
                req.body, dct, req.state["cloudevent"] = u
                req.headers["content-type"] = dct
                return await nxt(req)
            try:
                ce = json.loads(req.body)
            except ValueError:
                return await nxt(req)
            if isinstance(ce, dict):
                req.state["cloudevent"] = {k: v for k, v in ce.items() if k not in ("data", "data_base64")}
                dct = ce.get("datacontenttype", "application/json")
                if "data_base64" in ce:
                    req.body = base64.b64decode(ce["data_base64"])
                elif "data" in ce:
                    d = ce["data"]
                    if isinstance(d, str) and "json" not in dct:
                        req.body = d.encode()
                    else:
                        req.body = json.dumps(d).encode()
                        req.state["json"] = (req.body, d)  # Request.json() reuses the parsed data
                req.headers["content-type"] = dct
        return await nxt(req)
    return mw
