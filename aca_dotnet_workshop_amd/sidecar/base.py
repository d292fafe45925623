"""Shared plumbing for sidecar components: runtime context, backing-service endpoint
resolution from Azure-style metadata, and the component type registry."""
from __future__ import annotations

import os
import re
from dataclasses import dataclass, field
from typing import Callable
from urllib.parse import urlsplit

from ..backing.client import BackingClient, backing_url
from ..backing.shards import PARTITIONED_FAMILIES, ShardedBackingClient, shard_urls
from ..web.client import HttpClient
from .components import Component, ComponentError


@dataclass
class RuntimeContext:
    app_id: str
    namespace: str = "default"
    identity: str | None = None
    backing_url: str = field(default_factory=backing_url)
    http: HttpClient = field(default_factory=HttpClient)
    environ: dict[str, str] = field(default_factory=lambda: dict(os.environ))

    def backing(self, comp: Component, key: str | None = None) -> BackingClient:
        """Endpoint of the backing service for this component: explicit ``ttBackingUrl``
        metadata, else a per-service-family URL (``TT_BACKING_URL_COSMOS`` /
        ``_SERVICEBUS`` / ``_STORAGE`` / ``_KEYVAULT`` / ``_SENDGRID``), else the shared
        ``TT_BACKING_URL`` -- Azure's services are separate endpoints, so they may be
        separate emulator processes.  ``TT_BACKING_SHARDS_COSMOS`` / ``_SERVICEBUS`` (URLs in
        rank order) make the store / broker partitioned over several backings."""
        family = service_family(comp.type)
        base = comp.get("ttBackingUrl") or self.environ.get(f"TT_BACKING_URL_{family}") or self.backing_url
        if not comp.get("ttBackingUrl"):
            # the same backing process on this host's Unix socket (platform/processes.py): the
            # data path's exchanges skip the loopback TCP stack
            uds = self.environ.get(f"TT_BACKING_UDS_{family}") if self.environ.get(f"TT_BACKING_URL_{family}") \
                else self.environ.get("TT_BACKING_UDS") if base == self.environ.get("TT_BACKING_URL") else None
            if uds:
                base = f"unix:{uds}:"
        if not comp.get("ttBackingUrl") and family in PARTITIONED_FAMILIES:
            urls = shard_urls(self.environ, family)
            if urls:  # a partitioned collection / namespace (backing/shards.py)
                return ShardedBackingClient(urls, identity=self.identity or "", key=key, http=self.http, home=base)
        return BackingClient(base, identity=self.identity or "", key=key, http=self.http)


class ComponentBase:
    """Every component is constructed from its resolved ``Component`` manifest."""

    def __init__(self, comp: Component, ctx: RuntimeContext) -> None:
        self.comp = comp
        self.ctx = ctx
        self.name = comp.name

    async def init(self) -> None:
        pass

    async def close(self) -> None:
        pass


_REGISTRY: dict[str, type] = {}


def register(*types: str) -> Callable[[type], type]:
    def deco(cls: type) -> type:
        for t in types:
            _REGISTRY[t] = cls
        return cls
    return deco


def create_component(comp: Component, ctx: RuntimeContext) -> ComponentBase:
    cls = _REGISTRY.get(comp.type)
    if cls is None:
        raise ComponentError(f"component {comp.name}: unsupported type {comp.type!r} "
                             f"(supported: {', '.join(sorted(_REGISTRY))})")
    return cls(comp, ctx)


def supported_types() -> list[str]:
    return sorted(_REGISTRY)


def service_family(component_type: str) -> str:
    t = component_type
    if t.startswith("state."):
        return "COSMOS"
    if t.startswith("pubsub."):
        return "SERVICEBUS"
    if t.startswith("secretstores."):
        return "KEYVAULT"
    if "sendgrid" in t:
        return "SENDGRID"
    if t == "bindings.cron":
        return "COSMOS"  # leases live in the document store
    return "STORAGE"


# -- Azure-style endpoint metadata -> emulator account names --------------------
def cosmos_account(url: str) -> str:
    host = urlsplit(url).hostname or url
    return host.split(".")[0]


def servicebus_namespace(comp: Component) -> tuple[str, str | None]:
    cs = comp.get("connectionString")
    if cs:
        parts = dict(p.split("=", 1) for p in cs.split(";") if "=" in p)
        ep = parts.get("Endpoint", "")
        host = urlsplit(ep).hostname or ep.replace("sb://", "").strip("/")
        return host.split(".")[0] or "default", parts.get("SharedAccessKey")
    ns = comp.get("namespaceName")
    if ns:
        return ns.split(".")[0], None
    return "default", None


def redis_namespace(comp: Component) -> str:
    host = comp.get("redisHost", "localhost:6379") or "localhost:6379"
    return "redis-" + re.sub(r"[^A-Za-z0-9]", "-", host)
