"""Component manifest loading -- both dialects the reference ships.

* **Dapr self-hosted CRD** (``components/*.yaml``): ``apiVersion/kind/metadata/spec`` with
  ``spec.metadata[]`` entries carrying ``value`` / ``secretKeyRef{name,key}`` /
  ``envRef``, a top-level ``auth.secretStore`` and ``scopes`` (reference
  components/dapr-statestore-cosmos.yaml:1-18).  ``kind: Subscription`` (declarative
  subscriptions), ``kind: Configuration`` and ``kind: Resiliency`` documents are
  recognised too.
* **Azure Container Apps schema** (``aca-components/*.yaml``): ``componentType``,
  ``version``, ``metadata[]`` with ``value`` / ``secretRef``, ``secretStoreComponent``
  and ``scopes`` (reference aca-components/containerapps-bindings-in-storagequeue.yaml:1-16).
  The component *name* is not part of the file -- it is given at registration time
  (``--dapr-component-name``, reference docs/aca/04-aca-dapr-stateapi/index.md:531); the
  environment manifest supplies it, falling back to the file stem.

Drift between the dialects is resolved by loading exactly what a
file says; the environment manifest picks one file per component name.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from pathlib import Path
from typing import Any, Iterable

import yaml


@dataclass
class MetadataItem:
    name: str
    value: Any = None
    secret_name: str | None = None
    secret_key: str | None = None
    env_ref: str | None = None


@dataclass
class Component:
    name: str
    type: str
    version: str = "v1"
    items: list[MetadataItem] = field(default_factory=list)
    scopes: list[str] = field(default_factory=list)
    secret_store: str | None = None
    ignore_errors: bool = False
    init_timeout: float = 5.0
    dialect: str = "dapr"
    source: str = ""
    metadata: dict[str, str] = field(default_factory=dict)  # resolved

    @property
    def category(self) -> str:
        return self.type.split(".", 1)[0]

    def in_scope(self, app_id: str) -> bool:
        return not self.scopes or app_id in self.scopes

    def needs_secrets(self) -> bool:
        return any(i.secret_name for i in self.items)

    def resolve(self, secrets: dict[str, str] | None = None, environ: dict[str, str] | None = None) -> dict[str, str]:
        """Resolve values, ``envRef`` and secret references into ``self.metadata``.
        ``secrets`` maps metadata item name -> already-fetched secret value."""
        env = os.environ if environ is None else environ
        out: dict[str, str] = {}
        for it in self.items:
            if it.secret_name:
                if secrets is None or it.name not in secrets:
                    raise ComponentError(f"component {self.name}: metadata {it.name} references secret "
                                         f"{it.secret_name!r} but no secret store is available")
                out[it.name] = secrets[it.name]
            elif it.env_ref:
                out[it.name] = env.get(it.env_ref, "")
            else:
                out[it.name] = _to_str(it.value)
        self.metadata = out
        return out

    def get(self, key: str, default: str | None = None) -> str | None:
        """Case-insensitive metadata lookup (Dapr metadata keys are case-insensitive)."""
        if key in self.metadata:
            return self.metadata[key]
        low = key.lower()
        for k, v in self.metadata.items():
            if k.lower() == low:
                return v
        return default

    def get_bool(self, key: str, default: bool = False) -> bool:
        v = self.get(key)
        if v is None or v == "":
            return default
        return v.strip().lower() in ("true", "1", "yes", "on")

    def get_int(self, key: str, default: int) -> int:
        v = self.get(key)
        if v is None or str(v).strip() == "":
            return default
        return int(float(v))

    def describe(self) -> dict[str, Any]:
        return {"name": self.name, "type": self.type, "version": self.version}


@dataclass
class SubscriptionSpec:
    pubsubname: str
    topic: str
    route: str
    metadata: dict[str, str] = field(default_factory=dict)
    dead_letter_topic: str | None = None
    scopes: list[str] = field(default_factory=list)
    rules: list[dict[str, Any]] = field(default_factory=list)
    declarative: bool = False


class ComponentError(Exception):
    pass


def _to_str(v: Any) -> str:
    if v is None:
        return ""
    if isinstance(v, bool):
        return "true" if v else "false"
    return str(v)


def _items(entries: Iterable[dict[str, Any]] | None) -> list[MetadataItem]:
    out = []
    for e in entries or []:
        if not isinstance(e, dict) or "name" not in e:
            raise ComponentError(f"invalid metadata entry {e!r}")
        it = MetadataItem(str(e["name"]))
        if "secretKeyRef" in e:
            ref = e["secretKeyRef"] or {}
            it.secret_name = ref.get("name")
            it.secret_key = ref.get("key") or ref.get("name")
        elif "secretRef" in e:
            it.secret_name = str(e["secretRef"])
            it.secret_key = it.secret_name
        elif "envRef" in e:
            it.env_ref = str(e["envRef"])
        else:
            it.value = e.get("value")
        out.append(it)
    return out


def parse_documents(docs: Iterable[Any], source: str = "", default_name: str | None = None) -> tuple[
        list[Component], list[SubscriptionSpec], list[dict[str, Any]]]:
    comps: list[Component] = []
    subs: list[SubscriptionSpec] = []
    others: list[dict[str, Any]] = []
    for doc in docs:
        if not doc:
            continue
        if not isinstance(doc, dict):
            raise ComponentError(f"{source}: manifest is not a mapping")
        if "componentType" in doc:  # ACA dialect
            name = doc.get("name") or default_name or Path(source).stem
            comps.append(Component(name=name, type=doc["componentType"], version=str(doc.get("version", "v1")),
                                   items=_items(doc.get("metadata")), scopes=list(doc.get("scopes") or []),
                                   secret_store=doc.get("secretStoreComponent"),
                                   ignore_errors=bool(doc.get("ignoreErrors", False)),
                                   init_timeout=_timeout(doc.get("initTimeout")), dialect="aca", source=source))
            continue
        kind = doc.get("kind")
        meta = doc.get("metadata") or {}
        spec = doc.get("spec") or {}
        if kind == "Component":
            comps.append(Component(name=meta.get("name") or default_name or Path(source).stem, type=spec["type"],
                                   version=str(spec.get("version", "v1")), items=_items(spec.get("metadata")),
                                   scopes=list(doc.get("scopes") or []),
                                   secret_store=(doc.get("auth") or {}).get("secretStore"),
                                   ignore_errors=bool(spec.get("ignoreErrors", False)),
                                   init_timeout=_timeout(spec.get("initTimeout")), dialect="dapr", source=source))
        elif kind == "Subscription":
            routes = spec.get("routes") or {}
            route = spec.get("route") or (routes.get("default") if isinstance(routes, dict) else None) or ""
            rules = routes.get("rules", []) if isinstance(routes, dict) else []
            subs.append(SubscriptionSpec(spec["pubsubname"], spec["topic"], route.lstrip("/"),
                                         {k: _to_str(v) for k, v in (spec.get("metadata") or {}).items()},
                                         spec.get("deadLetterTopic"), list(doc.get("scopes") or []), rules, True))
        elif kind in ("Configuration", "Resiliency", "HTTPEndpoint"):
            others.append(doc)
        else:
            raise ComponentError(f"{source}: unsupported manifest kind {kind!r}")
    return comps, subs, others


def _timeout(v: Any) -> float:
    if v is None:
        return 5.0
    s = str(v).strip()
    from ..utils.cron import parse_duration
    try:
        return parse_duration(s).total_seconds()
    except ValueError:
        return float(s)


def load_file(path: str | os.PathLike, name: str | None = None) -> tuple[list[Component], list[SubscriptionSpec], list[dict[str, Any]]]:
    p = Path(path)
    with open(p, encoding="utf-8") as f:
        docs = list(yaml.safe_load_all(f))
    return parse_documents(docs, str(p), name)


def load_paths(paths: Iterable[str | os.PathLike]) -> tuple[list[Component], list[SubscriptionSpec], list[dict[str, Any]]]:
    """Load every ``*.yaml``/``*.yml`` under the given files/directories (``--resources-path``)."""
    comps: list[Component] = []
    subs: list[SubscriptionSpec] = []
    others: list[dict[str, Any]] = []
    for base in paths:
        bp = Path(base)
        files = [bp] if bp.is_file() else sorted(list(bp.glob("*.yaml")) + list(bp.glob("*.yml")))
        for f in files:
            c, s, o = load_file(f)
            comps += c
            subs += s
            others += o
    names: dict[str, str] = {}
    for c in comps:
        if c.name in names and names[c.name] != c.source:
            raise ComponentError(f"duplicate component name {c.name!r} in {names[c.name]} and {c.source}")
        names[c.name] = c.source
    return comps, subs, others


def from_dict(d: dict[str, Any], name: str | None = None) -> Component:
    """Inline component definition (environment manifest / tests), either dialect."""
    comps, _, _ = parse_documents([d], "<inline>", name)
    if len(comps) != 1:
        raise ComponentError("inline definition must describe exactly one component")
    return comps[0]
