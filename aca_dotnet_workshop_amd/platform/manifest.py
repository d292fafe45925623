"""Environment manifest: the Bicep (``bicep/main.bicep`` + modules) equivalent.

A manifest declares, in one YAML document, what the reference's IaC provisions
(SURVEY.md §2.5 E1-E13):

* ``environment``    -- the Container Apps environment: Log Analytics retention (E3,
  30 days), App-Insights-style tracing incl. sidecar spans (``daprAIInstrumentationKey``),
  RBAC enforcement mode;
* ``resources``      -- Key Vault + secrets (E4, E13), Service Bus namespace/topic/
  subscriptions (E5), Cosmos account/db/container (E6), Storage account/queues/containers
  (E7) -- provisioned into the backing-services emulator;
* ``daprComponents`` -- component name -> ACA-dialect file (E8);
* ``containerApps``  -- per app: ``image`` (from the environment's ``containerRegistry``, pulled
  with the app identity's AcrPull role) or ``module`` (the dev loop: code from the source tree), ingress (internal/external), Dapr
  settings, managed identity + role assignments, env/secrets, resources, scale rules
  (E9-E12, KEDA ``azure-servicebus`` rule of processor-backend-service.bicep:159-183);
* ``outputs``        -- like main.bicep:243-256.

Parameters: ``parameters:`` defaults, overridden by a parameters file (the
``main.parameters.json`` shape: ``{"parameters": {"x": {"value": ...}}}`` or flat JSON/YAML)
and by ``--param k=v``.  Strings may contain ``${name}`` references and a handful of
functions: ``${uniqueString(seed)}``, ``${empty(x)}``, ``${notEmpty(x)}``, ``${toLower(x)}``, ``${if(c, a, b)}``,
``${concat(a,b,...)}``, ``${coalesce(a,b,...)}``.

``validate`` lints the manifest (the ``az bicep build`` + ARM ``Validate`` stage of
.github/workflows/infra-deploy.yml:40-77) and ``what_if`` diffs it against the recorded
state of a running environment (the ``what-if`` stage, :80-99).
"""
from __future__ import annotations

import copy
import hashlib
import json
import re
from dataclasses import dataclass, field
from pathlib import Path
from typing import Any

import yaml

from ..sidecar.components import ComponentError, load_file
from ..utils.cron import CronError, CronSchedule

_EXPR = re.compile(r"\$\{([^{}]+)\}")
KNOWN_SCALE_TYPES = {"azure-servicebus", "azure-queue", "http", "cpu", "memory", "cron"}


class ManifestError(ValueError):
    def __init__(self, errors: list[str]) -> None:
        super().__init__("; ".join(errors))
        self.errors = errors


def unique_string(*parts: str) -> str:
    """Deterministic 13-char id like Bicep's ``uniqueString(resourceGroup().id)``."""
    h = hashlib.sha256("|".join(parts).encode()).hexdigest()
    return "".join(c for c in h if c.isalnum())[:13]


def _split_args(s: str) -> list[str]:
    out, depth, cur = [], 0, ""
    for ch in s:
        if ch == "," and depth == 0:
            out.append(cur.strip())
            cur = ""
            continue
        depth += ch == "("
        depth -= ch == ")"
        cur += ch
    if cur.strip():
        out.append(cur.strip())
    return out


def _eval(expr: str, params: dict[str, Any]) -> Any:
    expr = expr.strip()
    m = re.fullmatch(r"(\w+)\((.*)\)", expr)
    if m:
        fn, args = m.group(1), [_eval(a, params) for a in _split_args(m.group(2))]
        if fn == "uniqueString":
            return unique_string(*map(str, args))
        if fn == "empty":
            return not args[0]
        if fn == "notEmpty":
            return bool(args[0])
        if fn == "toLower":
            return str(args[0]).lower()
        if fn == "concat":
            return "".join(map(str, args))
        if fn == "coalesce":
            return next((a for a in args if a not in (None, "")), "")
        if fn == "if":  # Bicep's  cond ? a : b
            if len(args) != 3:
                raise ManifestError([f"if() takes 3 arguments in ${{{expr}}}"])
            return args[1] if args[0] else args[2]
        raise ManifestError([f"unknown function {fn}() in ${{{expr}}}"])
    if (expr.startswith("'") and expr.endswith("'")) or (expr.startswith('"') and expr.endswith('"')):
        return expr[1:-1]
    if expr in params:
        return params[expr]
    raise ManifestError([f"unknown parameter {expr!r}"])


def substitute(node: Any, params: dict[str, Any]) -> Any:
    if isinstance(node, str):
        m = _EXPR.fullmatch(node)
        if m:  # whole-string expression keeps its type (bool/int/list)
            return _eval(m.group(1), params)
        return _EXPR.sub(lambda mm: _fmt(_eval(mm.group(1), params)), node)
    if isinstance(node, list):  # Bicep's conditional deployment: items with a false ``if:`` drop out
        out = []
        for x in node:
            x = substitute(x, params)
            if isinstance(x, dict) and "if" in x:
                if not _truthy_cond(x.pop("if")):
                    continue
            out.append(x)
        return out
    if isinstance(node, dict):
        d = {k: substitute(v, params) for k, v in node.items()}
        for k, v in list(d.items()):  # a conditional object member (``resource x = if (...) {}``)
            if isinstance(v, dict) and "if" in v:
                if _truthy_cond(v.pop("if")):
                    continue
                del d[k]
        return d
    return node


def _truthy_cond(v: Any) -> bool:
    if isinstance(v, str):
        return v.strip().lower() not in ("", "false", "0", "no")
    return bool(v)


def _fmt(v: Any) -> str:
    if isinstance(v, bool):
        return "true" if v else "false"
    return str(v)


def load_parameters(path: str | Path | None) -> dict[str, Any]:
    if not path:
        return {}
    text = Path(path).read_text()
    data = json.loads(text) if str(path).endswith(".json") else yaml.safe_load(text)
    data = data or {}
    if "parameters" in data and isinstance(data["parameters"], dict):
        data = data["parameters"]
    return {k: (v["value"] if isinstance(v, dict) and "value" in v else v) for k, v in data.items()}


@dataclass
class Manifest:
    raw: dict[str, Any]
    path: Path
    params: dict[str, Any]
    doc: dict[str, Any] = field(default_factory=dict)

    @property
    def base_dir(self) -> Path:
        return self.path.parent

    @property
    def name(self) -> str:
        return (self.doc.get("metadata") or {}).get("name", "environment")

    @property
    def environment(self) -> dict[str, Any]:
        return self.doc.get("environment") or {}

    @property
    def resources(self) -> dict[str, Any]:
        return self.doc.get("resources") or {}

    @property
    def apps(self) -> list[dict[str, Any]]:
        return list(self.doc.get("containerApps") or [])

    def app(self, name: str) -> dict[str, Any]:
        for a in self.apps:
            if a["name"] == name:
                return a
        raise KeyError(name)

    @property
    def components(self) -> list[dict[str, Any]]:
        return list(self.doc.get("daprComponents") or [])

    def component_path(self, entry: dict[str, Any]) -> Path:
        return (self.base_dir / entry["file"]).resolve()

    def outputs(self) -> dict[str, Any]:
        return dict(self.doc.get("outputs") or {})

    def role_assignments(self) -> list[dict[str, str]]:
        out = []
        for a in self.apps:
            ident = identity_of(a)
            for ra in a.get("roleAssignments") or []:
                out.append({"principal": ident, "role": ra["role"], "scope": ra["scope"]})
        for ra in (self.environment.get("rbac") or {}).get("roleAssignments") or []:
            out.append(dict(ra))
        return out


def identity_of(app: dict[str, Any]) -> str:
    ident = app.get("identity") or {}
    return ident.get("name") or f"{app['name']}-identity"


def load_manifest(path: str | Path, parameters_file: str | Path | None = None,
                  overrides: dict[str, Any] | None = None) -> Manifest:
    p = Path(path).resolve()
    raw = yaml.safe_load(p.read_text()) or {}
    params = dict(raw.get("parameters") or {})
    params.update(load_parameters(parameters_file))
    params.update(overrides or {})
    # parameters may reference each other (one pass in declaration order is enough here)
    for k in list(params):
        params[k] = substitute(params[k], params)
    doc = copy.deepcopy({k: v for k, v in raw.items() if k != "parameters"})
    doc = substitute(doc, params)
    return Manifest(raw, p, params, doc)


def validate(m: Manifest) -> list[str]:
    """Lint: structure, references, scale rules, component files/scopes.  [] = valid."""
    errs: list[str] = []
    if m.doc.get("kind") != "Environment":
        errs.append("kind must be 'Environment'")
    names = [a.get("name") for a in m.apps]
    if len(set(names)) != len(names):
        errs.append(f"duplicate container app names: {names}")
    app_ids = set()
    for a in m.apps:
        n = a.get("name", "<unnamed>")
        if not a.get("module") and not a.get("image"):
            errs.append(f"{n}: 'image' or 'module' (the app's code from the source tree) is required")
        if a.get("image"):
            server = str(a["image"]).split("/", 1)[0]
            regs = [r for r in a.get("registries") or [] if r.get("server") == server]
            if not regs:
                errs.append(f"{n}: image {a['image']} needs a 'registries' entry for {server}")
            acr = m.resources.get("containerRegistry") or {}
            if not acr.get("name") or server != f"{acr['name']}.azurecr.io":
                errs.append(f"{n}: image registry {server} is not the environment's containerRegistry")
            for r in regs:
                if r.get("identity") and r["identity"] != identity_of(a):
                    errs.append(f"{n}: registry identity {r['identity']!r} is not the app's identity")
        ing = a.get("ingress")
        if ing is not None and not isinstance(ing.get("external", False), bool):
            errs.append(f"{n}: ingress.external must be a boolean")
        d = a.get("dapr") or {}
        if d.get("enabled"):
            app_ids.add(d.get("appId") or n)
        sc = a.get("scale") or {}
        lo, hi = int(sc.get("minReplicas", 1)), int(sc.get("maxReplicas", max(1, int(sc.get("minReplicas", 1)))))
        if lo < 0 or hi < 1 or lo > hi:
            errs.append(f"{n}: invalid replica bounds min={lo} max={hi}")
        for r in sc.get("rules") or []:
            t = (r.get("custom") or {}).get("type") or r.get("type")
            if t not in KNOWN_SCALE_TYPES:
                errs.append(f"{n}: scale rule {r.get('name')}: unsupported type {t!r}")
            meta = (r.get("custom") or r).get("metadata") or {}
            if t == "azure-servicebus":
                for k in ("topicName", "subscriptionName", "messageCount"):
                    if k not in meta and not (k == "topicName" and "queueName" in meta):
                        errs.append(f"{n}: scale rule {r.get('name')}: metadata.{k} is required")
            if t == "azure-queue" and "queueName" not in meta:
                errs.append(f"{n}: scale rule {r.get('name')}: metadata.queueName is required")
        for e in a.get("env") or []:
            if "secretRef" in e and e["secretRef"] not in {s["name"] for s in a.get("secrets") or []}:
                errs.append(f"{n}: env {e.get('name')} references unknown secret {e['secretRef']!r}")
    comp_names: set[str] = set()
    for c in m.components:
        cp = m.component_path(c)
        if not cp.exists():
            errs.append(f"component {c.get('name')}: file {c.get('file')} not found")
            continue
        try:
            comps, _, _ = load_file(cp, c.get("name"))
        except (ComponentError, yaml.YAMLError, KeyError) as ex:
            errs.append(f"component {c.get('name')}: {ex}")
            continue
        for comp in comps:
            comp_names.add(comp.name)
            unknown = [s for s in comp.scopes if s not in app_ids]
            if unknown:
                errs.append(f"component {comp.name}: scopes reference unknown app-ids {unknown}")
            if comp.type == "bindings.cron":
                sched = next((i.value for i in comp.items if i.name == "schedule"), None)
                try:
                    CronSchedule.parse(str(sched))
                except CronError as ex:
                    errs.append(f"component {comp.name}: {ex}")
            if comp.secret_store and comp.secret_store not in {x.get("name") for x in m.components}:
                errs.append(f"component {comp.name}: secretStoreComponent {comp.secret_store!r} is not declared")
    if len(comp_names) != len(m.components):
        errs.append("component names must be unique")
    sb = m.resources.get("serviceBus") or {}
    for t in sb.get("topics") or []:
        if not t.get("name"):
            errs.append("serviceBus topic without name")
    return errs


def desired_state(m: Manifest) -> dict[str, Any]:
    """Flattened resource inventory used by what-if and recorded after a deployment."""
    res: dict[str, Any] = {}
    r = m.resources
    acr = r.get("containerRegistry")
    if acr and acr.get("name"):
        res[f"containerRegistry/{acr['name']}"] = {"loginServer": f"{acr['name']}.azurecr.io"}
    kv = r.get("keyVault")
    if kv:
        res[f"keyVault/{kv['name']}"] = {"secrets": sorted(s["name"] for s in kv.get("secrets") or [])}
    sb = r.get("serviceBus")
    if sb:
        for t in sb.get("topics") or []:
            res[f"serviceBus/{sb['namespace']}/topics/{t['name']}"] = {
                "subscriptions": sorted(s if isinstance(s, str) else s["name"] for s in t.get("subscriptions") or [])}
        for q in sb.get("queues") or []:
            res[f"serviceBus/{sb['namespace']}/queues/{q if isinstance(q, str) else q['name']}"] = {}
    cos = r.get("cosmosDb")
    if cos:
        for db in cos.get("databases") or []:
            for c in db.get("containers") or []:
                res[f"cosmosDb/{cos['account']}/{db['name']}/{c['name']}"] = {
                    "partitionKey": c.get("partitionKey", "/id"), "maxThroughput": c.get("autoscaleMaxThroughput")}
    st = r.get("storage")
    if st:
        for q in st.get("queues") or []:
            res[f"storage/{st['account']}/queues/{q}"] = {}
        for c in st.get("containers") or []:
            res[f"storage/{st['account']}/containers/{c}"] = {}
    for c in m.components:
        res[f"daprComponents/{c['name']}"] = {"file": c["file"],
                                              "sha": hashlib.sha256(m.component_path(c).read_bytes()).hexdigest()[:12]
                                              if m.component_path(c).exists() else None}
    for a in m.apps:
        res[f"containerApps/{a['name']}"] = {"template": template_hash(a), "ingress": a.get("ingress"),
                                             "scale": a.get("scale"), "identity": identity_of(a)}
        if a.get("image"):
            res[f"containerApps/{a['name']}"]["image"] = a["image"]
    for ra in m.role_assignments():
        res[f"roleAssignments/{ra['principal']}/{ra['role']}/{ra['scope']}"] = {}
    return res


def template_hash(app: dict[str, Any]) -> str:
    """Revision-scope fields: a change here creates a new revision (ACA semantics)."""
    scoped = {k: app.get(k) for k in ("module", "args", "env", "resources", "dapr", "secrets", "revisionSuffix")}
    if app.get("image"):  # a new image reference is a new revision (the dev loop's apps have none)
        scoped["image"] = app["image"]
    return hashlib.sha256(json.dumps(scoped, sort_keys=True, default=str).encode()).hexdigest()[:10]


def what_if(m: Manifest, current: dict[str, Any] | None) -> list[dict[str, Any]]:
    """Diff desired vs recorded state: Create / Modify / Delete / NoChange entries."""
    desired = desired_state(m)
    cur = current or {}
    out = []
    for k in sorted(set(desired) | set(cur)):
        if k not in cur:
            out.append({"change": "Create", "resource": k, "after": desired[k]})
        elif k not in desired:
            out.append({"change": "Delete", "resource": k, "before": cur[k]})
        elif desired[k] != cur[k]:
            out.append({"change": "Modify", "resource": k, "before": cur[k], "after": desired[k]})
        else:
            out.append({"change": "NoChange", "resource": k})
    return out
