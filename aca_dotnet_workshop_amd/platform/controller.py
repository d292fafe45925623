"""Environment controller: the Azure Container Apps control plane, locally.

``EnvironmentController(manifest, env_dir).up()`` performs what ``az deployment group
create -f bicep/main.bicep`` + the ACA platform do for the reference
(SURVEY.md §3.5 "Deploy"): start the backing services, provision resources and secrets,
register role assignments, install the Dapr components, deploy every container app as
a revision with ``minReplicas`` replicas (app + sidecar process pairs), open ingress,
and then keep reconciling:

* **supervision** -- crashed replicas are restarted with backoff (ACA restart policy);
* **autoscaling** -- one scaler per app with scale rules (KEDA, see ``scaler.py``);
* **revisions** -- re-applying a manifest whose revision-scope fields changed starts a new
  revision, shifts ingress to it once ready and retires the old one (single-revision mode);
  ``traffic`` weights split ingress between revisions (multiple-revision mode);
* a **control API** on ``<env>/control.sock`` (``status``, ``scale``, ``restart``,
  ``apply``, ``shutdown``) used by the CLI -- the ``az containerapp ...`` equivalent.
"""
from __future__ import annotations

import asyncio
import json
import logging
import os
import secrets as pysecrets
import shutil
import time
from dataclasses import dataclass, field
from pathlib import Path
from typing import Any, Callable

import yaml

from ..backing.client import BackingClient
from ..backing.shards import PARTITIONED_FAMILIES, ShardedBackingClient
from ..web.app import WebApp
from ..web.http import Request, Response, empty, json_response
from ..web.server import HttpServer
from .ingress import Backend, IngressRoute, make_ingress_async
from .limits import Limits, ResourceLimiter
from .pki import EnvironmentPki
from .manifest import Manifest, ManifestError, desired_state, identity_of, template_hash, validate
from .processes import LocalStack, ReplicaProc
from .registry import LocalRegistry, RegistryError
from .scaler import Autoscaler, ScaleRule, cron_metric

log = logging.getLogger("platform")
ADMIN = "platform-admin"


class ImagePullError(Exception):
    """A revision's image could not be pulled (unknown image, or the app identity lacks AcrPull):
    ACA reports the revision as failed to provision."""


@dataclass
class Revision:
    name: str
    template: str
    created: float = field(default_factory=time.time)
    replicas: list[ReplicaProc] = field(default_factory=list)
    active: bool = True


@dataclass
class AppRuntime:
    spec: dict[str, Any]
    revisions: list[Revision] = field(default_factory=list)
    ingress: Ingress | None = None
    ingress_sig: str | None = None  # the ingress config the listener was opened with
    autoscaler: Autoscaler | None = None
    desired: int = 1
    restarts: int = 0
    last_metrics: dict[str, float] = field(default_factory=dict)
    scale_events: list[dict[str, Any]] = field(default_factory=list)
    # every scaler poll (wall time, whether a trigger was active, replicas before, decided, the
    # poll's own recommendation): KEDA's polling and the HPA's scale-down stabilization window are
    # observable -- a scale-in comes one window after the last poll that recommended more
    polls: list[tuple[float, bool, int, int, int]] = field(default_factory=list)

    @property
    def name(self) -> str:
        return self.spec["name"]

    @property
    def current(self) -> Revision | None:
        act = [r for r in self.revisions if r.active]
        return act[-1] if act else None


class EnvironmentController:
    def __init__(self, manifest: Manifest, env_dir: str | os.PathLike, polling_interval: float | None = None,
                 cooldown: float | None = None, log_level: str = "warning",
                 registry_root: str | os.PathLike | None = None,
                 shard_exchange: Callable[[str], list[str]] | None = None) -> None:
        self.m = manifest
        # partitioned shared environment (backing/shards.py): called with this environment's
        # backing URL once it is up, returns every shard's URL in rank order (bench.py
        # --shared-env exchanges them over torch.distributed)
        self.shard_exchange = shard_exchange
        self.shards: list[str] = []
        self.dir = Path(env_dir).resolve()
        self.dir.mkdir(parents=True, exist_ok=True)
        (self.dir / "components").mkdir(exist_ok=True)
        keda = manifest.environment.get("keda") or {}
        self.polling = float(polling_interval if polling_interval is not None else keda.get("pollingIntervalSeconds", 30))
        self.cooldown = float(cooldown if cooldown is not None else keda.get("cooldownPeriodSeconds", 300))
        self.log_level = log_level
        ai = manifest.environment.get("appInsights") or {}
        env = {"TT_TELEMETRY_DIR": str(self.dir / "telemetry") if ai.get("enabled", True) else "",
               "TT_TRACE_SAMPLE_RATE": str(float(ai.get("samplingPercentage", 100)) / 100.0),
               "TT_LOG_FORMAT": "console"}
        self.stack = LocalStack(self.dir / "runtime", components=[str(self.dir / "components")], env=env)
        rl = manifest.environment.get("resourceLimits") or {}
        self.limiter = ResourceLimiter(manifest.name, enforce_memory=_truthy(rl.get("memory", True)),
                                       enforce_cpu=_truthy(rl.get("cpu", False)))
        self._oom: set[str] = set()
        # environment CA: sidecar mTLS identities (Dapr Sentry) and the ingress certificate
        tls = manifest.environment.get("tls") or {}
        self.mtls = _truthy(tls.get("daprMtls", True))
        self.pki = EnvironmentPki(self.dir / "pki", trust_domain=f"{manifest.name}.local")
        self.apps: dict[str, AppRuntime] = {}
        self.backing: BackingClient | None = None
        self.storage_keys: dict[str, str] = {}
        self.registry_root = registry_root
        self.registry: LocalRegistry | None = None
        self._pulled: dict[str, dict[str, Any]] = {}  # manifest digest -> unpacked container
        self.events: list[dict[str, Any]] = []
        self.stop_event = asyncio.Event()
        self._tasks: list[asyncio.Task] = []
        self._control: HttpServer | None = None
        self._lock = asyncio.Lock()
        self.started = time.time()

    # ------------------------------------------------------------------ events
    def event(self, kind: str, **kw: Any) -> None:
        e = {"ts": time.time(), "kind": kind, **kw}
        self.events.append(e)
        del self.events[:-500]
        log.info("%s %s", kind, kw)
        with open(self.dir / "events.jsonl", "a") as f:
            f.write(json.dumps(e) + "\n")

    # ------------------------------------------------------------------ up / down
    async def up(self, serve_control: bool = True) -> None:
        errs = validate(self.m)
        if errs:
            raise ManifestError(errs)
        await self._start_backing()
        await self._provision()
        self._install_components()
        for spec in self.m.apps:
            await self._deploy_app(spec)
        self._write_state()
        self._tasks.append(asyncio.ensure_future(self._supervise()))
        for rt in self.apps.values():
            if rt.autoscaler is not None:
                self._tasks.append(asyncio.ensure_future(self._scale_loop(rt)))
        self._tasks.append(asyncio.ensure_future(self._retention_loop()))
        if self.limiter.enforce_cpu and self.limiter.mode == "watchdog" and self.limiter.duty is None:
            self._tasks.append(asyncio.ensure_future(self._throttle_loop()))
        self.event("ResourceLimitsApplied", **self.limiter.describe())
        if serve_control:
            await self._serve_control()
        self.event("EnvironmentReady", name=self.m.name, apps=list(self.apps))

    async def down(self) -> None:
        for t in self._tasks:
            t.cancel()
        for rt in self.apps.values():
            if rt.ingress:
                await rt.ingress.stop()
        self.limiter.release_all()
        await asyncio.to_thread(self.stack.stop)
        if self._control is not None:
            await self._control.close(1.0)
        if self.backing is not None:
            await self.backing.close()
        self.event("EnvironmentStopped", name=self.m.name)

    async def run_forever(self) -> None:
        await self.stop_event.wait()
        await self.down()

    # ------------------------------------------------------------------ backing + provisioning
    async def _start_backing(self) -> None:
        policy = {"mode": (self.m.environment.get("rbac") or {}).get("mode", "open"),
                  "roleAssignments": [{"principal": ADMIN, "role": "Owner", "scope": ""}] + self.m.role_assignments(),
                  "keys": {}}
        st = self.m.resources.get("storage")
        if st:
            key_file = self.dir / "storage-keys.json"
            keys = json.loads(key_file.read_text()) if key_file.exists() else {}
            keys.setdefault(st["account"], pysecrets.token_urlsafe(24))
            key_file.write_text(json.dumps(keys))
            self.storage_keys = keys
            policy["keys"][f"storage/{st['account']}"] = keys[st["account"]]
        url = await asyncio.to_thread(self.stack.start_backing, str(self.dir / "backing"), policy)
        self.backing = BackingClient(url, identity=ADMIN)
        if self.shard_exchange is not None:
            urls = [u.rstrip("/") for u in await asyncio.to_thread(self.shard_exchange, url)]
            if len(urls) > 1:
                # the document store and the broker are partitioned over every rank's backing;
                # provisioning (topics, subscriptions, RU/s split) reaches all of them
                self.shards = urls
                for fam in PARTITIONED_FAMILIES:
                    self.stack.base_env[f"TT_BACKING_SHARDS_{fam}"] = ",".join(urls)
                self.backing = ShardedBackingClient(urls, identity=ADMIN, home=url)
        self.event("BackingServicesStarted", url=url, rbac=policy["mode"], shards=self.shards)

    async def _provision(self) -> None:
        r = self.m.resources
        b = self.backing
        sb = r.get("serviceBus")
        if sb:
            for t in sb.get("topics") or []:
                await b.sb_create_topic(sb["namespace"], t["name"])
                for s in t.get("subscriptions") or []:
                    s = {"name": s} if isinstance(s, str) else s
                    await b.sb_create_subscription(sb["namespace"], t["name"], s["name"],
                                                   int(s.get("lockDurationSeconds", 60)) * 1000,
                                                   int(s.get("maxDeliveryCount", 10)))
            for q in sb.get("queues") or []:
                q = {"name": q} if isinstance(q, str) else q
                await b.sb_create_queue(sb["namespace"], q["name"], int(q.get("lockDurationSeconds", 60)) * 1000,
                                        int(q.get("maxDeliveryCount", 10)))
        cdb = r.get("cosmosDb")
        if cdb:  # provisioned throughput: autoscale max (cosmos-db.bicep:68-72) or manual RU/s
            for d in cdb.get("databases") or []:
                for c in d.get("containers") or []:
                    ru = c.get("autoscaleMaxThroughput") or c.get("throughput") or 0
                    await b.doc_set_throughput(cdb["account"], d["name"], c["name"], float(ru))
        acr = r.get("containerRegistry")
        if acr and acr.get("name"):
            self.registry = LocalRegistry(acr["name"], self.registry_root)
            self.event("ContainerRegistryAttached", loginServer=self.registry.login_server,
                       repositories=[x["repository"] for x in self.registry.repositories()])
        kv = r.get("keyVault")
        if kv:
            for s in kv.get("secrets") or []:
                if "fromStorageAccountKey" in s:
                    val = self.storage_keys.get(s["fromStorageAccountKey"], "")
                else:
                    val = str(s.get("value", ""))
                await b.kv_set(kv["name"], s["name"], val)
        self.event("ResourcesProvisioned", resources=sorted(desired_state(self.m)))

    def _install_components(self) -> None:
        cdir = self.dir / "components"
        for f in cdir.glob("*.yaml"):
            f.unlink()
        for c in self.m.components:
            doc = yaml.safe_load(self.m.component_path(c).read_text())
            if "componentType" in doc:
                doc["name"] = c["name"]
                items = doc.setdefault("metadata", [])
            else:
                doc.setdefault("metadata", {})["name"] = c["name"]
                items = doc.setdefault("spec", {}).setdefault("metadata", [])
            # manifest-level metadata overrides (dapr-components.bicep sets metadata per deployment)
            for ov in c.get("metadata") or []:
                hit = next((m for m in items if m.get("name") == ov["name"]), None)
                if hit is None:
                    items.append({"name": ov["name"], "value": str(ov.get("value", ""))})
                else:
                    hit["value"] = str(ov.get("value", ""))
            (cdir / f"{c['name']}.yaml").write_text(yaml.safe_dump(doc, sort_keys=False))
        self.event("DaprComponentsInstalled", components=[c["name"] for c in self.m.components])

    # ------------------------------------------------------------------ apps
    def _generated_secret(self, app: str, name: str) -> str:
        """A ``generate: true`` app secret: random, created once per environment and kept in the
        environment directory (every replica and revision of the app gets the same value)."""
        f = self.dir / "generated-secrets.json"
        vals = json.loads(f.read_text()) if f.exists() else {}
        key = f"{app}/{name}"
        if key not in vals:
            vals[key] = pysecrets.token_hex(32)
            tmp = self.dir / "generated-secrets.json.tmp"
            tmp.write_text(json.dumps(vals))
            os.chmod(tmp, 0o600)
            os.replace(tmp, f)
        return vals[key]

    def _app_env(self, spec: dict[str, Any]) -> dict[str, str]:
        secrets = {s["name"]: self._generated_secret(spec["name"], s["name"]) if _truthy(s.get("generate", False))
                   else str(s.get("value", "")) for s in spec.get("secrets") or []}
        env: dict[str, str] = {"TT_APP_SECRETS": json.dumps(secrets), "TT_ROLE_NAME": spec["name"]}
        for e in spec.get("env") or []:
            v = secrets.get(e["secretRef"], "") if "secretRef" in e else e.get("value", "")
            env[e["name"]] = "true" if v is True else "false" if v is False else str(v)
        app_id = (spec.get("dapr") or {}).get("appId") or spec["name"]
        if self.mtls:
            w = self.pki.workload(app_id)
            env.update({"TT_MTLS_CERT": w.cert, "TT_MTLS_KEY": w.key, "TT_MTLS_CA": w.ca})
        for other in self.m.apps:
            if other.get("ingress") is not None:
                env[f"TT_INTERNAL_URL_{other['name'].upper().replace('-', '_')}"] = \
                    f"unix:{self._ingress_uds(other['name'])}:"
        return env

    def _ingress_uds(self, app: str) -> str:
        return str(self.stack.sock_dir / f"{app}.ingress.sock")

    def _pull(self, spec: dict[str, Any]) -> dict[str, Any]:
        """Pull the app's image from the environment's registry with the app identity: the
        ``registries`` entry names the identity, which needs **AcrPull** on the registry
        (container-apps.bicep:113-127).  Unpacked once per digest under ``runtime/images``."""
        ref = spec["image"]
        ident = identity_of(spec)
        try:
            if self.registry is None:
                raise ImagePullError(f"{spec['name']}: image {ref}: the environment has no containerRegistry")
            server = ref.split("/", 1)[0]
            reg = next((r for r in spec.get("registries") or [] if r.get("server") == server), None)
            if reg is None:
                raise ImagePullError(f"{spec['name']}: no registry credentials for {server}")
            scope = f"registry/{self.registry.name}"
            if not any(ra["principal"] == ident and ra["role"] == "AcrPull" and ra["scope"] == scope
                       for ra in self.m.role_assignments()):
                raise ImagePullError(f"{spec['name']}: UNAUTHORIZED: identity {ident!r} has no AcrPull role on {scope}")
            digest = self.registry.resolve(ref)
            if digest in self._pulled:
                return dict(self._pulled[digest], image=ref)
            rootfs, cfg = self.registry.unpack(digest, self.dir / "runtime" / "images")
        except (ImagePullError, RegistryError) as e:
            self.event("ImagePullFailed", app=spec["name"], image=ref, error=str(e))
            raise ImagePullError(str(e)) from None
        c = {"image": ref, "digest": digest, "rootfs": str(rootfs), "config": cfg["config"]}
        self._pulled[digest] = c
        self.event("ImagePulled", app=spec["name"], image=ref, digest=digest, identity=ident)
        return c

    def _start_replica(self, rt: AppRuntime, rev: Revision) -> ReplicaProc:
        spec = rt.spec
        dapr = spec.get("dapr") or {}
        level = self.log_level if not dapr.get("enableApiLogging") else "info"
        container = self._pull(spec) if spec.get("image") else None
        rp = self.stack.start_replica(dapr.get("appId") or spec["name"], extra_env=self._app_env(spec),
                                      module=spec.get("module"), log_level=level, identity=identity_of(spec),
                                      api_logging=bool(dapr.get("enableApiLogging")),
                                      grpc=str(dapr.get("apiProtocol", "http")).lower() == "grpc",
                                      container=container)
        rp.revision = rev.name  # type: ignore[attr-defined]
        rev.replicas.append(rp)
        self.limiter.add(rp.name, rp.proc.pid, Limits.from_spec(spec))
        self.event("ReplicaStarted", app=rt.name, revision=rev.name, replica=rp.name)
        return rp

    async def _deploy_app(self, spec: dict[str, Any]) -> AppRuntime:
        rt = self.apps.get(spec["name"]) or AppRuntime(spec)
        rt.spec = spec
        self.apps[spec["name"]] = rt
        sc = spec.get("scale") or {}
        lo = int(sc.get("minReplicas", 1))
        hi = int(sc.get("maxReplicas", max(lo, 1)))
        rules = [ScaleRule.from_manifest(r) for r in sc.get("rules") or []]
        rt.autoscaler = Autoscaler(lo, hi, rules, self.cooldown) if rules else None
        rt.desired = max(lo, 1) if rules or lo > 0 else lo
        tmpl = template_hash(spec)
        rev_name = f"{spec['name']}--{spec.get('revisionSuffix') or tmpl[:7]}"
        cur = rt.current
        if cur is not None and cur.template == tmpl:
            await self._reconcile_ingress(rt)  # app-level config: no new revision
            return rt
        rev = Revision(rev_name, tmpl)
        rt.revisions.append(rev)
        for _ in range(rt.desired):
            self._start_replica(rt, rev)
        await asyncio.to_thread(self.stack.wait_ready, 120.0, list(rev.replicas))
        self.event("RevisionProvisioned", app=rt.name, revision=rev.name, replicas=len(rev.replicas))
        if spec.get("ingress") is not None:
            await self._ensure_ingress(rt)
        mode = spec.get("activeRevisionsMode", "single")
        if cur is not None and mode == "single":
            cur.active = False
            await self._retire(rt, cur)
        self._refresh_backends(rt)
        return rt

    async def _retire(self, rt: AppRuntime, rev: Revision) -> None:
        self._refresh_backends(rt)
        for rp in list(rev.replicas):
            self.limiter.remove(rp.name)
            await asyncio.to_thread(self.stack.stop_replica, rp)
        rev.replicas.clear()
        self.event("RevisionDeactivated", app=rt.name, revision=rev.name)

    @staticmethod
    def _ingress_sig(ing: dict[str, Any] | None) -> str | None:
        """What needs a new listener when it changes (traffic weights are applied live)."""
        if ing is None:
            return None
        return json.dumps({k: ing.get(k) for k in ("external", "port", "transport", "allowInsecure")}, sort_keys=True,
                          default=str)

    async def _reconcile_ingress(self, rt: AppRuntime) -> None:
        """``az containerapp ingress update/enable/disable``: an ingress change is app-level
        configuration -- the listener is replaced, the running revision stays."""
        want = rt.spec.get("ingress")
        if rt.ingress is not None and self._ingress_sig(want) != rt.ingress_sig:
            await rt.ingress.stop()
            rt.ingress = None
            self.event("IngressRemoved" if want is None else "IngressUpdated", app=rt.name)
        if want is not None and rt.ingress is None:
            await self._ensure_ingress(rt)
        self._refresh_backends(rt)

    async def _ensure_ingress(self, rt: AppRuntime) -> None:
        if rt.ingress is not None:
            return
        ing = rt.spec["ingress"]
        rt.ingress_sig = self._ingress_sig(ing)
        route = IngressRoute(rt.name, bool(ing.get("external", False)))
        ingress = await make_ingress_async(route, self.stack.sock_dir)
        if rt.ingress is not None:  # another reconcile pass got there while this one built
            return
        rt.ingress = ingress
        port = int(ing.get("port") or 0)
        tls = None
        if route.external and str(ing.get("transport", "auto")).lower() != "http":
            tls = self.pki.server(f"ingress-{rt.name}", [rt.name])  # certificate files (CertPair)
        await rt.ingress.start(port or None, self._ingress_uds(rt.name), tls=tls,
                               allow_insecure=_truthy(ing.get("allowInsecure", False)))
        self.event("IngressReady", app=rt.name, external=route.external, port=rt.ingress.public_port,
                   tls=tls is not None, insecurePort=rt.ingress.insecure_port, **rt.ingress.describe())

    def _refresh_backends(self, rt: AppRuntime) -> None:
        if rt.ingress is None:
            return
        backends = []
        for rev in rt.revisions:
            if not rev.active:
                continue
            for rp in rev.replicas:
                port = rp.app_port
                if rp.alive() and port:
                    # the replica's local socket when it serves one (the environment network
                    # between the ingress and a replica is this host's), else its TCP port
                    uds = rp.app_uds if rp.app_uds and os.path.exists(rp.app_uds) else None
                    backends.append(Backend(rev.name, f"unix:{uds}:" if uds else f"http://127.0.0.1:{port}"))
        traffic = (rt.spec.get("ingress") or {}).get("traffic") or []
        rt.ingress.set_backends(backends, {t["revision"]: int(t.get("weight", 0)) for t in traffic})

    async def scale_to(self, rt: AppRuntime, n: int, reason: str) -> None:
        async with self._lock:
            rev = rt.current
            if rev is None:
                return
            live = [r for r in rev.replicas if r.alive()]
            if n > len(live):
                new = [self._start_replica(rt, rev) for _ in range(n - len(live))]
                await asyncio.to_thread(self.stack.wait_ready, 120.0, new)
            elif n < len(live):
                for rp in live[n:][::-1]:
                    rev.replicas.remove(rp)
                    self.limiter.remove(rp.name)
                    await asyncio.to_thread(self.stack.stop_replica, rp)
            rt.desired = n
            rt.scale_events.append({"ts": time.time(), "replicas": n, "reason": reason})
            self._refresh_backends(rt)
            self.event("Scaled", app=rt.name, replicas=n, reason=reason)

    # ------------------------------------------------------------------ loops
    async def _supervise(self) -> None:
        backoff: dict[str, float] = {}
        while True:
            await asyncio.sleep(0.5)
            for name, used in await asyncio.to_thread(self.limiter.check_memory):
                self._oom.add(name)
                st = self.limiter.replicas.get(name)
                self.event("ReplicaOOMKilled", replica=name, rssBytes=used,
                           limitBytes=st.limits.memory if st else None)
            if not self.stack.backing_alive():
                # the managed services' equivalent: restart in place over the durable logs
                code = self.stack.backing_proc.poll() if self.stack.backing_proc is not None else None
                self.event("BackingServicesCrashed", code=code)
                try:
                    await asyncio.to_thread(self.stack.restart_backing)
                    await self._provision()  # idempotent: entities already replayed from the logs
                    self.event("BackingServicesRestarted", url=self.stack.backing_url)
                except Exception as e:
                    self.event("BackingServicesFailedToStart", error=str(e))
            for rt in self.apps.values():
                rev = rt.current
                if rev is None:
                    continue
                for rp in list(rev.replicas):
                    if rp.alive():
                        continue
                    wait = backoff.get(rp.name, 0.5)
                    self.limiter.remove(rp.name)
                    self.event("ReplicaCrashed", app=rt.name, replica=rp.name, code=rp.proc.returncode,
                               reason="OOMKilled" if rp.name in self._oom else "Error")
                    self._oom.discard(rp.name)
                    async with self._lock:
                        rev.replicas.remove(rp)
                        await asyncio.sleep(wait)
                        new = self._start_replica(rt, rev)
                    backoff[new.name] = min(wait * 2, 30.0)
                    rt.restarts += 1
                    try:
                        await asyncio.to_thread(self.stack.wait_ready, 120.0, [new])
                    except Exception as e:
                        self.event("ReplicaFailedToStart", app=rt.name, replica=new.name, error=str(e))
                    self._refresh_backends(rt)

    def retention_days(self) -> float:
        return float((self.m.environment.get("logAnalytics") or {}).get("retentionInDays") or 0)

    def prune_telemetry(self, now: float | None = None) -> dict:
        """Log Analytics retention (``retentionInDays``) over the environment's telemetry dir."""
        from ..telemetry.retention import prune
        res = prune(self.dir / "telemetry", self.retention_days(), now)
        if res["removed"]:
            self.event("TelemetryPruned", retentionInDays=self.retention_days(), files=len(res["removed"]))
        return res

    async def _retention_loop(self) -> None:
        while True:
            try:
                await asyncio.to_thread(self.prune_telemetry)
            except Exception as e:
                log.warning("telemetry retention: %r", e)
            await asyncio.sleep(3600)

    async def _throttle_loop(self) -> None:
        """CPU duty cycle of every replica (watchdog mode, ``resourceLimits.cpu: true``)."""
        from .limits import PERIOD_S
        while True:  # a few ticks per period: a replica overruns its quota by at most a tick
            await asyncio.to_thread(self.limiter.throttle_tick)
            await asyncio.sleep(PERIOD_S / 4)

    async def metric(self, rt: AppRuntime, rule: ScaleRule) -> float:
        md = rule.metadata
        if rule.type == "azure-servicebus":
            ns = md.get("namespace") or (self.m.resources.get("serviceBus") or {}).get("namespace", "default")
            entity = md["queueName"] if md.get("queueName") else f"{md['topicName']}/subscriptions/{md['subscriptionName']}"
            c = await self.backing.sb_counts(ns, entity)
            return float(c.get("active", 0) + (c.get("locked", 0) if md.get("includeLocked") else 0))
        if rule.type == "azure-queue":
            acct = md.get("accountName") or (self.m.resources.get("storage") or {}).get("account")
            return float((await self.backing.queue_count(acct, md["queueName"])).get("active", 0))
        if rule.type == "http":
            if rt.ingress is None:
                return 0.0
            return float(rt.ingress.inflight)  # total in-flight; the rule target is per replica
        if rule.type in ("cpu", "memory"):
            import psutil
            vals = []
            for rp in (rt.current.replicas if rt.current else []):
                try:
                    p = psutil.Process(rp.proc.pid)
                    procs = [p] + p.children(recursive=True)
                    if rule.type == "cpu":
                        vals.append(sum(x.cpu_percent(interval=None) for x in procs) / max(float(rt.spec.get("resources", {}).get("cpu", 1.0)), 0.01))
                    else:
                        mem = sum(x.memory_info().rss for x in procs)
                        lim = _parse_mem(str(rt.spec.get("resources", {}).get("memory", "0.5Gi")))
                        vals.append(100.0 * mem / lim)
                except (psutil.Error, ValueError):
                    continue
            return sum(vals) / len(vals) if vals else 0.0
        if rule.type == "cron":
            return cron_metric(rule)
        return 0.0

    async def _scale_loop(self, rt: AppRuntime) -> None:
        while True:
            try:
                metrics = {r.name: await self.metric(rt, r) for r in rt.autoscaler.rules}
                rt.last_metrics = metrics
                cur = len([r for r in (rt.current.replicas if rt.current else []) if r.alive()])
                want = rt.autoscaler.decide(metrics, cur)
                rt.polls.append((time.time(), any(v > 0 for v in metrics.values()), cur, want,
                                 rt.autoscaler.last_rec))
                del rt.polls[:-2000]
                if want != cur:
                    await self.scale_to(rt, want, f"metrics={metrics}")
            except asyncio.CancelledError:
                raise
            except Exception as e:
                log.warning("scaler %s: %r", rt.name, e)
            await asyncio.sleep(self.polling)

    # ------------------------------------------------------------------ state + control API
    def status(self) -> dict[str, Any]:
        apps = {}
        for rt in self.apps.values():
            ing = rt.ingress
            apps[rt.name] = {
                "revisions": [{"name": r.name, "active": r.active, "created": r.created,
                               "replicas": [{"name": p.name, "pid": p.proc.pid, "alive": p.alive(), "appPort": p.app_port,
                                             "sidecar": p.sidecar_uds,
                                             **({"image": p.container["digest"], "isolation": p.container["isolation"]}
                                                if p.container else {})}
                                            for p in r.replicas]} for r in rt.revisions],
                "image": rt.spec.get("image") or None,
                "desiredReplicas": rt.desired, "restarts": rt.restarts,
                "scale": rt.spec.get("scale"), "lastMetrics": rt.last_metrics, "scaleEvents": rt.scale_events[-20:],
                "ingress": None if ing is None else {
                    "external": ing.route.external,
                    "fqdn": f"{'https' if ing.tls else 'http'}://127.0.0.1:{ing.public_port}",
                    "httpUrl": f"http://127.0.0.1:{ing.insecure_port}" if ing.insecure_port else None,
                    "internalUrl": f"unix:{self._ingress_uds(rt.name)}:", "inflight": ing.inflight,
                    "requests": ing.requests, **ing.describe()},
            }
        limits = {**self.limiter.describe(),
                  "replicas": {n: {"cpu": st.limits.cpu, "memoryBytes": st.limits.memory, "peakRssBytes": st.peak_rss,
                                   "throttledPeriods": self.limiter.throttled_periods(n)}
                               for n, st in self.limiter.replicas.items()}}
        return {"name": self.m.name, "envDir": str(self.dir), "backingUrl": self.stack.backing_url,
                "tls": {"caCert": str(self.pki.ca_crt), "daprMtls": self.mtls},
                "resourceLimits": limits,
                "uptimeSeconds": round(time.time() - self.started, 1), "apps": apps,
                "outputs": self.m.outputs(), "events": self.events[-30:]}

    async def live_metrics(self) -> dict[str, Any]:
        """Live Metrics snapshot (App Insights' Live Metrics blade): per replica, the sidecar's and
        the app's Prometheus counters plus CPU seconds of the replica's processes."""
        import psutil

        from ..telemetry.metrics import parse_exposition
        from ..web.client import HttpClient
        http = HttpClient(timeout=2.0)
        out: dict[str, Any] = {"ts": time.time(), "apps": {}}
        try:
            for rt in self.apps.values():
                reps = {}
                for r in (rt.current.replicas if rt.current else []):
                    if not r.alive():
                        continue
                    rec: dict[str, Any] = {}
                    app_url = (f"http://127.0.0.1:{r.app_port}/metrics" if r.container else
                               f"unix:{self.stack.sock_dir / (r.name + '.a.sock')}:/metrics")
                    for label, url in (("sidecar", f"unix:{r.sidecar_uds}:/metrics"), ("app", app_url)):
                        try:
                            resp = await http.get(url)
                            rec[label] = parse_exposition(resp.text) if resp.status == 200 else {}
                        except Exception:
                            rec[label] = {}
                    try:
                        procs = [psutil.Process(r.proc.pid)] + psutil.Process(r.proc.pid).children(recursive=True)
                        rec["cpuSeconds"] = sum(sum(p.cpu_times()[:2]) for p in procs)
                    except psutil.Error:
                        rec["cpuSeconds"] = 0.0
                    reps[r.name] = rec
                out["apps"][rt.name] = reps
        finally:
            await http.close()
        return out

    def _write_state(self) -> None:
        st = {"desired": desired_state(self.m), "status": self.status()}
        tmp = self.dir / "state.json.tmp"
        tmp.write_text(json.dumps(st, indent=1, default=str))
        os.replace(tmp, self.dir / "state.json")

    async def apply(self, manifest: Manifest) -> dict[str, Any]:
        errs = validate(manifest)
        if errs:
            raise ManifestError(errs)
        self.m = manifest
        await self._provision()
        self._install_components()
        changed = []
        for spec in manifest.apps:
            before = self.apps.get(spec["name"])
            prev = before.current.name if before and before.current else None
            rt = await self._deploy_app(spec)
            if rt.current and rt.current.name != prev:
                changed.append(rt.current.name)
        self._write_state()
        return {"newRevisions": changed}

    async def _serve_control(self) -> None:
        app = WebApp("platform-control")
        ctl = self

        async def status(req: Request) -> Response:
            return json_response(ctl.status())

        async def scale(req: Request) -> Response:
            rt = ctl.apps.get(req.path_params["app"])
            if rt is None:
                return json_response({"error": "no such app"}, 404)
            body = req.json() or {}
            sc = dict(rt.spec.get("scale") or {})
            if "min" in body:
                sc["minReplicas"] = int(body["min"])
            if "max" in body:
                sc["maxReplicas"] = int(body["max"])
            rt.spec["scale"] = sc
            lo, hi = int(sc.get("minReplicas", 1)), int(sc.get("maxReplicas", 1))
            if rt.autoscaler:
                rt.autoscaler.min_replicas, rt.autoscaler.max_replicas = lo, hi
            cur = len([r for r in (rt.current.replicas if rt.current else []) if r.alive()])
            target = min(hi, max(lo, int(body.get("replicas", cur))))
            if target != cur:
                await ctl.scale_to(rt, target, "manual")
            return json_response({"app": rt.name, "replicas": target, "min": lo, "max": hi})

        async def restart(req: Request) -> Response:
            rt = ctl.apps.get(req.path_params["app"])
            if rt is None or rt.current is None:
                return json_response({"error": "no such app"}, 404)
            n = len(rt.current.replicas)
            await ctl.scale_to(rt, 0, "restart")
            await ctl.scale_to(rt, max(n, 1), "restart")
            return json_response({"app": rt.name, "revision": rt.current.name, "replicas": n})

        async def do_apply(req: Request) -> Response:
            from .manifest import load_manifest
            body = req.json() or {}
            m = load_manifest(body["file"], body.get("parameters"), body.get("overrides"))
            try:
                return json_response(await ctl.apply(m))
            except ManifestError as e:
                return json_response({"errors": e.errors}, 400)

        async def shutdown(req: Request) -> Response:
            asyncio.get_running_loop().call_later(0.05, ctl.stop_event.set)
            return empty(202)

        async def live(req: Request) -> Response:
            return json_response(await ctl.live_metrics())

        app.add_route("/status", status, ("GET",))
        app.add_route("/metrics/live", live, ("GET",))
        app.add_route("/apps/{app}/scale", scale, ("POST",))
        app.add_route("/apps/{app}/restart", restart, ("POST",))
        app.add_route("/apply", do_apply, ("POST",))
        app.add_route("/shutdown", shutdown, ("POST",))
        self._control = HttpServer(app, asyncio.get_running_loop())
        await self._control.listen_unix(str(self.dir / "control.sock"))


def _parse_mem(s: str) -> float:
    s = s.strip()
    for suf, mul in (("Gi", 2 ** 30), ("Mi", 2 ** 20), ("Ki", 2 ** 10), ("G", 1e9), ("M", 1e6)):
        if s.endswith(suf):
            return float(s[:-len(suf)]) * mul
    return float(s)


def reset_env_dir(env_dir: str | os.PathLike) -> None:
    """``az group delete``: remove an environment's state (only when it is stopped)."""
    p = Path(env_dir)
    if (p / "control.sock").exists():
        raise RuntimeError("environment is running; run `down` first")
    shutil.rmtree(p, ignore_errors=True)


def _truthy(v) -> bool:
    return v is True or str(v).strip().lower() in ("1", "true", "yes", "on")
