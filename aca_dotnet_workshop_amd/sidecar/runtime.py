"""The sidecar runtime -- the ``daprd`` equivalent.

One sidecar runs next to every app replica.  It exposes the building-block HTTP API to
its app and an internal endpoint to peer sidecars:

==============================================  ==============================================
API                                             reference usage
==============================================  ==============================================
``/v1.0/invoke/{app-id}/method/{path}``          every ``InvokeMethodAsync`` (§2.10 rows 1-10)
``dapr-app-id`` header proxying                  ``CreateInvokeHttpClient`` variants (Index.cshtml.cs:37-45)
``/v1.0/state/{store}[...]`` + query             TasksStoreManager.cs (§2.10 row 12)
``/v1.0/publish/{pubsub}/{topic}``               TasksStoreManager.cs:155 (row 11)
``/v1.0-alpha1/publish/bulk/...``                bulk publish
``/v1.0/bindings/{name}``                        ExternalTasksProcessorController.cs:43 (row 8)
``/v1.0/secrets/{store}/{key}`` + bulk           secret store building block
``/v1.0/metadata``, ``/v1.0/healthz``            runtime introspection / readiness
gRPC ``dapr.proto.runtime.v1.Dapr``              ``DaprClient``'s transport (``grpc_api.py``)
==============================================  ==============================================

Inbound to the app: ``GET /dapr/subscribe`` discovery then CloudEvent deliveries to the
subscribed routes (in-1, in-4), ``OPTIONS``-probed input-binding routes (in-2) and cron
triggers (in-3).  Components are loaded from ``--resources-path`` directories in either
manifest dialect, filtered by ``scopes``; secret references are resolved through the
configured secret stores.
"""
from __future__ import annotations

import asyncio
import json
import logging
import os
import time
import uuid
from typing import Any
from urllib.parse import parse_qsl

from ..models.dotnet import format_datetime, utcnow
from ..telemetry.metrics import REGISTRY
from ..telemetry.tracing import Tracer, parse_traceparent
from ..web.app import WebApp
from ..web.client import ConnectionClosed, HttpClient
from ..web.http import Request, Response, empty, json_response
from ..web.server import HttpServer
from .base import RuntimeContext, create_component
from .bindings import Binding, BindingError
from .components import Component, ComponentError, SubscriptionSpec, load_paths
from .pubsub import DROP, RETRY, SUCCESS, Consumer, PubSub, message_body
from .registry import NameResolver
from .secrets import APP_SECRETS_STORE, AppSecretsStore, SecretStore
from .state import EtagMismatch, SetRequest, StateStore

log = logging.getLogger("sidecar")
api_log = logging.getLogger("sidecar.http-info")

RUNTIME_VERSION = "1.0.0-tt"
_HOP = {"host", "content-length", "connection", "transfer-encoding", "keep-alive", "dapr-api-token", "dapr-app-id",
        "expect", "upgrade", "te", "trailer", "proxy-authorization"}

M_INVOKE = REGISTRY.counter("sidecar_invoke_total", "service invocations proxied by the sidecar")
M_INVOKE_LAT = REGISTRY.histogram("sidecar_invoke_seconds", "service invocation latency")
M_PUBLISH = REGISTRY.counter("sidecar_publish_total", "messages published")
M_DELIVER = REGISTRY.counter("sidecar_delivery_total", "pub/sub deliveries to the app by outcome")
M_BINDING = REGISTRY.counter("sidecar_binding_total", "binding operations")
M_STATE = REGISTRY.counter("sidecar_state_total", "state operations")


def err(status: int, code: str, message: str) -> Response:
    return json_response({"errorCode": code, "message": message}, status)


class Sidecar:
    def __init__(self, app_id: str, *, app_port: int | None = None, app_uds: str | None = None,
                 http_port: int | None = 3500, http_host: str = "127.0.0.1", uds: str | None = None,
                 internal_port: int | None = 0, internal_uds: str | None = None,
                 resources_paths: list[str] | None = None, components: list[Component] | None = None,
                 subscriptions: list[SubscriptionSpec] | None = None, registry_dir: str | None = None,
                 resolver: NameResolver | None = None, api_token: str | None = None, app_token: str | None = None,
                 mesh_token: str | None = None, app_max_concurrency: int | None = None,
                 identity: str | None = None, backing_url: str | None = None, environ: dict[str, str] | None = None,
                 telemetry_dir: str | None = None, instance: str | None = None,
                 app_health_path: str | None = None, data_plane: str | None = None,
                 api_logging: bool = False, grpc_port: int | None = None, grpc_uds: str | None = None,
                 mtls: dict[str, str] | None = None, app_ssl: bool | None = None) -> None:
        self.app_id = app_id
        self.app_port = app_port
        self.app_uds = app_uds
        self.http_port = http_port
        self.http_host = http_host
        self.uds = uds
        self.internal_port = internal_port
        self.internal_uds = internal_uds
        self.resources_paths = resources_paths or []
        self.extra_components = components or []
        self.extra_subscriptions = subscriptions or []
        self.environ = dict(os.environ if environ is None else environ)
        self.resolver = resolver or NameResolver(registry_dir or self.environ.get("TT_REGISTRY_DIR"))
        self.api_token = api_token
        self.app_token = app_token
        self.mesh_token = mesh_token
        self.instance = instance or f"{app_id}-{uuid.uuid4().hex[:8]}"
        self.app_health_path = app_health_path
        self.api_logging = api_logging
        self.grpc_port = grpc_port  # None: no gRPC API; 0: ephemeral port
        self.grpc_uds = grpc_uds
        self.grpc_server = None
        self.bound_grpc_port: int | None = None
        self.extended_metadata: dict[str, str] = {}
        # mutual TLS between sidecars (Dapr Sentry equivalent): this app-id's workload certificate
        # from the environment CA (platform/pki.py), presented and required on the internal endpoint
        env_mtls = {k: self.environ.get(f"TT_MTLS_{k.upper()}", "") for k in ("cert", "key", "ca")}
        self.mtls = mtls or (env_mtls if all(env_mtls.values()) else None)
        # --app-ssl: the app serves HTTPS (its own dev certificate, not verified -- Dapr's behaviour)
        self.app_ssl = bool(app_ssl) if app_ssl is not None else self.environ.get("TT_APP_SSL", "") in ("1", "true")
        self._mesh_server_tls = None
        mesh_client_tls = None
        if self.mtls:
            from ..platform.pki import CertPair
            pair = CertPair(self.mtls["cert"], self.mtls["key"], self.mtls["ca"])
            self._mesh_server_tls = pair.server_context(require_client_cert=True)
            mesh_client_tls = pair.client_context()
        self.http = HttpClient(timeout=300, tls=mesh_client_tls)
        self.app_http = self.http
        if self.app_ssl:
            import ssl
            insecure = ssl.SSLContext(ssl.PROTOCOL_TLS_CLIENT)
            insecure.check_hostname = False
            insecure.verify_mode = ssl.CERT_NONE
            self.app_http = HttpClient(timeout=300, tls=insecure)
        kw: dict[str, Any] = {"app_id": app_id, "identity": identity, "http": self.http, "environ": self.environ}
        if backing_url:
            kw["backing_url"] = backing_url
        self.ctx = RuntimeContext(**kw)
        self.tracer = Tracer(f"{app_id}.sidecar", telemetry_dir or self.environ.get("TT_TELEMETRY_DIR") or None,
                             float(self.environ.get("TT_TRACE_SAMPLE_RATE", "1.0")), self.instance)
        self.app_sem = asyncio.Semaphore(app_max_concurrency) if app_max_concurrency else None
        # "native": hot API paths served by the C++ data plane (native/src/dataplane.cpp), this
        # process keeps the control plane behind a private socket.  Not used with
        # --app-max-concurrency (the app-channel semaphore lives here).
        self.data_plane = (data_plane or self.environ.get("TT_SIDECAR_DATAPLANE") or "python").lower()
        self._dp_proc: asyncio.subprocess.Process | None = None
        self._dp_dir: str | None = None
        self._dp_control = ""
        self.components: dict[str, Component] = {}
        self.secret_stores: dict[str, SecretStore] = {}
        self.state_stores: dict[str, StateStore] = {}
        self.pubsubs: dict[str, PubSub] = {}
        self.bindings: dict[str, Binding] = {}
        self.subscriptions: list[SubscriptionSpec] = []
        self.consumers: list[Consumer] = []
        self.input_bindings: list[str] = []
        self.failed_components: dict[str, str] = {}
        self._servers: list[HttpServer] = []
        self._bg: list[asyncio.Task] = []
        self.ready = asyncio.Event()
        self.app_ready = asyncio.Event()
        self.stopped = asyncio.Event()
        self.bound_http_port: int | None = None
        self.bound_internal: str | None = None
        self.started_at = time.time()

    # ================================================================ lifecycle
    async def start(self) -> None:
        await self._load_components()
        api = self._build_api()
        internal = self._build_internal()
        loop = asyncio.get_running_loop()
        if self.data_plane == "native" and self.app_sem is None:
            await self._start_native_data_plane(api)
        else:
            await self._start_python_servers(api, internal, loop)
        if (self.grpc_port is not None or self.grpc_uds) and self.grpc_server is None:
            from .grpc_api import DaprGrpcServer
            self.grpc_server = DaprGrpcServer(self, api)
            self.bound_grpc_port = await self.grpc_server.start(self.grpc_port or 0, uds=self.grpc_uds)
        self.resolver.register(self.app_id, self.instance, self.bound_internal,
                               {"httpPort": self.bound_http_port, "dataPlane": self.active_data_plane})
        self.ready.set()
        log.info("sidecar %s up: api=%s%s grpc=%s internal=%s plane=%s components=%s", self.app_id,
                 self.bound_http_port, f" uds={self.uds}" if self.uds else "", self.bound_grpc_port,
                 self.bound_internal, self.active_data_plane,
                 sorted(self.components))
        if self.app_port is not None or self.app_uds:
            self._bg.append(asyncio.ensure_future(self._app_startup()))

    @property
    def active_data_plane(self) -> str:
        return "native" if self._dp_proc is not None else "python"

    async def _start_python_servers(self, api: WebApp, internal: WebApp, loop) -> None:
        srv = HttpServer(api, loop)
        if self.http_port is not None:
            self.bound_http_port = await srv.listen_tcp(self.http_host, self.http_port)
        if self.uds:
            await srv.listen_unix(self.uds)
        self._servers.append(srv)
        isrv = HttpServer(internal, loop)
        tls = self._mesh_server_tls
        if self.internal_uds:
            await isrv.listen_unix(self.internal_uds, ssl=tls)
            self.bound_internal = f"unix:{self.internal_uds}:"
        if self.internal_port is not None and (self.internal_port or not self.internal_uds):
            p = await isrv.listen_tcp("127.0.0.1", self.internal_port, ssl=tls)
            if self.bound_internal is None:
                self.bound_internal = f"http://127.0.0.1:{p}"
        if tls is not None and self.bound_internal:
            self.bound_internal = f"mtls:{self.app_id}@{self.bound_internal}"
        self._servers.append(isrv)

    def data_plane_config(self, fallback: str) -> dict[str, Any]:
        """What the native data plane needs to serve invoke/state/publish on its own."""
        from .pubsub import BackingTransport
        from .state import BackingStateStore
        stores = {}
        for name, st in self.state_stores.items():
            if isinstance(st, BackingStateStore):
                stores[name] = {"backing": st.client.base, "account": st.account, "db": st.db, "coll": st.coll,
                                "prefix": st.prefix, "identity": st.client.identity or "", "key": st.client.key or "",
                                "shards": list(getattr(st.client, "bases", []))}
        buses = {}
        for name, ps in self.pubsubs.items():
            t = getattr(ps, "transport", None)
            if isinstance(t, BackingTransport):
                buses[name] = {"backing": t.client.base, "ns": t.ns, "identity": t.client.identity or "",
                               "key": t.client.key or "", "shards": list(getattr(t.client, "bases", []))}
        listen = []
        if self.uds:
            listen.append("unix:" + self.uds)
        if self.http_port is not None:
            listen.append(f"tcp:{self.http_host}:{self.http_port}")
        internal = []
        if self.internal_uds:
            internal.append("unix:" + self.internal_uds)
        if self.internal_port is not None and (self.internal_port or not self.internal_uds):
            internal.append(f"tcp:127.0.0.1:{self.internal_port}")
        app = None
        if self.app_uds:
            app = "unix:" + self.app_uds
        elif self.app_port is not None:
            app = f"https+insecure://127.0.0.1:{self.app_port}" if self.app_ssl else f"tcp:127.0.0.1:{self.app_port}"
        ex = self.tracer.exporter
        return {"appId": self.app_id, "app": app, "appToken": self.app_token, "apiToken": self.api_token,
                "meshToken": self.mesh_token, "registryDir": str(self.resolver.dir) if self.resolver.dir else None,
                "fallback": fallback, "invokeNative": self.resolver.dir is not None, "appTimeout": 300.0,
                "listen": listen, "internal": internal, "stores": stores, "pubsubs": buses,
                "apiLogging": self.api_logging, **({"mtls": dict(self.mtls)} if self.mtls else {}),
                "trace": {"dir": ex.directory, "sampleRate": self.tracer.sample_rate, "role": self.tracer.role,
                          "instance": self.instance}}

    async def _start_native_data_plane(self, api: WebApp) -> None:
        import tempfile
        from ..native.build import build_dataplane
        # no silent fallback: a requested native plane must run (TT_DATAPLANE_BIN: an alternative
        # build of the same source, e.g. the sanitizer build used by the tests)
        exe = self.environ.get("TT_DATAPLANE_BIN") or build_dataplane()
        self._dp_dir = tempfile.mkdtemp(prefix="ttdp-")
        private = os.path.join(self._dp_dir, "cp.sock")
        grpc_listen = []
        if self.grpc_port is not None or self.grpc_uds:
            # the gRPC API port is served natively too (h2.hpp); RPCs it does not decode itself
            # come back here through /_tt/grpc/{Method} (grpc_api.py dispatch_raw)
            from .grpc_api import DaprGrpcServer
            self.grpc_server = DaprGrpcServer(self, api)
            if self.grpc_uds:
                grpc_listen.append("unix:" + self.grpc_uds)
            if self.grpc_port is not None:
                grpc_listen.append(f"tcp:127.0.0.1:{self.grpc_port}")
        srv = HttpServer(api, asyncio.get_running_loop())
        await srv.listen_unix(private)
        self._servers.append(srv)
        cfg = self.data_plane_config("unix:" + private)
        cfg["portFile"] = os.path.join(self._dp_dir, "ports.json")
        cfg["grpcListen"] = grpc_listen
        cfg["control"] = "unix:" + os.path.join(self._dp_dir, "ctl.sock")
        self._dp_control = cfg["control"] + ":"
        ex = self.tracer.exporter
        if ex.keep_in_memory:
            # no telemetry directory: the data plane writes its spans to a private file that is
            # relayed into this tracer's in-memory sink on access
            relay = os.path.join(self._dp_dir, "spans.jsonl")
            cfg["trace"].update({"file": relay, "flushEach": True})
            ex.attach_source(_span_file_reader(relay))
        cfg_path = os.path.join(self._dp_dir, "config.json")
        with open(cfg_path, "w") as f:
            json.dump(cfg, f)
        self._dp_proc = await asyncio.create_subprocess_exec(str(exe), cfg_path)
        deadline = time.monotonic() + 30
        while not os.path.exists(cfg["portFile"]):
            if self._dp_proc.returncode is not None:
                raise RuntimeError(f"native data plane exited with {self._dp_proc.returncode}")
            if time.monotonic() > deadline:
                raise TimeoutError("native data plane did not start")
            await asyncio.sleep(0.01)
        with open(cfg["portFile"]) as f:
            ports = json.load(f)
        if self.http_port is not None:
            self.bound_http_port = ports["http"]
        self.bound_internal = ports["internal"] or None
        if self.grpc_port is not None:
            self.bound_grpc_port = ports.get("grpc")

    async def stop(self, grace: float = 5.0) -> None:
        if self.stopped.is_set():
            return
        self.stopped.set()
        self.resolver.unregister()
        for t in self._bg:
            t.cancel()
        for c in self.consumers:
            await c.stop(grace)
        for b in self.bindings.values():
            await b.close()
        if self.grpc_server is not None:
            await self.grpc_server.stop(min(grace, 1.0))
        if self._dp_proc is not None and self._dp_proc.returncode is None:
            self._dp_proc.terminate()
            try:
                await asyncio.wait_for(self._dp_proc.wait(), grace + 1)
            except asyncio.TimeoutError:
                self._dp_proc.kill()
                await self._dp_proc.wait()
        for srv in self._servers:
            await srv.close(grace)
        if self._dp_dir:
            import shutil
            shutil.rmtree(self._dp_dir, ignore_errors=True)
        for group in (self.pubsubs, self.state_stores, self.secret_stores):
            for comp in group.values():
                try:
                    await comp.close()
                except Exception:
                    pass
        self.tracer.flush()
        await self.http.close()
        if self.app_http is not self.http:
            await self.app_http.close()

    # ================================================================ components
    async def _load_components(self) -> None:
        comps, subs, _ = load_paths(self.resources_paths) if self.resources_paths else ([], [], [])
        comps = comps + self.extra_components
        self.subscriptions = [s for s in subs + self.extra_subscriptions if not s.scopes or self.app_id in s.scopes]
        comps = [c for c in comps if c.in_scope(self.app_id)]
        self.components = {c.name: c for c in comps}
        # 1) secret stores (their own metadata may only use plain values / env refs)
        self.secret_stores[APP_SECRETS_STORE] = AppSecretsStore(self.ctx)
        for c in comps:
            if c.category == "secretstores":
                await self._init_component(c, resolve_secrets=False)
        # 2) everything else, resolving secret references
        for c in comps:
            if c.category != "secretstores":
                await self._init_component(c, resolve_secrets=True)

    async def _init_component(self, c: Component, resolve_secrets: bool) -> None:
        try:
            secrets: dict[str, str] | None = None
            if resolve_secrets and c.needs_secrets():
                secrets = {}
                for it in c.items:
                    if it.secret_name:
                        store = c.secret_store or APP_SECRETS_STORE
                        secrets[it.name] = await self._secret_value(store, it.secret_name, it.secret_key or it.secret_name)
            c.resolve(secrets, self.environ)
            inst = create_component(c, self.ctx)
            await asyncio.wait_for(inst.init(), max(c.init_timeout, 5.0))
        except Exception as e:
            self.failed_components[c.name] = f"{type(e).__name__}: {e}"
            if c.ignore_errors:
                log.warning("component %s (%s) failed to init, ignored: %s", c.name, c.type, e)
                return
            raise ComponentError(f"component {c.name} ({c.type}) failed to initialize: {e}") from e
        cat = c.category
        if cat == "secretstores":
            self.secret_stores[c.name] = inst  # type: ignore[assignment]
        elif cat == "state":
            self.state_stores[c.name] = inst  # type: ignore[assignment]
        elif cat == "pubsub":
            self.pubsubs[c.name] = inst  # type: ignore[assignment]
        elif cat == "bindings":
            self.bindings[c.name] = inst  # type: ignore[assignment]
        else:
            raise ComponentError(f"unsupported component category {cat}")

    async def _secret_value(self, store: str, name: str, key: str) -> str:
        s = self.secret_stores.get(store)
        if s is None:
            raise ComponentError(f"secret store {store!r} not found")
        got = await s.get(name)
        if got is None:
            raise ComponentError(f"secret {name!r} not found in store {store!r}")
        return got.get(key) if key in got else next(iter(got.values()))

    # ================================================================ app channel
    def app_base(self) -> str:
        if self.app_uds:
            return f"unix:{self.app_uds}:"
        return f"{'https' if self.app_ssl else 'http'}://127.0.0.1:{self.app_port}"

    async def call_app(self, method: str, path: str, headers: list[tuple[str, str]], body: bytes,
                       timeout: float | None = None):
        if self.app_token:
            headers = headers + [("dapr-api-token", self.app_token)]
        url = self.app_base() + "/" + path.lstrip("/")
        if self.app_sem is None:
            return await self.app_http.request(method, url, headers=headers, body=body, timeout=timeout)
        async with self.app_sem:
            return await self.app_http.request(method, url, headers=headers, body=body, timeout=timeout)

    async def _wait_for_app(self, timeout: float = 120.0) -> None:
        deadline = time.monotonic() + timeout
        while not self.stopped.is_set():
            try:
                if self.app_uds:
                    r, w = await asyncio.wait_for(asyncio.open_unix_connection(self.app_uds), 1.0)
                else:
                    r, w = await asyncio.wait_for(asyncio.open_connection("127.0.0.1", self.app_port), 1.0)
                w.close()
                if self.app_health_path:
                    resp = await self.app_http.request("GET", self.app_base() + self.app_health_path, timeout=2.0)
                    if resp.status >= 300:
                        raise ConnectionError("app not healthy yet")
                return
            except (OSError, asyncio.TimeoutError, ConnectionError):
                if time.monotonic() > deadline:
                    raise TimeoutError(f"app {self.app_id} did not start listening")
                await asyncio.sleep(0.05)

    async def _app_startup(self) -> None:
        try:
            await self._wait_for_app()
            await self._discover_subscriptions()
            await self._start_input_bindings()
            self.app_ready.set()
        except asyncio.CancelledError:
            raise
        except Exception:
            log.exception("sidecar %s: app startup handshake failed", self.app_id)

    async def _discover_subscriptions(self) -> None:
        subs = list(self.subscriptions)
        try:
            r = await self.call_app("GET", "/dapr/subscribe", [], b"", timeout=10)
            if r.status == 200 and r.body:
                for s in r.json() or []:
                    route = s.get("route") or ((s.get("routes") or {}).get("default")) or ""
                    rules = (s.get("routes") or {}).get("rules") or []
                    if not route and rules:
                        route = rules[0].get("path", "")
                    subs.append(SubscriptionSpec(s["pubsubname"], s["topic"], route.lstrip("/"),
                                                 {k: str(v) for k, v in (s.get("metadata") or {}).items()},
                                                 s.get("deadLetterTopic"), [], rules))
        except (OSError, ConnectionClosed, asyncio.TimeoutError) as e:
            log.info("sidecar %s: no /dapr/subscribe (%s)", self.app_id, e)
        self.subscriptions = subs
        for s in subs:
            ps = self.pubsubs.get(s.pubsubname)
            if ps is None:
                log.warning("sidecar %s: subscription to %s/%s skipped: pubsub component not loaded for this app",
                            self.app_id, s.pubsubname, s.topic)
                continue
            await self._subscribe_with_retry(ps, s)

    async def _subscribe_native(self, ps: PubSub, s: SubscriptionSpec) -> None:
        """Hand the subscription's delivery loop to the native data plane."""
        t = ps.transport
        entity = await ps.ensure_entity(s.topic)
        spec = {"name": f"{ps.name}/{s.topic}", "pubsub": ps.name, "topic": s.topic, "route": s.route,
                "entity": entity, "ns": t.ns, "backing": t.client.base, "identity": t.client.identity or "",
                "key": t.client.key or "", "deadLetterTopic": s.dead_letter_topic or "",
                "raw": s.metadata.get("rawPayload", "").lower() == "true", **ps.consumer_settings()}
        shards = list(getattr(t.client, "bases", []))
        specs = [spec]
        if shards:  # partitioned namespace: a receiver per shard, the replica's limits split over them
            n = len(shards)
            specs = [dict(spec, name=f"{spec['name']}#{i}", backing=url,
                          maxConcurrent=max(1, -(-spec["maxConcurrent"] // n)), prefetch=max(1, -(-spec["prefetch"] // n)))
                     for i, url in enumerate(shards)]
        for sp in specs:
            r = await self.http.request("POST", self._dp_control + "/subscribe", body=json.dumps(sp).encode(),
                                        headers=[("Content-Type", "application/json")])
            if r.status != 204:
                raise RuntimeError(f"native data plane refused subscription: {r.status} {r.body[:200]!r}")

    async def _subscribe_with_retry(self, ps: PubSub, s: SubscriptionSpec, delay: float = 1.0) -> None:
        from .pubsub import BackingTransport
        if self._dp_proc is not None and isinstance(getattr(ps, "transport", None), BackingTransport):
            try:
                await self._subscribe_native(ps, s)
                log.info("sidecar %s: subscribed %s/%s -> /%s (native)", self.app_id, s.pubsubname, s.topic, s.route)
                return
            except Exception as e:
                log.error("sidecar %s: subscribing %s/%s failed (%s); retrying in %.0fs", self.app_id, s.pubsubname,
                          s.topic, e, delay)

                async def again() -> None:
                    await asyncio.sleep(delay)
                    if not self.stopped.is_set():
                        await self._subscribe_with_retry(ps, s, min(delay * 2, 30.0))
                self._bg.append(asyncio.ensure_future(again()))
                return
        try:
            cs = await ps.subscribe(s.topic, self._make_delivery(ps, s), s.metadata, self._make_dead_letter(ps, s))
        except Exception as e:
            log.error("sidecar %s: subscribing %s/%s failed (%s); retrying in %.0fs", self.app_id, s.pubsubname,
                      s.topic, e, delay)

            async def later() -> None:
                await asyncio.sleep(delay)
                if not self.stopped.is_set():
                    await self._subscribe_with_retry(ps, s, min(delay * 2, 30.0))
            self._bg.append(asyncio.ensure_future(later()))
            return
        self.consumers.extend(cs)
        log.info("sidecar %s: subscribed %s/%s -> /%s", self.app_id, s.pubsubname, s.topic, s.route)

    def _make_delivery(self, ps: PubSub, sub: SubscriptionSpec):
        raw_sub = sub.metadata.get("rawPayload", "").lower() == "true"

        async def deliver(m: dict[str, Any]) -> str:
            body = message_body(m)
            ctype = m.get("contentType") or "application/json"
            parent = None
            if ctype.startswith("application/cloudevents"):
                try:
                    ce = json.loads(body)
                    parent = parse_traceparent(ce.get("traceparent"))
                except ValueError:
                    ce = None
            else:
                ce = None
            if ce is None and not raw_sub:
                ce = make_cloudevent(body, ctype, ps.name, sub.topic, "unknown", None, m.get("id"))
                body = json.dumps(ce).encode()
                ctype = "application/cloudevents+json"
            span = self.tracer.start_span(f"pubsub/{sub.topic}", "consumer", parent)
            span.set("messaging.delivery_count", m.get("deliveryCount"))
            try:
                headers = [("Content-Type", "application/cloudevents+json" if ce is not None and not raw_sub else ctype),
                           ("traceparent", span.traceparent), ("pubsubname", ps.name), ("topic", sub.topic)]
                try:
                    r = await self.call_app("POST", sub.route, headers, body)
                except (OSError, ConnectionClosed, asyncio.TimeoutError) as e:
                    span.fail(e)
                    M_DELIVER.inc(app=self.app_id, outcome="retry")
                    return RETRY
                span.set("http.status", r.status)
                outcome = RETRY
                if 200 <= r.status < 300:
                    outcome = SUCCESS
                    if r.body and "json" in r.headers.get("content-type", ""):
                        try:
                            st = (r.json() or {}).get("status", "") if isinstance(r.json(), dict) else ""
                        except ValueError:
                            st = ""
                        st = str(st).upper()
                        outcome = {"RETRY": RETRY, "DROP": DROP}.get(st, SUCCESS)
                elif r.status == 404:
                    outcome = DROP
                if outcome != SUCCESS:
                    span.status = "error"
                M_DELIVER.inc(app=self.app_id, outcome=outcome)
                return outcome
            finally:
                span.end()
        return deliver

    def _make_dead_letter(self, ps: PubSub, sub: SubscriptionSpec):
        if not sub.dead_letter_topic:
            return None

        async def forward(m: dict[str, Any]) -> bool:
            await ps.publish(sub.dead_letter_topic, message_body(m), m.get("contentType") or "application/json", {})
            return True
        return forward

    async def _start_input_bindings(self) -> None:
        for name, b in self.bindings.items():
            if not b.is_input:
                continue
            route = b.route()
            try:
                r = await self.call_app("OPTIONS", route, [], b"", timeout=10)
            except (OSError, ConnectionClosed, asyncio.TimeoutError):
                continue
            if r.status == 404:
                log.info("sidecar %s: app does not listen on %s; input binding %s not started", self.app_id, route, name)
                continue
            await b.start(self._make_binding_delivery(name, route))
            self.input_bindings.append(name)
            log.info("sidecar %s: input binding %s -> %s", self.app_id, name, route)

    def _make_binding_delivery(self, name: str, route: str):
        async def deliver(data: bytes, metadata: dict[str, str]) -> bool:
            span = self.tracer.start_span(f"bindings/{name}", "consumer", None)
            try:
                headers = [("Content-Type", "application/json"), ("traceparent", span.traceparent)]
                headers += [(k, v) for k, v in metadata.items() if v is not None]
                r = await self.call_app("POST", route, headers, data)
                span.set("http.status", r.status)
                ok = 200 <= r.status < 300
                if not ok:
                    span.status = "error"
                M_BINDING.inc(app=self.app_id, binding=name, direction="input", ok=str(ok))
                return ok
            except Exception as e:
                span.fail(e)
                return False
            finally:
                span.end()
        return deliver

    # ================================================================ API app
    def _build_api(self) -> WebApp:
        app = WebApp(f"{self.app_id}.sidecar")
        sc = self

        async def tracing_mw(req: Request, nxt) -> Response:
            if req.path.startswith("/v1.0/healthz"):
                return await nxt(req)
            if sc.api_token and req.headers.get("dapr-api-token") != sc.api_token:
                return err(401, "ERR_API_TOKEN", "invalid api token")
            parent = parse_traceparent(req.headers.get("traceparent"))
            span = sc.tracer.start_span(f"{req.method} {req.path.split('?')[0][:80]}", "server", parent)
            req.state["span"] = span
            t0 = time.perf_counter() if sc.api_logging else 0.0
            try:
                resp = await nxt(req)
                span.set("http.status", resp.status)
                if resp.status >= 500:
                    span.status = "error"
                if sc.api_logging:
                    api_log.info("HTTP API Called method=%s path=%s status=%d duration_ms=%.3f app_id=%s",
                                 req.method, req.path, resp.status, (time.perf_counter() - t0) * 1e3, sc.app_id)
                return resp
            except BaseException as e:
                span.fail(e)
                raise
            finally:
                span.end()
        app.use(tracing_mw)

        invoke_methods = ("GET", "POST", "PUT", "DELETE", "PATCH", "HEAD", "OPTIONS")
        app.add_route("/v1.0/invoke/{appId}/method/{*method}", self.h_invoke, invoke_methods)
        app.add_route("/v1.0/state/{store}", self.h_state_save, ("POST", "PUT"))
        app.add_route("/v1.0/state/{store}/bulk", self.h_state_bulk, ("POST", "PUT"))
        app.add_route("/v1.0/state/{store}/transaction", self.h_state_tx, ("POST", "PUT"))
        app.add_route("/v1.0/state/{store}/{key}", self.h_state_get, ("GET",))
        app.add_route("/v1.0/state/{store}/{key}", self.h_state_delete, ("DELETE",))
        for ver in ("v1.0-alpha1", "v1.0-beta1"):
            app.add_route(f"/{ver}/state/{{store}}/query", self.h_state_query, ("POST", "PUT"))
        app.add_route("/v1.0/publish/{pubsub}/{*topic}", self.h_publish, ("POST", "PUT"))
        app.add_route("/v1.0-alpha1/publish/bulk/{pubsub}/{*topic}", self.h_publish_bulk, ("POST", "PUT"))
        app.add_route("/v1.0/bindings/{name}", self.h_binding, ("POST", "PUT"))
        app.add_route("/v1.0/secrets/{store}/bulk", self.h_secret_bulk, ("GET",))
        app.add_route("/v1.0/secrets/{store}/{key}", self.h_secret, ("GET",))
        app.add_route("/v1.0/metadata", self.h_metadata, ("GET",))
        app.add_route("/v1.0/metadata/{key}", self.h_metadata_set, ("PUT",))
        app.add_route("/v1.0/healthz", self.h_healthz, ("GET",))
        app.add_route("/v1.0/healthz/outbound", self.h_healthz, ("GET",))
        app.add_route("/v1.0/shutdown", self.h_shutdown, ("POST",))
        app.add_route("/metrics", self.h_metrics, ("GET",))
        app.add_route("/_tt/grpc/{method}", self.h_grpc_bridge, ("POST",))
        app.add_route("/{*path}", self.h_header_proxy, invoke_methods)
        return app

    def _build_internal(self) -> WebApp:
        app = WebApp(f"{self.app_id}.sidecar.internal")
        app.add_route("/{*path}", self.h_internal, ("GET", "POST", "PUT", "DELETE", "PATCH", "HEAD", "OPTIONS"))
        return app

    # ---------------------------------------------------------------- invoke
    @staticmethod
    def _fwd_headers(req: Request) -> list[tuple[str, str]]:
        out = []
        for k, v in req.headers.items():
            if k in _HOP or k == "traceparent":
                continue
            if isinstance(v, list):
                out.extend((k, x) for x in v)
            else:
                out.append((k, v))
        return out

    @staticmethod
    def _relay(r) -> Response:
        headers = []
        for k, v in r.headers.items():
            if k in _HOP or k == "content-length":
                continue
            if isinstance(v, list):
                headers.extend((k, x) for x in v)
            else:
                headers.append((k, v))
        return Response(r.body, r.status, headers)

    async def h_invoke(self, req: Request) -> Response:
        target = req.path_params["appId"]
        method_path = req.path_params["method"]
        return await self._invoke(req, target, method_path)

    async def h_grpc_bridge(self, req: Request) -> Response:
        """RPCs the native data plane's gRPC port does not decode itself (grpc_api.py dispatch_raw)."""
        if self.grpc_server is None or self._dp_proc is None:
            return err(404, "ERR_NOT_FOUND", f"no route for {req.path}")
        return await self.grpc_server.dispatch_raw(req)

    async def h_header_proxy(self, req: Request) -> Response:
        target = req.headers.get("dapr-app-id")
        if not target:
            return err(404, "ERR_NOT_FOUND", f"no route for {req.path}")
        return await self._invoke(req, target, req.path.lstrip("/"))

    async def _invoke(self, req: Request, target: str, method_path: str) -> Response:
        t0 = time.perf_counter()
        target = target.split(".")[0]
        qs = ("?" + req.query_string) if req.query_string else ""
        span = req.state.get("span")
        headers = self._fwd_headers(req) + [("dapr-caller-app-id", self.app_id)]
        if span is not None:
            headers.append(("traceparent", span.traceparent))
            span.set("invoke.target", target)
        try:
            if target == self.app_id:
                r = await self.call_app(req.method, method_path + qs, headers, req.body)
            else:
                r = await self._call_peer(target, req.method, method_path + qs, headers, req.body)
        except LookupError as e:
            return err(500, "ERR_DIRECT_INVOKE", str(e))
        except (OSError, ConnectionClosed, asyncio.TimeoutError) as e:
            M_INVOKE.inc(app=self.app_id, target=target, status="error")
            return err(500, "ERR_DIRECT_INVOKE", f"failed to invoke, id: {target}, err: {e!r}")
        M_INVOKE.inc(app=self.app_id, target=target, status=str(r.status))
        M_INVOKE_LAT.observe(time.perf_counter() - t0, app=self.app_id, target=target)
        return self._relay(r)

    async def _call_peer(self, target: str, method: str, path: str, headers: list[tuple[str, str]], body: bytes):
        cands = self.resolver.candidates(target)
        if not cands:
            self.resolver.invalidate(target)
            cands = self.resolver.candidates(target)
            if not cands:
                raise LookupError(f"failed to resolve address for app-id {target!r}")
        if self.mesh_token:
            headers = headers + [("tt-mesh-token", self.mesh_token)]
        last: Exception | None = None
        for ep in cands[:3]:
            try:
                return await self.http.request(method, ep + "/" + path.lstrip("/"), headers=headers, body=body)
            except (ConnectionRefusedError, FileNotFoundError, ConnectionClosed) as e:
                # replica went away: try the next one (resiliency for transient failures)
                last = e
                self.resolver.invalidate(target)
        raise last or ConnectionError("no reachable replica")

    async def h_internal(self, req: Request) -> Response:
        if self.mtls:
            # the caller's workload certificate must name the app-id it claims (no spoofing)
            caller = req.headers.get("dapr-caller-app-id")
            peer = (req.state.get("tls") or {}).get("peer")
            if peer is None or (caller and caller not in peer):
                return err(403, "ERR_MESH_AUTH", "caller identity not proven by its mTLS certificate")
        if self.mesh_token and req.headers.get("tt-mesh-token") != self.mesh_token:
            return err(403, "ERR_MESH_AUTH", "sidecar-to-sidecar call not authenticated")
        parent = parse_traceparent(req.headers.get("traceparent"))
        span = self.tracer.start_span(f"{req.method} /{req.path_params['path']}", "server", parent)
        span.set("caller", req.headers.get("dapr-caller-app-id", ""))
        try:
            headers = [(k, v) for k, v in self._fwd_headers(req) if k != "tt-mesh-token"]
            headers.append(("traceparent", span.traceparent))
            qs = ("?" + req.query_string) if req.query_string else ""
            try:
                r = await self.call_app(req.method, req.path_params["path"] + qs, headers, req.body)
            except (OSError, ConnectionClosed, asyncio.TimeoutError) as e:
                span.fail(e)
                return err(502, "ERR_APP_CHANNEL", f"app {self.app_id} unreachable: {e!r}")
            span.set("http.status", r.status)
            return self._relay(r)
        finally:
            span.end()

    # ---------------------------------------------------------------- state
    def _store(self, req: Request) -> StateStore | Response:
        name = req.path_params["store"]
        s = self.state_stores.get(name)
        if s is None:
            return err(400, "ERR_STATE_STORE_NOT_FOUND", f"state store {name} is not found")
        return s

    async def h_state_save(self, req: Request) -> Response:
        s = self._store(req)
        if isinstance(s, Response):
            return s
        try:
            items = req.json()
        except ValueError as e:
            return err(400, "ERR_MALFORMED_REQUEST", str(e))
        if not isinstance(items, list):
            return err(400, "ERR_MALFORMED_REQUEST", "request body must be an array of state items")
        reqs = []
        for it in items:
            if not isinstance(it, dict) or not it.get("key"):
                return err(400, "ERR_MALFORMED_REQUEST", "state item without key")
            meta = it.get("metadata") or {}
            opts = it.get("options") or {}
            etag = it.get("etag")
            if isinstance(etag, dict):
                etag = etag.get("value")
            reqs.append(SetRequest(it["key"], json.dumps(it.get("value"), separators=(",", ":")), etag or None,
                                   opts.get("concurrency") == "first-write",
                                   int(float(meta.get("ttlInSeconds", 0) or 0) * 1000)))
        try:
            await s.set_many(reqs)
        except EtagMismatch as e:
            return err(409, "ERR_STATE_SAVE", f"failed saving state in state store {s.name}: {e}")
        except Exception as e:
            return err(500, "ERR_STATE_SAVE", f"failed saving state in state store {s.name}: {e}")
        M_STATE.inc(app=self.app_id, op="save", n=str(min(len(reqs), 10)))
        return empty(204)

    async def h_state_get(self, req: Request) -> Response:
        s = self._store(req)
        if isinstance(s, Response):
            return s
        try:
            r = await s.get(req.path_params["key"])
        except Exception as e:
            return err(500, "ERR_STATE_GET", str(e))
        M_STATE.inc(app=self.app_id, op="get")
        if r is None:
            return empty(204)
        return Response(r[0], 200, [("ETag", r[1])], "application/json")

    async def h_state_delete(self, req: Request) -> Response:
        s = self._store(req)
        if isinstance(s, Response):
            return s
        try:
            await s.delete(req.path_params["key"], req.headers.get("if-match") or None)
        except EtagMismatch as e:
            return err(409, "ERR_STATE_DELETE", str(e))
        except Exception as e:
            return err(500, "ERR_STATE_DELETE", str(e))
        M_STATE.inc(app=self.app_id, op="delete")
        return empty(204)

    async def h_state_bulk(self, req: Request) -> Response:
        s = self._store(req)
        if isinstance(s, Response):
            return s
        body = req.json() or {}
        try:
            return json_response(await s.bulk_get(list(body.get("keys") or [])))
        except Exception as e:
            return err(500, "ERR_STATE_BULK_GET", str(e))

    async def h_state_tx(self, req: Request) -> Response:
        s = self._store(req)
        if isinstance(s, Response):
            return s
        body = req.json() or {}
        try:
            await s.transact(body.get("operations") or [])
        except EtagMismatch as e:
            return err(409, "ERR_STATE_TRANSACTION", str(e))
        except ValueError as e:
            return err(400, "ERR_MALFORMED_REQUEST", str(e))
        except Exception as e:
            return err(500, "ERR_STATE_TRANSACTION", str(e))
        return empty(204)

    async def h_state_query(self, req: Request) -> Response:
        s = self._store(req)
        if isinstance(s, Response):
            return s
        if not s.supports_query:
            return err(500, "ERR_STATE_STORE_NOT_SUPPORTED", f"state store {s.name} does not support query")
        try:
            body = await s.query(req.body or b"{}")
        except Exception as e:
            status = getattr(e, "status", 500)
            return err(400 if status == 400 else 500, "ERR_STATE_QUERY", str(e))
        M_STATE.inc(app=self.app_id, op="query")
        return Response(body, 200, None, "application/json")

    # ---------------------------------------------------------------- pub/sub
    async def h_publish(self, req: Request) -> Response:
        name = req.path_params["pubsub"]
        topic = req.path_params["topic"]
        ps = self.pubsubs.get(name)
        if ps is None:
            return err(404 if name else 404, "ERR_PUBSUB_NOT_FOUND", f"pubsub {name} not found")
        if not topic:
            return err(404, "ERR_TOPIC_EMPTY", "topic is empty")
        meta = _metadata_from_query(req.query_string)
        ctype = req.headers.get("content-type") or "application/json"
        body, out_ctype = self._envelope(req.body, ctype, name, topic, meta, req.state.get("span"))
        try:
            await ps.publish(topic, body, out_ctype, meta)
        except Exception as e:
            return err(500, "ERR_PUBSUB_PUBLISH_MESSAGE", f"error when publish to topic {topic} in pubsub {name}: {e}")
        M_PUBLISH.inc(app=self.app_id, pubsub=name, topic=topic)
        return empty(204)

    def _envelope(self, body: bytes, ctype: str, pubsub: str, topic: str, meta: dict[str, str], span) -> tuple[bytes, str]:
        if meta.get("rawPayload", "").lower() == "true":
            return body, ctype
        tp = span.traceparent if span is not None else None
        if ctype.split(";")[0].strip().lower() == "application/cloudevents+json":
            try:
                ce = json.loads(body)
                ce.setdefault("specversion", "1.0")
                ce.setdefault("id", str(uuid.uuid4()))
                ce.setdefault("source", self.app_id)
                ce.setdefault("type", "com.dapr.event.sent")
                ce["topic"], ce["pubsubname"] = topic, pubsub
                if tp:
                    ce.setdefault("traceparent", tp)
                return json.dumps(ce).encode(), "application/cloudevents+json"
            except ValueError:
                pass
        ce = make_cloudevent(body, ctype, pubsub, topic, self.app_id, tp)
        return json.dumps(ce, separators=(",", ":")).encode(), "application/cloudevents+json"

    async def h_publish_bulk(self, req: Request) -> Response:
        name = req.path_params["pubsub"]
        topic = req.path_params["topic"]
        ps = self.pubsubs.get(name)
        if ps is None:
            return err(404, "ERR_PUBSUB_NOT_FOUND", f"pubsub {name} not found")
        entries = req.json() or []
        failed = []
        for e in entries:
            ctype = e.get("contentType") or "application/json"
            ev = e.get("event")
            raw = json.dumps(ev).encode() if "json" in ctype else (ev if isinstance(ev, str) else json.dumps(ev)).encode()
            body, out_ctype = self._envelope(raw, ctype, name, topic, e.get("metadata") or {}, req.state.get("span"))
            try:
                await ps.publish(topic, body, out_ctype, e.get("metadata") or {})
            except Exception as ex:
                failed.append({"entryId": e.get("entryId"), "error": str(ex)})
        M_PUBLISH.inc(len(entries) - len(failed), app=self.app_id, pubsub=name, topic=topic)
        if failed:
            return json_response({"failedEntries": failed, "errorCode": "ERR_PUBSUB_PUBLISH_MESSAGE"}, 500)
        return empty(204)

    # ---------------------------------------------------------------- bindings
    async def h_binding(self, req: Request) -> Response:
        name = req.path_params["name"]
        b = self.bindings.get(name)
        if b is None or not b.is_output:
            return err(400, "ERR_INVOKE_OUTPUT_BINDING", f"output binding {name} not found")
        try:
            body = req.json() or {}
        except ValueError as e:
            return err(400, "ERR_MALFORMED_REQUEST", str(e))
        op = body.get("operation") or ""
        data = body.get("data")
        if data is None:
            raw = b""
        elif isinstance(data, str):
            raw = data.encode()
        else:
            raw = json.dumps(data, separators=(",", ":")).encode()
        meta = {k: str(v) for k, v in (body.get("metadata") or {}).items()}
        try:
            out, out_meta = await b.invoke(op, raw, meta)
        except BindingError as e:
            M_BINDING.inc(app=self.app_id, binding=name, direction="output", ok="False")
            return err(e.status if e.status < 500 else 500, "ERR_INVOKE_OUTPUT_BINDING", str(e))
        except Exception as e:
            M_BINDING.inc(app=self.app_id, binding=name, direction="output", ok="False")
            return err(500, "ERR_INVOKE_OUTPUT_BINDING", f"error invoking output binding {name}: {e}")
        M_BINDING.inc(app=self.app_id, binding=name, direction="output", ok="True")
        hdrs = [(f"metadata.{k}", v) for k, v in (out_meta or {}).items()]
        if out is None:
            return Response(b"", 204, hdrs)
        return Response(out, 200, hdrs, "application/json")

    # ---------------------------------------------------------------- secrets
    async def h_secret(self, req: Request) -> Response:
        s = self.secret_stores.get(req.path_params["store"])
        if s is None or req.path_params["store"] == APP_SECRETS_STORE:
            return err(401, "ERR_SECRET_STORE_NOT_FOUND", f"secret store {req.path_params['store']} not found")
        try:
            v = await s.get(req.path_params["key"], _metadata_from_query(req.query_string))
        except Exception as e:
            return err(500, "ERR_SECRET_GET", str(e))
        if v is None:
            return err(500, "ERR_SECRET_GET", f"secret {req.path_params['key']} not found")
        return json_response(v)

    async def h_secret_bulk(self, req: Request) -> Response:
        s = self.secret_stores.get(req.path_params["store"])
        if s is None or req.path_params["store"] == APP_SECRETS_STORE:
            return err(401, "ERR_SECRET_STORE_NOT_FOUND", f"secret store {req.path_params['store']} not found")
        return json_response(await s.bulk())

    # ---------------------------------------------------------------- runtime
    async def h_metadata(self, req: Request) -> Response:
        consumers = {c.name: c.stats for c in self.consumers}
        if self._dp_proc is not None:
            try:
                r = await self.http.request("GET", self._dp_control + "/stats", timeout=2.0)
                consumers.update(r.json().get("consumers", {}))
            except Exception as e:  # metadata stays available even if the data plane is wedged
                log.warning("native data plane stats unavailable: %r", e)
        comps = [self.components[n].describe() for n in sorted(self.components) if n not in self.failed_components]
        subs = [{"pubsubname": s.pubsubname, "topic": s.topic, "rules": [{"path": "/" + s.route}],
                 "deadLetterTopic": s.dead_letter_topic or "", "type": "DECLARATIVE" if s.declarative else "PROGRAMMATIC"}
                for s in self.subscriptions]
        return json_response({
            "id": self.app_id, "runtimeVersion": RUNTIME_VERSION, "components": comps, "subscriptions": subs,
            "inputBindings": self.input_bindings, "failedComponents": self.failed_components,
            "extended": {**self.extended_metadata, "instance": self.instance, "appReady": self.app_ready.is_set(),
                         "dataPlane": self.active_data_plane,
                         "consumers": consumers},
            "appConnectionProperties": {"port": self.app_port, "uds": self.app_uds, "protocol": "http"},
            "grpcPort": self.bound_grpc_port,
        })

    async def h_metadata_set(self, req: Request) -> Response:
        """``PUT /v1.0/metadata/{key}``: app-defined attributes shown under ``extended``."""
        self.extended_metadata[req.path_params["key"]] = req.body.decode("utf-8", "replace")
        return empty(204)

    async def h_healthz(self, req: Request) -> Response:
        """Dapr's health API: ``/v1.0/healthz`` is 204 once the sidecar is initialized AND its app
        channel is up (daprd waits for the app port first); ``/v1.0/healthz/outbound`` only needs
        the sidecar's own side (components loaded), for apps that call it during their startup."""
        if not self.ready.is_set():
            return empty(500)
        has_app = self.app_port is not None or bool(self.app_uds)
        if req.path.rstrip("/").endswith("/outbound") or not has_app or self.app_ready.is_set():
            return empty(204)
        return empty(500)

    async def h_shutdown(self, req: Request) -> Response:
        asyncio.get_running_loop().call_later(0.05, lambda: asyncio.ensure_future(self.stop()))
        return empty(204)

    async def h_metrics(self, req: Request) -> Response:
        return Response(REGISTRY.expose().encode(), 200, None, "text/plain; version=0.0.4")


def _span_file_reader(path: str):
    pos = 0

    def read() -> list[dict[str, Any]]:
        nonlocal pos
        try:
            with open(path, "rb") as f:
                f.seek(pos)
                data = f.read()
        except FileNotFoundError:
            return []
        end = data.rfind(b"\n") + 1
        pos += end
        return [json.loads(line) for line in data[:end].splitlines() if line.strip()]
    return read


def _metadata_from_query(qs: str) -> dict[str, str]:
    out = {}
    for k, v in parse_qsl(qs, keep_blank_values=True):
        if k.startswith("metadata."):
            out[k[9:]] = v
    return out


def make_cloudevent(body: bytes, ctype: str, pubsub: str, topic: str, source: str, traceparent: str | None,
                    event_id: str | None = None) -> dict[str, Any]:
    """CloudEvents 1.0 envelope as the sidecar writes it (reference
    docs/aca/05-aca-dapr-pubsubapi/index.md:60-69 shows the ``data`` payload)."""
    base = ctype.split(";")[0].strip().lower()
    ce: dict[str, Any] = {"specversion": "1.0", "id": event_id or str(uuid.uuid4()), "source": source,
                          "type": "com.dapr.event.sent", "datacontenttype": base or "application/json",
                          "topic": topic, "pubsubname": pubsub, "time": format_datetime(utcnow())}
    if "json" in base:
        try:
            ce["data"] = json.loads(body) if body else None
        except ValueError:
            ce["data"] = body.decode("utf-8", "replace")
    elif base.startswith("text/") or not body:
        ce["data"] = body.decode("utf-8", "replace")
    else:
        import base64
        ce["data_base64"] = base64.b64encode(body).decode()
    if traceparent:
        ce["traceparent"] = traceparent
        ce["traceid"] = traceparent
    return ce
