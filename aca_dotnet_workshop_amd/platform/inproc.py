"""In-process environment: backing services + every app + its sidecar in ONE event loop.

The multi-process platform (``platform.environment``) is the production shape; this
runner reproduces the same topology (app <-> sidecar over Unix sockets, sidecar <->
sidecar through the name registry, sidecars -> backing services over HTTP) inside one
process, which makes end-to-end tests deterministic and fast.  It is also what
``__graft_entry__.smoke()`` drives.
"""
from __future__ import annotations

import asyncio
import os
import tempfile
from dataclasses import dataclass, field
from pathlib import Path
from typing import Any, Callable

from ..backing.auth import AccessPolicy
from ..backing.server import BackingServices
from ..sdk.client import SidecarClient
from ..sidecar.components import Component
from ..sidecar.runtime import Sidecar
from ..utils.config import Configuration
from ..web.app import WebApp
from ..web.client import HttpClient
from ..web.server import HttpServer

REPO_ROOT = Path(__file__).resolve().parents[2]
DEFAULT_COMPONENTS = REPO_ROOT / "deploy" / "components"


@dataclass
class AppSpec:
    app_id: str
    factory: Callable[..., WebApp]          # create_app(config=..., client=...) style factory
    config: dict[str, Any] = field(default_factory=dict)
    replicas: int = 1
    client_kw: str = "client"                # factory kwarg receiving the SidecarClient (None = pass via manager)
    env: dict[str, str] = field(default_factory=dict)


@dataclass
class Replica:
    app_id: str
    index: int
    app: WebApp
    server: HttpServer
    sidecar: Sidecar
    port: int
    client: SidecarClient


class InProcessEnvironment:
    def __init__(self, root: str | os.PathLike | None = None, components_paths: list[str] | None = None,
                 extra_components: list[Component] | None = None, policy: dict[str, Any] | None = None,
                 persist: bool = False) -> None:
        self._tmp = None
        if root is None:
            self._tmp = tempfile.TemporaryDirectory(prefix="tt-env-")
            root = self._tmp.name
        self.root = Path(root)
        self.sock_dir = Path(tempfile.mkdtemp(prefix="tts-"))  # short path: AF_UNIX limit is 108 bytes
        self.components_paths = components_paths if components_paths is not None else [str(DEFAULT_COMPONENTS)]
        self.extra_components = extra_components or []
        self.policy = policy
        self.persist = persist
        self.backing: BackingServices | None = None
        self.backing_server: HttpServer | None = None
        self.backing_url = ""
        self.replicas: dict[str, list[Replica]] = {}
        self.http = HttpClient()

    async def start_backing(self) -> str:
        data = str(self.root / "backing") if self.persist else None
        self.backing = BackingServices(data, AccessPolicy.from_dict(self.policy))
        self.backing_server = HttpServer(self.backing.build_app(), asyncio.get_running_loop())
        port = await self.backing_server.listen_tcp("127.0.0.1", 0)
        self.backing_url = f"http://127.0.0.1:{port}"
        return self.backing_url

    async def add_app(self, spec: AppSpec) -> list[Replica]:
        out = []
        for i in range(spec.replicas):
            out.append(await self._start_replica(spec, len(self.replicas.get(spec.app_id, [])) + i))
        self.replicas.setdefault(spec.app_id, []).extend(out)
        return out

    async def _start_replica(self, spec: AppSpec, idx: int) -> Replica:
        tag = f"{spec.app_id}-{idx}"
        sc_uds = str(self.sock_dir / f"{tag}.d.sock")
        app_uds = str(self.sock_dir / f"{tag}.a.sock")
        int_uds = str(self.sock_dir / f"{tag}.i.sock")
        client = SidecarClient(base_url=f"unix:{sc_uds}:")
        cfg = Configuration([{"Environment": "Development", "TT_SIDECAR_UDS": sc_uds}, spec.config])
        kwargs: dict[str, Any] = {"config": cfg}
        if spec.client_kw:
            kwargs[spec.client_kw] = client
        app = spec.factory(**kwargs)
        srv = HttpServer(app, asyncio.get_running_loop())
        await app.startup()
        port = await srv.listen_tcp("127.0.0.1", 0)
        await srv.listen_unix(app_uds)
        env = dict(os.environ)
        env.update(spec.env)
        sc = Sidecar(spec.app_id, app_uds=app_uds, http_port=None, uds=sc_uds, internal_port=None,
                     internal_uds=int_uds, resources_paths=self.components_paths,
                     components=[_clone(c) for c in self.extra_components], registry_dir=str(self.root / "registry"),
                     identity=spec.env.get("TT_IDENTITY", spec.app_id), backing_url=self.backing_url, environ=env,
                     instance=f"{spec.app_id}-{idx}")
        await sc.start()
        return Replica(spec.app_id, idx, app, srv, sc, port, client)

    async def wait_ready(self, timeout: float = 20.0) -> None:
        async def one(r: Replica) -> None:
            await asyncio.wait_for(r.sidecar.app_ready.wait(), timeout)
        await asyncio.gather(*(one(r) for rs in self.replicas.values() for r in rs))

    def url(self, app_id: str, index: int = 0) -> str:
        return f"http://127.0.0.1:{self.replicas[app_id][index].port}"

    def sidecar(self, app_id: str, index: int = 0) -> Sidecar:
        return self.replicas[app_id][index].sidecar

    async def remove_replica(self, app_id: str, index: int = -1) -> None:
        r = self.replicas[app_id].pop(index)
        await r.sidecar.stop(grace=1.0)
        await r.server.close(grace=1.0)
        await r.app.shutdown()

    async def stop(self) -> None:
        for rs in self.replicas.values():
            for r in rs:
                await r.sidecar.stop(grace=1.0)
                await r.server.close(grace=1.0)
                await r.app.shutdown()
        self.replicas.clear()
        if self.backing_server is not None:
            await self.backing_server.close(grace=1.0)
        await self.http.close()
        import shutil
        shutil.rmtree(self.sock_dir, ignore_errors=True)
        if self._tmp is not None:
            self._tmp.cleanup()

    async def __aenter__(self) -> "InProcessEnvironment":
        await self.start_backing()
        return self

    async def __aexit__(self, *exc) -> None:
        await self.stop()


def _clone(c: Component) -> Component:
    import copy
    return copy.deepcopy(c)


def tasks_tracker_specs(api_backend: str = "store", processor: dict[str, Any] | None = None,
                        frontend: bool = True, processor_replicas: int = 1,
                        api: dict[str, Any] | None = None) -> list[AppSpec]:
    """The reference topology: Backend API + Processor (+ Frontend)."""
    from ..services.backend_api.app import create_app as api_factory
    from ..services.backend_api.managers import FakeTasksManager, TasksStoreManager
    from ..services.processor.app import create_app as proc_factory

    def api_app(config, client):
        mgr = TasksStoreManager.from_config(client, config) if api_backend == "store" else FakeTasksManager()
        return api_factory(config=config, manager=mgr)

    specs = [AppSpec("tasksmanager-backend-api", api_app, dict(api or {})),
             AppSpec("tasksmanager-backend-processor", proc_factory, dict(processor or {}), processor_replicas)]
    if frontend:
        from ..services.frontend.app import create_app as fe_factory
        specs.append(AppSpec("tasksmanager-frontend-webapp", fe_factory))
    return specs
