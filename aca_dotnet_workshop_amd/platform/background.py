"""An environment controller on a background thread: ``up`` from a manifest, then hand back the
running topology to synchronous code (the benchmark, tests) while the controller keeps
reconciling -- supervision, scale loops, ingress, limits -- on its own event loop.

    with BackgroundEnvironment(load_manifest("deploy/main.yaml", params, overrides), env_dir) as env:
        env.replicas("tasksmanager-frontend-webapp")   # [ReplicaProc] with app ports, sidecar sockets
        env.backing_url
"""
from __future__ import annotations

import asyncio
import threading
from typing import Any

from .controller import EnvironmentController
from .manifest import Manifest
from .processes import ReplicaProc


class BackgroundEnvironment:
    def __init__(self, manifest: Manifest, env_dir: str, timeout: float = 300.0, **controller_kw: Any) -> None:
        self.manifest = manifest
        self.env_dir = env_dir
        self.timeout = timeout
        self.kw = controller_kw
        self.ctl: EnvironmentController | None = None
        self._loop: asyncio.AbstractEventLoop | None = None
        self._ready = threading.Event()
        self._error: BaseException | None = None
        self._thread = threading.Thread(target=self._main, name="environment-controller", daemon=True)

    # -- lifecycle --------------------------------------------------------------------------
    def start(self) -> "BackgroundEnvironment":
        self._thread.start()
        if not self._ready.wait(self.timeout):
            raise TimeoutError(f"environment not up within {self.timeout}s")
        if self._error is not None:
            self._thread.join(30)
            raise RuntimeError(f"environment failed to start: {self._error!r}") from self._error
        return self

    def stop(self) -> None:
        if self._loop is not None and self.ctl is not None and self._thread.is_alive():
            self._loop.call_soon_threadsafe(self.ctl.stop_event.set)
        self._thread.join(120)

    def __enter__(self) -> "BackgroundEnvironment":
        return self.start()

    def __exit__(self, *exc) -> None:
        self.stop()

    def _main(self) -> None:
        loop = self._loop = asyncio.new_event_loop()
        asyncio.set_event_loop(loop)
        try:
            loop.run_until_complete(self._run())
        finally:
            loop.close()

    async def _run(self) -> None:
        try:
            self.ctl = EnvironmentController(self.manifest, self.env_dir, **self.kw)
            await self.ctl.up(serve_control=False)
        except BaseException as e:  # reported to start()
            self._error = e
            self._ready.set()
            if self.ctl is not None:
                try:
                    await self.ctl.down()
                except Exception:
                    pass
            return
        self._ready.set()
        await self.ctl.run_forever()

    # -- topology -----------------------------------------------------------------------------
    def call(self, fn, *args, timeout: float = 120.0):
        """Run ``fn(*args)`` (a coroutine function) on the controller's loop and wait for it."""
        return asyncio.run_coroutine_threadsafe(fn(*args), self._loop).result(timeout)

    def replicas(self, app: str) -> list[ReplicaProc]:
        rt = self.ctl.apps[app]
        return [r for r in (rt.current.replicas if rt.current else []) if r.alive()]

    @property
    def backing_url(self) -> str:
        return self.ctl.stack.backing_url

    @property
    def stack(self):
        return self.ctl.stack

    def status(self) -> dict[str, Any]:
        return self.call(self._status)

    async def _status(self) -> dict[str, Any]:
        return self.ctl.status()
