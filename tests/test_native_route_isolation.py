"""A slow state save (a sidecar sleeping through the store's 429 retries) holds up only its own
create on the API's native route (apphost.hpp ``api_create``): the save goes over an
ordinary connection, not a pipelined one, so the creates behind it -- their saves and their
publishes -- are answered on time."""
import asyncio
import json

from aca_dotnet_workshop_amd.utils.config import Configuration
from aca_dotnet_workshop_amd.web import WebApp
from aca_dotnet_workshop_amd.web.client import HttpClient
from aca_dotnet_workshop_amd.web.http import Response
from aca_dotnet_workshop_amd.web.server import HttpServer

from helpers import run
from test_native_routes import UNSAMPLED, _serve


def test_a_throttled_save_does_not_delay_the_creates_behind_it(tmp_path, monkeypatch):
    monkeypatch.setenv("TT_APP_HOST", "native")
    monkeypatch.setenv("TT_NATIVE_ROUTES", "1")
    monkeypatch.setenv("TT_TRACE_SAMPLE_RATE", "0")
    side_sock, app_sock = str(tmp_path / "side.sock"), str(tmp_path / "app.sock")
    slow_s = 1.5

    async def main():
        loop = asyncio.get_running_loop()
        t0 = loop.time()
        seen = {"saves": 0}
        publishes, saves_done = [], []
        side = WebApp("slow-sidecar")

        async def any_route(req):
            if req.target.startswith("/v1.0/state/"):
                seen["saves"] += 1
                if seen["saves"] == 1:  # the first save sleeps through "429 retries"
                    await asyncio.sleep(slow_s)
                saves_done.append(loop.time() - t0)
            elif req.target.startswith("/v1.0/publish/"):
                publishes.append(loop.time() - t0)
            return Response(b"", 204)
        side.add_route("/{*path}", any_route, ("GET", "POST", "PUT", "DELETE"))
        srv = HttpServer(side, loop)
        await srv.listen_unix(side_sock)
        from aca_dotnet_workshop_amd.sdk.client import SidecarClient
        from aca_dotnet_workshop_amd.services.backend_api import create_app
        from aca_dotnet_workshop_amd.services.backend_api.managers import TasksStoreManager
        from aca_dotnet_workshop_amd.telemetry import tracing
        tracing.configure("native-isolation-test", None, 0.0)
        client = SidecarClient(f"unix:{side_sock}:")
        cfg = Configuration([{"APP_PORT": "0", "Environment": "Production", "TT_APP_UDS": app_sock}])
        app = create_app(config=cfg, manager=TasksStoreManager(client))
        stop, ports = asyncio.Event(), []
        task = asyncio.create_task(_serve(app, app_sock, stop, ports))
        for _ in range(200):
            if ports:
                break
            await asyncio.sleep(0.01)
        c = HttpClient()
        body = json.dumps({"taskName": "t", "taskCreatedBy": "a@b.c", "taskDueDate": "2030-01-01T00:00:00",
                           "taskAssignedTo": "x@y.z"}).encode()

        async def create(i):
            if i:
                await asyncio.sleep(0.05)  # after the slow one has its save in flight
            t = loop.time()
            r = await c.post(f"unix:{app_sock}:/api/tasks", body=body,
                             headers={"Content-Type": "application/json", "traceparent": UNSAMPLED})
            return r.status, loop.time() - t
        try:
            got = await asyncio.gather(*(create(i) for i in range(24)))
        finally:
            await c.close()
            stop.set()
            await task
            await srv.close(1)
        return got, publishes, saves_done
    got, publishes, saves_done = run(main())
    assert all(st == 201 for st, _ in got), got
    assert got[0][1] >= slow_s  # the throttled one waits for its save
    others = [dt for _, dt in got[1:]]
    assert max(others) < slow_s / 2, others  # nobody queued behind it
    assert len(publishes) == 24 and sorted(publishes)[22] < slow_s, publishes  # 23 published before it returned
