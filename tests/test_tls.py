"""TLS everywhere the reference has it:

* HTTPS app endpoints + ``UseHttpsRedirection`` (reference Backend.Api/Program.cs:26,
  launchSettings https profiles), on both I/O hosts (asyncio / native epoll + OpenSSL);
* ``dapr run --app-ssl`` (snippets/dapr-run-backend-api.md:12,24): the sidecar reaches the app
  over HTTPS on both data planes;
* sidecar-to-sidecar mutual TLS lives in test_dataplane.py::test_sidecar_mutual_tls, the HTTPS
  external ingress in test_platform.py."""
import asyncio
import ssl

import pytest

from aca_dotnet_workshop_amd.platform.pki import EnvironmentPki
from aca_dotnet_workshop_amd.services.backend_api.app import create_app
from aca_dotnet_workshop_amd.services.backend_api.managers import FakeTasksManager
from aca_dotnet_workshop_amd.services.hosting import serve_host
from aca_dotnet_workshop_amd.utils.config import Configuration
from aca_dotnet_workshop_amd.web import HttpClient

from helpers import run

HOSTS = ["python", "native"]


async def _serve(monkeypatch, host, tmp_path, urls):
    monkeypatch.setenv("TT_APP_HOST", host)
    cfg = Configuration([{"Environment": "Development", "urls": urls, "TT_DEV_CERTS_DIR": str(tmp_path / "dev")}])
    app = create_app(config=cfg, manager=FakeTasksManager())
    stop = asyncio.Event()
    got = asyncio.get_running_loop().create_future()
    task = asyncio.ensure_future(serve_host(app, stop, got.set_result))
    ports = await asyncio.wait_for(got, 20)
    return stop, task, ports


@pytest.mark.parametrize("host", HOSTS)
def test_https_endpoint_and_https_redirection(host, monkeypatch, tmp_path):
    async def main():
        stop, task, (https_port, http_port) = await _serve(monkeypatch, host, tmp_path,
                                                            "https://127.0.0.1:0;http://127.0.0.1:0")
        ca = EnvironmentPki(tmp_path / "dev", trust_domain="localhost-dev").ca_crt
        ctx = ssl.create_default_context(cafile=str(ca))
        c = HttpClient(tls=ctx)
        try:
            r = await c.get(f"https://127.0.0.1:{https_port}/api/tasks?createdBy=tjoudeh@bitoftech.net")
            assert r.status == 200 and len(r.json()) == 10  # module 1, over TLS (certificate verified)
            r = await c.get(f"http://127.0.0.1:{http_port}/api/tasks?createdBy=x")
            assert r.status == 307
            assert r.headers["location"] == f"https://127.0.0.1:{https_port}/api/tasks?createdBy=x"
            # an untrusting client refuses the dev certificate
            with pytest.raises(ssl.SSLError):
                await HttpClient(tls=ssl.create_default_context()).get(f"https://127.0.0.1:{https_port}/healthz")
        finally:
            await c.close()
            stop.set()
            await task
    run(main())


@pytest.mark.parametrize("plane", ["python", "native"])
def test_sidecar_app_ssl(plane, monkeypatch, tmp_path):
    from aca_dotnet_workshop_amd.sidecar import Sidecar

    async def main():
        stop, task, (https_port,) = await _serve(monkeypatch, "python", tmp_path, "https://127.0.0.1:0")
        sc = Sidecar("tasksmanager-backend-api", app_port=https_port, app_ssl=True, http_port=0,
                     registry_dir=str(tmp_path / "reg"), components=[], data_plane=plane,
                     internal_uds=str(tmp_path / "i.sock"))
        await sc.start()
        c = HttpClient()
        try:
            await asyncio.wait_for(sc.app_ready.wait(), 10)
            assert sc.active_data_plane == plane
            r = await c.get(f"http://127.0.0.1:{sc.bound_http_port}/v1.0/invoke/tasksmanager-backend-api/method/"
                            "api/tasks?createdBy=tjoudeh@bitoftech.net")
            assert r.status == 200 and len(r.json()) == 10
        finally:
            await c.close()
            await sc.stop(1.0)
            stop.set()
            await task
    run(main())
