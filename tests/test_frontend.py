"""Frontend variants: module-2 direct HTTP mode (named HttpClient on BaseUrlExternalHttp) and
the production error page."""
import pytest

from aca_dotnet_workshop_amd.services.backend_api import FakeTasksManager
from aca_dotnet_workshop_amd.services.backend_api import create_app as api_app
from aca_dotnet_workshop_amd.services.frontend import create_app as fe_app
from aca_dotnet_workshop_amd.utils.config import Configuration

from helpers import run, served


def test_http_mode_requires_base_url():
    with pytest.raises(RuntimeError, match="BaseUrlExternalHttp"):
        fe_app(config=Configuration([{"Frontend": {"BackendMode": "http"}}]))


def test_http_mode_lists_seeded_tasks():
    async def main():
        async with served(api_app(config=Configuration([{}]), manager=FakeTasksManager())) as (api, _):
            cfg = Configuration([{"Frontend": {"BackendMode": "http"}, "BackendApiConfig": {"BaseUrlExternalHttp": api}}])
            async with served(fe_app(config=cfg)) as (web, c):
                r = await c.get(web + "/Tasks/Index", headers={"Cookie": "TasksCreatedByCookie=tjoudeh@bitoftech.net"})
                assert r.status == 200 and r.text.count("Task number:") == 10
    run(main())


def test_error_page_outside_development():
    async def main():
        cfg = Configuration([{"Environment": "Production", "Frontend": {"BackendMode": "http"},
                              "BackendApiConfig": {"BaseUrlExternalHttp": "http://127.0.0.1:9"}}])
        async with served(fe_app(config=cfg)) as (web, c):
            r = await c.get(web + "/Tasks/Index", headers={"Cookie": "TasksCreatedByCookie=a@b"})
            assert r.status == 500 and "An error occurred while processing your request." in r.text
    run(main())
