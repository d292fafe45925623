"""Test helpers: run a WebApp in-process on an ephemeral port."""
import asyncio
import contextlib

from aca_dotnet_workshop_amd.web import HttpClient, HttpServer


@contextlib.asynccontextmanager
async def served(app, uds=None):
    srv = HttpServer(app, asyncio.get_running_loop())
    await app.startup()
    port = await srv.listen_tcp("127.0.0.1", 0)
    if uds:
        await srv.listen_unix(uds)
    client = HttpClient()
    try:
        yield f"http://127.0.0.1:{port}", client
    finally:
        await client.close()
        await srv.close()
        await app.shutdown()


def run(coro):
    return asyncio.run(coro)
