"""Failure handling across processes (SURVEY.md §7.4 fault tests): a competing-consumer replica
is killed (SIGKILL of its sidecar, data plane and app) while it holds locked messages; the
surviving replica finishes the subscription once the dead consumer's peek-locks expire --
no message is lost, none is dead-lettered (at-least-once delivery)."""
import asyncio
import os
import shutil
import signal
from pathlib import Path

from aca_dotnet_workshop_amd.backing.client import BackingClient
from aca_dotnet_workshop_amd.platform.processes import LocalStack

from helpers import run

ROOT = Path(__file__).resolve().parents[1]
ENTITY = "tasksavedtopic/subscriptions/tasksmanager-backend-processor"
CE = ('{"specversion":"1.0","id":"%d","source":"t","type":"t","datacontenttype":"application/json",'
      '"data":{"taskName":"t%d","taskAssignedTo":"a@x","taskDueDate":"2030-01-01T00:00:00"}}')


def _components(tmp: Path) -> str:
    d = tmp / "components"
    shutil.copytree(ROOT / "deploy" / "components", d)
    f = d / "dapr-pubsub-svcbus.yaml"
    text = f.read_text().replace("  metadata:\n  - name: connectionString",
                                 "  metadata:\n  - name: lockDurationInSec\n    value: \"2\"\n  - name: connectionString")
    f.write_text(text)
    return str(d)


def test_killed_consumer_messages_are_redelivered(tmp_path):
    n = 400
    stack = LocalStack(root=tmp_path / "stack", components=[_components(tmp_path)])
    try:
        backing = stack.start_backing()
        cfg = {"Logging:LogLevel:Default": "Warning", "TasksNotifier:Mode": "log", "SendGrid:SimulatedDelayMs": "20"}
        victim = stack.start_replica("tasksmanager-backend-processor", cfg)
        stack.start_replica("tasksmanager-backend-processor", cfg)
        stack.wait_ready()

        async def main():
            b = BackingClient(backing, identity="tasksmanager-backend-api")
            await b.sb_publish_batch("taskstracker", "tasksavedtopic",
                                     [{"body": CE % (i, i), "contentType": "application/cloudevents+json"}
                                      for i in range(n)])
            for _ in range(400):
                c = await b.sb_counts("taskstracker", ENTITY)
                if c["completed"] >= n // 4 and c["locked"] > 0:
                    break
                await asyncio.sleep(0.02)
            os.killpg(victim.proc.pid, signal.SIGKILL)  # sidecar, data plane and app of one replica
            for _ in range(600):
                c = await b.sb_counts("taskstracker", ENTITY)
                if c["completed"] >= n:
                    break
                await asyncio.sleep(0.05)
            await b.http.close()
            return c

        c = run(main())
        assert c["completed"] == n and c["dead_letter"] == 0 and c["active"] == 0, c
        assert c["received"] >= n  # redeliveries of the dead replica's locked messages included
        assert victim.proc.wait(timeout=10) == -signal.SIGKILL
    finally:
        stack.stop()


def test_backing_services_crash_and_restart_in_place(tmp_path):
    """The backing-services process (Cosmos / Service Bus equivalents) is SIGKILLed mid-run and
    restarted on the same port over its data directory: saved tasks and undelivered messages come
    back from the engines' durable logs, the sidecars' native data planes reconnect, and the
    createTask flow works again end to end."""
    from aca_dotnet_workshop_amd.web.client import HttpClient
    stack = LocalStack(root=tmp_path / "stack")
    try:
        backing = stack.start_backing(str(tmp_path / "data"))
        cfg = {"Logging:LogLevel:Default": "Warning", "TasksNotifier:Mode": "log"}
        api = stack.start_replica("tasksmanager-backend-api", cfg)
        stack.wait_ready()
        url = f"unix:{api.sidecar_uds}:/v1.0/invoke/tasksmanager-backend-api/method/api/tasks"
        body = b'{"taskName":"%s","taskCreatedBy":"dur@x","taskDueDate":"2030-01-01T00:00:00","taskAssignedTo":"a@x"}'

        def crash_and_restart():
            os.kill(stack.backing_proc.pid, signal.SIGKILL)
            stack.backing_proc.wait(timeout=10)
            return stack.restart_backing()

        async def main():
            c = HttpClient()
            b = BackingClient(backing, identity="tasksmanager-backend-api")

            async def create(name):
                r = await c.post(url, body=body % name.encode(), headers={"Content-Type": "application/json"})
                return r.status
            # the processor's subscription, provisioned as the platform does (no processor runs:
            # the events wait in it)
            await b.sb_create_topic("taskstracker", "tasksavedtopic")
            await b.sb_create_subscription("taskstracker", "tasksavedtopic", "tasksmanager-backend-processor", 60000, 10)
            assert [await create(f"t{i}") for i in range(20)] == [201] * 20
            assert (await b.sb_counts("taskstracker", ENTITY))["active"] == 20
            assert await asyncio.to_thread(crash_and_restart) == backing
            for _ in range(100):  # the data plane's pooled connections to the dead process fail once
                if await create("after") == 201:
                    break
                await asyncio.sleep(0.05)
            else:
                raise AssertionError("createTask did not recover after the backing restart")
            r = await c.get(url + "?createdBy=dur@x")
            names = sorted(t["taskName"] for t in r.json())
            counts = await b.sb_counts("taskstracker", ENTITY)
            await c.close()
            await b.http.close()
            return names, counts
        names, counts = run(main())
        assert names == sorted([f"t{i}" for i in range(20)] + ["after"])
        assert counts["active"] == 21
    finally:
        stack.stop()
