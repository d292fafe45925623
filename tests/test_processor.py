"""Processor notifier variants (docs-only controllers of the reference): SendGrid output
binding behind the feature flag, simulated work when disabled, direct SendGrid API."""
import asyncio
import time

from aca_dotnet_workshop_amd.platform.inproc import InProcessEnvironment, tasks_tracker_specs

from helpers import run

API = "tasksmanager-backend-api"
PROC = "tasksmanager-backend-processor"


async def _run_with(processor_cfg, n=2):
    env = InProcessEnvironment()
    url = await env.start_backing()
    if callable(processor_cfg):
        processor_cfg = processor_cfg(url)
    for s in tasks_tracker_specs(processor=processor_cfg, frontend=False):
        await env.add_app(s)
    await env.wait_ready()
    c = env.replicas[API][0].client
    t0 = time.perf_counter()
    for i in range(n):
        await c.invoke_method("POST", API, "api/tasks", {"taskName": f"n{i}", "taskCreatedBy": "c@x",
                                                         "taskDueDate": "2030-03-04T00:00:00", "taskAssignedTo": "dev@x"})
    sc = env.sidecar(PROC)
    for _ in range(500):
        if sum(x.stats["succeeded"] for x in sc.consumers) >= n:
            break
        await asyncio.sleep(0.01)
    return env, time.perf_counter() - t0


def test_sendgrid_binding_enabled():
    async def main():
        env, _ = await _run_with({"TasksNotifier": {"Mode": "sendgrid-binding"}, "SendGrid": {"IntegrationEnabled": True}})
        try:
            out = env.backing.outbox
            assert len(out) == 2
            msg = out[0]["message"]
            assert msg["personalizations"][0]["subject"] == "Task 'n0' is assigned to you!"
            assert msg["personalizations"][0]["to"][0]["email"] == "dev@x"
            assert "completed by the end of: 04/03/2030" in msg["content"][0]["value"]
            assert msg["from"]["email"] == "notifications@taskstracker.local"
        finally:
            await env.stop()
    run(main())


def test_sendgrid_disabled_simulates_work():
    async def main():
        env, dt = await _run_with({"TasksNotifier": {"Mode": "sendgrid-binding"},
                                   "SendGrid": {"IntegrationEnabled": False, "SimulatedDelayMs": 300}}, n=1)
        try:
            assert env.backing.outbox == [] and dt >= 0.3
        finally:
            await env.stop()
    run(main())


def test_sendgrid_api_mode():
    async def main():
        env, _ = await _run_with(lambda url: {"TasksNotifier": {"Mode": "sendgrid-api"},
                                              "SendGrid": {"Endpoint": url, "ApiKey": "SG.k"}}, n=1)
        try:
            msg = env.backing.outbox[0]["message"]
            assert [c["type"] for c in msg["content"]] == ["text/plain", "text/html"]
        finally:
            await env.stop()
    run(main())


def test_sendgrid_failure_is_retried():
    async def main():
        env2, _ = await _run_with({"TasksNotifier": {"Mode": "sendgrid-api"}, "SendGrid": {"Endpoint": "http://127.0.0.1:9"}},
                                  n=1)
        try:
            # SendGrid unreachable -> 400 -> broker redelivers (delivery count grows, nothing completed)
            await asyncio.sleep(0.5)
            b = env2.backing.broker("taskstracker")
            c = b.counts(f"tasksavedtopic/subscriptions/{PROC}")
            assert c["completed"] == 0 and c["received"] >= 2
        finally:
            await env2.stop()
    run(main())
