"""Platform layer: manifest (Bicep equivalent), KEDA/HPA scaler semantics, and a
multi-process environment deployed by the controller (ACA equivalent) -- module 2
(internal ingress 403), module 9 (KEDA 1 -> 5 -> 1 replicas), module 10 (what-if/apply).
"""
import asyncio
import collections
import json
import os
import re
import signal
import time
import urllib.error
import urllib.parse
import urllib.request
from pathlib import Path

import pytest

from aca_dotnet_workshop_amd.platform.manifest import (ManifestError, identity_of, load_manifest, substitute, unique_string,
                                                       validate, what_if)
from aca_dotnet_workshop_amd.platform.scaler import Autoscaler, ScaleRule, cron_metric

from helpers import run

ROOT = Path(__file__).resolve().parents[1]
MAIN = ROOT / "deploy" / "main.yaml"
PARAMS = ROOT / "deploy" / "main.parameters.json"


def test_manifest_parameters_and_functions():
    m = load_manifest(MAIN, PARAMS, {"sendGridKeySecretValue": "SG.key", "prefix": "dev-"})
    assert m.name == "dev-cae-tasks-tracker"
    proc = m.app("tasksmanager-backend-processor")
    env = {e["name"]: e["value"] for e in proc["env"]}
    assert env["SendGrid__IntegrationEnabled"] is True  # notEmpty(sendGridKeySecretValue)
    assert proc["scale"]["maxReplicas"] == 5 and proc["scale"]["rules"][0]["custom"]["metadata"]["messageCount"] == 10
    kv = m.resources["keyVault"]["secrets"][0]
    assert kv["value"] == "SG.key"
    m2 = load_manifest(MAIN, PARAMS)
    assert m2.resources["keyVault"]["secrets"][0]["value"] == "dummy"  # coalesce(empty, 'dummy') like the bicep module
    assert {ra["role"] for ra in m2.role_assignments() if ra["principal"] == "tasksmanager-backend-api-mi"} == {
        "Cosmos DB Built-in Data Contributor", "Azure Service Bus Data Sender"}
    assert unique_string("rg") == unique_string("rg") and len(unique_string("rg")) == 13
    assert substitute("${concat('a', x)}-${toLower(y)}", {"x": "b", "y": "C"}) == "ab-c"
    with pytest.raises(ManifestError):
        substitute("${nope}", {})


def test_validate_and_what_if(tmp_path):
    m = load_manifest(MAIN, PARAMS)
    assert validate(m) == []
    changes = what_if(m, None)
    assert all(c["change"] == "Create" for c in changes)
    from aca_dotnet_workshop_amd.platform.manifest import desired_state
    cur = desired_state(m)
    assert {c["change"] for c in what_if(m, cur)} == {"NoChange"}
    m2 = load_manifest(MAIN, PARAMS, {"notifierSimulatedDelayMs": 5})
    mod = [c["resource"] for c in what_if(m2, cur) if c["change"] == "Modify"]
    assert mod == ["containerApps/tasksmanager-backend-processor"]
    bad = tmp_path / "bad.yaml"
    text = MAIN.read_text().replace("type: azure-servicebus", "type: kafka").replace(
        "aca-components/containerapps-scheduled-cron.yaml", "aca-components/missing.yaml")
    bad.write_text(text)
    (tmp_path / "aca-components").symlink_to(ROOT / "deploy" / "aca-components")
    errs = validate(load_manifest(bad, PARAMS))
    assert any("unsupported type 'kafka'" in e for e in errs)
    assert any("missing.yaml not found" in e for e in errs)


def test_keda_hpa_semantics():
    rule = ScaleRule("topic", "azure-servicebus", {"messageCount": "10"})
    a = Autoscaler(1, 5, [rule], cooldown=300)
    assert a.decide({"topic": 0}, 1, now=0) == 1
    assert a.decide({"topic": 35}, 1, now=30) == 4          # ceil(35/10)
    assert a.decide({"topic": 10_000}, 4, now=60) == 5      # clamp to maxReplicas
    assert a.decide({"topic": 0}, 5, now=90) == 5           # stabilization window holds replicas
    assert a.decide({"topic": 0}, 5, now=359) == 5
    assert a.decide({"topic": 0}, 5, now=361) == 1          # one cooldown after the last high recommendation
    z = Autoscaler(0, 3, [rule], cooldown=10)
    assert z.decide({"topic": 0}, 0, now=100) == 0          # scale-to-zero stays at zero
    assert z.decide({"topic": 1}, 0, now=101) == 1          # activation
    assert z.decide({"topic": 0}, 1, now=105) == 1
    assert z.decide({"topic": 0}, 1, now=120) == 0
    http = ScaleRule("http", "http", {"concurrentRequests": "10"})
    assert Autoscaler(1, 10, [http]).decide({"http": 55}, 1, now=0) == 6
    assert ScaleRule.from_manifest({"name": "h", "http": {"metadata": {"concurrentRequests": "3"}}}).target() == 3


def test_cron_scaler_window():
    from datetime import datetime, timezone
    r = ScaleRule("c", "cron", {"start": "0 8 * * *", "end": "0 18 * * *", "desiredReplicas": "4"})
    assert cron_metric(r, datetime(2024, 5, 1, 12, 0, tzinfo=timezone.utc)) == 4
    assert cron_metric(r, datetime(2024, 5, 1, 20, 0, tzinfo=timezone.utc)) == 0


# --------------------------------------------------------------------- integration
def _get(url, **kw):
    return urllib.request.urlopen(url, timeout=10, **kw)


@pytest.fixture(scope="module")
def lifecycle_acr(tmp_path_factory):
    """Chiseled images of the three services, pushed to a registry (module 12 -> module 10)."""
    from aca_dotnet_workshop_amd.platform import image
    from aca_dotnet_workshop_amd.platform.registry import LocalRegistry
    reg = LocalRegistry("lifecycleacr", tmp_path_factory.mktemp("acr"))
    out = tmp_path_factory.mktemp("images")
    for svc, name in image.SERVICES.items():
        reg.push(image.build_image(svc, "chiseled", out).path, f"tasksmanager/{name}", "r2")
    return reg


def test_image_pull_needs_acrpull(tmp_path, lifecycle_acr):
    """An app pulls its image only with AcrPull on the registry for its own identity; an unknown
    tag fails the pull (the revision's provisioning error in ACA)."""
    from aca_dotnet_workshop_amd.platform.controller import EnvironmentController, ImagePullError
    from aca_dotnet_workshop_amd.platform.registry import LocalRegistry
    m = load_manifest(MAIN, PARAMS, {"containerRegistryName": lifecycle_acr.name, "imageTag": "r2"})
    assert validate(m) == []
    ctl = EnvironmentController(m, tmp_path / "env", registry_root=lifecycle_acr.dir.parent)
    ctl.registry = LocalRegistry(lifecycle_acr.name, lifecycle_acr.dir.parent)
    api = m.app("tasksmanager-backend-api")
    c = ctl._pull(api)
    root = Path(c["rootfs"])
    assert (root / "app" / "aca_dotnet_workshop_amd" / "services" / "backend_api").is_dir()
    assert not (root / "bin" / "sh").exists() and c["config"]["User"] != "0:0"
    api["roleAssignments"] = [ra for ra in api["roleAssignments"] if ra["role"] != "AcrPull"]
    with pytest.raises(ImagePullError, match="no AcrPull"):
        ctl._pull(api)  # the earlier pull by digest does not bypass the check
    fe = m.app("tasksmanager-frontend-webapp")
    fe["image"] = fe["image"].replace(":r2", ":missing")
    with pytest.raises(ImagePullError, match="manifest unknown"):
        ctl._pull(fe)
    assert [e["kind"] for e in ctl.events] == ["ImagePulled", "ImagePullFailed", "ImagePullFailed"]
    m2 = load_manifest(MAIN, PARAMS, {"containerRegistryName": lifecycle_acr.name})
    m2.app("tasksmanager-backend-api")["registries"] = []
    assert any("needs a 'registries' entry" in e for e in validate(m2))


@pytest.mark.slow
@pytest.mark.parametrize("source", ["module", "image"])
def test_environment_lifecycle(tmp_path, source, request):
    """The whole environment, with the apps' code from the source tree (the dev loop) or pulled
    as chiseled images from the environment's registry with each identity's AcrPull role -- then
    the API also talks gRPC to its sidecar."""
    from aca_dotnet_workshop_amd.platform.controller import EnvironmentController
    over = {"notifierSimulatedDelayMs": 150}
    reg_root = None
    if source == "image":
        acr = request.getfixturevalue("lifecycle_acr")
        over.update({"containerRegistryName": acr.name, "imageTag": "r2", "backendApiDaprApiProtocol": "grpc"})
        reg_root = acr.dir.parent

    async def main():
        m = load_manifest(MAIN, PARAMS, over)
        ctl = EnvironmentController(m, tmp_path / "env", polling_interval=0.5, cooldown=3, registry_root=reg_root)
        await ctl.up()
        try:
            st = ctl.status()
            if source == "image":  # every replica runs its image's entrypoint in the image's root fs
                for name, app in st["apps"].items():
                    assert app["image"] == f"{acr.login_server}/tasksmanager/{name}:r2"
                    reps = app["revisions"][-1]["replicas"]
                    assert reps and all(r["image"].startswith("sha256:") for r in reps)
                    assert all(r["isolation"] == ("chroot" if os.geteuid() == 0 else "none") for r in reps)
                pulls = [e for e in ctl.events if e["kind"] == "ImagePulled"]
                assert sorted(e["identity"] for e in pulls) == sorted(identity_of(a) for a in m.apps)
            api = st["apps"]["tasksmanager-backend-api"]["ingress"]
            fe = st["apps"]["tasksmanager-frontend-webapp"]["ingress"]
            # module 2: internal ingress is 403 from outside the environment
            with pytest.raises(urllib.error.HTTPError) as ei:
                await asyncio.to_thread(_get, api["fqdn"] + "/api/tasks?createdBy=x")
            assert ei.value.code == 403
            # external ingress: HTTPS with the environment CA's certificate; plain HTTP -> 301
            import ssl
            assert fe["fqdn"].startswith("https://")
            tls = ssl.create_default_context(cafile=st["tls"]["caCert"])
            r = await asyncio.to_thread(_get, fe["fqdn"] + "/", context=tls)
            assert r.status == 200
            noredir = urllib.request.build_opener(_NoRedirect)
            r = await asyncio.to_thread(noredir.open, fe["httpUrl"] + "/Tasks/Index")
            assert r.status == 301 and r.headers["Location"] == fe["fqdn"] + "/Tasks/Index"
            with pytest.raises(urllib.error.URLError):  # not trusted without the environment CA
                await asyncio.to_thread(_get, fe["fqdn"] + "/")
            # the frontend -> API -> state store path works under RBAC (managed identities), the
            # sidecars talk mutual TLS (per-app-id workload certificates)
            data = b"TasksCreatedBy=env%40test"
            req = urllib.request.Request(fe["fqdn"] + "/", data=data, method="POST",
                                         headers={"Content-Type": "application/x-www-form-urlencoded"})
            opener = urllib.request.build_opener(_NoRedirect, urllib.request.HTTPSHandler(context=tls))
            resp = await asyncio.to_thread(opener.open, req)
            assert resp.status == 302
            # create + list through frontend -> (sidecar mTLS) -> API -> state store
            cookie = resp.headers["Set-Cookie"].split(";", 1)[0]
            req = urllib.request.Request(fe["fqdn"] + "/Tasks/Create", headers={"Cookie": cookie})
            r = await asyncio.to_thread(opener.open, req)
            af = re.search(r"\.AspNetCore\.Antiforgery=([0-9a-f]+)", r.headers["Set-Cookie"]).group(1)
            token = re.search(r'name="__RequestVerificationToken" value="([0-9a-f]+)"', r.read().decode()).group(1)
            cookie += f"; .AspNetCore.Antiforgery={af}"
            form = urllib.parse.urlencode({"__RequestVerificationToken": token, "TaskAdd.TaskName": "via mtls",
                                           "TaskAdd.TaskAssignedTo": "a@x", "TaskAdd.TaskDueDate": "2030-01-01"}).encode()
            req = urllib.request.Request(fe["fqdn"] + "/Tasks/Create", data=form, method="POST",
                                         headers={"Content-Type": "application/x-www-form-urlencoded",
                                                  "Cookie": cookie})
            assert (await asyncio.to_thread(opener.open, req)).status == 302
            req = urllib.request.Request(fe["fqdn"] + "/Tasks/Index", headers={"Cookie": cookie})
            page = (await asyncio.to_thread(opener.open, req)).read().decode()
            assert "via mtls" in page
            if source == "image":  # the API saved it through its sidecar's gRPC API
                from aca_dotnet_workshop_amd.web.client import HttpClient
                http = HttpClient(timeout=5.0)
                try:
                    api_rep = ctl.apps["tasksmanager-backend-api"].current.replicas[0]
                    text = (await http.get(f"unix:{api_rep.sidecar_uds}:/metrics")).text
                    assert 'op="grpc.SaveState"' in text and 'op="grpc.PublishEvent"' in text, text[-1500:]
                    app_metrics = await http.get(f"http://127.0.0.1:{api_rep.app_port}/metrics")
                    assert app_metrics.status == 200
                finally:
                    await http.close()
            regs = [json.loads(f.read_text()) for f in (tmp_path / "env" / "runtime" / "registry").glob("*/*.json")]
            assert regs and all(r["endpoint"].startswith(f"mtls:{r['appId']}@") for r in regs)
            b = ctl.backing
            entity = "tasksavedtopic/subscriptions/tasksmanager-backend-processor"
            for _ in range(100):  # the created task's tasksaved event is delivered first
                if (await b.sb_counts("taskstracker", entity))["completed"] == 1:
                    break
                await asyncio.sleep(0.1)
            # module 9: burst on the topic scales the processor out, then back in after the cooldown
            def ce(i):
                return json.dumps({"specversion": "1.0", "id": f"x{i}", "source": "t", "type": "t",
                                   "datacontenttype": "application/json",
                                   "data": {"taskName": f"burst-{i}", "taskAssignedTo": "a@x",
                                            "taskDueDate": "2030-01-01T00:00:00"}})
            await b.sb_publish_batch("taskstracker", "tasksavedtopic",
                                     [{"body": ce(i), "contentType": "application/cloudevents+json"} for i in range(800)])
            proc = ctl.apps["tasksmanager-backend-processor"]
            peak = 1
            for _ in range(100):
                await asyncio.sleep(0.1)
                peak = max(peak, len([r for r in proc.current.replicas if r.alive()]))
                c = await b.sb_counts("taskstracker", "tasksavedtopic/subscriptions/tasksmanager-backend-processor")
                if c["completed"] >= 801 and peak > 1:
                    break
            assert peak == 5
            assert c["completed"] == 801 and c["dead_letter"] == 0
            # competing consumers across the 5 replicas: every message handled, none twice
            # (the processor logs each delivery it starts; no lock expired, so no redelivery)
            seen = collections.Counter()
            for f in ctl.stack.log_dir.glob("tasksmanager-backend-processor*.log"):
                seen.update(re.findall(r"Task Name 'burst-(\d+)'", f.read_text(errors="replace")))
            assert len(seen) == 800 and set(seen.values()) == {1}, (len(seen), seen.most_common(3))
            # live metrics (App Insights Live Metrics): native deliveries counted per replica
            from aca_dotnet_workshop_amd.platform.__main__ import live_rates
            s0 = await ctl.live_metrics()
            procs = s0["apps"]["tasksmanager-backend-processor"]
            assert sum(r["sidecar"].get("sidecar_native_requests_total", 0) for r in procs.values()) >= 800
            assert all(r["cpuSeconds"] > 0 for r in procs.values())
            s1 = await ctl.live_metrics()
            rates = live_rates(s0, s1)
            assert rates["tasksmanager-backend-processor"]["replicas"] == len(s1["apps"]["tasksmanager-backend-processor"])
            for _ in range(300):  # the cooldown, then the scaler's next poll (slower on a loaded host)
                await asyncio.sleep(0.1)
                if len([r for r in proc.current.replicas if r.alive()]) == 1:
                    break
            assert len([r for r in proc.current.replicas if r.alive()]) == 1
            # restart policy: a crashed replica is replaced
            api_rt = ctl.apps["tasksmanager-backend-api"]
            victim = api_rt.current.replicas[0]
            os.killpg(victim.proc.pid, signal.SIGKILL)
            for _ in range(200):
                await asyncio.sleep(0.1)
                if api_rt.restarts >= 1 and all(r.alive() for r in api_rt.current.replicas):
                    break
            assert api_rt.restarts >= 1 and api_rt.current.replicas[0].name != victim.name
            # resource limits (0.25 vCPU / 0.5Gi per replica): a replica over its memory limit is
            # killed and restarted like an OOM-killed container
            lim = ctl.status()["resourceLimits"]
            assert lim["mode"] in ("cgroup2", "cgroup1-cpu", "watchdog") and len(lim["replicas"]) >= 3
            assert all(r["memoryBytes"] == 512 << 20 and r["cpu"] == 0.25 for r in lim["replicas"].values())
            oom = api_rt.current.replicas[0]
            ctl.limiter.replicas[oom.name].limits.memory = 1 << 20  # as if it had grown past 0.5Gi
            for _ in range(200):
                await asyncio.sleep(0.1)
                if api_rt.restarts >= 2 and all(r.alive() for r in api_rt.current.replicas):
                    break
            ev = [e for e in ctl.events if e["kind"] in ("ReplicaOOMKilled", "ReplicaCrashed") and e["replica"] == oom.name]
            assert [e["kind"] for e in ev] == ["ReplicaOOMKilled", "ReplicaCrashed"] and ev[1]["reason"] == "OOMKilled"
            assert api_rt.current.replicas[0].name != oom.name
            # Cosmos provisioned throughput from the manifest (autoscale max 4000 RU/s)
            ts = (await b.doc_stats("taskstracker-state-store", "tasksmanagerdb", "taskscollection"))["throughput"]
            assert ts["ru_per_s"] == 4000
            # Log Analytics retention (retentionInDays: 30): day files past the window are pruned
            from aca_dotnet_workshop_amd.telemetry.retention import utc_day
            tdir = tmp_path / "env" / "telemetry"
            stale = tdir / f"logs-old-1-{utc_day(time.time() - 31 * 86400)}.jsonl"
            stale.write_text("{}\n")
            assert ctl.retention_days() == 30 and stale.name in ctl.prune_telemetry()["removed"]
            assert any(tdir.glob(f"spans-*-{utc_day()}.jsonl"))  # today's telemetry stays
            # module 10: a changed template deploys a new revision and retires the old one
            old = proc.current.name
            res = await ctl.apply(load_manifest(MAIN, PARAMS, {**over, "notifierSimulatedDelayMs": 10}))
            assert proc.current.name != old and res["newRevisions"] == [proc.current.name]
            assert [r.active for r in proc.revisions] == [False, True]
            assert (tmp_path / "env" / "state.json").exists()
            # the backing services crash: the supervisor restarts them in place over their logs
            os.kill(ctl.stack.backing_proc.pid, signal.SIGKILL)
            for _ in range(300):
                await asyncio.sleep(0.1)
                if any(e["kind"] == "BackingServicesRestarted" for e in ctl.events):
                    break
            kinds = [e["kind"] for e in ctl.events]
            assert "BackingServicesCrashed" in kinds and "BackingServicesRestarted" in kinds
            c2 = await b.sb_counts("taskstracker", "tasksavedtopic/subscriptions/tasksmanager-backend-processor")
            assert c2["active"] == 0 and c2["dead_letter"] == 0  # settled messages stay settled after replay
        finally:
            await ctl.down()
    run(main())


class _NoRedirect(urllib.request.HTTPRedirectHandler):
    def redirect_request(self, *a, **k):
        return None

    def http_error_302(self, req, fp, code, msg, headers):
        return fp

    http_error_301 = http_error_302


@pytest.mark.slow
def test_keda_reference_timings_30s_polling_300s_cooldown(tmp_path):
    """Module 9 at ACA's own KEDA timings (docs/aca/09-aca-autoscale-keda/index.md:224-226):
    30 s polling and a 300 s cooldown, not the bench's shortened ones.  A scaled-down burst
    (3,000 messages of 1 s simulated work each, the module-9 notifier) on the processor's
    subscription scales it 1 -> 5 (messageCount 10 per replica, processor-backend-service.bicep:
    159-183); after the backlog drains it stays at 5 until a full cooldown past the last poll
    that saw messages, then returns to 1; every message is completed once."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_keda", os.path.join(os.path.dirname(__file__), "..", "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    k = bench.keda_stage(str(tmp_path), 0, 3000, polling_s=30.0, cooldown_s=300.0, budget_s=600.0)
    assert "error" not in k, k
    assert k["peak_replicas"] == 5 and k["exactly_once"], k
    assert k["keda_polling_s"] == 30.0 and k["keda_cooldown_s"] == 300.0
    # no scale-in before 300 s after the last poll that asked for more than one replica (the HPA
    # scale-down stabilization window KEDA's cooldown sets); and it comes within the next polls
    assert k["scale_in_after_last_recommendation_s"] is not None, k
    assert 300.0 <= k["scale_in_after_last_recommendation_s"] <= 300.0 + 2 * 30.0 + 15.0, k
    # the backlog drained long before: the replicas stayed up for the window, not for the work
    assert k["drain_s"] < k["scaled_in_to_1_s"] - 200.0, k
    assert k["replica_timeline"][0][1] == 1 and k["replica_timeline"][-1][1] == 1
    print(k)  # the timings (pytest -s): last active poll, last scale-out recommendation, scale-in
