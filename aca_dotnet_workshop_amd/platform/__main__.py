"""``python -m aca_dotnet_workshop_amd.platform`` -- the ``az deployment`` / ``az containerapp``
equivalent CLI.

    validate  -f deploy/main.yaml [-p params.json]          lint (az bicep build + ARM Validate)
    what-if   -f ... [--env-dir DIR]                        diff vs the running/recorded env
    up        -f ... --env-dir DIR [--detach]                deploy and run the environment
    status    --env-dir DIR                                  apps, revisions, replicas, ingress URLs
    show      APP --env-dir DIR [--query ingress.fqdn]       one app (az containerapp show --query)
    exec      APP --env-dir DIR -- CMD...                    run CMD in a replica's context (az containerapp exec)
    image     [--service S] [--verify] [--push ACR --variant V --tag T]   build (and push) the images
    acr       NAME                                           a registry's repositories and tags
    scale     APP --env-dir DIR [--min N] [--max N] [--replicas N]
    restart   APP --env-dir DIR                              restart the active revision
    apply     -f ... --env-dir DIR                           re-deploy changed apps as new revisions
    logs      APP --env-dir DIR [--tail N] [--follow]        container logs (az containerapp logs show)
    outputs   --env-dir DIR
    down      --env-dir DIR [--delete]                       stop (and delete = az group delete)
    appmap / failures / performance --env-dir DIR            telemetry views (App Insights blades)
    metrics   [APP] --env-dir DIR [--interval S]             live metrics: request/failure/delivery rates, CPU
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import subprocess
import sys
import time
from pathlib import Path

from .manifest import ManifestError, load_manifest, validate, what_if


def _uds_request(sock: str, method: str, path: str, body: dict | None = None, timeout: float = 600.0) -> tuple[int, dict]:
    import socket
    s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    s.settimeout(timeout)
    s.connect(sock)
    data = json.dumps(body).encode() if body is not None else b""
    s.sendall(f"{method} {path} HTTP/1.1\r\nHost: x\r\nConnection: close\r\nContent-Type: application/json\r\n"
              f"Content-Length: {len(data)}\r\n\r\n".encode() + data)
    buf = b""
    while True:
        ch = s.recv(65536)
        if not ch:
            break
        buf += ch
    s.close()
    head, _, payload = buf.partition(b"\r\n\r\n")
    status = int(head.split(b" ")[1])
    return status, (json.loads(payload) if payload.strip() else {})


def _ctl(env_dir: str) -> str:
    sock = str(Path(env_dir) / "control.sock")
    if not os.path.exists(sock):
        sys.exit(f"no running environment in {env_dir} (control.sock missing)")
    return sock


def _params(a) -> dict:
    out = {}
    for kv in a.param or []:
        k, _, v = kv.partition("=")
        out[k] = v
    return out


def cmd_validate(a) -> int:
    m = load_manifest(a.file, a.parameters, _params(a))
    errs = validate(m)
    if errs:
        for e in errs:
            print("ERROR:", e)
        return 1
    print(f"manifest {a.file} is valid: {len(m.apps)} apps, {len(m.components)} components")
    return 0


def cmd_whatif(a) -> int:
    m = load_manifest(a.file, a.parameters, _params(a))
    cur = None
    if a.env_dir and (Path(a.env_dir) / "state.json").exists():
        cur = json.loads((Path(a.env_dir) / "state.json").read_text()).get("desired")
    changes = what_if(m, cur)
    sym = {"Create": "+", "Delete": "-", "Modify": "~", "NoChange": "="}
    for c in changes:
        if c["change"] != "NoChange" or a.verbose:
            print(f"  {sym[c['change']]} {c['resource']}")
    counts = {k: sum(1 for c in changes if c["change"] == k) for k in sym}
    print(f"Resource changes: {counts['Create']} to create, {counts['Modify']} to modify, "
          f"{counts['Delete']} to delete, {counts['NoChange']} no change.")
    return 0


async def _up(a) -> int:
    from ..telemetry import configure_logging
    from .controller import EnvironmentController
    configure_logging("platform")
    m = load_manifest(a.file, a.parameters, _params(a))
    ctl = EnvironmentController(m, a.env_dir, a.polling_interval, a.cooldown, registry_root=a.registry_root)
    import signal
    loop = asyncio.get_running_loop()
    for sig in (signal.SIGTERM, signal.SIGINT):
        loop.add_signal_handler(sig, ctl.stop_event.set)
    try:
        await ctl.up()
    except Exception:
        await ctl.down()
        raise
    st = ctl.status()
    print(json.dumps({"ready": True, "apps": {k: v["ingress"] for k, v in st["apps"].items()}, "outputs": st["outputs"]}),
          flush=True)
    await ctl.run_forever()
    return 0


def cmd_up(a) -> int:
    if a.detach:
        Path(a.env_dir).mkdir(parents=True, exist_ok=True)
        args = [sys.executable, "-m", "aca_dotnet_workshop_amd.platform", "up", "-f", a.file, "--env-dir", a.env_dir]
        if a.parameters:
            args += ["-p", a.parameters]
        for kv in a.param or []:
            args += ["--param", kv]
        if a.polling_interval is not None:
            args += ["--polling-interval", str(a.polling_interval)]
        if a.cooldown is not None:
            args += ["--cooldown", str(a.cooldown)]
        if a.registry_root:
            args += ["--registry-root", a.registry_root]
        logf = open(Path(a.env_dir) / "controller.log", "ab")
        p = subprocess.Popen(args, stdout=logf, stderr=subprocess.STDOUT, start_new_session=True)
        deadline = time.time() + a.timeout
        while time.time() < deadline:
            if p.poll() is not None:
                sys.exit(f"controller exited with {p.returncode}; see {a.env_dir}/controller.log")
            sock = Path(a.env_dir) / "control.sock"
            if sock.exists():
                try:
                    st, body = _uds_request(str(sock), "GET", "/status", timeout=5)
                    if st == 200 and any(e["kind"] == "EnvironmentReady" for e in body.get("events", [])):
                        print(json.dumps({"pid": p.pid, "apps": {k: v["ingress"] for k, v in body["apps"].items()}}))
                        return 0
                except OSError:
                    pass
            time.sleep(0.2)
        sys.exit("timed out waiting for the environment")
    return asyncio.run(_up(a))


def cmd_status(a) -> int:
    st, body = _uds_request(_ctl(a.env_dir), "GET", "/status")
    if a.json:
        print(json.dumps(body, indent=1))
        return 0
    print(f"environment {body['name']}  backing={body['backingUrl']}  uptime={body['uptimeSeconds']}s")
    for name, app in body["apps"].items():
        ing = app["ingress"]
        where = "no ingress" if ing is None else (ing["fqdn"] if ing["external"] else f"internal ({ing['internalUrl']})")
        print(f"  {name}: desired={app['desiredReplicas']} restarts={app['restarts']}  {where}")
        for r in app["revisions"]:
            alive = sum(1 for p in r["replicas"] if p["alive"])
            print(f"    revision {r['name']} {'active' if r['active'] else 'inactive'}: {alive}/{len(r['replicas'])} replicas")
    return 0


def cmd_scale(a) -> int:
    body = {k: v for k, v in (("min", a.min), ("max", a.max), ("replicas", a.replicas)) if v is not None}
    st, res = _uds_request(_ctl(a.env_dir), "POST", f"/apps/{a.app}/scale", body)
    print(json.dumps(res))
    return 0 if st == 200 else 1


def cmd_restart(a) -> int:
    st, res = _uds_request(_ctl(a.env_dir), "POST", f"/apps/{a.app}/restart", {})
    print(json.dumps(res))
    return 0 if st == 200 else 1


def cmd_apply(a) -> int:
    st, res = _uds_request(_ctl(a.env_dir), "POST", "/apply",
                           {"file": str(Path(a.file).resolve()), "parameters": a.parameters and str(Path(a.parameters).resolve()),
                            "overrides": _params(a)})
    print(json.dumps(res))
    return 0 if st == 200 else 1


def cmd_logs(a) -> int:
    logs = Path(a.env_dir) / "runtime" / "logs"
    files = sorted(logs.glob(f"{a.app}-*.log"))
    if not files:
        sys.exit(f"no logs for {a.app}")
    for f in files:
        lines = f.read_text(errors="replace").splitlines()
        for ln in lines[-a.tail:]:
            print(f"[{f.stem}] {ln}")
    if a.follow:
        pos = {f: f.stat().st_size for f in files}
        try:
            while True:
                time.sleep(0.5)
                for f in sorted(logs.glob(f"{a.app}-*.log")):
                    size = f.stat().st_size
                    if size > pos.get(f, 0):
                        with open(f, errors="replace") as fh:
                            fh.seek(pos.get(f, 0))
                            for ln in fh.read().splitlines():
                                print(f"[{f.stem}] {ln}", flush=True)
                        pos[f] = size
        except KeyboardInterrupt:
            pass
    return 0


def cmd_show(a) -> int:
    """``az containerapp show -n APP --query <path>``: one app's live description; ``--query``
    takes a dotted path (``ingress.fqdn``, ``ingress.httpUrl``, ``desiredReplicas``) and prints the
    bare value, for shell use (``FQDN=$(... show tasksmanager-frontend-webapp --query ingress.fqdn)``)."""
    st, body = _uds_request(_ctl(a.env_dir), "GET", "/status")
    app = body["apps"].get(a.app)
    if app is None:
        print(f"no app {a.app!r} in this environment", file=sys.stderr)
        return 1
    v = app
    for part in (a.query.split(".") if a.query else []):
        if isinstance(v, list) and part.isdigit() and int(part) < len(v):
            v = v[int(part)]
        elif isinstance(v, dict) and part in v:
            v = v[part]
        else:
            print(f"{a.query!r} not found", file=sys.stderr)
            return 1
    print(v if isinstance(v, (str, int, float)) else json.dumps(v, indent=1))
    return 0


def cmd_exec(a) -> int:
    """``az containerapp exec``: run a command inside a replica's context -- its sidecar is
    reachable through ``DAPR_HTTP_UDS`` (a Unix socket: ``curl --unix-socket "$DAPR_HTTP_UDS"
    http://localhost/v1.0/...``), as ``localhost:3500`` is from inside a Container App."""
    st, body = _uds_request(_ctl(a.env_dir), "GET", "/status")
    app = body["apps"].get(a.app)
    reps = [p for r in (app or {}).get("revisions", []) if r["active"] for p in r["replicas"] if p["alive"]]
    if not reps:
        print(f"no running replica of {a.app!r}", file=sys.stderr)
        return 1
    rep = next((p for p in reps if p["name"] == a.replica), None) if a.replica else reps[0]
    if rep is None:
        print(f"no replica {a.replica!r}", file=sys.stderr)
        return 1
    cmd = a.command
    env = dict(os.environ, DAPR_HTTP_UDS=rep["sidecar"], TT_REPLICA_NAME=rep["name"], CONTAINER_APP_NAME=a.app)
    return subprocess.call(cmd or ["bash"], env=env)


def cmd_outputs(a) -> int:
    st, body = _uds_request(_ctl(a.env_dir), "GET", "/status")
    print(json.dumps(body["outputs"], indent=1))
    return 0


def cmd_down(a) -> int:
    sock = Path(a.env_dir) / "control.sock"
    if sock.exists():
        try:
            _uds_request(str(sock), "POST", "/shutdown", {})
        except OSError:
            pass
        for _ in range(300):
            try:
                _uds_request(str(sock), "GET", "/status", timeout=1)
            except OSError:
                break
            time.sleep(0.1)
        if sock.exists():
            sock.unlink()
    if a.delete:
        from .controller import reset_env_dir
        reset_env_dir(a.env_dir)
    print("environment stopped" + (" and deleted" if a.delete else ""))
    return 0


def live_rates(s0: dict, s1: dict) -> dict[str, dict[str, float]]:
    """Per-app rates between two /metrics/live snapshots."""
    dt = max(1e-6, s1["ts"] - s0["ts"])
    out: dict[str, dict[str, float]] = {}

    def tot(snap, app, part, key):
        return sum(r.get(part, {}).get(key, 0.0) for r in snap["apps"].get(app, {}).values())

    def fails(snap, app):
        n = 0.0
        for r in snap["apps"].get(app, {}).values():
            for k, v in r.get("app", {}).items():
                if k.startswith("http_requests_total{") and 'status="5' in k:
                    n += v
        return n

    for app in s1["apps"]:
        out[app] = {
            "replicas": len(s1["apps"][app]),
            "requests_per_s": (tot(s1, app, "app", "http_requests_total") - tot(s0, app, "app", "http_requests_total")) / dt,
            "failures_per_s": (fails(s1, app) - fails(s0, app)) / dt,
            "sidecar_native_per_s": (tot(s1, app, "sidecar", "sidecar_native_requests_total")
                                     - tot(s0, app, "sidecar", "sidecar_native_requests_total")) / dt,
            "cpu_cores": (sum(r.get("cpuSeconds", 0.0) for r in s1["apps"][app].values())
                          - sum(r.get("cpuSeconds", 0.0) for r in s0["apps"].get(app, {}).values())) / dt,
        }
    return out


def cmd_metrics(a) -> int:
    st, s0 = _uds_request(_ctl(a.env_dir), "GET", "/metrics/live")
    if st != 200:
        print(json.dumps(s0), file=sys.stderr)
        return 1
    time.sleep(a.interval)
    st, s1 = _uds_request(_ctl(a.env_dir), "GET", "/metrics/live")
    rates = live_rates(s0, s1)
    if a.app:
        rates = {k: v for k, v in rates.items() if k == a.app}
    if a.json:
        print(json.dumps(rates, indent=1))
        return 0
    print(f"{'app':36} {'repl':>4} {'req/s':>10} {'fail/s':>8} {'native/s':>10} {'cpu':>6}")
    for app, r in sorted(rates.items()):
        print(f"{app:36} {r['replicas']:>4} {r['requests_per_s']:>10.1f} {r['failures_per_s']:>8.1f} "
              f"{r['sidecar_native_per_s']:>10.1f} {r['cpu_cores']:>6.2f}")
    return 0


def cmd_telemetry(a) -> int:
    from ..telemetry import appmap
    tdir = Path(a.env_dir) / "telemetry"
    fn = {"appmap": appmap.application_map, "failures": appmap.failures, "performance": appmap.performance}[a.cmd]
    print(json.dumps(fn(tdir), indent=1))
    return 0


def cmd_image(a) -> int:
    """Build (``az acr build`` / ``docker build``), optionally verify, and with ``--push REGISTRY``
    push each service's ``--variant`` image as ``tasksmanager/<app id>:<tag>``."""
    from . import image
    reg = None
    if a.push:
        from .registry import LocalRegistry
        reg = LocalRegistry(a.push, a.registry_root)
    tags = a.tag or ["latest"]
    for row in image.report(a.out, a.service, a.verify):
        if reg is not None and row["variant"] == a.variant:
            repo = f"tasksmanager/{image.SERVICES[row['service']]}"
            row["pushed"] = [f"{reg.login_server}/{repo}:{t}@{reg.push(row['archive'], repo, t)}" for t in tags]
        print(json.dumps(row), flush=True)
    return 0


def cmd_acr(a) -> int:
    """``az acr create`` / ``az acr import`` / ``az acr repository list``."""
    from .registry import LocalRegistry, RegistryError
    reg = LocalRegistry(a.name, a.registry_root)
    if a.action == "create":
        print(f"ACR {reg.login_server} created" if reg.create() else f"ACR {reg.login_server} already exists.")
        return 0
    if a.action == "import":
        if not reg.exists():
            print(f"ERROR: registry {a.name} does not exist", file=sys.stderr)
            return 1
        server, _, rest = a.source.partition("/")
        src = LocalRegistry(server.split(".", 1)[0], a.registry_root)
        try:
            digest = reg.import_image(src, a.source, a.image, force=a.force)
        except RegistryError as e:
            print(f"ERROR: {e}", file=sys.stderr)
            return 1
        print(f"imported {a.source} -> {reg.login_server}/{a.image}@{digest}")
        return 0
    print(json.dumps({"loginServer": reg.login_server, "repositories": reg.repositories()}, indent=1))
    return 0


def main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser(prog="tt-platform", description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    sub = ap.add_subparsers(dest="cmd", required=True)

    def manifest_args(p, need_env=False):
        p.add_argument("-f", "--file", default="deploy/main.yaml")
        p.add_argument("-p", "--parameters", default=None)
        p.add_argument("--param", action="append", help="k=v parameter override")
        p.add_argument("--env-dir", required=need_env, default=None)

    p = sub.add_parser("validate")
    manifest_args(p)
    p.set_defaults(fn=cmd_validate)
    p = sub.add_parser("what-if")
    manifest_args(p)
    p.add_argument("-v", "--verbose", action="store_true")
    p.set_defaults(fn=cmd_whatif)
    p = sub.add_parser("up")
    manifest_args(p, True)
    p.add_argument("--detach", action="store_true")
    p.add_argument("--timeout", type=float, default=180.0)
    p.add_argument("--polling-interval", type=float, default=None)
    p.add_argument("--cooldown", type=float, default=None)
    p.add_argument("--registry-root", default=None,
                   help="where container registries live ($TT_CONTAINER_REGISTRY_ROOT); apps with an image pull from there")
    p.set_defaults(fn=cmd_up)
    p = sub.add_parser("apply")
    manifest_args(p, True)
    p.set_defaults(fn=cmd_apply)
    for name, fn in (("status", cmd_status), ("outputs", cmd_outputs), ("down", cmd_down),
                     ("appmap", cmd_telemetry), ("failures", cmd_telemetry), ("performance", cmd_telemetry)):
        p = sub.add_parser(name)
        p.add_argument("--env-dir", required=True)
        if name == "status":
            p.add_argument("--json", action="store_true")
        if name == "down":
            p.add_argument("--delete", action="store_true")
        p.set_defaults(fn=fn)
    p = sub.add_parser("show")
    p.add_argument("app")
    p.add_argument("--env-dir", required=True)
    p.add_argument("--query", default=None)
    p.set_defaults(fn=cmd_show)
    p = sub.add_parser("exec")
    p.add_argument("app")
    p.add_argument("--env-dir", required=True)
    p.add_argument("--replica", default=None)
    p.set_defaults(fn=cmd_exec)  # the command follows "--"
    p = sub.add_parser("scale")
    p.add_argument("app")
    p.add_argument("--env-dir", required=True)
    p.add_argument("--min", type=int)
    p.add_argument("--max", type=int)
    p.add_argument("--replicas", type=int)
    p.set_defaults(fn=cmd_scale)
    p = sub.add_parser("restart")
    p.add_argument("app")
    p.add_argument("--env-dir", required=True)
    p.set_defaults(fn=cmd_restart)
    p = sub.add_parser("metrics")
    p.add_argument("app", nargs="?")
    p.add_argument("--env-dir", required=True)
    p.add_argument("--interval", type=float, default=2.0)
    p.add_argument("--json", action="store_true")
    p.set_defaults(fn=cmd_metrics)
    p = sub.add_parser("logs")
    p.add_argument("app")
    p.add_argument("--env-dir", required=True)
    p.add_argument("--tail", type=int, default=50)
    p.add_argument("--follow", action="store_true")
    p.set_defaults(fn=cmd_logs)
    p = sub.add_parser("image", help="build OCI images of the services (standard + chiseled; module 12)")
    p.add_argument("--service", action="append", choices=["backend_api", "processor", "frontend"])
    p.add_argument("--out", default="dist/images")
    p.add_argument("--verify", action="store_true", help="run each image under chroot and probe it (root)")
    p.add_argument("--push", metavar="REGISTRY", default=None, help="push to this registry (ACR name)")
    p.add_argument("--variant", choices=["standard", "chiseled"], default="chiseled", help="which variant --push pushes")
    p.add_argument("--tag", action="append", default=None, help="tag to push (repeatable; default latest)")
    p.add_argument("--registry-root", default=None, help="where registries live ($TT_CONTAINER_REGISTRY_ROOT)")
    p.set_defaults(fn=cmd_image)
    p = sub.add_parser("acr", help="registries: create, import an image, list repositories and tags")
    p.add_argument("action", nargs="?", choices=["list", "create", "import"], default="list")
    p.add_argument("name")
    p.add_argument("--source", help="import: <registry login server>/<repo>:<tag>")
    p.add_argument("--image", help="import: <repo>[:tag] in this registry")
    p.add_argument("--force", action="store_true")
    p.add_argument("--registry-root", default=None)
    p.set_defaults(fn=cmd_acr)
    argv = list(sys.argv[1:] if argv is None else argv)
    tail: list[str] = []
    if "--" in argv:  # exec APP ... -- CMD ARGS: everything after "--" is the command
        i = argv.index("--")
        argv, tail = argv[:i], argv[i + 1:]
    a = ap.parse_args(argv)
    a.command = tail
    try:
        return a.fn(a)
    except ManifestError as e:
        for err in e.errors:
            print("ERROR:", err, file=sys.stderr)
        return 1


if __name__ == "__main__":
    sys.exit(main())
