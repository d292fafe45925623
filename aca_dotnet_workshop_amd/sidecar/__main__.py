"""``python -m aca_dotnet_workshop_amd.sidecar`` -- the ``dapr run`` / ``daprd`` CLI equivalent.

``run`` starts a sidecar and (optionally) the application command as a child process,
exactly like the reference's local recipe (snippets/dapr-run-backend-api.md):

    python -m aca_dotnet_workshop_amd.sidecar run --app-id tasksmanager-backend-api \\
        --app-port 7088 --dapr-http-port 3500 --resources-path deploy/components \\
        -- python -m aca_dotnet_workshop_amd.services.backend_api --urls http://127.0.0.1:7088

The child receives ``DAPR_HTTP_PORT`` (and ``TT_SIDECAR_UDS`` when ``--unix-socket-dir``
is used), ``APP_ID``, ``APP_PORT``; with ``--app-env-file`` (an app running from its container
image) it gets that environment only, plus the Dapr ports.  The sidecar stops when the app exits and vice versa.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import logging
import os
import tempfile
import signal
import subprocess
import sys

from ..telemetry import configure_logging
from ..telemetry.profiler import maybe_profile
from .runtime import Sidecar

log = logging.getLogger("sidecar.cli")


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog="tt-sidecar", description="Sidecar runtime (daprd equivalent)")
    sub = ap.add_subparsers(dest="cmd", required=True)
    r = sub.add_parser("run", help="run a sidecar, optionally with the app as a child process")
    r.add_argument("--app-id", required=True)
    r.add_argument("--app-port", type=int, default=None)
    r.add_argument("--app-uds", default=None, help="app listens on this Unix socket instead of a port")
    r.add_argument("--dapr-http-port", type=int, default=3500)
    r.add_argument("--dapr-internal-port", "--dapr-internal-grpc-port", dest="internal_port", type=int, default=0,
                   help="sidecar-to-sidecar port (0 = ephemeral)")
    r.add_argument("--dapr-grpc-port", type=int, default=None,
                   help="serve the gRPC API (dapr.proto.runtime.v1.Dapr) on this port (0 = ephemeral; off if unset)")
    r.add_argument("--unix-socket-dir", default=None, help="expose the sidecar API and internal port as Unix sockets here")
    r.add_argument("--resources-path", "--components-path", dest="resources", action="append", default=[])
    r.add_argument("--registry-dir", default=os.environ.get("TT_REGISTRY_DIR") or default_registry_dir(),
                   help="name-resolution directory shared by the sidecars of one host (self-hosted Dapr's mDNS); "
                        "default: $TT_REGISTRY_DIR or /tmp/tt-registry-<uid>")
    r.add_argument("--backing-url", default=os.environ.get("TT_BACKING_URL"))
    r.add_argument("--identity", default=os.environ.get("TT_IDENTITY"))
    r.add_argument("--app-max-concurrency", type=int, default=None)
    r.add_argument("--app-health-check-path", default=None)
    r.add_argument("--log-level", default="info")
    r.add_argument("--enable-api-logging", action="store_true",
                   help="log every sidecar API call (Dapr's enableApiLogging)")
    r.add_argument("--replica-name", default=os.environ.get("TT_REPLICA_NAME"))
    r.add_argument("--app-ssl", action="store_true", default=os.environ.get("TT_APP_SSL", "") in ("1", "true"),
                   help="the app serves HTTPS on --app-port (its certificate is not verified, as in Dapr)")
    r.add_argument("--mtls-cert", default=os.environ.get("TT_MTLS_CERT"),
                   help="workload certificate for mutual TLS with peer sidecars (with --mtls-key/--mtls-ca)")
    r.add_argument("--mtls-key", default=os.environ.get("TT_MTLS_KEY"))
    r.add_argument("--mtls-ca", default=os.environ.get("TT_MTLS_CA"))
    r.add_argument("--data-plane", choices=("native", "python"),
                   default=os.environ.get("TT_SIDECAR_DATAPLANE") or "native",
                   help="native: hot HTTP/gRPC API paths served by the C++ data plane (default); python: all in-process")
    r.add_argument("--app-env-file", default=None,
                   help="JSON object: the app's whole environment (a container's: nothing inherited from the "
                        "sidecar's, no Unix-socket paths; the app reaches the sidecar on DAPR_HTTP_PORT/DAPR_GRPC_PORT)")
    r.add_argument("command", nargs=argparse.REMAINDER, help="-- <app command>")
    return ap


async def _run(a: argparse.Namespace) -> int:
    cmd = list(a.command)
    if cmd and cmd[0] == "--":
        cmd = cmd[1:]
    sock_api = sock_int = None
    tag = a.replica_name or f"{a.app_id}-{os.getpid()}"
    if a.unix_socket_dir:
        os.makedirs(a.unix_socket_dir, exist_ok=True)
        sock_api = os.path.join(a.unix_socket_dir, f"{tag}.d.sock")
        sock_int = os.path.join(a.unix_socket_dir, f"{tag}.i.sock")
    sc = Sidecar(a.app_id, app_port=a.app_port, app_uds=a.app_uds, http_port=a.dapr_http_port, uds=sock_api,
                 internal_port=a.internal_port if not sock_int else None, internal_uds=sock_int,
                 resources_paths=a.resources, registry_dir=a.registry_dir, api_token=os.environ.get("DAPR_API_TOKEN"),
                 app_token=os.environ.get("APP_API_TOKEN"), mesh_token=os.environ.get("TT_MESH_TOKEN"),
                 app_max_concurrency=a.app_max_concurrency, identity=a.identity, backing_url=a.backing_url,
                 instance=a.replica_name, app_health_path=a.app_health_check_path,
                 api_logging=a.enable_api_logging, grpc_port=a.dapr_grpc_port, app_ssl=a.app_ssl,
                 mtls={"cert": a.mtls_cert, "key": a.mtls_key, "ca": a.mtls_ca}
                 if a.mtls_cert and a.mtls_key and a.mtls_ca else None,
                 grpc_uds=os.path.join(a.unix_socket_dir, f"{tag}.g.sock") if a.unix_socket_dir and a.dapr_grpc_port is not None
                 else None, data_plane=a.data_plane)
    await sc.start()
    loop = asyncio.get_running_loop()
    stop = asyncio.Event()
    for sig in (signal.SIGTERM, signal.SIGINT):
        loop.add_signal_handler(sig, stop.set)
    proc = None
    if cmd:
        container = a.app_env_file is not None
        if container:
            with open(a.app_env_file) as fh:
                env = {str(k): str(v) for k, v in json.load(fh).items()}
        else:
            env = dict(os.environ)
        env.update({"DAPR_HTTP_PORT": str(sc.bound_http_port or ""), "APP_ID": a.app_id,
                    "APP_PORT": str(a.app_port or ""), "TT_APP_ID": a.app_id})
        if sock_api and not container:
            env["TT_SIDECAR_UDS"] = sock_api
        if sc.bound_grpc_port:
            env["DAPR_GRPC_PORT"] = str(sc.bound_grpc_port)
        if sc.grpc_uds and not container:  # the co-located app's gRPC, like its HTTP, on the socket
            env["TT_SIDECAR_GRPC_UDS"] = sc.grpc_uds
        if a.app_uds:
            env["TT_APP_UDS"] = a.app_uds
        proc = await asyncio.create_subprocess_exec(*cmd, env=env)
        waiter = asyncio.ensure_future(proc.wait())
        stopper = asyncio.ensure_future(stop.wait())
        done_sc = asyncio.ensure_future(sc.stopped.wait())
        await asyncio.wait([waiter, stopper, done_sc], return_when=asyncio.FIRST_COMPLETED)
        if proc.returncode is None:
            proc.send_signal(signal.SIGTERM)
            try:
                await asyncio.wait_for(proc.wait(), 10)
            except asyncio.TimeoutError:
                proc.kill()
                await proc.wait()
        for t in (stopper, done_sc):
            t.cancel()
    else:
        stopper = asyncio.ensure_future(stop.wait())
        done_sc = asyncio.ensure_future(sc.stopped.wait())
        await asyncio.wait([stopper, done_sc], return_when=asyncio.FIRST_COMPLETED)
    await sc.stop()
    return proc.returncode if proc is not None and proc.returncode is not None else 0


def default_registry_dir() -> str:
    """One registry per user and host, like self-hosted Dapr's mDNS zone."""
    return os.path.join(tempfile.gettempdir(), f"tt-registry-{os.getuid()}")


def main(argv: list[str] | None = None) -> int:
    a = build_parser().parse_args(argv)
    configure_logging(f"{a.app_id}.sidecar")
    logging.getLogger().setLevel(getattr(logging, a.log_level.upper(), logging.INFO))
    try:
        with maybe_profile(f"{a.replica_name or a.app_id}.sidecar"):
            return asyncio.run(_run(a))
    except KeyboardInterrupt:
        return 0


if __name__ == "__main__":
    sys.exit(main())
