"""The sidecar's gRPC API (``dapr.proto.runtime.v1.Dapr``) against its HTTP API.

Every building-block call the reference's ``DaprClient`` makes over gRPC (state save / get /
delete / query, publish, output binding; Backend.Api TasksStoreManager.cs, Processor
ExternalTasksProcessorController.cs:43) is run through both ``SidecarClient`` (HTTP) and
``GrpcSidecarClient`` (gRPC) against one sidecar; results, ETag semantics, delivered CloudEvents
and error statuses must agree."""
import json

import grpc
import pytest

from aca_dotnet_workshop_amd.sdk import SidecarClient, cloud_events_middleware, map_subscribe_handler, topic
from aca_dotnet_workshop_amd.sdk import proto as P
from aca_dotnet_workshop_amd.sdk.client import InvocationError, client_from_config
from aca_dotnet_workshop_amd.sdk.grpc_client import GrpcSidecarClient
from aca_dotnet_workshop_amd.web import WebApp, empty, json_response

from helpers import run
from test_sidecar import Harness, _inline, _until

COSMOS = {"url": "https://acct.documents.azure.com:443/", "masterKey": "k", "database": "db", "collection": "c"}


def test_proto_descriptors_match_dapr_wire_numbers():
    # field numbers are wire contract: spot-check the ones the reference's calls use
    f = P.rt("SaveStateRequest").DESCRIPTOR.fields_by_name
    assert (f["store_name"].number, f["states"].number) == (1, 2)
    s = P.common("StateItem").DESCRIPTOR.fields_by_name
    assert [s[n].number for n in ("key", "value", "etag", "metadata", "options")] == [1, 2, 3, 4, 5]
    p = P.rt("PublishEventRequest").DESCRIPTOR.fields_by_name
    assert [p[n].number for n in ("pubsub_name", "topic", "data", "data_content_type", "metadata")] == [1, 2, 3, 4, 5]
    assert P.rt("InvokeServiceRequest").DESCRIPTOR.fields_by_name["message"].number == 3
    b = P.rt("InvokeBindingRequest").DESCRIPTOR.fields_by_name
    assert [b[n].number for n in ("name", "data", "metadata", "operation")] == [1, 2, 3, 4]
    svc = P.POOL.FindServiceByName(P.SERVICE)
    assert {m.name for m in svc.methods} >= {"SaveState", "GetState", "DeleteState", "QueryStateAlpha1",
                                             "PublishEvent", "InvokeBinding", "InvokeService", "GetSecret"}
    # round trip through the wire format
    m = P.rt("SaveStateRequest")(store_name="s")
    it = m.states.add(key="k", value=b'{"a":1}')
    it.metadata["ttlInSeconds"] = "5"
    it.options.concurrency = 1
    again = P.rt("SaveStateRequest").FromString(m.SerializeToString())
    assert again == m and again.states[0].metadata["ttlInSeconds"] == "5"


def _app(received: list):
    app = WebApp("grpcapp")
    app.use(cloud_events_middleware())

    @topic("bus", "saved")
    async def saved(req):
        received.append(req.json())
        return empty(200)
    app.add_route("/saved", saved, ("POST",))

    async def echo(req):
        return json_response({"method": req.method, "q": req.query_get("x"), "body": req.json()})
    app.add_route("/echo", echo, ("GET", "POST", "PUT"))

    async def nope(req):
        return json_response({"err": "nope"}, 404)
    app.add_route("/nope", nope, ("GET",))
    map_subscribe_handler(app)
    return app


PLANES = ["python", "native"]


@pytest.mark.parametrize("plane", PLANES)
def test_grpc_and_http_clients_agree(plane, tmp_path):
    received: list = []
    secrets = tmp_path / "secrets.json"
    secrets.write_text('{"dbkey": "s3cr3t", "other": "x"}')
    comps = [_inline("statestore", "state.azure.cosmosdb", COSMOS),
             _inline("bus", "pubsub.azure.servicebus", {"connectionString": "Endpoint=sb://ns1.servicebus.windows.net/"}),
             _inline("files", "bindings.localstorage", {"rootPath": str(tmp_path / "blobs")}),
             _inline("secrets", "secretstores.local.file", {"secretsFile": str(secrets)})]

    async def main():
        async with Harness(_app(received), comps, app_id="grpcapp", grpc_port=0, data_plane=plane) as h:
            assert h.sc.bound_grpc_port and h.sc.active_data_plane == plane
            http = SidecarClient(h.base)
            g = GrpcSidecarClient(f"127.0.0.1:{h.sc.bound_grpc_port}", transport="grpcio")
            await g.wait_for_sidecar(5)
            # the native app host's HTTP/2 client (h2.hpp GrpcClient) as a third transport
            n = GrpcSidecarClient(f"127.0.0.1:{h.sc.bound_grpc_port}", transport="native")
            await n.wait_for_sidecar(5)
            for c, tag in ((http, "h"), (g, "g"), (n, "n")):
                doc = {"taskId": tag, "taskName": f"name {tag}", "isCompleted": False, "n": 3}
                await c.save_state("statestore", f"k-{tag}", doc)
                got, etag = await c.get_state_and_etag("statestore", f"k-{tag}")
                assert got == doc and etag
                # first-write concurrency with a stale ETag -> 409 from both transports
                with pytest.raises(InvocationError) as ei:
                    await c.save_state("statestore", f"k-{tag}", doc, etag="999999", concurrency="first-write")
                assert ei.value.status == 409
                await c.save_state("statestore", f"k-{tag}", {**doc, "n": 4}, etag=etag, concurrency="first-write")
                assert (await c.get_state("statestore", f"k-{tag}"))["n"] == 4
                assert await c.get_state("statestore", f"missing-{tag}") is None
                bulk = await c.get_bulk_state("statestore", [f"k-{tag}", f"missing-{tag}"])
                assert bulk[0].data["n"] == 4 and bulk[1].data is None
                # the raw forms the task codecs read: the HTTP API's JSON whichever protocol
                # carried it (gRPC: daprpb.hpp bulk_state_response_json / query_response_json)
                raw = json.loads(await c.get_bulk_state_raw("statestore", [f"k-{tag}", f"missing-{tag}"]))
                assert raw[0] == {"key": f"k-{tag}", "data": {**doc, "n": 4}, "etag": bulk[0].etag}
                assert raw[1]["key"] == f"missing-{tag}" and raw[1].get("data") is None
                await c.save_state_body("statestore", json.dumps([{"key": f"b-{tag}", "value": {"v": tag}}]).encode())
                rq = json.loads(await c.query_state_raw("statestore", {"filter": {"EQ": {"v": tag}}}))
                assert [(r["key"], r["data"]) for r in rq["results"]] == [(f"b-{tag}", {"v": tag})]
                await c.execute_state_transaction("statestore", [
                    {"operation": "upsert", "request": {"key": f"t1-{tag}", "value": {"taskCreatedBy": tag, "v": 1}}},
                    {"operation": "upsert", "request": {"key": f"t2-{tag}", "value": {"taskCreatedBy": tag, "v": 2}}}])
                q = await c.query_state("statestore", {"filter": {"EQ": {"taskCreatedBy": tag}},
                                                       "sort": [{"key": "v", "order": "DESC"}]})
                assert [r.data["v"] for r in q.results] == [2, 1]
                await c.delete_state("statestore", f"t1-{tag}")
                assert await c.get_state("statestore", f"t1-{tag}") is None
                with pytest.raises(InvocationError) as ei:
                    await c.save_state("nostore", "a", 1)
                assert ei.value.status == 400
                # pub/sub: both deliver the same CloudEvent data to the subscriber
                await c.publish_event("bus", "saved", {"taskName": f"t-{tag}"})
                await _until(lambda: {"taskName": f"t-{tag}"} in received)
                res = await c.publish_events("bus", "saved", [{"i": 1}, {"i": 2}])
                assert res["failedEntries"] == []
                with pytest.raises(InvocationError) as ei:
                    await c.publish_event("nobus", "saved", {})
                assert ei.value.status == 404
                # output binding with metadata in and out
                out = await c.invoke_binding("files", "create", {"task": tag}, {"fileName": f"{tag}.json"})
                assert out["fileName"].endswith(f"{tag}.json")
                assert await c.invoke_binding("files", "get", None, {"fileName": f"{tag}.json"}) == {"task": tag}
                # secrets
                assert await c.get_secret("secrets", "dbkey") == {"dbkey": "s3cr3t"}
                assert (await c.get_bulk_secret("secrets"))["other"] == {"other": "x"}
                # service invocation (self), verb + query string + body
                r = await c.invoke_method("PUT", "grpcapp", "echo?x=7", {"a": 1})
                assert r == {"method": "PUT", "q": "7", "body": {"a": 1}}
                raw = await c.invoke_method_raw("GET", "grpcapp", "nope")
                assert raw.status == 404
                await c.set_metadata(f"attr-{tag}", "v")
                meta = await c.get_metadata()
                assert meta["id"] == "grpcapp" and meta["extended"][f"attr-{tag}"] == "v"
                assert {x["name"] for x in meta["components"]} >= {"statestore", "bus", "files", "secrets"}
            for tag in "ghn":  # same bytes written through every transport
                assert (tmp_path / "blobs" / f"{tag}.json").read_bytes() == b'{"task":"%s"}' % tag.encode()
            await _until(lambda: sum(1 for x in received if "i" in x) == 6)
            if plane == "native":
                # the hot RPCs were decoded by the C++ plane (h2.hpp / dataplane.cpp) and ran its
                # native state / publish paths; the rest were bridged to grpc_api.py
                metrics = (await h.http.get(h.base + "/metrics")).body.decode()
                for op in ("grpc.SaveState", "grpc.GetState", "grpc.DeleteState", "grpc.QueryStateAlpha1", "grpc.GetBulkState",
                           "grpc.PublishEvent", "grpc.InvokeService", "grpc.GetSecret", "state.save",
                           "state.get", "state.delete", "state.query", "publish"):
                    assert f'op="{op}"' in metrics, op
            await http.close()
            await g.close()
            await n.close()
    run(main())


@pytest.mark.parametrize("plane", PLANES)
def test_grpc_api_token_and_client_factory(plane):
    comps = [_inline("kv", "state.in-memory", {})]

    async def main():
        async with Harness(WebApp("t"), comps, app_id="t", api_token="tok", grpc_port=0, data_plane=plane) as h:
            target = f"127.0.0.1:{h.sc.bound_grpc_port}"
            bad = GrpcSidecarClient(target, api_token="")
            with pytest.raises(InvocationError) as ei:
                await bad.save_state("kv", "a", 1)
            assert ei.value.status == 401
            await bad.close()
            env = {"DAPR_API_PROTOCOL": "grpc", "DAPR_GRPC_PORT": str(h.sc.bound_grpc_port)}
            c = client_from_config(None, env)
            assert isinstance(c, GrpcSidecarClient)
            c.api_token = "tok"
            await c.save_state("kv", "a", {"x": 1})
            assert await c.get_state("kv", "a") == {"x": 1}
            # raw stub call: grpc status code for an unknown store
            ch = grpc.aio.insecure_channel(target)
            req_cls, resp_cls = P.rpc_types("GetState")
            stub = ch.unary_unary(P.method_path("GetState"), request_serializer=req_cls.SerializeToString,
                                  response_deserializer=resp_cls.FromString)
            with pytest.raises(grpc.aio.AioRpcError) as ei:
                await stub(req_cls(store_name="missing", key="a"), metadata=[("dapr-api-token", "tok")])
            assert ei.value.code() == grpc.StatusCode.INVALID_ARGUMENT
            await ch.close()
            await c.close()
            assert isinstance(client_from_config(None, {}), SidecarClient)
    run(main())


@pytest.mark.parametrize("plane", PLANES)
def test_backend_api_over_grpc_transport(plane):
    """The Backend API's store manager on the gRPC transport: createTask persists + publishes."""
    from aca_dotnet_workshop_amd.services.backend_api.app import create_app
    received: list = []
    comps = [_inline("statestore", "state.azure.cosmosdb", COSMOS),
             _inline("dapr-pubsub-servicebus", "pubsub.azure.servicebus",
                     {"connectionString": "Endpoint=sb://ns2.servicebus.windows.net/"})]
    sub = WebApp("sub")
    sub.use(cloud_events_middleware())

    @topic("dapr-pubsub-servicebus", "tasksavedtopic")
    async def saved(req):
        received.append(req.json())
        return empty(200)
    sub.add_route("/tasksaved", saved, ("POST",))
    map_subscribe_handler(sub)

    async def main():
        async with Harness(sub, comps, app_id="tasksmanager-backend-api", grpc_port=0, data_plane=plane) as h:
            g = GrpcSidecarClient(f"127.0.0.1:{h.sc.bound_grpc_port}")
            api = create_app([], overrides={"TasksManager:Backend": "store", "Dapr:ApiProtocol": "grpc",
                                            "Logging:LogLevel:Default": "Warning"})
            mgr = api.services["tasks_manager"]
            assert isinstance(mgr.client, GrpcSidecarClient)
            mgr.client = g
            from datetime import datetime
            tid = await mgr.create_new_task("grpc task", "me@x", "you@x", datetime(2030, 1, 1))
            t = await mgr.get_task_by_id(tid)
            assert t.task_name == "grpc task"
            tasks = await mgr.get_tasks_by_creator("me@x")
            assert [x.task_id for x in tasks] == [t.task_id]
            assert await _until(lambda: len(received) == 1)
            assert received[0]["taskName"] == "grpc task" and received[0]["taskId"] == str(tid)
            # the request path of a running service: inside an unsampled trace the native transport
            # sends pre-encoded SaveState / PublishEvent straight to the app host (no span)
            from aca_dotnet_workshop_amd.telemetry import tracing
            n = GrpcSidecarClient(f"127.0.0.1:{h.sc.bound_grpc_port}", transport="native")
            mgr.client = n
            span = tracing.Tracer("t", None, sample_rate=0.0).start_span("POST", "server")
            try:
                assert not span.sampled
                tid2 = await mgr.create_new_task_from_body(
                    b'{"taskName":"fast grpc","taskCreatedBy":"me@x","taskDueDate":"2030-01-02","taskAssignedTo":"a@x"}')
            finally:
                span.end()
            assert (await mgr.get_task_by_id(tid2)).task_name == "fast grpc"
            assert await _until(lambda: len(received) == 2)
            assert received[1]["taskId"] == tid2 and received[1]["taskDueDate"] == "2030-01-02T00:00:00"
            await g.close()
            await n.close()
    run(main())
