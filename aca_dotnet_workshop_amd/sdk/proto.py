"""Protobuf messages of the sidecar's gRPC API, built at import time (no ``protoc``).

The reference's services talk to ``daprd`` through ``Dapr.Client.DaprClient``, which uses the
sidecar's gRPC API (port ``50001``/``50002``/``50003`` in the reference's launch plan,
.vscode/tasks.json:126-165) for state, pub/sub, bindings and secrets; only
``InvokeMethodAsync`` goes over HTTP.  This module declares the subset of the
``dapr.proto.runtime.v1.Dapr`` service those calls need -- same package, service, method and
message names and the same field numbers as the public Dapr 1.14 protos -- and builds the
message classes from a hand-written ``FileDescriptorProto``.  ``protoc``/``grpc_tools`` are not
available in this image, and generating descriptors in code keeps the schema reviewable in one
place.

Used by ``sidecar/grpc_api.py`` (server) and ``sdk/grpc_client.py`` (client).
"""
from __future__ import annotations

from typing import Any

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

F = descriptor_pb2.FieldDescriptorProto
_T = {"string": F.TYPE_STRING, "bytes": F.TYPE_BYTES, "int32": F.TYPE_INT32, "int64": F.TYPE_INT64,
      "bool": F.TYPE_BOOL, "double": F.TYPE_DOUBLE}

COMMON = "dapr.proto.common.v1"
RUNTIME = "dapr.proto.runtime.v1"
SERVICE = f"{RUNTIME}.Dapr"

# field spec: (name, number, type, label) where type is a scalar name, "map<string,X>",
# ".pkg.Message" (message) or "enum:.pkg.Enum"; label "repeated" or "" (proto3 singular)
_COMMON_MSGS: dict[str, list[tuple]] = {
    "HTTPExtension": [("verb", 1, "enum:.dapr.proto.common.v1.HTTPExtension.Verb", ""), ("querystring", 2, "string", "")],
    "InvokeRequest": [("method", 1, "string", ""), ("data", 2, ".google.protobuf.Any", ""),
                      ("content_type", 3, "string", ""), ("http_extension", 4, ".dapr.proto.common.v1.HTTPExtension", "")],
    "InvokeResponse": [("data", 1, ".google.protobuf.Any", ""), ("content_type", 2, "string", "")],
    "Etag": [("value", 1, "string", "")],
    "StateOptions": [("concurrency", 1, "enum:.dapr.proto.common.v1.StateOptions.StateConcurrency", ""),
                     ("consistency", 2, "enum:.dapr.proto.common.v1.StateOptions.StateConsistency", "")],
    "StateItem": [("key", 1, "string", ""), ("value", 2, "bytes", ""), ("etag", 3, ".dapr.proto.common.v1.Etag", ""),
                  ("metadata", 4, "map<string,string>", ""), ("options", 5, ".dapr.proto.common.v1.StateOptions", "")],
}
_COMMON_ENUMS = {
    "HTTPExtension.Verb": ["NONE", "GET", "HEAD", "POST", "PUT", "DELETE", "CONNECT", "OPTIONS", "TRACE", "PATCH"],
    "StateOptions.StateConcurrency": ["CONCURRENCY_UNSPECIFIED", "CONCURRENCY_FIRST_WRITE", "CONCURRENCY_LAST_WRITE"],
    "StateOptions.StateConsistency": ["CONSISTENCY_UNSPECIFIED", "CONSISTENCY_EVENTUAL", "CONSISTENCY_STRONG"],
}

_C = ".dapr.proto.common.v1."
_R = ".dapr.proto.runtime.v1."
_RUNTIME_MSGS: dict[str, list[tuple]] = {
    "InvokeServiceRequest": [("id", 1, "string", ""), ("message", 3, _C + "InvokeRequest", "")],
    "GetStateRequest": [("store_name", 1, "string", ""), ("key", 2, "string", ""),
                        ("consistency", 3, "enum:" + _C + "StateOptions.StateConsistency", ""),
                        ("metadata", 4, "map<string,string>", "")],
    "GetStateResponse": [("data", 1, "bytes", ""), ("etag", 2, "string", ""), ("metadata", 3, "map<string,string>", "")],
    "GetBulkStateRequest": [("store_name", 1, "string", ""), ("keys", 2, "string", "repeated"),
                            ("parallelism", 3, "int32", ""), ("metadata", 4, "map<string,string>", "")],
    "BulkStateItem": [("key", 1, "string", ""), ("data", 2, "bytes", ""), ("etag", 3, "string", ""),
                      ("error", 4, "string", ""), ("metadata", 5, "map<string,string>", "")],
    "GetBulkStateResponse": [("items", 1, _R + "BulkStateItem", "repeated")],
    "DeleteStateRequest": [("store_name", 1, "string", ""), ("key", 2, "string", ""), ("etag", 3, _C + "Etag", ""),
                           ("options", 4, _C + "StateOptions", ""), ("metadata", 5, "map<string,string>", "")],
    "DeleteBulkStateRequest": [("store_name", 1, "string", ""), ("states", 2, _C + "StateItem", "repeated")],
    "SaveStateRequest": [("store_name", 1, "string", ""), ("states", 2, _C + "StateItem", "repeated")],
    "QueryStateRequest": [("store_name", 1, "string", ""), ("query", 2, "string", ""),
                          ("metadata", 3, "map<string,string>", "")],
    "QueryStateItem": [("key", 1, "string", ""), ("data", 2, "bytes", ""), ("etag", 3, "string", ""),
                       ("error", 4, "string", "")],
    "QueryStateResponse": [("results", 1, _R + "QueryStateItem", "repeated"), ("token", 2, "string", ""),
                           ("metadata", 3, "map<string,string>", "")],
    "TransactionalStateOperation": [("operationType", 1, "string", ""), ("request", 2, _C + "StateItem", "")],
    "ExecuteStateTransactionRequest": [("storeName", 1, "string", ""),
                                       ("operations", 2, _R + "TransactionalStateOperation", "repeated"),
                                       ("metadata", 3, "map<string,string>", "")],
    "PublishEventRequest": [("pubsub_name", 1, "string", ""), ("topic", 2, "string", ""), ("data", 3, "bytes", ""),
                            ("data_content_type", 4, "string", ""), ("metadata", 5, "map<string,string>", "")],
    "BulkPublishRequestEntry": [("entry_id", 1, "string", ""), ("event", 2, "bytes", ""),
                                ("content_type", 3, "string", ""), ("metadata", 4, "map<string,string>", "")],
    "BulkPublishRequest": [("pubsub_name", 1, "string", ""), ("topic", 2, "string", ""),
                           ("entries", 3, _R + "BulkPublishRequestEntry", "repeated"),
                           ("metadata", 4, "map<string,string>", "")],
    "BulkPublishResponseFailedEntry": [("entry_id", 1, "string", ""), ("error", 2, "string", "")],
    "BulkPublishResponse": [("failedEntries", 1, _R + "BulkPublishResponseFailedEntry", "repeated")],
    "InvokeBindingRequest": [("name", 1, "string", ""), ("data", 2, "bytes", ""),
                             ("metadata", 3, "map<string,string>", ""), ("operation", 4, "string", "")],
    "InvokeBindingResponse": [("data", 1, "bytes", ""), ("metadata", 2, "map<string,string>", "")],
    "GetSecretRequest": [("store_name", 1, "string", ""), ("key", 2, "string", ""),
                         ("metadata", 3, "map<string,string>", "")],
    "GetSecretResponse": [("data", 1, "map<string,string>", "")],
    "GetBulkSecretRequest": [("store_name", 1, "string", ""), ("metadata", 2, "map<string,string>", "")],
    "SecretResponse": [("secrets", 1, "map<string,string>", "")],
    "GetBulkSecretResponse": [("data", 1, "map<string," + _R + "SecretResponse>", "")],
    "GetMetadataRequest": [],
    "RegisteredComponents": [("name", 1, "string", ""), ("type", 2, "string", ""), ("version", 3, "string", ""),
                             ("capabilities", 4, "string", "repeated")],
    "PubsubSubscriptionRule": [("match", 1, "string", ""), ("path", 2, "string", "")],
    "PubsubSubscriptionRules": [("rules", 1, _R + "PubsubSubscriptionRule", "repeated")],
    "PubsubSubscription": [("pubsub_name", 1, "string", ""), ("topic", 2, "string", ""),
                           ("metadata", 3, "map<string,string>", ""), ("rules", 4, _R + "PubsubSubscriptionRules", ""),
                           ("dead_letter_topic", 5, "string", "")],
    "AppConnectionHealthProperties": [("health_check_path", 1, "string", ""), ("health_probe_interval", 2, "string", ""),
                                      ("health_probe_timeout", 3, "string", ""), ("health_threshold", 4, "int32", "")],
    "AppConnectionProperties": [("port", 1, "int32", ""), ("protocol", 2, "string", ""), ("channel_address", 3, "string", ""),
                                ("max_concurrency", 4, "int32", ""),
                                ("health", 5, _R + "AppConnectionHealthProperties", "")],
    "GetMetadataResponse": [("id", 1, "string", ""),
                            ("registered_components", 3, _R + "RegisteredComponents", "repeated"),
                            ("extended_metadata", 4, "map<string,string>", ""),
                            ("subscriptions", 5, _R + "PubsubSubscription", "repeated"),
                            ("app_connection_properties", 7, _R + "AppConnectionProperties", ""),
                            ("runtime_version", 8, "string", ""), ("enabled_features", 9, "string", "repeated")],
    "SetMetadataRequest": [("key", 1, "string", ""), ("value", 2, "string", "")],
    "ShutdownRequest": [],
}

# rpc name -> (request message, response message)
RPCS: dict[str, tuple[str, str]] = {
    "InvokeService": (_R + "InvokeServiceRequest", _C + "InvokeResponse"),
    "GetState": (_R + "GetStateRequest", _R + "GetStateResponse"),
    "GetBulkState": (_R + "GetBulkStateRequest", _R + "GetBulkStateResponse"),
    "SaveState": (_R + "SaveStateRequest", ".google.protobuf.Empty"),
    "QueryStateAlpha1": (_R + "QueryStateRequest", _R + "QueryStateResponse"),
    "DeleteState": (_R + "DeleteStateRequest", ".google.protobuf.Empty"),
    "DeleteBulkState": (_R + "DeleteBulkStateRequest", ".google.protobuf.Empty"),
    "ExecuteStateTransaction": (_R + "ExecuteStateTransactionRequest", ".google.protobuf.Empty"),
    "PublishEvent": (_R + "PublishEventRequest", ".google.protobuf.Empty"),
    "BulkPublishEventAlpha1": (_R + "BulkPublishRequest", _R + "BulkPublishResponse"),
    "InvokeBinding": (_R + "InvokeBindingRequest", _R + "InvokeBindingResponse"),
    "GetSecret": (_R + "GetSecretRequest", _R + "GetSecretResponse"),
    "GetBulkSecret": (_R + "GetBulkSecretRequest", _R + "GetBulkSecretResponse"),
    "GetMetadata": (_R + "GetMetadataRequest", _R + "GetMetadataResponse"),
    "SetMetadata": (_R + "SetMetadataRequest", ".google.protobuf.Empty"),
    "Shutdown": (_R + "ShutdownRequest", ".google.protobuf.Empty"),
}


def _camel(name: str) -> str:
    head, *rest = name.split("_")
    return head + "".join(p[:1].upper() + p[1:] for p in rest)


def _add_fields(msg: descriptor_pb2.DescriptorProto, fields: list[tuple]) -> None:
    for name, num, typ, label in fields:
        f = msg.field.add(name=name, number=num, json_name=_camel(name))
        f.label = F.LABEL_REPEATED if label == "repeated" else F.LABEL_OPTIONAL
        if typ.startswith("map<"):
            k, v = typ[4:-1].split(",")
            entry = msg.nested_type.add(name="".join(p[:1].upper() + p[1:] for p in name.split("_")) + "Entry")
            entry.options.map_entry = True
            entry.field.add(name="key", number=1, label=F.LABEL_OPTIONAL, type=_T[k], json_name="key")
            vf = entry.field.add(name="value", number=2, label=F.LABEL_OPTIONAL, json_name="value")
            if v in _T:
                vf.type = _T[v]
            else:
                vf.type = F.TYPE_MESSAGE
                vf.type_name = v
            f.label = F.LABEL_REPEATED
            f.type = F.TYPE_MESSAGE
            f.type_name = f".{msg.name}.{entry.name}"  # fixed up to the full name below
        elif typ.startswith("enum:"):
            f.type = F.TYPE_ENUM
            f.type_name = typ[5:]
        elif typ.startswith("."):
            f.type = F.TYPE_MESSAGE
            f.type_name = typ
        else:
            f.type = _T[typ]


def _file(name: str, package: str, msgs: dict[str, list[tuple]], enums: dict[str, list[str]],
          deps: list[str]) -> descriptor_pb2.FileDescriptorProto:
    fd = descriptor_pb2.FileDescriptorProto(name=name, package=package, syntax="proto3")
    fd.dependency.extend(deps)
    for mname, fields in msgs.items():
        m = fd.message_type.add(name=mname)
        _add_fields(m, fields)
        for f in m.field:  # map entry type names are nested in this message
            if f.type == F.TYPE_MESSAGE and f.type_name.startswith(f".{mname}.") and f.type_name.endswith("Entry"):
                f.type_name = f".{package}{f.type_name}"
    for ename, values in enums.items():
        owner, _, short = ename.rpartition(".")
        target = next(m for m in fd.message_type if m.name == owner) if owner else fd
        e = target.enum_type.add(name=short)
        for i, v in enumerate(values):
            e.value.add(name=v, number=i)
    return fd


def _build_pool() -> descriptor_pool.DescriptorPool:
    from google.protobuf import any_pb2, empty_pb2
    pool = descriptor_pool.DescriptorPool()
    for mod in (any_pb2, empty_pb2):
        fdp = descriptor_pb2.FileDescriptorProto()
        mod.DESCRIPTOR.CopyToProto(fdp)
        pool.Add(fdp)
    common = _file("tt/dapr/common.proto", COMMON, _COMMON_MSGS, _COMMON_ENUMS,
                   ["google/protobuf/any.proto"])
    pool.Add(common)
    runtime = _file("tt/dapr/runtime.proto", RUNTIME, _RUNTIME_MSGS, {},
                    ["google/protobuf/any.proto", "google/protobuf/empty.proto", "tt/dapr/common.proto"])
    svc = runtime.service.add(name="Dapr")
    for rpc, (req, resp) in RPCS.items():
        svc.method.add(name=rpc, input_type=req, output_type=resp)
    pool.Add(runtime)
    return pool


POOL = _build_pool()
_classes: dict[str, Any] = {}


def message(full_name: str) -> Any:
    """Message class by full name (``dapr.proto.runtime.v1.SaveStateRequest``)."""
    full_name = full_name.lstrip(".")
    cls = _classes.get(full_name)
    if cls is None:
        cls = message_factory.GetMessageClass(POOL.FindMessageTypeByName(full_name))
        _classes[full_name] = cls
    return cls


def rt(name: str) -> Any:
    return message(f"{RUNTIME}.{name}")


def common(name: str) -> Any:
    return message(f"{COMMON}.{name}")


def rpc_types(rpc: str) -> tuple[Any, Any]:
    req, resp = RPCS[rpc]
    return message(req), message(resp)


def method_path(rpc: str) -> str:
    return f"/{SERVICE}/{rpc}"


def verb_name(verb: int) -> str:
    return _COMMON_ENUMS["HTTPExtension.Verb"][verb]


def verb_number(name: str) -> int:
    return _COMMON_ENUMS["HTTPExtension.Verb"].index(name.upper())
