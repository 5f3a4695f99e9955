"""Messages / service of Serve's built-in gRPC API (reference: src/ray/protobuf/
serve.proto ``RayServeAPIService``: ``ListApplications`` and ``Healthz``).

There is no ``protoc`` in this image, so the descriptor is built with
``descriptor_pb2`` at import time and registered in the default pool — the
result is the same as a generated ``*_pb2`` module: real protobuf message
classes (wire-compatible with the reference's messages), a client stub and an
``add_RayServeAPIServiceServicer_to_server`` function.
"""
from __future__ import annotations

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

PACKAGE = "ray.serve"
SERVICE = "RayServeAPIService"


def _build():
    pool = descriptor_pool.Default()
    try:
        pool.FindMessageTypeByName(f"{PACKAGE}.ListApplicationsRequest")
    except KeyError:
        f = descriptor_pb2.FileDescriptorProto(name="caamd_serve_api.proto", package=PACKAGE, syntax="proto3")
        f.message_type.add(name="ListApplicationsRequest")
        m = f.message_type.add(name="ListApplicationsResponse")
        m.field.add(name="application_names", number=1, type=descriptor_pb2.FieldDescriptorProto.TYPE_STRING,
                    label=descriptor_pb2.FieldDescriptorProto.LABEL_REPEATED)
        f.message_type.add(name="HealthzRequest")
        m = f.message_type.add(name="HealthzResponse")
        m.field.add(name="message", number=1, type=descriptor_pb2.FieldDescriptorProto.TYPE_STRING,
                    label=descriptor_pb2.FieldDescriptorProto.LABEL_OPTIONAL)
        s = f.service.add(name=SERVICE)
        s.method.add(name="ListApplications", input_type=f".{PACKAGE}.ListApplicationsRequest",
                     output_type=f".{PACKAGE}.ListApplicationsResponse")
        s.method.add(name="Healthz", input_type=f".{PACKAGE}.HealthzRequest",
                     output_type=f".{PACKAGE}.HealthzResponse")
        pool.Add(f)
    get = lambda n: message_factory.GetMessageClass(pool.FindMessageTypeByName(f"{PACKAGE}.{n}"))  # noqa: E731
    return (get("ListApplicationsRequest"), get("ListApplicationsResponse"), get("HealthzRequest"),
            get("HealthzResponse"))


ListApplicationsRequest, ListApplicationsResponse, HealthzRequest, HealthzResponse = _build()


class RayServeAPIServiceStub:
    def __init__(self, channel):
        base = f"/{PACKAGE}.{SERVICE}/"
        self.ListApplications = channel.unary_unary(
            base + "ListApplications", request_serializer=ListApplicationsRequest.SerializeToString,
            response_deserializer=ListApplicationsResponse.FromString)
        self.Healthz = channel.unary_unary(
            base + "Healthz", request_serializer=HealthzRequest.SerializeToString,
            response_deserializer=HealthzResponse.FromString)


def add_RayServeAPIServiceServicer_to_server(servicer, server):
    import grpc

    handlers = {
        "ListApplications": grpc.unary_unary_rpc_method_handler(
            servicer.ListApplications, request_deserializer=ListApplicationsRequest.FromString,
            response_serializer=ListApplicationsResponse.SerializeToString),
        "Healthz": grpc.unary_unary_rpc_method_handler(
            servicer.Healthz, request_deserializer=HealthzRequest.FromString,
            response_serializer=HealthzResponse.SerializeToString),
    }
    server.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(f"{PACKAGE}.{SERVICE}", handlers),))
