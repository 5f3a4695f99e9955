"""A protoc-style module for the Serve gRPC tests (no protoc in the image: the
descriptor is built with descriptor_pb2). Mirrors the shape of the reference's
test protos: a unary ``__call__``, a ``Multiplexing`` call and a server-streaming
``Streaming`` method on ``userdefined.UserDefinedService``."""
from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

_F = descriptor_pb2.FieldDescriptorProto
PKG = "userdefined"


def _build():
    pool = descriptor_pool.Default()
    try:
        pool.FindMessageTypeByName(f"{PKG}.UserDefinedMessage")
    except KeyError:
        f = descriptor_pb2.FileDescriptorProto(name="caamd_test_user_defined.proto", package=PKG, syntax="proto3")
        m = f.message_type.add(name="UserDefinedMessage")
        m.field.add(name="name", number=1, type=_F.TYPE_STRING, label=_F.LABEL_OPTIONAL)
        m.field.add(name="num", number=2, type=_F.TYPE_INT64, label=_F.LABEL_OPTIONAL)
        m = f.message_type.add(name="UserDefinedResponse")
        m.field.add(name="greeting", number=1, type=_F.TYPE_STRING, label=_F.LABEL_OPTIONAL)
        m.field.add(name="num_x2", number=2, type=_F.TYPE_INT64, label=_F.LABEL_OPTIONAL)
        s = f.service.add(name="UserDefinedService")
        for name, stream in (("__call__", False), ("Multiplexing", False), ("Streaming", True)):
            s.method.add(name=name, input_type=f".{PKG}.UserDefinedMessage",
                         output_type=f".{PKG}.UserDefinedResponse", server_streaming=stream)
        pool.Add(f)
    get = lambda n: message_factory.GetMessageClass(pool.FindMessageTypeByName(f"{PKG}.{n}"))  # noqa: E731
    return get("UserDefinedMessage"), get("UserDefinedResponse")


UserDefinedMessage, UserDefinedResponse = _build()


class UserDefinedServiceStub:
    def __init__(self, channel):
        base = f"/{PKG}.UserDefinedService/"
        ser, de = UserDefinedMessage.SerializeToString, UserDefinedResponse.FromString
        self.__call__ = channel.unary_unary(base + "__call__", request_serializer=ser, response_deserializer=de)
        self.Multiplexing = channel.unary_unary(base + "Multiplexing", request_serializer=ser,
                                                response_deserializer=de)
        self.Streaming = channel.unary_stream(base + "Streaming", request_serializer=ser, response_deserializer=de)


def add_UserDefinedServiceServicer_to_server(servicer, server):
    import grpc

    de, ser = UserDefinedMessage.FromString, UserDefinedResponse.SerializeToString
    handlers = {
        "__call__": grpc.unary_unary_rpc_method_handler(servicer.__call__, request_deserializer=de,
                                                        response_serializer=ser),
        "Multiplexing": grpc.unary_unary_rpc_method_handler(servicer.Multiplexing, request_deserializer=de,
                                                            response_serializer=ser),
        "Streaming": grpc.unary_stream_rpc_method_handler(servicer.Streaming, request_deserializer=de,
                                                          response_serializer=ser),
    }
    server.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(f"{PKG}.UserDefinedService", handlers),))
