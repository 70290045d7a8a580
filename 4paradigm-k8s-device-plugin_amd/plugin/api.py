"""kubelet device-plugin API v1beta1, built at runtime (no protoc in this environment).

Wire contract: ``k8s.io/kubelet/pkg/apis/deviceplugin/v1beta1/api.proto`` (reference
vendor tree, ``api.proto:23-211``) and ``constants.go:19-37``. The message and service
definitions below use exactly the same package, names, field numbers and types, so the
bytes on the wire are identical to what the kubelet's gogo-generated code produces and
consumes (pinned by ``tests/test_plugin_api.py`` against hand-encoded golden bytes).

Exports message classes (``Device``, ``AllocateRequest``, ...), the gRPC method paths,
server-side handler builders and thin client stubs for both services
(``Registration`` served by the kubelet, ``DevicePlugin`` served by us).
"""
import grpc
from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

VERSION = "v1beta1"
HEALTHY = "Healthy"
UNHEALTHY = "Unhealthy"
DEVICE_PLUGIN_PATH = "/var/lib/kubelet/device-plugins/"
KUBELET_SOCKET = DEVICE_PLUGIN_PATH + "kubelet.sock"
PRE_START_CONTAINER_TIMEOUT_S = 30
SUPPORTED_VERSIONS = (VERSION,)

_F = descriptor_pb2.FieldDescriptorProto
_STR, _BOOL, _I32, _I64, _MSG = _F.TYPE_STRING, _F.TYPE_BOOL, _F.TYPE_INT32, _F.TYPE_INT64, _F.TYPE_MESSAGE
_OPT, _REP = _F.LABEL_OPTIONAL, _F.LABEL_REPEATED

# name -> [(field, number, type, label, message type name or None)]
_MESSAGES = {
    "DevicePluginOptions": [("pre_start_required", 1, _BOOL, _OPT, None),
                            ("get_preferred_allocation_available", 2, _BOOL, _OPT, None)],
    "RegisterRequest": [("version", 1, _STR, _OPT, None), ("endpoint", 2, _STR, _OPT, None),
                        ("resource_name", 3, _STR, _OPT, None), ("options", 4, _MSG, _OPT, "DevicePluginOptions")],
    "Empty": [],
    "ListAndWatchResponse": [("devices", 1, _MSG, _REP, "Device")],
    "TopologyInfo": [("nodes", 1, _MSG, _REP, "NUMANode")],
    "NUMANode": [("ID", 1, _I64, _OPT, None)],
    "Device": [("ID", 1, _STR, _OPT, None), ("health", 2, _STR, _OPT, None),
               ("topology", 3, _MSG, _OPT, "TopologyInfo")],
    "PreStartContainerRequest": [("devicesIDs", 1, _STR, _REP, None)],
    "PreStartContainerResponse": [],
    "PreferredAllocationRequest": [("container_requests", 1, _MSG, _REP, "ContainerPreferredAllocationRequest")],
    "ContainerPreferredAllocationRequest": [("available_deviceIDs", 1, _STR, _REP, None),
                                            ("must_include_deviceIDs", 2, _STR, _REP, None),
                                            ("allocation_size", 3, _I32, _OPT, None)],
    "PreferredAllocationResponse": [("container_responses", 1, _MSG, _REP, "ContainerPreferredAllocationResponse")],
    "ContainerPreferredAllocationResponse": [("deviceIDs", 1, _STR, _REP, None)],
    "AllocateRequest": [("container_requests", 1, _MSG, _REP, "ContainerAllocateRequest")],
    "ContainerAllocateRequest": [("devicesIDs", 1, _STR, _REP, None)],
    "AllocateResponse": [("container_responses", 1, _MSG, _REP, "ContainerAllocateResponse")],
    "ContainerAllocateResponse": [("envs", 1, "map", _REP, None), ("mounts", 2, _MSG, _REP, "Mount"),
                                  ("devices", 3, _MSG, _REP, "DeviceSpec"), ("annotations", 4, "map", _REP, None)],
    "Mount": [("container_path", 1, _STR, _OPT, None), ("host_path", 2, _STR, _OPT, None),
              ("read_only", 3, _BOOL, _OPT, None)],
    "DeviceSpec": [("container_path", 1, _STR, _OPT, None), ("host_path", 2, _STR, _OPT, None),
                   ("permissions", 3, _STR, _OPT, None)],
}

# service -> [(method, request, response, server_streaming)]
_SERVICES = {
    "Registration": [("Register", "RegisterRequest", "Empty", False)],
    "DevicePlugin": [("GetDevicePluginOptions", "Empty", "DevicePluginOptions", False),
                     ("ListAndWatch", "Empty", "ListAndWatchResponse", True),
                     ("GetPreferredAllocation", "PreferredAllocationRequest", "PreferredAllocationResponse", False),
                     ("Allocate", "AllocateRequest", "AllocateResponse", False),
                     ("PreStartContainer", "PreStartContainerRequest", "PreStartContainerResponse", False)],
}


def _camel(name):
    return "".join(p[:1].upper() + p[1:] for p in name.split("_"))


def _build_file():
    fd = descriptor_pb2.FileDescriptorProto(name="amdvgpu/deviceplugin/v1beta1/api.proto", package=VERSION,
                                            syntax="proto3")
    for mname, fields in _MESSAGES.items():
        m = fd.message_type.add(name=mname)
        for fname, num, ftype, label, tname in fields:
            if ftype == "map":
                entry = m.nested_type.add(name=_camel(fname) + "Entry")
                entry.options.map_entry = True
                entry.field.add(name="key", number=1, type=_STR, label=_OPT, json_name="key")
                entry.field.add(name="value", number=2, type=_STR, label=_OPT, json_name="value")
                m.field.add(name=fname, number=num, type=_MSG, label=_REP,
                            type_name=f".{VERSION}.{mname}.{entry.name}")
            else:
                f = m.field.add(name=fname, number=num, type=ftype, label=label)
                if tname:
                    f.type_name = f".{VERSION}.{tname}"
    for sname, methods in _SERVICES.items():
        s = fd.service.add(name=sname)
        for meth, req, resp, stream in methods:
            s.method.add(name=meth, input_type=f".{VERSION}.{req}", output_type=f".{VERSION}.{resp}",
                         server_streaming=stream)
    return fd


POOL = descriptor_pool.DescriptorPool()
FILE = POOL.Add(_build_file())
_FD = POOL.FindFileByName("amdvgpu/deviceplugin/v1beta1/api.proto")

_classes = {}
for _name in _MESSAGES:
    _classes[_name] = message_factory.GetMessageClass(_FD.message_types_by_name[_name])
globals().update(_classes)

DevicePluginOptions = _classes["DevicePluginOptions"]
RegisterRequest = _classes["RegisterRequest"]
Empty = _classes["Empty"]
ListAndWatchResponse = _classes["ListAndWatchResponse"]
TopologyInfo = _classes["TopologyInfo"]
NUMANode = _classes["NUMANode"]
Device = _classes["Device"]
PreStartContainerRequest = _classes["PreStartContainerRequest"]
PreStartContainerResponse = _classes["PreStartContainerResponse"]
PreferredAllocationRequest = _classes["PreferredAllocationRequest"]
ContainerPreferredAllocationRequest = _classes["ContainerPreferredAllocationRequest"]
PreferredAllocationResponse = _classes["PreferredAllocationResponse"]
ContainerPreferredAllocationResponse = _classes["ContainerPreferredAllocationResponse"]
AllocateRequest = _classes["AllocateRequest"]
ContainerAllocateRequest = _classes["ContainerAllocateRequest"]
AllocateResponse = _classes["AllocateResponse"]
ContainerAllocateResponse = _classes["ContainerAllocateResponse"]
Mount = _classes["Mount"]
DeviceSpec = _classes["DeviceSpec"]


def method_path(service, method):
    return f"/{VERSION}.{service}/{method}"


def _handler(fn, req, resp, stream):
    des, ser = _classes[req].FromString, _classes[resp].SerializeToString
    if stream:
        return grpc.unary_stream_rpc_method_handler(fn, request_deserializer=des, response_serializer=ser)
    return grpc.unary_unary_rpc_method_handler(fn, request_deserializer=des, response_serializer=ser)


def service_handler(service, impl):
    """Generic gRPC handler for ``service`` whose methods are attributes of ``impl``."""
    handlers = {}
    for meth, req, resp, stream in _SERVICES[service]:
        handlers[meth] = _handler(getattr(impl, meth), req, resp, stream)
    return grpc.method_handlers_generic_handler(f"{VERSION}.{service}", handlers)


class Stub:
    """Client stub for ``service`` over ``channel`` (methods named as in the proto)."""

    def __init__(self, channel, service):
        for meth, req, resp, stream in _SERVICES[service]:
            ser, des = _classes[req].SerializeToString, _classes[resp].FromString
            mk = channel.unary_stream if stream else channel.unary_unary
            setattr(self, meth, mk(method_path(service, meth), request_serializer=ser, response_deserializer=des))


def registration_stub(channel):
    return Stub(channel, "Registration")


def device_plugin_stub(channel):
    return Stub(channel, "DevicePlugin")


def unix_target(path):
    return f"unix://{path}" if not path.startswith("unix:") else path
