"""kubelet PodResources API v1 (``List``) and monitor-mode attribution of container
directories to the pods that really hold their vGPUs.

The kubelet's ``Allocate`` carries only device IDs, so in monitor mode the plugin guesses
the pod and container an allocation is for (``k8s.PodMatcher``: the next unallocated GPU
containers of the oldest pending pod with that request; the reference does the same with
the whole pod, ``server.go:381-405``). Two pending pods with equal requests make that guess
ambiguous, and the kubelet is free to allocate the younger one first. Once the container
exists the kubelet knows the answer: its PodResources service (``/var/lib/kubelet/
pod-resources/kubelet.sock``, GA since Kubernetes 1.20) lists, per pod and container, the
device IDs of every extended resource. The contract writes the allocated IDs into the
container's host directory (``.devices``); ``attribute`` matches them against ``List``
and names the directory's true owner, which the monitor exports and garbage collection
trusts. The reference has no such check (monitor mode).

Wire contract: ``k8s.io/kubelet/pkg/apis/podresources/v1/api.proto`` (package ``v1``,
service ``PodResourcesLister``); built at runtime like ``api.py``, same field numbers.
"""
import os

import grpc
from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

from .api import unix_target

PACKAGE = "v1"
SOCKET = "/var/lib/kubelet/pod-resources/kubelet.sock"
DEVICES_FILE = ".devices"
OWNER_FILE = ".owner"

_F = descriptor_pb2.FieldDescriptorProto
_STR, _I64, _MSG = _F.TYPE_STRING, _F.TYPE_INT64, _F.TYPE_MESSAGE
_OPT, _REP = _F.LABEL_OPTIONAL, _F.LABEL_REPEATED

_MESSAGES = {
    "ListPodResourcesRequest": [],
    "ListPodResourcesResponse": [("pod_resources", 1, _MSG, _REP, "PodResources")],
    "PodResources": [("name", 1, _STR, _OPT, None), ("namespace", 2, _STR, _OPT, None),
                     ("containers", 3, _MSG, _REP, "ContainerResources")],
    "ContainerResources": [("name", 1, _STR, _OPT, None), ("devices", 2, _MSG, _REP, "ContainerDevices"),
                           ("cpu_ids", 3, _I64, _REP, None)],
    "ContainerDevices": [("resource_name", 1, _STR, _OPT, None), ("device_ids", 2, _STR, _REP, None),
                         ("topology", 3, _MSG, _OPT, "TopologyInfo")],
    "TopologyInfo": [("nodes", 1, _MSG, _REP, "NUMANode")],
    "NUMANode": [("ID", 1, _I64, _OPT, None)],
}


def _build():
    fd = descriptor_pb2.FileDescriptorProto(name="amdvgpu/podresources/v1/api.proto", package=PACKAGE,
                                            syntax="proto3")
    for mname, fields in _MESSAGES.items():
        m = fd.message_type.add(name=mname)
        for fname, num, ftype, label, tname in fields:
            f = m.field.add(name=fname, number=num, type=ftype, label=label)
            if tname:
                f.type_name = f".{PACKAGE}.{tname}"
    s = fd.service.add(name="PodResourcesLister")
    s.method.add(name="List", input_type=f".{PACKAGE}.ListPodResourcesRequest",
                 output_type=f".{PACKAGE}.ListPodResourcesResponse")
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    fdesc = pool.FindFileByName(fd.name)
    return {n: message_factory.GetMessageClass(fdesc.message_types_by_name[n]) for n in _MESSAGES}


_classes = _build()
ListPodResourcesRequest = _classes["ListPodResourcesRequest"]
ListPodResourcesResponse = _classes["ListPodResourcesResponse"]
PodResources = _classes["PodResources"]
ContainerResources = _classes["ContainerResources"]
ContainerDevices = _classes["ContainerDevices"]
LIST_METHOD = f"/{PACKAGE}.PodResourcesLister/List"


def lister_handler(list_fn):
    """gRPC handler serving ``List`` with ``list_fn(request, context)`` (the stub kubelet)."""
    h = grpc.unary_unary_rpc_method_handler(list_fn, request_deserializer=ListPodResourcesRequest.FromString,
                                            response_serializer=ListPodResourcesResponse.SerializeToString)
    return grpc.method_handlers_generic_handler(f"{PACKAGE}.PodResourcesLister", {"List": h})


def list_pod_resources(socket=SOCKET, timeout=2.0):
    """[{namespace, name, containers: [{name, devices: {resource: [ids]}}]}] from the
    kubelet, or None when the service is not reachable."""
    if not os.path.exists(socket):
        return None
    try:
        with grpc.insecure_channel(unix_target(socket)) as ch:
            call = ch.unary_unary(LIST_METHOD, request_serializer=ListPodResourcesRequest.SerializeToString,
                                  response_deserializer=ListPodResourcesResponse.FromString)
            resp = call(ListPodResourcesRequest(), timeout=timeout)
    except grpc.RpcError:
        return None
    out = []
    for p in resp.pod_resources:
        ctrs = []
        for c in p.containers:
            devs = {}
            for d in c.devices:
                devs.setdefault(d.resource_name, []).extend(d.device_ids)
            ctrs.append({"name": c.name, "devices": devs})
        out.append({"namespace": p.namespace, "name": p.name, "containers": ctrs})
    return out


def write_devices(host_dir, ids):
    """Records the device IDs an Allocate gave the container owning ``host_dir``."""
    tmp = os.path.join(host_dir, DEVICES_FILE + ".tmp")
    with open(tmp, "w") as f:
        f.write("".join(f"{i}\n" for i in sorted(ids)))
    os.replace(tmp, os.path.join(host_dir, DEVICES_FILE))


def read_devices(host_dir):
    try:
        with open(os.path.join(host_dir, DEVICES_FILE)) as f:
            return frozenset(x.strip() for x in f if x.strip())
    except OSError:
        return None


def attribute(root, pods, resources):
    """{tag: owner} for the container directories under ``root``.

    ``owner`` is {"namespace", "pod", "container", "source"}: ``source`` "podresources" when
    a container of ``pods`` (a ``list_pod_resources`` result) holds exactly the directory's
    recorded device IDs of one of ``resources``, else "allocate" (the tag the plugin gave
    the directory at Allocate, split back into namespace / pod / container). A directory
    whose devices PodResources attributes to another pod than its tag names also gets
    ``"mismatch": True`` and an ``.owner`` file, so the mistake is visible on the node."""
    held = {}
    for p in pods or []:
        for c in p["containers"]:
            for res, ids in c["devices"].items():
                if res in resources and ids:
                    held[frozenset(ids)] = (p["namespace"], p["name"], c["name"])
    out = {}
    try:
        tags = sorted(os.listdir(root))
    except OSError:
        return out
    for tag in tags:
        d = os.path.join(root, tag)
        if not os.path.isdir(d):
            continue
        parts = tag.split("_")
        guess = tuple(parts) if len(parts) == 3 else ("", "_".join(parts[:-1]), parts[-1])
        ids = read_devices(d)
        who = held.get(ids) if ids else None
        if who is None:
            out[tag] = {"namespace": guess[0], "pod": guess[1], "container": guess[2], "source": "allocate"}
            continue
        owner = {"namespace": who[0], "pod": who[1], "container": who[2], "source": "podresources"}
        if who != guess:
            owner["mismatch"] = True
            try:
                with open(os.path.join(d, OWNER_FILE), "w") as f:
                    f.write(f"{who[0]}/{who[1]}/{who[2]}\n")
            except OSError:
                pass
        out[tag] = owner
    return out
