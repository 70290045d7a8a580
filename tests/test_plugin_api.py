"""Wire compatibility of the runtime-built v1beta1 protos (no protoc available).

Golden bytes are hand-encoded from the field numbers/types of the kubelet's api.proto
(reference vendor/k8s.io/kubelet/pkg/apis/deviceplugin/v1beta1/api.proto:23-211), so a
wrong field number or type fails here rather than against a real kubelet.
"""
from amdvgpu.plugin import api


def tag(field, wire):
    return bytes([(field << 3) | wire])


def ld(field, payload):
    return tag(field, 2) + bytes([len(payload)]) + payload


def test_device_golden():
    d = api.Device(ID="GPU-1-0", health=api.HEALTHY, topology=api.TopologyInfo(nodes=[api.NUMANode(ID=1)]))
    want = ld(1, b"GPU-1-0") + ld(2, b"Healthy") + ld(3, ld(1, tag(1, 0) + b"\x01"))
    assert d.SerializeToString() == want
    assert api.Device.FromString(want) == d


def test_register_request_golden():
    r = api.RegisterRequest(version="v1beta1", endpoint="amd-vgpu.sock", resource_name="amd.com/gpu",
                            options=api.DevicePluginOptions(get_preferred_allocation_available=True))
    want = (ld(1, b"v1beta1") + ld(2, b"amd-vgpu.sock") + ld(3, b"amd.com/gpu") + ld(4, tag(2, 0) + b"\x01"))
    assert r.SerializeToString() == want


def test_allocate_response_golden():
    c = api.ContainerAllocateResponse()
    c.envs["K"] = "V"
    c.mounts.add(container_path="/c", host_path="/h", read_only=True)
    c.devices.add(container_path="/dev/kfd", host_path="/dev/kfd", permissions="rw")
    c.annotations["a"] = "b"
    want = (ld(1, ld(1, b"K") + ld(2, b"V")) + ld(2, ld(1, b"/c") + ld(2, b"/h") + tag(3, 0) + b"\x01")
            + ld(3, ld(1, b"/dev/kfd") + ld(2, b"/dev/kfd") + ld(3, b"rw")) + ld(4, ld(1, b"a") + ld(2, b"b")))
    assert c.SerializeToString() == want
    r = api.AllocateResponse(container_responses=[c])
    assert r.SerializeToString() == ld(1, want)


def test_preferred_allocation_golden():
    r = api.PreferredAllocationRequest(container_requests=[api.ContainerPreferredAllocationRequest(
        available_deviceIDs=["a", "b"], must_include_deviceIDs=["a"], allocation_size=2)])
    inner = ld(1, b"a") + ld(1, b"b") + ld(2, b"a") + tag(3, 0) + b"\x02"
    assert r.SerializeToString() == ld(1, inner)
    resp = api.PreferredAllocationResponse(container_responses=[api.ContainerPreferredAllocationResponse(
        deviceIDs=["x"])])
    assert resp.SerializeToString() == ld(1, ld(1, b"x"))


def test_allocate_request_and_prestart_golden():
    r = api.AllocateRequest(container_requests=[api.ContainerAllocateRequest(devicesIDs=["d0", "d1"])])
    assert r.SerializeToString() == ld(1, ld(1, b"d0") + ld(1, b"d1"))
    p = api.PreStartContainerRequest(devicesIDs=["d0"])
    assert p.SerializeToString() == ld(1, b"d0")
    assert api.Empty().SerializeToString() == b""


def test_constants():
    assert api.VERSION == "v1beta1"
    assert api.KUBELET_SOCKET == "/var/lib/kubelet/device-plugins/kubelet.sock"
    assert api.method_path("DevicePlugin", "ListAndWatch") == "/v1beta1.DevicePlugin/ListAndWatch"
    assert api.method_path("Registration", "Register") == "/v1beta1.Registration/Register"
