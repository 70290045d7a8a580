"""kubelet PodResources v1 client and monitor-mode attribution (no GPU, no kubelet: a
gRPC PodResourcesLister on a unix socket stands in for the kubelet)."""
import os
from concurrent import futures

import grpc
import pytest

from amdvgpu.plugin import podresources as pr
from amdvgpu.plugin.config import PluginConfig
from amdvgpu.plugin.contract import build_container_response, gc_shared_dirs
from amdvgpu.plugin.devices import FakeBackend
from amdvgpu.plugin.monitor import render_metrics
from amdvgpu.plugin.vdevice import device_to_vdevices


def _resp(pods):
    """pods: [(namespace, name, [(container, {resource: [ids]})])]"""
    r = pr.ListPodResourcesResponse()
    for ns, name, ctrs in pods:
        p = r.pod_resources.add(name=name, namespace=ns)
        for cname, devs in ctrs:
            c = p.containers.add(name=cname)
            for res, ids in devs.items():
                c.devices.add(resource_name=res, device_ids=ids)
    return r


def test_wire_format_matches_the_kubelet_proto():
    """Field numbers of k8s.io/kubelet/pkg/apis/podresources/v1/api.proto, hand-encoded:
    ListPodResourcesResponse.pod_resources=1; PodResources name=1 namespace=2 containers=3;
    ContainerResources name=1 devices=2; ContainerDevices resource_name=1 device_ids=2."""
    devices = b"\x0a\x0bamd.com/gpu" + b"\x12\x02d1"
    ctr = b"\x0a\x01c" + b"\x12" + bytes([len(devices)]) + devices
    pod = b"\x0a\x01p" + b"\x12\x02ns" + b"\x1a" + bytes([len(ctr)]) + ctr
    golden = b"\x0a" + bytes([len(pod)]) + pod
    assert _resp([("ns", "p", [("c", {"amd.com/gpu": ["d1"]})])]).SerializeToString() == golden
    back = pr.ListPodResourcesResponse.FromString(golden)
    assert back.pod_resources[0].containers[0].devices[0].device_ids == ["d1"]


@pytest.fixture
def kubelet(tmp_path):
    """A PodResourcesLister on a unix socket; ``kubelet.pods`` is what List returns."""
    class K:
        pods = []
    sock = str(tmp_path / "pod-resources" / "kubelet.sock")
    os.makedirs(os.path.dirname(sock))
    srv = grpc.server(futures.ThreadPoolExecutor(max_workers=2))
    srv.add_generic_rpc_handlers((pr.lister_handler(lambda req, ctx: _resp(K.pods)),))
    srv.add_insecure_port(f"unix://{sock}")
    srv.start()
    K.socket = sock
    yield K
    srv.stop(0)


def test_list_over_the_socket(kubelet, tmp_path):
    kubelet.pods = [("ns", "a", [("main", {"amd.com/gpu": ["GPU-1-0", "GPU-2-1"], "example.com/nic": ["n0"]})]),
                    ("kube-system", "dp", [("x", {})])]
    got = pr.list_pod_resources(kubelet.socket)
    assert got[0] == {"namespace": "ns", "name": "a",
                      "containers": [{"name": "main", "devices": {"amd.com/gpu": ["GPU-1-0", "GPU-2-1"],
                                                                  "example.com/nic": ["n0"]}}]}
    assert pr.list_pod_resources(str(tmp_path / "nowhere.sock")) is None


def _monitor_cfg(tmp_path):
    cfg = PluginConfig(monitor_mode=True, vgpu_dir=str(tmp_path / "vgpu")).validate()
    devs = FakeBackend(n=2).devices()
    vds = device_to_vdevices(devs, cfg.device_split_count, 1.0, 1.0)
    return cfg, vds, {d.uuid: d for d in devs}


def test_allocate_records_the_kubelet_ids_and_attribution_corrects_a_wrong_match(kubelet, tmp_path):
    """Two pending pods with equal requests: the Allocate-time match names the older one,
    but the kubelet allocated the younger first. PodResources (the device IDs the kubelet
    assigned) names each directory's true owner; the monitor exports it."""
    cfg, vds, by = _monitor_cfg(tmp_path)
    root = os.path.join(cfg.vgpu_dir, "shared")
    # Allocate #1 (really for pod "young") was matched to "old"; #2 (for "old") to "young".
    build_container_response(cfg, [vds[0]], by, pod_tag="ns_old_main", kubelet_ids=[vds[0].id])
    build_container_response(cfg, [vds[2]], by, pod_tag="ns_young_main", kubelet_ids=[vds[2].id])
    build_container_response(cfg, [vds[1]], by, pod_tag="ns_solo_main")  # no IDs recorded
    assert pr.read_devices(os.path.join(root, "ns_old_main")) == {vds[0].id}
    kubelet.pods = [("ns", "young", [("main", {"amd.com/gpu": [vds[0].id]})]),
                    ("ns", "old", [("main", {"amd.com/gpu": [vds[2].id]})])]
    got = pr.attribute(root, pr.list_pod_resources(kubelet.socket), {"amd.com/gpu"})
    assert got["ns_old_main"] == {"namespace": "ns", "pod": "young", "container": "main",
                                  "source": "podresources", "mismatch": True}
    assert got["ns_young_main"]["pod"] == "old" and got["ns_young_main"]["mismatch"]
    assert got["ns_solo_main"] == {"namespace": "ns", "pod": "solo", "container": "main", "source": "allocate"}
    with open(os.path.join(root, "ns_old_main", pr.OWNER_FILE)) as f:
        assert f.read() == "ns/young/main\n"
    # A right match is just confirmed.
    kubelet.pods = [("ns", "old", [("main", {"amd.com/gpu": [vds[0].id]})])]
    assert pr.attribute(root, pr.list_pod_resources(kubelet.socket), {"amd.com/gpu"})["ns_old_main"] == {
        "namespace": "ns", "pod": "old", "container": "main", "source": "podresources"}
    # The monitor's info metric (a region file makes the directory a container).
    open(os.path.join(root, "ns_old_main", "x.cache"), "w").close()
    text = render_metrics(root, kubelet.socket)
    assert ('vgpu_container_info{container="ns_old_main",namespace="ns",pod="old",pod_container="main",'
            'source="podresources",mismatch="false"} 1') in text


def test_gc_keeps_directories_whose_devices_are_held(tmp_path):
    """A directory the pod list would drop (its tag names no live pod) stays while the
    kubelet reports its recorded device IDs as held by a live container."""
    import time
    root = tmp_path / "shared"
    now = time.time()
    old = now - 3 * 24 * 3600
    for tag, ids in (("ns_held_main", ["GPU-a-0"]), ("ns_gone_main", ["GPU-a-1"])):
        (root / tag).mkdir(parents=True)
        pr.write_devices(str(root / tag), ids)
        os.utime(root / tag, (old, old))
    removed = gc_shared_dirs(str(root), [], now=now, held={frozenset(["GPU-a-0"])})
    assert removed == ["ns_gone_main"] and os.listdir(root) == ["ns_held_main"]
