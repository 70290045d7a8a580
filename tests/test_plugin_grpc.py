"""Control plane end to end against a stub kubelet over unix sockets (BASELINE.json
config 1: ListAndWatch/Allocate with 2 fake devices, no GPU)."""
import os
import threading
import time

import pytest

from amdvgpu.plugin import api
from amdvgpu.plugin.config import PluginConfig
from amdvgpu.plugin.devices import FakeBackend
from amdvgpu.plugin.kubelet_stub import StubKubelet
from amdvgpu.plugin.main import Supervisor


@pytest.fixture
def plugin_dir(tmp_path):
    d = tmp_path / "dp"
    d.mkdir()
    return str(d)


def start(plugin_dir, backend=None, **kw):
    cfg = PluginConfig(device_plugin_path=plugin_dir + "/", backend="fake", health_interval_s=0.1,
                       vgpu_dir=os.path.join(os.path.dirname(plugin_dir), "vgpu"), **kw).validate()
    kubelet = StubKubelet(plugin_dir).start()
    sup = Supervisor(cfg, backend=backend or FakeBackend(n=2), install_signals=False)
    stop = threading.Event()
    th = threading.Thread(target=sup.run, args=(stop,), daemon=True)
    th.start()
    return cfg, kubelet, sup, stop, th


def shutdown(kubelet, stop, th):
    stop.set()
    th.join(timeout=10)
    kubelet.stop()


def test_register_list_and_allocate(plugin_dir):
    cfg, k, sup, stop, th = start(plugin_dir, device_split_count=2)
    try:
        reg = k.wait_registered("amd.com/gpu")
        assert reg.version == "v1beta1" and reg.endpoint == "amd-vgpu.sock"
        assert reg.options.get_preferred_allocation_available
        devs = k.wait_devices("amd.com/gpu", predicate=lambda d: len(d) == 4)
        assert all(h == api.HEALTHY for h in devs.values())
        ids, resp = k.allocate("amd.com/gpu", 1)
        envs = dict(resp.envs)
        uuid = ids[0].rsplit("-", 1)[0]
        assert envs["ROCR_VISIBLE_DEVICES"] == uuid
        assert envs["VGPU_DEVICE_MAP"] == f"0:{uuid}"
        total = FakeBackend(n=2).devices()[0].memory_total >> 20
        assert envs["VGPU_DEVICE_MEMORY_LIMIT_0"] == f"{total // 2}m"
        assert envs["VGPU_DEVICE_CU_LIMIT_0"] == "50"
        # the region: a file the plugin created, mounted over its path in the container
        region = envs["VGPU_SHARED_CACHE"]
        assert region.startswith("/usr/local/vgpu/regions/") and region.endswith(".cache")
        assert "VGPU_OVERSUBSCRIBE" not in envs
        mounts = {m.container_path: (m.host_path, m.read_only) for m in resp.mounts}
        assert mounts[region] == (os.path.join(cfg.vgpu_dir, "regions", os.path.basename(region)), False)
        assert os.path.isfile(mounts[region][0])
        assert mounts["/usr/local/vgpu/libvgpu_hip.so"] == (os.path.join(cfg.vgpu_dir, "libvgpu_hip.so"), True)
        assert mounts["/etc/ld.so.preload"] == (os.path.join(cfg.vgpu_dir, "ld.so.preload"), True)
        # the plugin-owned limits file (read-only): the ceiling the shim enforces
        assert envs["VGPU_LIMITS_FILE"] == "/vgpu/limits" and mounts["/vgpu/limits"][1] is True
        limits = dict(l.split("=", 1) for l in open(mounts["/vgpu/limits"][0]).read().splitlines())
        assert limits["VGPU_DEVICE_MEMORY_LIMIT_0"] == f"{total // 2}m" and limits["VGPU_SHARED_CACHE"] == region
        assert limits["VGPU_TASK_PRIORITY_MIN"] == "1"
        assert limits["VGPU_REGION_INODE"] == str(os.stat(mounts[region][0]).st_ino)
        specs = [d.container_path for d in resp.devices]
        assert specs[0] == "/dev/kfd" and any(p.startswith("/dev/dri/renderD") for p in specs)
        # second vGPU on the other slot of some GPU gets a disjoint CU range
        ids2, resp2 = k.allocate("amd.com/gpu", 1)
        assert ids2 != ids
    finally:
        shutdown(k, stop, th)


def test_multi_gpu_request_spreads_over_gpus(plugin_dir):
    cfg, k, sup, stop, th = start(plugin_dir, device_split_count=2, backend=FakeBackend(n=4, topology="xgmi"))
    try:
        k.wait_registered("amd.com/gpu")
        k.wait_devices("amd.com/gpu", predicate=lambda d: len(d) == 8)
        ids, resp = k.allocate("amd.com/gpu", 2)
        uuids = {i.rsplit("-", 1)[0] for i in ids}
        assert len(uuids) == 2
        envs = dict(resp.envs)
        assert len(envs["ROCR_VISIBLE_DEVICES"].split(",")) == 2
        assert "VGPU_DEVICE_MEMORY_LIMIT_1" in envs
    finally:
        shutdown(k, stop, th)


def test_health_unhealthy_then_recovered(plugin_dir):
    be = FakeBackend(n=2)
    cfg, k, sup, stop, th = start(plugin_dir, backend=be)
    try:
        k.wait_registered("amd.com/gpu")
        k.wait_devices("amd.com/gpu", predicate=lambda d: len(d) == 4)
        bad = be.devices()[1].uuid
        be.inject(bad, False, "GPU_PRE_RESET")
        devs = k.wait_devices("amd.com/gpu", predicate=lambda d: sum(h == api.UNHEALTHY for h in d.values()) == 2)
        assert {i for i, h in devs.items() if h == api.UNHEALTHY} == {f"{bad}-0", f"{bad}-1"}
        be.inject(bad, True, "GPU_POST_RESET")
        k.wait_devices("amd.com/gpu", predicate=lambda d: all(h == api.HEALTHY for h in d.values()))
    finally:
        shutdown(k, stop, th)


def test_healthchecks_disabled(plugin_dir, monkeypatch):
    be = FakeBackend(n=1)
    cfg, k, sup, stop, th = start(plugin_dir, backend=be, disable_healthchecks="all")
    try:
        k.wait_registered("amd.com/gpu")
        k.wait_devices("amd.com/gpu")
        be.inject(be.devices()[0].uuid, False, "x")
        time.sleep(0.5)
        assert all(h == api.HEALTHY for h in k.devices["amd.com/gpu"].values())
    finally:
        shutdown(k, stop, th)


def test_kubelet_restart_triggers_reregistration(plugin_dir):
    cfg, k, sup, stop, th = start(plugin_dir)
    try:
        k.wait_registered("amd.com/gpu")
        n0 = sup.restarts
        k.restart()  # re-creates kubelet.sock
        k.wait_registered("amd.com/gpu", timeout=15)
        # The kubelet records the registration before Supervisor.start_plugins returns
        # and counts the restart; give the supervisor thread a moment to finish it.
        deadline = time.time() + 10
        while sup.restarts <= n0 and time.time() < deadline:
            time.sleep(0.05)
        assert sup.restarts > n0
        k.wait_devices("amd.com/gpu")
    finally:
        shutdown(k, stop, th)


def test_unknown_device_rejected(plugin_dir):
    import grpc
    cfg, k, sup, stop, th = start(plugin_dir)
    try:
        k.wait_registered("amd.com/gpu")
        stub = k.stub_for("amd.com/gpu")
        with pytest.raises(grpc.RpcError) as e:
            stub.Allocate(api.AllocateRequest(container_requests=[api.ContainerAllocateRequest(devicesIDs=["x"])]))
        assert e.value.code() == grpc.StatusCode.INVALID_ARGUMENT
        assert isinstance(stub.PreStartContainer(api.PreStartContainerRequest()), api.PreStartContainerResponse)
    finally:
        shutdown(k, stop, th)


def test_mixed_partition_strategy(plugin_dir):
    class Mixed(FakeBackend):
        def __init__(self):
            super().__init__(n=1)
            part = FakeBackend(n=1, partitions_per_gpu=4, compute_partition="CPX", uuid_prefix="GPU-cafe").devices()
            for i, p in enumerate(part):
                p.index = 1 + i
                p.memory_partition = "NPS2"
            self._devs = self._devs + part

    cfg, k, sup, stop, th = start(plugin_dir, backend=Mixed(), partition_strategy="mixed")
    try:
        k.wait_registered("amd.com/gpu")
        reg = k.wait_registered("amd.com/cpx-nps2")
        assert reg.endpoint == "amd-cpx-nps2.sock"
        assert not reg.options.get_preferred_allocation_available
        devs = k.wait_devices("amd.com/cpx-nps2", predicate=lambda d: len(d) == 4)
        ids, resp = k.allocate("amd.com/cpx-nps2", 1)
        envs = dict(resp.envs)
        assert "VGPU_DEVICE_MEMORY_LIMIT_0" not in envs and "ROCR_VISIBLE_DEVICES" in envs
        assert len(k.wait_devices("amd.com/gpu")) == 2
    finally:
        shutdown(k, stop, th)


def test_eight_gpu_node_advertises_32_vgpus(plugin_dir):
    """BASELINE config 5 control-plane half: an 8xMI355X node (xGMI all-to-all, two NUMA
    nodes) split 4-way advertises 32 vGPUs; 4-vGPU requests land on 4 distinct GPUs of one
    NUMA node, 8 such pods exhaust the node without double-booking a vGPU."""
    be = FakeBackend(n=8, topology="xgmi", numa_split=4)
    cfg, k, sup, stop, th = start(plugin_dir, backend=be, device_split_count=4)
    try:
        k.wait_registered("amd.com/gpu")
        devs = k.wait_devices("amd.com/gpu", predicate=lambda d: len(d) == 32)
        assert len(devs) == 32
        numa = {d.uuid: d.numa_node for d in be.devices()}
        seen = set()
        for _ in range(8):
            ids, resp = k.allocate("amd.com/gpu", 4)
            assert not (set(ids) & seen)
            seen |= set(ids)
            gpus = {i.rsplit("-", 1)[0] for i in ids}
            if len(gpus) == 4:
                assert len({numa[g] for g in gpus}) == 1
        assert len(seen) == 32
        with pytest.raises(RuntimeError):
            k.allocate("amd.com/gpu", 1)
    finally:
        shutdown(k, stop, th)


def test_grpc_server_watchdog_restarts_and_budget(plugin_dir, monkeypatch):
    """Socket deleted under the plugin -> served again and re-registered; more than 5
    restarts within the hour -> fatal, the supervisor exits (server.go:180-207)."""
    from amdvgpu.plugin import server
    monkeypatch.setattr(server, "WATCHDOG_PERIOD_S", 0.1)  # from the first tick on
    cfg, k, sup, stop, th = start(plugin_dir)
    try:
        k.wait_registered("amd.com/gpu")
        p = sup.plugins[0]
        n0 = len(k.registrations)
        os.unlink(p.socket)
        k.wait_registered("amd.com/gpu", count=n0 + 1, timeout=15)
        assert os.path.exists(p.socket)
        p._restarts = [time.monotonic()] * 5  # budget already spent this hour
        os.unlink(p.socket)
        th.join(timeout=20)
        assert not th.is_alive() and p.fatal
    finally:
        shutdown(k, stop, th)


def test_stop_honoured_while_the_kubelet_is_down(plugin_dir):
    """No kubelet socket: registration keeps failing and is retried every second, but a
    stop request (or a signal) still ends the supervisor promptly."""
    cfg = PluginConfig(device_plugin_path=plugin_dir + "/", backend="fake", health_interval_s=0.1,
                       vgpu_dir=os.path.join(os.path.dirname(plugin_dir), "vgpu")).validate()
    sup = Supervisor(cfg, backend=FakeBackend(n=1), install_signals=False)
    stop = threading.Event()
    th = threading.Thread(target=sup.run, args=(stop,), daemon=True)
    th.start()
    time.sleep(2.5)
    assert th.is_alive() and sup.restarts == 0   # still retrying
    stop.set()
    th.join(timeout=10)   # at most one registration attempt (dial timeouts) in flight
    assert not th.is_alive()


def test_duplicate_vgpus_rejected_on_request(plugin_dir):
    """--duplicate-vgpus=reject: two vGPUs of one GPU in one container fail Allocate with a
    clear error (the container would otherwise see one device with the summed share)."""
    import grpc
    cfg, k, sup, stop, th = start(plugin_dir, device_split_count=4, backend=FakeBackend(n=1),
                                  duplicate_vgpus="reject")
    try:
        k.wait_registered("amd.com/gpu")
        devs = k.wait_devices("amd.com/gpu", predicate=lambda d: len(d) == 4)
        ids = sorted(devs)[:2]
        with pytest.raises(grpc.RpcError) as e:
            k.allocate_ids("amd.com/gpu", ids)
        assert e.value.code() == grpc.StatusCode.INVALID_ARGUMENT
        assert "several vGPUs of one GPU" in e.value.details() and "--duplicate-vgpus=split" in e.value.details()
    finally:
        shutdown(k, stop, th)


def test_duplicate_vgpus_split_into_separate_devices(plugin_dir):
    """--duplicate-vgpus=split: the same two-vGPU pod on a one-GPU node gets both vGPUs as
    separate devices - the map names the GPU twice with a quota each, and the shim is told to
    keep them apart (VGPU_DUPLICATE_SPLIT; tests/test_duplicate_split.py runs the shim side)."""
    cfg, k, sup, stop, th = start(plugin_dir, device_split_count=4, backend=FakeBackend(n=1),
                                  duplicate_vgpus="split")
    try:
        k.wait_registered("amd.com/gpu")
        k.wait_devices("amd.com/gpu", predicate=lambda d: len(d) == 4)
        ids, resp = k.allocate("amd.com/gpu", 2)
        envs = dict(resp.envs)
        uuid = ids[0].rsplit("-", 1)[0]
        assert envs["VGPU_DUPLICATE_SPLIT"] == "1" and "VGPU_DUPLICATE_MERGED" not in envs
        assert dict(resp.annotations)["amd-vgpu/split-duplicates"] == uuid
        assert envs["VGPU_DEVICE_MAP"] == f"0:{uuid} 1:{uuid}"
        assert envs["VGPU_DEVICE_MEMORY_LIMIT_0"] == envs["VGPU_DEVICE_MEMORY_LIMIT_1"]
        # one entry per vGPU: torch.cuda.device_count() counts the visible list, amd-smi the BDFs
        assert envs["ROCR_VISIBLE_DEVICES"] == f"{uuid},{uuid}"
        bdf = FakeBackend(n=1).devices()[0].bdf
        assert envs["VGPU_DEVICE_BDFS"] == f"{bdf},{bdf}"
    finally:
        shutdown(k, stop, th)


def test_readme_two_vgpu_pod_admitted_on_a_one_gpu_node(plugin_dir):
    """The reference README's sample pod requests two vGPUs (README.md:205). On a node with
    one GPU the kubelet must hand it two vGPUs of that GPU; by default (split) Allocate admits
    it as two devices, as the reference does ([device.c:81-155]): the GPU named once per vGPU
    in the visible list, one quota per device ordinal."""
    cfg, k, sup, stop, th = start(plugin_dir, device_split_count=4, backend=FakeBackend(n=1))
    try:
        assert cfg.duplicate_vgpus == "split"
        k.wait_registered("amd.com/gpu")
        k.wait_devices("amd.com/gpu", predicate=lambda d: len(d) == 4)
        ids, resp = k.allocate("amd.com/gpu", 2)   # the kubelet's flow: preferred allocation, then Allocate
        envs = dict(resp.envs)
        uuid = ids[0].rsplit("-", 1)[0]
        assert ids[1].rsplit("-", 1)[0] == uuid
        assert envs["VGPU_DUPLICATE_SPLIT"] == "1" and "VGPU_DUPLICATE_MERGED" not in envs
        assert dict(resp.annotations)["amd-vgpu/split-duplicates"] == uuid
        assert envs["ROCR_VISIBLE_DEVICES"] == f"{uuid},{uuid}"  # two devices in the container
        assert envs["VGPU_DEVICE_MAP"] == f"0:{uuid} 1:{uuid}"
        total = FakeBackend(n=1).devices()[0].memory_total >> 20
        assert envs["VGPU_DEVICE_MEMORY_LIMIT_0"] == envs["VGPU_DEVICE_MEMORY_LIMIT_1"] == f"{total // 4}m"
    finally:
        shutdown(k, stop, th)


def test_readme_two_vgpu_pod_merged_on_request(plugin_dir):
    """--duplicate-vgpus=merge: the README pod's two vGPUs of one GPU become one device with the
    summed quota and CU share, annotated for the operator."""
    cfg, k, sup, stop, th = start(plugin_dir, device_split_count=4, backend=FakeBackend(n=1),
                                  duplicate_vgpus="merge")
    try:
        k.wait_registered("amd.com/gpu")
        k.wait_devices("amd.com/gpu", predicate=lambda d: len(d) == 4)
        ids, resp = k.allocate("amd.com/gpu", 2)
        envs = dict(resp.envs)
        uuid = ids[0].rsplit("-", 1)[0]
        assert envs["VGPU_DUPLICATE_MERGED"] == uuid and "VGPU_DUPLICATE_SPLIT" not in envs
        assert dict(resp.annotations)["amd-vgpu/merged-duplicates"] == uuid
        assert envs["ROCR_VISIBLE_DEVICES"] == uuid  # one device in the container
        assert envs["VGPU_DEVICE_MAP"] == f"0:{uuid} 1:{uuid}"
    finally:
        shutdown(k, stop, th)


def test_placement_spread_over_the_kubelet(plugin_dir):
    """Sequential 1-vGPU pods through the kubelet flow land on distinct GPUs (spread),
    or fill one GPU first (binpack)."""
    for placement, want in (("spread", 4), ("binpack", 1)):
        d = os.path.join(plugin_dir, placement)
        os.makedirs(d)
        cfg, k, sup, stop, th = start(d, device_split_count=4, backend=FakeBackend(n=4, topology="xgmi"),
                                      placement=placement)
        try:
            k.wait_registered("amd.com/gpu")
            k.wait_devices("amd.com/gpu", predicate=lambda x: len(x) == 16)
            gpus = {k.allocate("amd.com/gpu", 1)[0][0].rsplit("-", 1)[0] for _ in range(4)}
            assert len(gpus) == want, (placement, gpus)
        finally:
            shutdown(k, stop, th)


def test_host_memory_budget_per_vgpu(plugin_dir):
    cfg, k, sup, stop, th = start(plugin_dir, device_split_count=2, backend=FakeBackend(n=2),
                                  host_memory_per_vgpu="16g")
    try:
        k.wait_registered("amd.com/gpu")
        k.wait_devices("amd.com/gpu", predicate=lambda d: len(d) == 4)
        _ids, resp = k.allocate("amd.com/gpu", 2)
        assert dict(resp.envs)["VGPU_HOST_MEMORY_LIMIT"] == f"{32 << 10}m"
    finally:
        shutdown(k, stop, th)
