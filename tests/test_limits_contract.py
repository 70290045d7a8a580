"""The plugin side of plugin-owned limits: the limits file, the plugin-created region, the
latency-class resource, and the node-wide host-memory budget.

Reference: the reference's Allocate emits limits as env only (``server.go:486-507``), its
CUDA_TASK_PRIORITY is whatever the pod says, and --device-memory-scaling promises host
memory without a bound (``server.go:505-507``). See tests/test_tamper.py for the shim side.
"""
import json
import os
import subprocess
import time

import pytest

from amdvgpu.plugin import api
from amdvgpu.plugin.config import PluginConfig
from amdvgpu.plugin.devices import FakeBackend
from amdvgpu.plugin.host_memory import check_spill_fits, host_budget_per_vgpu
from amdvgpu.plugin.kubelet_stub import NodeHarness, StubKubelet
from amdvgpu.plugin.main import Supervisor
from amdvgpu.shim.launcher import apply_contract
from amdvgpu.shim.native import LIB_DIR

GiB = 1 << 30
HARNESS = os.path.join(LIB_DIR, "fakerocm", "shim_harness")


def _limits(resp):
    mounts = {m.container_path: m for m in resp.mounts}
    m = mounts["/vgpu/limits"]
    assert m.read_only
    return dict(l.split("=", 1) for l in open(m.host_path).read().splitlines())


def test_latency_vgpus_are_a_separate_resource(tmp_path):
    """--latency-vgpus-per-gpu 1 with split 4: three vGPUs per GPU under amd.com/gpu, one
    under amd.com/gpu-latency; only the latter grants the latency class (and makes it the
    container's default)."""
    import threading
    pdir = tmp_path / "dp"
    pdir.mkdir()
    cfg = PluginConfig(device_plugin_path=str(pdir) + "/", backend="fake", vgpu_dir=str(tmp_path / "vgpu"),
                       device_split_count=4, latency_vgpus_per_gpu=1, health_interval_s=0.1).validate()
    k = StubKubelet(str(pdir)).start()
    sup = Supervisor(cfg, backend=FakeBackend(n=2), install_signals=False)
    stop = threading.Event()
    th = threading.Thread(target=sup.run, args=(stop,), daemon=True)
    th.start()
    try:
        k.wait_registered("amd.com/gpu")
        reg = k.wait_registered("amd.com/gpu-latency")
        assert reg.endpoint == "amd-vgpu-latency.sock"
        normal = k.wait_devices("amd.com/gpu", predicate=lambda d: len(d) == 6)
        latency = k.wait_devices("amd.com/gpu-latency", predicate=lambda d: len(d) == 2)
        assert all(i.endswith(("-0", "-1", "-2")) for i in normal) and all(i.endswith("-3") for i in latency)
        _, r_norm = k.allocate("amd.com/gpu", 1)
        _, r_lat = k.allocate("amd.com/gpu-latency", 1)
        assert _limits(r_norm)["VGPU_TASK_PRIORITY_MIN"] == "1" and "VGPU_TASK_PRIORITY" not in dict(r_norm.envs)
        assert _limits(r_lat)["VGPU_TASK_PRIORITY_MIN"] == "0" and dict(r_lat.envs)["VGPU_TASK_PRIORITY"] == "0"
    finally:
        stop.set()
        th.join(10)
        k.stop()


def test_allow_latency_class_grants_every_container(tmp_path):
    with NodeHarness(FakeBackend(n=1), device_split_count=2, allow_latency_class=True,
                     workdir=str(tmp_path)) as node:
        resp = node.kubelet.allocate_ids(node.resource, node.vgpu_ids(FakeBackend(n=1).devices()[0].uuid)[:1])
        assert _limits(resp)["VGPU_TASK_PRIORITY_MIN"] == "0"


def test_invalid_latency_split_is_refused():
    with pytest.raises(ValueError):
        PluginConfig(device_split_count=2, latency_vgpus_per_gpu=2).validate()


def test_spill_must_fit_in_the_nodes_ram():
    """Memory scaling 3 on eight 288 GiB GPUs promises 4.6 TiB of pinned host memory: refused
    on a 2 TiB node (fraction 0.5), accepted at scaling 1.2 (460 GiB); fraction 0 lifts the
    bound (the reference's behaviour)."""
    devs = FakeBackend(n=8).devices()
    cfg = PluginConfig(device_split_count=4, device_memory_scaling=3.0, host_memory_total="2048g").validate()
    with pytest.raises(ValueError, match="promises"):
        check_spill_fits(cfg, devs)
    check_spill_fits(PluginConfig(device_split_count=4, device_memory_scaling=1.2, host_memory_total="2048g"), devs)
    check_spill_fits(PluginConfig(device_split_count=4, device_memory_scaling=3.0, host_memory_total="2048g",
                                  host_memory_fraction=0.0), devs)


def test_auto_host_budget_per_vgpu():
    devs = FakeBackend(n=8).devices()
    cfg = PluginConfig(device_split_count=4, host_memory_total="2048g").validate()
    assert host_budget_per_vgpu(cfg, devs) == 1024 * GiB // 32                      # half the RAM over 32 vGPUs
    spill = PluginConfig(device_split_count=4, device_memory_scaling=1.2, host_memory_total="512g").validate()
    per = host_budget_per_vgpu(spill, devs)
    assert per >= int(devs[0].memory_total * 0.2) // 4                             # never below one vGPU's spill
    assert host_budget_per_vgpu(PluginConfig(host_memory_per_vgpu="16g"), devs) == 16 * GiB
    assert host_budget_per_vgpu(PluginConfig(host_memory_per_vgpu="0"), devs) == 0
    assert host_budget_per_vgpu(PluginConfig(host_memory_fraction=0.0, host_memory_total="1t"), devs) == 0


def test_contract_carries_the_auto_host_budget(tmp_path):
    with NodeHarness(FakeBackend(n=2), device_split_count=4, host_memory_total="256g",
                     workdir=str(tmp_path)) as node:
        envs, _ = node.pod(node.vgpu_ids(FakeBackend(n=2).devices()[0].uuid)[:1])
        assert envs["VGPU_HOST_MEMORY_LIMIT"] == f"{(128 * GiB // 8) >> 20}m"


def test_emulated_container_is_held_to_the_plugins_limits(tmp_path):
    """A whole Allocate contract applied by the container emulator (shim/launcher.py) to the
    fake runtime: the tenant's env asks for 64 GiB and no CU limit; the plugin's limits file
    (a host-path copy standing in for the read-only mount) holds it to the vGPU's quota,
    and its region is the file the plugin created."""
    kfd = tmp_path / "kfd"
    kfd.mkdir()
    b = FakeBackend(n=1, memory=8 * GiB)
    with NodeHarness(b, device_split_count=4, cu_mode="spatial", workdir=str(tmp_path / "node")) as node:
        envs, mounts = node.pod(node.vgpu_ids(b.devices()[0].uuid)[:1])
        env = apply_contract(envs, mounts)
        env.update(FAKE_ROCR_GPUS="1", FAKE_ROCR_HBM=str(8 * GiB), FAKE_ROCR_UUIDS=b.devices()[0].uuid,
                   FAKE_KFD_ROOT=str(kfd), VGPU_KFD_ROOT=str(kfd), VGPU_DEVICE_MEMORY_LIMIT_0="64g",
                   VGPU_DEVICE_CU_LIMIT_0="0", VGPU_CU_MODE="off")
        env.pop("ROCR_VISIBLE_DEVICES", None)
        p = subprocess.run([HARNESS, "meminfo", "malloc=1536m", "malloc=1024m", "stream", "queues"], env=env,
                           capture_output=True, text=True, timeout=60)
        assert p.returncode == 0, p.stderr[-3000:]
        out = [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]
        region = dict(mounts)[envs["VGPU_SHARED_CACHE"]]
        assert os.path.getsize(region) > 0                      # the plugin's file was used
    assert [o for o in out if "total" in o][0]["total"] == 2 * GiB
    assert [o["malloc"] for o in out if "malloc" in o] == ["ok", "oom"]
    assert [q["cus"] for q in [o for o in out if "queues" in o][0]["queues"]] == [64]


def test_limits_file_carries_the_board_and_admission(tmp_path):
    """The node board (where the GPU-time ledger lives), the container's slot in it, the
    exact share and the node's admission bound are ceilings like the quotas: the limits file
    carries them, so a tenant's own env cannot move it to a board of its making."""
    with NodeHarness(FakeBackend(n=1), device_split_count=16, gpu_concurrency=4,
                     workdir=str(tmp_path / "node")) as node:
        envs, mounts = node.pod(node.vgpu_ids(FakeBackend(n=1).devices()[0].uuid)[:1])
        limits_host = dict(mounts)["/vgpu/limits"]
        lim = dict(l.split("=", 1) for l in open(limits_host).read().splitlines())
    for k in ("VGPU_BOARD_DIR", "VGPU_BOARD_SLOT", "VGPU_GPU_CONCURRENCY", "VGPU_DEVICE_CU_SHARE_0"):
        assert lim.get(k) == envs[k], (k, lim.get(k), envs.get(k))



def test_gpu_concurrency_auto_reaches_the_container(tmp_path):
    """--gpu-concurrency=auto: the contract (env and limits file) says "auto", which the shim
    reads as pair turns while the GPU's containers launch more than VGPU_PAIRS_ON_RATE
    kernels/s together (tests/test_shim_fake.py::test_auto_pair_turns_follow_the_launch_rate)."""
    from amdvgpu.plugin.config import parse_config
    assert parse_config(["--gpu-concurrency", "auto"]).gpu_concurrency == -1
    assert parse_config([], {"GPU_CONCURRENCY": "auto"}).gpu_concurrency == -1
    with NodeHarness(FakeBackend(n=1), device_split_count=4, gpu_concurrency=-1,
                     workdir=str(tmp_path / "node")) as node:
        envs, mounts = node.pod(node.vgpu_ids(FakeBackend(n=1).devices()[0].uuid)[:1])
        lim = dict(l.split("=", 1) for l in open(dict(mounts)["/vgpu/limits"]).read().splitlines())
    assert envs["VGPU_GPU_CONCURRENCY"] == "auto" and lim["VGPU_GPU_CONCURRENCY"] == "auto"
