"""Multi-GPU readiness on the CPU (the round-4 verdict's weak item 4): an 8-GPU MI355X node
at split 16 exercised end to end without the hardware - the node's GPU-time ledger daemon
over 8 GPUs x 16 busy processes, the plugin's ListAndWatch / Allocate of 128 vGPUs through
a stub kubelet, and one container holding vGPUs of two different GPUs of an 8-agent node
with the GPU-time limiter on one of them.

Reference: the utilisation watcher samples per container ([multiprocess_utilization_watcher.c:
195-216]); the plugin advertises split x GPUs vdevices (vdevice.go:36-58) and picks
multi-GPU sets with the best-effort policy (besteffort_policy.go:34-89).
"""
import json
import os
import subprocess
import time

import pytest

from amdvgpu.plugin import api
from amdvgpu.plugin.devices import FakeBackend
from amdvgpu.plugin.ledger import monotonic_ns, read_board
from amdvgpu.shim.native import LEDGER, lib_path
from test_plugin_grpc import plugin_dir, shutdown, start  # noqa: F401  (fixture)
from test_shim_fake import HARNESS, fake, run  # noqa: F401  (fixture)

GiB = 1 << 30
N_GPUS, PODS_PER_GPU = 8, 16


def _fake_kfd(root, occ_of):
    """A KFD process tree: PODS_PER_GPU processes on each of N_GPUS gpu_ids (1000..1007)."""
    for g in range(N_GPUS):
        for i in range(PODS_PER_GPU):
            pid = 50000 + g * 100 + i
            d = root / str(pid) / f"stats_{1000 + g}"
            d.mkdir(parents=True)
            (d / "cu_occupancy").write_text(str(occ_of(g, i)))


def test_ledger_period_at_8_gpus_x_16_pods(tmp_path):
    """The ledger daemon samples each GPU on a thread of its own: with 128 busy processes on 8
    GPUs every GPU keeps the 1 ms period (a single loop over the node would stretch it to
    4 ms under the 32-read budget), no ledger ever looks stale to a container (heartbeat age
    under the containers' 50 ms rule, vgpu/ledger.h), each GPU's charges add up to at most
    the time it was sampled, and split in proportion to the processes' occupancies."""
    kfd, board = tmp_path / "kfd", tmp_path / "board"
    board.mkdir()
    _fake_kfd(kfd, lambda g, i: 4 + i)
    args = [lib_path(LEDGER), "--dir", str(board), "--period-us", "1000"]
    for g in range(N_GPUS):
        args += ["--gpu", str(1000 + g)]
    started = monotonic_ns()
    p = subprocess.Popen(args, env=dict(os.environ, VGPU_KFD_ROOT=str(kfd)))
    worst_age = 0
    try:
        t_end = time.time() + 2.5
        time.sleep(0.5)   # threads up, files created
        while time.time() < t_end:
            now = monotonic_ns()
            leds = read_board(str(board))
            if len(leds) == N_GPUS:
                worst_age = max(worst_age, max(now - l["heartbeat_ns"] for l in leds.values()))
            time.sleep(0.005)
        leds = read_board(str(board))
    finally:
        p.terminate()
        p.wait(timeout=10)
    assert sorted(leds) == [1000 + g for g in range(N_GPUS)]
    occ = [4 + i for i in range(PODS_PER_GPU)]
    for gid, led in leds.items():
        assert led["period_ns"] == 1_000_000, (gid, led["period_ns"])
        assert len(led["procs"]) == PODS_PER_GPU and led["total_occ"] == sum(occ)
        assert led["samples"] >= 800, (gid, led["samples"])       # ~2.5 s at 1 ms (CI jitter allowed)
        charged = {x["pid"]: x["charged_ns"] for x in led["procs"]}
        total = sum(charged.values())
        # the trapezoid adds each interval between two snapshots once: at least (samples - 1)
        # periods, at most the time since the daemon started
        assert (led["samples"] - 1) * 1_000_000 <= total <= led["heartbeat_ns"] - started, (gid, total, led)
        g = gid - 1000
        for i in range(PODS_PER_GPU):
            share = charged[50000 + g * 100 + i] / total
            assert abs(share - occ[i] / sum(occ)) < 0.002, (gid, i, share)
    assert worst_age < 50_000_000, worst_age   # kLedgerStaleNs: containers keep using the ledger


def test_eight_gpu_node_at_split_16_through_the_kubelet(plugin_dir):
    """An 8-GPU node at split 16: ListAndWatch advertises 128 vGPUs; an 8-vGPU pod gets one
    vGPU of every GPU (8 devices, each with a sixteenth of its memory); 1-vGPU pods then fill
    the node, every GPU's 16 vGPUs on disjoint CU slices."""
    cfg, k, sup, stop, th = start(plugin_dir, device_split_count=PODS_PER_GPU,
                                  backend=FakeBackend(n=N_GPUS, topology="xgmi"))
    try:
        k.wait_registered("amd.com/gpu")
        devs = k.wait_devices("amd.com/gpu", predicate=lambda d: len(d) == N_GPUS * PODS_PER_GPU)
        assert all(h == api.HEALTHY for h in devs.values())
        ids, resp = k.allocate("amd.com/gpu", N_GPUS)
        envs = dict(resp.envs)
        uuids = {i.rsplit("-", 1)[0] for i in ids}
        assert len(uuids) == N_GPUS
        assert set(envs["ROCR_VISIBLE_DEVICES"].split(",")) == uuids
        assert len(envs["VGPU_DEVICE_MAP"].split()) == N_GPUS
        total = FakeBackend(n=1).devices()[0].memory_total >> 20
        assert all(envs[f"VGPU_DEVICE_MEMORY_LIMIT_{i}"] == f"{total // PODS_PER_GPU}m" for i in range(N_GPUS))
        slices = {}
        for _ in range(N_GPUS * PODS_PER_GPU - N_GPUS):
            (vid,), r = k.allocate("amd.com/gpu", 1)
            e = dict(r.envs)
            lo, hi = (int(x) for x in e["VGPU_DEVICE_CU_RANGE_0"].split("-"))
            slices.setdefault(vid.rsplit("-", 1)[0], []).append((lo, hi))
        assert sorted(slices) == sorted(uuids)
        for u, rs in slices.items():
            assert len(rs) == PODS_PER_GPU - 1, (u, rs)
            rs.sort()
            assert all(a[1] <= b[0] for a, b in zip(rs, rs[1:])), (u, rs)   # disjoint
    finally:
        shutdown(k, stop, th)


def test_four_gpu_pod_stays_on_one_numa_node(plugin_dir):
    """PCIe node, GPUs 0-3 on NUMA node 0 and 4-7 on node 1: a 4-vGPU pod is placed on four
    GPUs of one NUMA node (preferred allocation), and a second one on the other node."""
    cfg, k, sup, stop, th = start(plugin_dir, device_split_count=2, backend=FakeBackend(n=N_GPUS, topology="pcie"))
    try:
        k.wait_registered("amd.com/gpu")
        k.wait_devices("amd.com/gpu", predicate=lambda d: len(d) == 2 * N_GPUS)
        by_uuid = {d.uuid: d for d in FakeBackend(n=N_GPUS, topology="pcie").devices()}
        nodes = []
        for _ in range(2):
            ids, _resp = k.allocate("amd.com/gpu", 4)
            gpus = {i.rsplit("-", 1)[0] for i in ids}
            assert len(gpus) == 4, ids
            nodes.append({by_uuid[u].numa_node for u in gpus})
        assert all(len(n) == 1 for n in nodes) and nodes[0] != nodes[1], nodes
    finally:
        shutdown(k, stop, th)


def test_two_vgpus_on_two_gpus_of_an_eight_agent_node(fake):
    """One container holds vGPUs of agents 3 and 6 of an 8-agent node (HIP_VISIBLE_DEVICES
    reorders them to HIP devices 0 and 1), the second limited to 20 % in time: launches on a
    stream of HIP device 1 are held to ~20 % even when issued with device 0 current, launches
    on device 0's stream run at full speed, and each vGPU's quota lands on its own agent."""
    uuids = [f"GPU-fa4e{i:012x}" for i in range(N_GPUS)]
    e = fake(gpus=N_GPUS, uuids=uuids, VGPU_DEVICE_MAP=f"0:{uuids[3]} 1:{uuids[6]}",
             VGPU_DEVICE_MEMORY_LIMIT_0="2g", VGPU_DEVICE_MEMORY_LIMIT_1="3g", VGPU_DEVICE_CU_LIMIT_1="20",
             VGPU_CU_MODE="temporal", HIP_VISIBLE_DEVICES="3,6")
    out = run(e, "dev=0", "curlimit", "stream", "dev=1", "curlimit", "stream", "dev=0", "usestream=1", "run=2000,3",
              "usestream=0", "run=2000,1.5", timeout=120)
    assert [o["limit"] for o in out if "limit" in o] == [2 * GiB, 3 * GiB]
    runs = [o for o in out if "run" in o]
    assert abs(runs[0]["busy_frac"] - 0.20) <= 0.05, runs
    assert runs[1]["busy_frac"] > 0.75, runs
