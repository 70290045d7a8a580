"""vGPU model (reference vdevice.go) and the Python/C++ CU-partition twins."""
import pytest

from amdvgpu.plugin.devices import FakeBackend
from amdvgpu.plugin.vdevice import (cu_partition_range, cu_range_for, cu_share_count, device_to_vdevices,
                                    physical_uuid, unique_device_uuids, vdevices_by_ids)

MiB = 1 << 20


def test_split_memory_formula():
    devs = FakeBackend(n=2).devices()
    vds = device_to_vdevices(devs, 4)
    assert len(vds) == 8
    total_mib = devs[0].memory_total // MiB
    assert all(v.memory == (total_mib // 4) * MiB for v in vds)
    assert vds[0].id == f"{devs[0].uuid}-0" and vds[5].id == f"{devs[1].uuid}-1"
    assert all(v.cu_pct == 25 for v in vds)


def test_memory_scaling_and_hbm_share():
    devs = FakeBackend(n=1).devices()
    vds = device_to_vdevices(devs, 2, memory_scaling=1.8)
    total_mib = devs[0].memory_total // MiB
    assert vds[0].memory == int(total_mib * 1.8 / 2) * MiB
    assert vds[0].hbm_limit == (total_mib // 2) * MiB


def test_disjoint_cu_ranges_per_slot():
    devs = FakeBackend(n=1).devices()
    vds = device_to_vdevices(devs, 4)
    ranges = [v.cu_range for v in vds]
    assert ranges == [(0, 64), (64, 128), (128, 192), (192, 256)]


def test_cores_scaling_widens_ranges():
    devs = FakeBackend(n=1).devices()
    vds = device_to_vdevices(devs, 4, cores_scaling=2.0)
    assert all(v.cu_pct == 50 for v in vds)
    assert all(v.cu_range[1] - v.cu_range[0] == 128 for v in vds)
    assert all(0 <= v.cu_range[0] and v.cu_range[1] <= 256 for v in vds)


def test_split_one_is_unlimited_compute():
    vds = device_to_vdevices(FakeBackend(n=1).devices(), 1)
    assert vds[0].cu_pct == 0 and vds[0].cu_range is None


def test_partitions_are_whole_devices():
    devs = FakeBackend(n=1, partitions_per_gpu=8, compute_partition="CPX").devices()
    vds = device_to_vdevices(devs, 4)
    assert len(vds) == 8 and all(v.memory == 0 and v.cu_pct == 0 for v in vds)


def test_lookup_helpers():
    vds = device_to_vdevices(FakeBackend(n=2).devices(), 2)
    got = vdevices_by_ids(vds, [vds[3].id, vds[0].id])
    assert [v.id for v in got] == [vds[3].id, vds[0].id]
    with pytest.raises(KeyError):
        vdevices_by_ids(vds, ["nope"])
    assert unique_device_uuids([vds[0], vds[1], vds[2]]) == [vds[0].uuid, vds[2].uuid]
    assert physical_uuid(vds[3].id) == vds[3].uuid


@pytest.mark.parametrize("cu,xcc", [(256, 8), (32, 1), (128, 4), (80, 8)])
def test_python_cu_math_matches_native(cu, xcc):
    from amdvgpu.shim import region
    for pct in (0, 1, 10, 25, 33, 50, 99, 100):
        assert cu_share_count(cu, xcc, pct) == region.cu_share_count(cu, xcc, pct)
    for split in range(1, 40):
        for slot in range(split):
            assert cu_partition_range(cu, xcc, split, slot) == region.cu_partition_range(cu, xcc, split, slot)


def test_partition_ranges_cover_chip_disjointly():
    for split in range(1, 33):
        rs = [cu_partition_range(256, 8, split, s) for s in range(split)]
        cov = [0] * 256
        for b, e in rs:
            assert b % 8 == 0 and e % 8 == 0 and e > b
            for i in range(b, e):
                cov[i] += 1
        assert all(c == 1 for c in cov)


def test_cu_range_for_clamps():
    assert cu_range_for(256, 8, 4, 3, 50) == (128, 256)


@pytest.mark.parametrize("split,pct", [(2, 50), (3, 34), (4, 25), (6, 17), (8, 13), (10, 10)])
def test_cu_share_rounds_up_so_shares_cover_the_gpu(split, pct):
    """A fully split GPU's temporal shares sum to >= 100 %, so N busy tenants are never
    throttled below the whole GPU (the reference's int() gives 8 x 12 % = 96 %)."""
    dev = FakeBackend(n=1).devices()
    vds = device_to_vdevices(dev, split)
    assert {v.cu_pct for v in vds} == {pct}
    assert sum(v.cu_pct for v in vds) >= 100
    # spatial slices stay disjoint
    rngs = sorted(v.cu_range for v in vds)
    assert all(a[1] <= b[0] for a, b in zip(rngs, rngs[1:]))


def test_exact_share_sent_only_with_the_ledger():
    """A split-16 vGPU's CU limit is a whole percent rounded up (7); with the node ledger the
    plugin also sends the exact share (6.25) for the limiter's grants."""
    from amdvgpu.plugin.devices import FakeBackend
    from amdvgpu.plugin.kubelet_stub import NodeHarness
    b = FakeBackend(n=1)
    u = b.devices()[0].uuid
    for ledger, share in ((False, None), (True, "6.25")):
        with NodeHarness(b, device_split_count=16, ledger=ledger) as node:
            envs, _ = node.pod(node.vgpu_ids(u)[:1])
        assert envs["VGPU_DEVICE_CU_LIMIT_0"] == "7" and envs.get("VGPU_DEVICE_CU_SHARE_0") == share
    with NodeHarness(b, device_split_count=4, ledger=True) as node:   # 25 % is exact already
        envs, _ = node.pod(node.vgpu_ids(u)[:1])
    assert envs["VGPU_DEVICE_CU_LIMIT_0"] == "25" and "VGPU_DEVICE_CU_SHARE_0" not in envs


def test_ledger_is_the_default_path():
    """Round 4 picks one default: the plugin runs the node ledger and sends exact shares
    unless --ledger=false (profiles/r4o)."""
    from amdvgpu.plugin.config import PluginConfig
    from amdvgpu.plugin.devices import FakeBackend
    from amdvgpu.plugin.kubelet_stub import NodeHarness
    assert PluginConfig().ledger is True
    b = FakeBackend(n=1)
    with NodeHarness(b, device_split_count=12) as node:
        envs, _ = node.pod(node.vgpu_ids(b.devices()[0].uuid)[:1])
    assert envs["VGPU_DEVICE_CU_LIMIT_0"] == "9" and envs["VGPU_DEVICE_CU_SHARE_0"] == "8.3333"
