"""vGPU model: each physical MI355X is advertised as ``split`` schedulable vGPUs.

Reference: ``vdevice.go`` — ``VDevice{dev, memory}`` (:29-33), ``Device2VDevice``
(:36-58, memory per vGPU = ``totalMiB * memScaling / split`` at :49, MIG devices get one
vdevice with memory 0), ``VDevicesByIDs`` (:61-75), ``UniqueDeviceIDs`` (:78-90); and the
SM limit ``int(100 * coresScaling / split)`` emitted for every vdevice (``server.go:492``;
rounded up here, see ``device_to_vdevices``).

MI355X additions:
* every vGPU carries its own CU share *and* a logical CU range. Slot ``i`` of a GPU gets
  the i-th XCD-balanced slice (``cu_partition_range``), so co-resident containers run on
  disjoint CUs (spatial partitioning through per-queue CU masks; the reference's limit
  is temporal and identical for all vdevices);
* with ``cores_scaling > 1`` (compute oversubscription) slices widen and overlap;
* with ``memory_scaling > 1`` the quota exceeds the HBM share; the HBM-resident part stays
  ``total / split`` and the rest spills to host memory (``hbm_limit``);
* compute/memory partitions (CPX/QPX/DPX x NPS) are whole devices already: one vdevice,
  no quota and no CU limit (the reference's MIG rule).

The CU arithmetic here is the Python twin of ``native/src/core/cumask.cpp``
(cross-checked by tests/test_vdevice.py).
"""
import math
from dataclasses import dataclass

MiB = 1 << 20


def cu_share_count(cu_count, num_xcc, pct):
    """CUs for ``pct`` percent, rounded down to a multiple of num_xcc (>= num_xcc)."""
    if cu_count <= 0:
        return 0
    num_xcc = max(1, num_xcc)
    if pct <= 0 or pct >= 100:
        return cu_count
    n = cu_count * pct // 100 // num_xcc * num_xcc
    return min(max(n, num_xcc), cu_count)


def cu_partition_range(cu_count, num_xcc, split, slot):
    """Logical CU range [begin, end) of tenant ``slot`` among ``split`` equal tenants."""
    num_xcc = max(1, num_xcc)
    if split <= 1:
        return 0, cu_count
    units = cu_count // num_xcc
    base, rem = divmod(units, split)
    if base == 0:
        u = slot % units
        return u * num_xcc, u * num_xcc + num_xcc
    start = slot * base + min(slot, rem)
    length = base + (1 if slot < rem else 0)
    return start * num_xcc, (start + length) * num_xcc


def cu_range_for(cu_count, num_xcc, split, slot, pct):
    """CU range for vGPU ``slot``: its partition slice, widened to ``pct`` when compute is
    oversubscribed (cores_scaling > 1), clamped inside the chip."""
    b, e = cu_partition_range(cu_count, num_xcc, split, slot)
    want = cu_share_count(cu_count, num_xcc, pct)
    if want <= e - b:
        return b, e
    b = min(b, cu_count - want)
    return b, b + want


@dataclass
class VDevice:
    id: str
    dev: object            # GpuDevice
    slot: int
    memory: int            # quota in bytes (0 = unlimited)
    hbm_limit: int         # HBM-resident cap in bytes (0 = same as quota)
    cu_pct: int            # 0 = unlimited
    cu_range: tuple        # (begin, end) logical CUs, or None
    cu_share: float = 0.0  # exact share in percent (100 * cores_scaling / split); 0 = unlimited
    cpu_node: int = -1     # NUMA node whose CPUs the container's processes run on (--numa-spread), -1 = any

    @property
    def uuid(self):
        return self.dev.uuid

    @property
    def memory_mib(self):
        return self.memory // MiB


def device_to_vdevices(devices, split, memory_scaling=1.0, cores_scaling=1.0):
    """Expands physical devices into vGPUs (reference Device2VDevice)."""
    out = []
    for d in devices:
        if d.is_partition:
            out.append(VDevice(f"{d.uuid}-0", d, 0, 0, 0, 0, None))
            continue
        total_mib = d.memory_total // MiB
        mem = int(total_mib * memory_scaling / split) * MiB
        hbm = int(total_mib / split) * MiB if memory_scaling > 1 else 0
        # Rounded up, unlike the reference's int(): the shares of a fully split GPU then
        # sum to >= 100 %, so N busy temporal tenants (each charged 1/N of the time)
        # are never throttled below the whole GPU (int() leaves up to N-1 % idle, e.g.
        # 8 x 12 % = 96 %). Spatial slices are unchanged (cu_share_count rounds down to
        # whole XCD columns, which fit the partition slice).
        pct = math.ceil(round(100 * cores_scaling / split, 6))
        if pct >= 100:
            pct = 0
        share = round(100 * cores_scaling / split, 4) if pct else 0.0
        for i in range(split):
            rng = cu_range_for(d.cu_count, d.num_xcc, split, i, pct) if pct else None
            out.append(VDevice(f"{d.uuid}-{i}", d, i, mem, hbm, pct, rng, share))
    return out


def vdevices_by_ids(vdevices, ids):
    index = {v.id: v for v in vdevices}
    out = []
    for i in ids:
        if i not in index:
            raise KeyError(f"unknown vGPU device id {i!r}")
        out.append(index[i])
    return out


def unique_device_uuids(vdevices):
    seen, out = set(), []
    for v in vdevices:
        if v.uuid not in seen:
            seen.add(v.uuid)
            out.append(v.uuid)
    return out


def physical_uuid(vdevice_id):
    """'<uuid>-<slot>' -> '<uuid>'."""
    base, _, slot = vdevice_id.rpartition("-")
    return base if slot.isdigit() and base else vdevice_id


def assign_cpu_nodes(vdevices, cpu_nodes):
    """--numa-spread: vGPU ``slot`` of a GPU gets CPU node ``order[slot % len(order)]``, where
    ``order`` is the GPU's own NUMA node followed by the node's other CPU nodes. Co-tenant
    pods of one GPU then launch from different CPU sockets: two launch-bound PyTorch pods
    whose threads share a socket run no faster together than one alone on MI355X, on two
    sockets at up to twice the rate, and a lone pod runs as fast from either socket
    (profiles/r5d). Partitions and GPUs without a NUMA node keep -1."""
    nodes = sorted(set(cpu_nodes))
    for v in vdevices:
        v.cpu_node = -1
        home = getattr(v.dev, "numa_node", -1)
        if len(nodes) < 2 or home < 0 or getattr(v.dev, "is_partition", False):
            continue
        order = ([home] if home in nodes else []) + [n for n in nodes if n != home]
        v.cpu_node = order[v.slot % len(order)]
    return vdevices
