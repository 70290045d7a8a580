"""Device discovery, topology and health for the control plane.

Reference: ``nvidia.go`` (``ResourceManager{Devices, CheckHealth}`` :43-46, ``Devices``
:81-136, ``buildDevice`` :148-164 with NUMA from ``/sys/bus/pci/devices/<bdf>/numa_node``,
``checkHealth`` :166-237) on top of NVML cgo bindings, and go-gpuallocator's link
discovery (``device.go:33-71``).

MI355X design: the authoritative inventory is the KFD topology in sysfs
(``/sys/class/kfd/kfd/topology/nodes/<n>/{gpu_id,properties,mem_banks,io_links}``), which
every ROCm process (and the shim) sees identically and which needs neither root nor a
GPU context: it gives the ROCr UUID (``unique_id``), BDF, NUMA node, CU/XCC counts, the
render minor for device specs, HBM size and the xGMI/PCIe link graph. Compute/memory
partitions (SPX/DPX/QPX/CPX x NPS1/NPS2) appear as separate KFD nodes sharing a BDF.
``AmdSmiBackend`` layers amdsmi on top for health events (GPU reset / ring hang / RAS)
when the bindings and driver permit; ``FakeBackend`` provides N fake GPUs with a
configurable topology for tests and the stub-kubelet config (no GPU).
"""
import glob
import json
import os
import time
import threading
from dataclasses import dataclass, field

# io_link types from the KFD topology (kfd_crat.h CRAT_IOLINK_TYPE_*)
IOLINK_PCIE = 2
IOLINK_XGMI = 11


@dataclass
class GpuDevice:
    index: int                    # node-local ordinal (KFD GPU order)
    uuid: str                     # ROCr UUID "GPU-<16 hex>" (what ROCR_VISIBLE_DEVICES takes)
    bdf: str = ""                 # "0000:5a:00.0"
    numa_node: int = -1
    memory_total: int = 0         # bytes of HBM visible to this device/partition
    cu_count: int = 256
    num_xcc: int = 8
    render_minor: int = -1        # /dev/dri/renderD<minor>
    card_index: int = -1          # /dev/dri/card<index>
    gpu_id: int = 0               # KFD gpu_id
    node_id: int = -1             # KFD topology node
    compute_partition: str = "SPX"
    memory_partition: str = "NPS1"
    partition_index: int = 0      # index among the partitions of one physical GPU
    product: str = "AMD Instinct MI355X"
    gfx_target: str = "gfx950"
    healthy: bool = True
    links: dict = field(default_factory=dict)  # peer index -> list of (type, weight/hops)

    @property
    def is_partition(self):
        return self.compute_partition != "SPX"

    @property
    def device_paths(self):
        paths = ["/dev/kfd"]
        if self.render_minor >= 0:
            paths.append(f"/dev/dri/renderD{self.render_minor}")
        if self.card_index >= 0:
            paths.append(f"/dev/dri/card{self.card_index}")
        return paths

    def to_dict(self):
        d = dict(self.__dict__)
        d["links"] = {str(k): v for k, v in self.links.items()}
        return d


class HealthEvent:
    def __init__(self, uuid, healthy, reason):
        self.uuid, self.healthy, self.reason = uuid, healthy, reason

    def __repr__(self):
        return f"HealthEvent({self.uuid}, healthy={self.healthy}, {self.reason})"


class Backend:
    """Interface of a device backend."""

    name = "base"

    def devices(self):
        raise NotImplementedError

    def poll_health(self, devices):
        """Returns a list of HealthEvent since the last call (non-blocking)."""
        return []

    def cpu_numa_nodes(self):
        """The node's NUMA nodes that have CPUs, sorted."""
        return cpu_numa_nodes()

    def close(self):
        pass


def cpu_numa_nodes(sys_root="/sys"):
    """NUMA nodes with at least one CPU (``/sys/devices/system/node/node<n>/cpulist``)."""
    out = []
    for d in glob.glob(os.path.join(sys_root, "devices", "system", "node", "node[0-9]*")):
        if _read(os.path.join(d, "cpulist"), ""):
            out.append(int(os.path.basename(d)[4:]))
    return sorted(out)


# ----------------------------------------------------------------------------- sysfs


def _read(path, default=None):
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return default


def _props(path):
    out = {}
    txt = _read(path, "")
    for line in txt.splitlines():
        parts = line.split()
        if len(parts) == 2:
            try:
                out[parts[0]] = int(parts[1])
            except ValueError:
                pass
    return out


def bdf_from_location(domain, location_id):
    bus, dev, fn = (location_id >> 8) & 0xFF, (location_id >> 3) & 0x1F, location_id & 0x7
    return f"{domain:04x}:{bus:02x}:{dev:02x}.{fn:x}"


def rocr_uuid(unique_id):
    return f"GPU-{unique_id:016x}" if unique_id else ""


# A GPU marked unhealthy by uncorrectable RAS errors returns to Healthy only after its
# UE counter stayed flat this long, or at once on an observed GPU reset (amdsmi
# POST_RESET): an uncorrectable error usually needs a reset, and flapping back after one
# flat poll would hand the device to new pods while it is still suspect.
def _env_seconds(name, default):
    try:
        v = float(os.environ.get(name, default))
    except ValueError:
        return float(default)
    return v if v >= 0 else float(default)


RAS_RECOVER_S = _env_seconds("VGPU_RAS_RECOVER_S", 300)


class SysfsBackend(Backend):
    """KFD-topology + DRM sysfs inventory and RAS-counter health (no root, no GPU context)."""

    name = "sysfs"

    def __init__(self, kfd_root="/sys/class/kfd/kfd/topology/nodes", drm_root="/sys/class/drm",
                 ras_recover_s=None, clock=time.monotonic):
        self.kfd_root, self.drm_root = kfd_root, drm_root
        self._ras = {}
        self._ras_bad_at = {}   # uuid -> time of the last UE increase (RAS-unhealthy devices)
        self.ras_recover_s = RAS_RECOVER_S if ras_recover_s is None else ras_recover_s
        self._clock = clock

    def _drm_dev(self, minor):
        return os.path.join(self.drm_root, f"renderD{minor}", "device")

    def devices(self):
        nodes = []
        for nd in sorted(glob.glob(os.path.join(self.kfd_root, "*")), key=lambda p: int(os.path.basename(p))):
            p = _props(os.path.join(nd, "properties"))
            gpu_id = int(_read(os.path.join(nd, "gpu_id"), "0") or 0)
            if not gpu_id or p.get("simd_count", 0) == 0:
                continue  # CPU node
            nodes.append((int(os.path.basename(nd)), nd, p, gpu_id))
        devs, seen_uuid = [], {}
        for idx, (node_id, nd, p, gpu_id) in enumerate(nodes):
            simd_per_cu = p.get("simd_per_cu", 4) or 4
            cu = p.get("simd_count", 0) // simd_per_cu
            minor = p.get("drm_render_minor", -1)
            mem = 0
            for mb in glob.glob(os.path.join(nd, "mem_banks", "*", "properties")):
                mem += _props(mb).get("size_in_bytes", 0)
            ddir = self._drm_dev(minor)
            vram = _read(os.path.join(ddir, "mem_info_vram_total"))
            if vram and vram.isdigit() and int(vram) > 0:
                mem = int(vram) if not mem else mem
            numa = _read(os.path.join(ddir, "numa_node"))
            cpart = (_read(os.path.join(ddir, "current_compute_partition"), "SPX") or "SPX").upper()
            mpart = (_read(os.path.join(ddir, "current_memory_partition"), "NPS1") or "NPS1").upper()
            cards = glob.glob(os.path.join(ddir, "drm", "card*"))
            card = int(os.path.basename(cards[0])[4:]) if cards else -1
            uuid = rocr_uuid(p.get("unique_id", 0)) or f"GPU-kfd{gpu_id:08x}"
            k = seen_uuid.get(uuid, 0)
            seen_uuid[uuid] = k + 1
            gfx = p.get("gfx_target_version", 0)
            d = GpuDevice(index=idx, uuid=uuid if k == 0 else f"{uuid}-p{k}", bdf=bdf_from_location(
                p.get("domain", 0), p.get("location_id", 0)), numa_node=int(numa) if numa and numa.lstrip(
                    "-").isdigit() else -1, memory_total=mem, cu_count=cu, num_xcc=p.get("num_xcc", 1) or 1,
                render_minor=minor, card_index=card, gpu_id=gpu_id, node_id=node_id, compute_partition=cpart,
                memory_partition=mpart, partition_index=k,
                gfx_target=f"gfx{gfx // 10000}{(gfx // 100) % 100:x}{gfx % 100:x}" if gfx else "gfx950")
            devs.append(d)
        by_node = {d.node_id: d for d in devs}
        for d in devs:
            for lk in glob.glob(os.path.join(self.kfd_root, str(d.node_id), "io_links", "*", "properties")):
                lp = _props(lk)
                peer = by_node.get(lp.get("node_to", -1))
                if peer is None or peer is d:
                    continue
                d.links.setdefault(peer.index, []).append((lp.get("type", 0), lp.get("weight", 0)))
            for lk in glob.glob(os.path.join(self.kfd_root, str(d.node_id), "p2p_links", "*", "properties")):
                lp = _props(lk)
                peer = by_node.get(lp.get("node_to", -1))
                if peer is None or peer is d or peer.index in d.links:
                    continue
                d.links.setdefault(peer.index, []).append((lp.get("type", 0), lp.get("weight", 0)))
        return devs

    def _ras_ue(self, d):
        total = 0
        for f in glob.glob(os.path.join(self._drm_dev(d.render_minor), "ras", "*_err_count")):
            for line in (_read(f, "") or "").splitlines():
                if line.startswith("ue:"):
                    try:
                        total += int(line.split()[1])
                    except (IndexError, ValueError):
                        pass
        return total

    def poll_health(self, devices):
        """Uncorrectable RAS errors -> Unhealthy; device node vanished -> Unhealthy. Recovery
        (the reference never recovers, server.go:262): a node that is back, with a flat UE
        count for one poll, is Healthy again (the driver re-created it); a RAS-unhealthy
        device once its UE count stayed flat for ``ras_recover_s`` (or at a reset event,
        AmdSmiBackend)."""
        events = []
        now = self._clock()
        for d in devices:
            present = os.path.exists(os.path.join(self.kfd_root, str(d.node_id), "gpu_id")) if d.node_id >= 0 else True
            ue = self._ras_ue(d) if present else None
            prev = self._ras.get(d.uuid)
            self._ras[d.uuid] = ue
            if present and prev is not None and ue is not None and ue > prev:
                self._ras_bad_at[d.uuid] = now
                if d.healthy:
                    events.append(HealthEvent(d.uuid, False, f"uncorrectable RAS errors {prev}->{ue}"))
            elif not present and d.healthy:
                events.append(HealthEvent(d.uuid, False, "device node disappeared"))
            elif present and not d.healthy and prev is not None and ue == prev:
                bad_at = self._ras_bad_at.get(d.uuid)
                if bad_at is None or now - bad_at >= self.ras_recover_s:
                    self._ras_bad_at.pop(d.uuid, None)
                    events.append(HealthEvent(d.uuid, True, "device recovered"))
        return events

    def reset_observed(self, uuid):
        """A GPU reset clears the RAS hold-off: the device may recover at once."""
        self._ras_bad_at.pop(uuid, None)


# ----------------------------------------------------------------------------- amdsmi


def _handle_key(h):
    """amdsmi processor handles are ctypes pointers; events carry a fresh wrapper object
    for the same device, so compare the pointer value, not the Python object."""
    v = getattr(h, "value", None)
    return v if v is not None else id(h)


class AmdSmiBackend(SysfsBackend):
    """sysfs inventory + amdsmi event notifications (reset / ring hang -> Unhealthy,
    post-reset -> Healthy; VM faults are application errors and are ignored, the
    analogue of XIDs 31/43/45 in nvidia.go:208-210)."""

    name = "amdsmi"

    def __init__(self, **kw):
        super().__init__(**kw)
        import amdsmi  # noqa: F401 (raises ImportError when absent)
        self._smi = amdsmi
        self._smi.amdsmi_init()
        self._handles = {}
        self._notif = False

    def devices(self):
        devs = super().devices()
        smi = self._smi
        try:
            for h in smi.amdsmi_get_processor_handles():
                bdf = smi.amdsmi_get_gpu_device_bdf(h)
                for d in devs:
                    if d.bdf.lower() == str(bdf).lower():
                        self._handles[d.uuid] = h
                        try:
                            d.product = smi.amdsmi_get_gpu_asic_info(h).get("market_name", d.product)
                        except Exception:
                            pass
        except Exception:
            pass
        if not self._notif and self._handles:
            try:
                for h in self._handles.values():
                    smi.amdsmi_init_gpu_event_notification(h)
                    mask = (smi.AmdSmiEvtNotificationType.GPU_PRE_RESET | smi.AmdSmiEvtNotificationType.GPU_POST_RESET
                            | smi.AmdSmiEvtNotificationType.RING_HANG)
                    smi.amdsmi_set_gpu_event_notification_mask(h, mask)
                self._notif = True
            except Exception:
                self._notif = False
        return devs

    def poll_health(self, devices):
        events = super().poll_health(devices)
        if not self._notif:
            return events
        smi = self._smi
        try:
            got = smi.amdsmi_get_gpu_event_notification(0)
        except Exception:
            return events
        by_handle = {_handle_key(h): u for u, h in self._handles.items()}
        for ev in got or []:
            uuid = by_handle.get(_handle_key(ev.get("processor_handle")))
            kind = str(ev.get("event", ""))
            if not uuid:
                continue
            if "PRE_RESET" in kind or "RING_HANG" in kind:
                events.append(HealthEvent(uuid, False, kind))
            elif "POST_RESET" in kind:
                self.reset_observed(uuid)
                events.append(HealthEvent(uuid, True, kind))
        return events

    def close(self):
        try:
            self._smi.amdsmi_shut_down()
        except Exception:
            pass


# ----------------------------------------------------------------------------- fake


class FakeBackend(Backend):
    """N fake MI355X GPUs. ``topology``: "xgmi" (8-GPU UBB: every pair one direct xGMI
    link), "pcie" (pairs by NUMA node), or an explicit {(i, j): [(type, weight)]} map."""

    name = "fake"

    def __init__(self, n=2, memory=309220868096, cu_count=256, num_xcc=8, topology="xgmi", numa_split=None,
                 compute_partition="SPX", partitions_per_gpu=1, uuid_prefix="GPU-fa4e"):
        self._lock = threading.Lock()
        self._pending = []
        devs = []
        numa_split = numa_split or max(1, n // 2)
        idx = 0
        for g in range(n):
            for p in range(partitions_per_gpu):
                devs.append(GpuDevice(
                    index=idx, uuid=f"{uuid_prefix}{g:04x}{p:08x}" if partitions_per_gpu > 1 else
                    f"{uuid_prefix}{g:012x}", bdf=f"0000:{0x05 + 0x10 * g:02x}:00.0",
                    numa_node=0 if g < numa_split else 1, memory_total=memory // partitions_per_gpu,
                    cu_count=cu_count // partitions_per_gpu, num_xcc=max(1, num_xcc // partitions_per_gpu),
                    render_minor=128 + idx, card_index=idx, gpu_id=1000 + idx, node_id=idx + 2,
                    compute_partition=compute_partition if partitions_per_gpu > 1 else "SPX", partition_index=p))
                idx += 1
        for a in devs:
            for b in devs:
                if a is b:
                    continue
                if isinstance(topology, dict):
                    lk = topology.get((a.index, b.index)) or topology.get((b.index, a.index))
                    if lk:
                        a.links[b.index] = list(lk)
                elif topology == "xgmi":
                    a.links[b.index] = [(IOLINK_XGMI, 15)]
                else:
                    a.links[b.index] = [(IOLINK_PCIE, 20 if a.numa_node == b.numa_node else 40)]
        self._devs = devs

    @classmethod
    def from_spec(cls, spec):
        if isinstance(spec, str):
            spec = json.loads(open(spec).read()) if os.path.exists(spec) else json.loads(spec)
        return cls(**spec)

    def devices(self):
        return [GpuDevice(**{k: v for k, v in d.__dict__.items() if k != "links"}, links=dict(d.links))
                for d in self._devs]

    def cpu_numa_nodes(self):
        return sorted({d.numa_node for d in self._devs if d.numa_node >= 0})

    def inject(self, uuid, healthy, reason="injected"):
        with self._lock:
            self._pending.append(HealthEvent(uuid, healthy, reason))

    def poll_health(self, devices):
        with self._lock:
            ev, self._pending = self._pending, []
        return ev


def detect_backend(name="auto", fake_spec=None):
    """Picks a backend: explicit name, else amdsmi when importable and a GPU node exists,
    else sysfs when a KFD GPU node exists, else None (no GPUs on this node)."""
    if name == "fake" or fake_spec:
        return FakeBackend.from_spec(fake_spec or {})
    if name == "sysfs":
        return SysfsBackend()
    if name == "amdsmi":
        return AmdSmiBackend()
    sysfs = SysfsBackend()
    try:
        has_gpu = bool(sysfs.devices())
    except OSError:
        has_gpu = False
    if not has_gpu:
        return None
    try:
        return AmdSmiBackend()
    except Exception:
        return sysfs
