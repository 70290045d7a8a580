"""ctypes binding of ``libvgpu_region.so``: the shared accounting region of a container.

The node-side view of what the shim enforces (same code path: the library is built from
the same ``native/src/core`` objects the shim links). Used by the monitor
(``plugin/monitor.py``), by tests, and by the benchmarks to read per-container usage,
limits, CU masks, throttle time and suspend state, and to drive the control API the
reference exported from libvgpu.so (``suspend_all``/``resume_all``/
``set_current_device_memory_limit``/``set_current_device_sm_limit_scale``,
SURVEY.md §2.3 N15).
"""
import ctypes as C
import os

from .native import REGION, lib_path

MAX_DEVICES = 16
MAX_PROCS = 1024
MEM_KINDS = ("data", "context", "module", "spill")


class ProcInfo(C.Structure):
    _fields_ = [
        ("pid", C.c_int32), ("hostpid", C.c_int32), ("status", C.c_int32), ("priority", C.c_int32),
        ("launches", C.c_uint64), ("throttle_ns", C.c_uint64), ("suspend_ns", C.c_uint64),
        ("oom_events", C.c_uint64), ("used", C.c_uint64 * 16), ("used_kind", (C.c_uint64 * 4) * 16),
        ("peak", C.c_uint64 * 16), ("host_used", C.c_uint64), ("host_peak", C.c_uint64),
    ]


CU_MODES = {0: "off", 1: "spatial", 2: "temporal", 3: "both"}


class DeviceInfo(C.Structure):
    _fields_ = [
        ("uuid", C.c_char * 64), ("mem_limit", C.c_uint64), ("phys_total", C.c_uint64), ("used", C.c_uint64),
        ("spilled", C.c_uint64), ("monitor_used", C.c_uint64), ("cu_limit_pct", C.c_int32),
        ("cu_count", C.c_int32), ("num_xcc", C.c_int32), ("cu_mask_count", C.c_int32),
        ("cu_mask", C.c_uint32 * 8), ("credit_ns", C.c_int64), ("charged_ns", C.c_uint64),
        ("wall_ns", C.c_uint64), ("util_pct", C.c_int32), ("cu_mode", C.c_int32), ("gpu_id", C.c_uint32), ("bdf", C.c_uint32), ("domain", C.c_uint32), ("configured", C.c_uint32),
        ("hbm_limit", C.c_uint64), ("crowd", C.c_int32), ("preempt", C.c_int32), ("depth_cap", C.c_int32),
        ("cu_share_bp", C.c_int32),
    ]


_lib = None


def lib():
    global _lib
    if _lib is None:
        L = C.CDLL(lib_path(REGION))
        P = C.c_void_p
        sig = {
            "vgpu_region_open": (P, [C.c_char_p, C.c_int, C.POINTER(C.c_int)]),
            "vgpu_region_close": (None, [P]),
            "vgpu_region_version": (C.c_uint32, []),
            "vgpu_region_size": (C.c_uint64, []),
            "vgpu_region_num_devices": (C.c_int, [P]),
            "vgpu_region_device_info": (C.c_int, [P, C.c_int, C.POINTER(DeviceInfo)]),
            "vgpu_region_proc_count": (C.c_int, [P]),
            "vgpu_region_procs": (C.c_int, [P, C.POINTER(ProcInfo), C.c_int]),
            "vgpu_region_set_memory_limit": (C.c_int, [P, C.c_int, C.c_uint64]),
            "vgpu_region_set_cu_limit": (C.c_int, [P, C.c_int, C.c_int]),
            "vgpu_region_set_cu_share": (C.c_int, [P, C.c_int, C.c_int]),
            "vgpu_region_set_hbm_limit": (C.c_int, [P, C.c_int, C.c_uint64]),
            "vgpu_region_suspend_all": (C.c_int, [P]),
            "vgpu_region_resume_all": (C.c_int, [P]),
            "vgpu_region_suspended": (C.c_int, [P]),
            "vgpu_region_set_priority": (C.c_int, [P, C.c_int]),
            "vgpu_region_get_priority": (C.c_int, [P]),
            "vgpu_region_set_recent_kernel": (C.c_int, [P, C.c_int]),
            "vgpu_region_get_recent_kernel": (C.c_int, [P]),
            "vgpu_region_set_utilization_switch": (C.c_int, [P, C.c_int]),
            "vgpu_region_reclaim": (C.c_int, [P]),
            "vgpu_region_host_info": (C.c_int, [P, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
            "vgpu_region_set_host_limit": (C.c_int, [P, C.c_uint64]),
            "vgpu_region_charge_host": (C.c_int, [P, C.c_int, C.c_uint64]),
            "vgpu_region_uncharge_host": (None, [P, C.c_int, C.c_uint64]),
            "vgpu_region_samples": (C.c_uint64, [P]),
            "vgpu_region_other_refreshes": (C.c_uint64, [P]),
            "vgpu_region_register": (C.c_int, [P, C.c_int32, C.c_int32]),
            "vgpu_region_unregister": (None, [P, C.c_int]),
            "vgpu_region_charge": (C.c_int, [P, C.c_int, C.c_int, C.c_uint64, C.c_int]),
            "vgpu_region_uncharge": (None, [P, C.c_int, C.c_int, C.c_uint64, C.c_int]),
            "vgpu_cu_share_count": (C.c_int, [C.c_int, C.c_int, C.c_int]),
            "vgpu_cu_partition_range": (None, [C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_int),
                                               C.POINTER(C.c_int)]),
            "vgpu_parse_size": (C.c_int64, [C.c_char_p]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def cu_share_count(cu_count, num_xcc, pct):
    return lib().vgpu_cu_share_count(cu_count, num_xcc, pct)


def cu_partition_range(cu_count, num_xcc, split, slot):
    b, e = C.c_int(), C.c_int()
    lib().vgpu_cu_partition_range(cu_count, num_xcc, split, slot, C.byref(b), C.byref(e))
    return b.value, e.value


def native_parse_size(text):
    return lib().vgpu_parse_size(str(text).encode())


class Region:
    """An attached shared-region file (``VGPU_SHARED_CACHE``)."""

    def __init__(self, path, create=False):
        self.path = os.fspath(path)
        err = C.c_int(0)
        self._h = lib().vgpu_region_open(self.path.encode(), 1 if create else 0, C.byref(err))
        if not self._h:
            raise OSError(-err.value, f"cannot open vGPU region {self.path}: {os.strerror(-err.value)}")

    def close(self):
        if self._h:
            lib().vgpu_region_close(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # --- queries -------------------------------------------------------------
    @property
    def num_devices(self):
        return lib().vgpu_region_num_devices(self._h)

    def device(self, dev):
        d = DeviceInfo()
        if lib().vgpu_region_device_info(self._h, dev, C.byref(d)) != 0:
            raise IndexError(dev)
        mask = 0
        for i, w in enumerate(d.cu_mask):
            mask |= int(w) << (32 * i)
        return {
            "index": dev, "uuid": d.uuid.decode(errors="replace"), "mem_limit": d.mem_limit,
            "phys_total": d.phys_total, "used": d.used, "spilled": d.spilled, "monitor_used": d.monitor_used,
            "cu_limit_pct": d.cu_limit_pct, "cu_count": d.cu_count, "num_xcc": d.num_xcc,
            "cu_mask_count": d.cu_mask_count, "cu_mask": mask, "credit_ns": d.credit_ns,
            "charged_ns": d.charged_ns, "wall_ns": d.wall_ns, "util_pct": d.util_pct,
            "cu_mode": CU_MODES.get(d.cu_mode, str(d.cu_mode)), "gpu_id": d.gpu_id, "bdf": d.bdf, "domain": d.domain,
            "configured": bool(d.configured), "hbm_limit": d.hbm_limit, "crowd": d.crowd,
            "preempt": bool(d.preempt), "depth_cap": d.depth_cap, "cu_share_bp": d.cu_share_bp,
        }

    def devices(self):
        return [self.device(i) for i in range(self.num_devices)]

    def procs(self):
        buf = (ProcInfo * MAX_PROCS)()
        n = lib().vgpu_region_procs(self._h, buf, MAX_PROCS)
        out = []
        for p in buf[:n]:
            out.append({
                "pid": p.pid, "hostpid": p.hostpid, "status": p.status, "priority": p.priority,
                "launches": p.launches, "throttle_ns": p.throttle_ns, "suspend_ns": p.suspend_ns,
                "oom_events": p.oom_events, "used": list(p.used),
                "used_kind": [dict(zip(MEM_KINDS, list(k))) for k in p.used_kind], "peak": list(p.peak),
                "host_used": p.host_used, "host_peak": p.host_peak,
            })
        return out

    def host(self):
        """Pinned host memory of the container: {"limit": bytes (0 = unlimited), "used": bytes}."""
        lim, used = C.c_uint64(), C.c_uint64()
        lib().vgpu_region_host_info(self._h, C.byref(lim), C.byref(used))
        return {"limit": lim.value, "used": used.value}

    @property
    def proc_count(self):
        return lib().vgpu_region_proc_count(self._h)

    def snapshot(self):
        return {
            "path": self.path, "version": lib().vgpu_region_version(), "suspended": self.suspended,
            "priority": self.priority, "recent_kernel": self.recent_kernel, "samples": self.samples,
            "other_refreshes": self.other_refreshes, "host": self.host(),
            "devices": self.devices(),
            "procs": self.procs(),
        }

    # --- control API ---------------------------------------------------------
    def set_memory_limit(self, dev, nbytes):
        return lib().vgpu_region_set_memory_limit(self._h, dev, int(nbytes))

    def set_host_limit(self, nbytes):
        return lib().vgpu_region_set_host_limit(self._h, int(nbytes))

    def set_cu_limit(self, dev, pct):
        return lib().vgpu_region_set_cu_limit(self._h, dev, int(pct))

    def set_cu_share(self, dev, bp):
        """Exact GPU-time share of the limiter's grants, basis points (0 = the CU limit)."""
        return lib().vgpu_region_set_cu_share(self._h, dev, int(bp))

    def set_hbm_limit(self, dev, nbytes):
        """HBM-resident share of an oversubscribed vGPU (0 = no cap)."""
        return lib().vgpu_region_set_hbm_limit(self._h, dev, int(nbytes))

    def suspend_all(self):
        return lib().vgpu_region_suspend_all(self._h)

    def resume_all(self):
        return lib().vgpu_region_resume_all(self._h)

    @property
    def suspended(self):
        return bool(lib().vgpu_region_suspended(self._h))

    @property
    def priority(self):
        return lib().vgpu_region_get_priority(self._h)

    @priority.setter
    def priority(self, v):
        lib().vgpu_region_set_priority(self._h, int(v))

    @property
    def recent_kernel(self):
        return lib().vgpu_region_get_recent_kernel(self._h)

    @recent_kernel.setter
    def recent_kernel(self, v):
        lib().vgpu_region_set_recent_kernel(self._h, int(v))

    @property
    def samples(self):
        """Occupancy-sampler ticks so far (temporal mode)."""
        return lib().vgpu_region_samples(self._h)

    @property
    def other_refreshes(self):
        """Sampler ticks that re-read the other processes' occupancy."""
        return lib().vgpu_region_other_refreshes(self._h)

    def set_utilization_switch(self, v):
        return lib().vgpu_region_set_utilization_switch(self._h, int(v))

    def reclaim(self):
        return lib().vgpu_region_reclaim(self._h)

    # --- accounting (same admission path as the shim) -------------------------
    def register(self, pid, hostpid=0):
        return lib().vgpu_region_register(self._h, int(pid), int(hostpid))

    def unregister(self, slot):
        lib().vgpu_region_unregister(self._h, slot)

    def charge(self, slot, dev, nbytes, kind=0):
        return lib().vgpu_region_charge(self._h, slot, dev, int(nbytes), kind)

    def uncharge(self, slot, dev, nbytes, kind=0):
        lib().vgpu_region_uncharge(self._h, slot, dev, int(nbytes), kind)

    def charge_host(self, slot, nbytes):
        return lib().vgpu_region_charge_host(self._h, slot, int(nbytes))

    def uncharge_host(self, slot, nbytes):
        lib().vgpu_region_uncharge_host(self._h, slot, int(nbytes))
