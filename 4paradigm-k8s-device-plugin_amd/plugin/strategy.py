"""Partition strategies: which resources the plugin advertises (the MIG-strategy analogue).

Reference: ``mig-strategy.go`` — ``none`` (one ``nvidia.com/gpu`` plugin over full
GPUs, :62-75), ``single`` (every GPU MIG-enabled with one profile, devices exposed as
``nvidia.com/gpu``, :78-164), ``mixed`` (full-GPU plugin plus one plugin per MIG profile
``nvidia.com/mig-<g>g.<gb>gb`` on socket ``nvidia-<res>.sock``, :167-239).

MI355X: compute partitions (SPX/DPX/QPX/CPX) x memory partitions (NPS1/NPS2) are set by
the driver; each partition is its own KFD node / render node, i.e. a GPU to ROCr.
* ``none``   every KFD device is a GPU and is split into vGPUs under ``amd.com/gpu``;
* ``single`` all devices must share one partition mode; partitions are whole devices
             under ``amd.com/gpu`` (no vGPU split), SPX-only nodes fall back to ``none``;
* ``mixed``  unpartitioned GPUs become vGPUs under ``amd.com/gpu``; each partition mode
             gets its own resource ``amd.com/<cpx>-<nps>`` (e.g. ``amd.com/cpx-nps2``),
             socket ``amd-<cpx>-<nps>.sock``, whole-device allocation.
"""
from dataclasses import replace

from .config import PARTITION_MIXED, PARTITION_NONE, PARTITION_SINGLE
from .server import DevicePluginServer

GPU_SOCKET = "amd-vgpu.sock"
LATENCY_SOCKET = "amd-vgpu-latency.sock"
LATENCY_SUFFIX = "-latency"


def partition_profile(d):
    return f"{d.compute_partition.lower()}-{d.memory_partition.lower()}"


def plugins_for(cfg, devices, backend=None, legacy_factory=None, pod_matcher=None):
    """Returns the DevicePluginServer list for the configured strategy. Checks that the
    node's RAM backs the host spill the memory scaling promises and resolves the per-vGPU
    host-memory budget first (plugin/host_memory.py)."""
    from .host_memory import check_spill_fits, host_budget_per_vgpu
    check_spill_fits(cfg, devices)
    cfg.host_budget_bytes = host_budget_per_vgpu(cfg, devices)
    strategy = cfg.partition_strategy
    if strategy == PARTITION_NONE:
        as_gpus = [replace(d, compute_partition="SPX") if d.is_partition else d for d in devices]
        return _flat([_gpu_plugin(cfg, as_gpus, backend, legacy_factory, pod_matcher)])
    if strategy == PARTITION_SINGLE:
        profiles = {partition_profile(d) for d in devices}
        if len(profiles) > 1:
            raise ValueError(f"partition strategy 'single' needs one partition mode on all GPUs, found "
                             f"{sorted(profiles)}")
        if not any(d.is_partition for d in devices):
            return _flat([_gpu_plugin(cfg, devices, backend, legacy_factory, pod_matcher)])
        return [DevicePluginServer(cfg, cfg.resource_name, GPU_SOCKET, devices, backend, partition_resource=True)]
    if strategy == PARTITION_MIXED:
        full = [d for d in devices if not d.is_partition]
        plugins = _flat([_gpu_plugin(cfg, full, backend, legacy_factory, pod_matcher)])
        by_profile = {}
        for d in devices:
            if d.is_partition:
                by_profile.setdefault(partition_profile(d), []).append(d)
        base = cfg.resource_name.split("/")[0]
        for prof, devs in sorted(by_profile.items()):
            plugins.append(DevicePluginServer(cfg, f"{base}/{prof}", f"amd-{prof}.sock", devs, backend,
                                              partition_resource=True))
        return plugins
    raise ValueError(f"unknown partition strategy {strategy!r}")


def _gpu_plugin(cfg, devices, backend, legacy_factory, pod_matcher):
    """The vGPU resource; with --latency-vgpus-per-gpu K > 0 the last K vGPUs of every GPU
    are served as <resource>-latency instead (a second plugin on its own socket), which grants
    the latency class: a namespace's ResourceQuota on it is the operator's control over who
    may run latency-critical work (VGPU_TASK_PRIORITY=0 is clamped to 1 elsewhere)."""
    k = getattr(cfg, "latency_vgpus_per_gpu", 0) or 0
    regular = None if not k else (lambda v, n=cfg.device_split_count - k: v.slot < n)
    p = DevicePluginServer(cfg, cfg.resource_name, GPU_SOCKET, devices, backend, pod_matcher=pod_matcher,
                           vdev_filter=regular)
    if legacy_factory is not None and cfg.enable_legacy_preferred:
        p.initialize()
        p.legacy = legacy_factory([v.id for v in p.vdevices])
    if not k:
        return p
    lat = DevicePluginServer(cfg, cfg.resource_name + LATENCY_SUFFIX, LATENCY_SOCKET, devices, backend,
                             pod_matcher=pod_matcher, vdev_filter=lambda v, n=cfg.device_split_count - k: v.slot >= n,
                             latency=True)
    return [p, lat]


def _flat(items):
    out = []
    for i in items:
        out.extend(i if isinstance(i, list) else [i])
    return out
