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


def partition_profile(d):
    return f"{d.compute_partition.lower()}-{d.memory_partition.lower()}"


def plugins_for(cfg, devices, backend=None, legacy_factory=None, pod_matcher=None):
    """Returns the DevicePluginServer list for the configured strategy."""
    strategy = cfg.partition_strategy
    if strategy == PARTITION_NONE:
        as_gpus = [replace(d, compute_partition="SPX") if d.is_partition else d for d in devices]
        return [_gpu_plugin(cfg, as_gpus, backend, legacy_factory, pod_matcher)]
    if strategy == PARTITION_SINGLE:
        profiles = {partition_profile(d) for d in devices}
        if len(profiles) > 1:
            raise ValueError(f"partition strategy 'single' needs one partition mode on all GPUs, found "
                             f"{sorted(profiles)}")
        if not any(d.is_partition for d in devices):
            return [_gpu_plugin(cfg, devices, backend, legacy_factory, pod_matcher)]
        return [DevicePluginServer(cfg, cfg.resource_name, GPU_SOCKET, devices, backend, partition_resource=True)]
    if strategy == PARTITION_MIXED:
        full = [d for d in devices if not d.is_partition]
        plugins = [_gpu_plugin(cfg, full, backend, legacy_factory, pod_matcher)]
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
    p = DevicePluginServer(cfg, cfg.resource_name, GPU_SOCKET, devices, backend, pod_matcher=pod_matcher)
    if legacy_factory is not None and cfg.enable_legacy_preferred:
        p.initialize()
        p.legacy = legacy_factory([v.id for v in p.vdevices])
    return p
