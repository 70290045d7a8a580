"""Host memory the vGPU containers of a node may pin: a budget per vGPU, and the check
that oversubscription's host spill fits in the node's RAM.

Reference: the shim OOM-checks every host allocation (class (b): cuMemAllocHost_v2,
cuMemHostAlloc, cuMemHostRegister_v2), and --device-memory-scaling > 1
turns every allocation into managed memory that the UVM driver pages to host RAM
(``server.go:505-507``) - with no bound on how much RAM that promises.

Here page-locked memory is one node-wide resource with two consumers: pinned buffers
(hipHostMalloc / hipHostRegister) and the host spill of oversubscribed vGPUs (pinned host
memory the GPU reads, ``hsa_hooks.cpp``). Both are charged to the container's host budget
(VGPU_HOST_MEMORY_LIMIT). By default the budget is ``--host-memory-fraction`` (0.5) of the
node's RAM divided among its vGPUs, and the plugin refuses to start with a memory scaling
whose total spill - split x (quota - HBM share) on every GPU, i.e. HBM x (scaling - 1) per
GPU - would not fit in that fraction: 8 MI355X at scaling 3 promise 4.6 TB of pinned RAM.
"""
import logging

from ..utils.sizes import parse_size

log = logging.getLogger("amdvgpu.plugin")


def node_memory_total(cfg, meminfo="/proc/meminfo"):
    """The node's RAM in bytes: --host-memory-total, else MemTotal (0 if unknown)."""
    if cfg.host_memory_total:
        return parse_size(cfg.host_memory_total)
    try:
        with open(meminfo) as f:
            for line in f:
                if line.startswith("MemTotal:"):
                    return int(line.split()[1]) * 1024
    except (OSError, ValueError, IndexError):
        pass
    return 0


def _vgpu_devices(devices):
    return [d for d in devices if not getattr(d, "is_partition", False)]


def spill_bytes(cfg, devices):
    """Host memory oversubscription promises over all GPUs of the node."""
    if cfg.device_memory_scaling <= 1:
        return 0
    return int(sum(d.memory_total for d in _vgpu_devices(devices)) * (cfg.device_memory_scaling - 1))


def check_spill_fits(cfg, devices, total=None):
    """Raises ValueError when the node cannot back the spill of every vGPU at once."""
    spill = spill_bytes(cfg, devices)
    if not spill or not cfg.host_memory_fraction:
        return
    total = node_memory_total(cfg) if total is None else total
    if not total:
        log.warning("node RAM unknown: the host spill of --device-memory-scaling %s (%d GiB) is not checked",
                    cfg.device_memory_scaling, spill >> 30)
        return
    room = int(total * cfg.host_memory_fraction)
    if spill > room:
        raise ValueError(f"--device-memory-scaling {cfg.device_memory_scaling} promises {spill >> 30} GiB of pinned "
                         f"host memory for spilled device memory, more than --host-memory-fraction "
                         f"{cfg.host_memory_fraction} of the node's {total >> 30} GiB ({room >> 30} GiB)")


def host_budget_per_vgpu(cfg, devices, total=None):
    """Bytes of pinned host memory per vGPU (0 = unlimited): the explicit
    --host-memory-per-vgpu, or (auto) the node fraction divided among its vGPUs, never less
    than one vGPU's spill."""
    if cfg.host_memory_per_vgpu != "auto":
        return cfg.host_memory_per_vgpu_bytes
    devs = _vgpu_devices(devices)
    n = len(devs) * max(1, cfg.device_split_count)
    total = node_memory_total(cfg) if total is None else total
    if not n or not total or not cfg.host_memory_fraction:
        return 0
    budget = int(total * cfg.host_memory_fraction) // n
    spill_per = spill_bytes(cfg, devs) // n
    return max(budget, spill_per)
