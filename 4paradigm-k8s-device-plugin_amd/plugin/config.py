"""Plugin flags with environment fallbacks and validation.

Reference: ``main.go:55-133`` (11 urfave/cli flags, each with an env var) and
``validateFlags`` (``main.go:143-161``). Same flag names where the concept carries
over; NVIDIA-specific names get AMD equivalents (``--mig-strategy`` is accepted as an
alias of ``--partition-strategy``) and MI355X-only knobs are added (CU-limit mode,
device backend, paths used by the stub-kubelet tests).
"""
import argparse
import os
from dataclasses import dataclass, field

PARTITION_NONE, PARTITION_SINGLE, PARTITION_MIXED = "none", "single", "mixed"
LIST_ENVVAR, LIST_AMD_RUNTIME, LIST_VOLUME_MOUNTS = "envvar", "amd-container-runtime", "volume-mounts"
ID_UUID, ID_INDEX = "uuid", "index"
CU_MODES = ("auto", "spatial", "temporal", "both", "off")
PLACEMENTS = ("spread", "binpack")
DUPLICATE_POLICIES = ("reject", "merge", "split")
NUMA_SPREAD_MODES = ("auto", "on", "off")
DEFAULT_RESOURCE = "amd.com/gpu"
DEFAULT_PLUGIN_DIR = "/var/lib/kubelet/device-plugins/"
DEFAULT_VGPU_DIR = "/usr/local/vgpu"


def _env_bool(v, default):
    if v is None:
        return default
    return str(v).strip().lower() in ("1", "true", "yes", "on")


@dataclass
class PluginConfig:
    partition_strategy: str = PARTITION_NONE
    fail_on_init_error: bool = True
    pass_device_specs: bool = True           # AMD has no runtime hook: default on
    device_list_strategy: str = LIST_ENVVAR
    device_id_strategy: str = ID_UUID
    driver_root: str = "/"
    device_split_count: int = 2
    device_memory_scaling: float = 1.0
    device_cores_scaling: float = 1.0
    enable_legacy_preferred: bool = False
    verbose: int = 0
    # MI355X additions
    cu_mode: str = "auto"
    backend: str = "auto"
    fake_devices: str = ""
    resource_name: str = DEFAULT_RESOURCE
    device_plugin_path: str = DEFAULT_PLUGIN_DIR
    vgpu_dir: str = DEFAULT_VGPU_DIR
    monitor_mode: bool = False
    pcibus_file: str = ""
    disable_healthchecks: str = ""          # DP_DISABLE_HEALTHCHECKS: "all" | "events"/"xids"
    health_interval_s: float = 5.0
    node_name: str = ""
    shared_cache_dir: str = "/tmp"
    placement: str = "spread"               # which GPU a 1-vGPU pod lands on (GetPreferredAllocation)
    duplicate_vgpus: str = "split"          # Allocate of two vGPUs of one GPU: split (one device per vGPU, as the
                                            # reference) | merge (one device, summed share) | reject
    host_memory_per_vgpu: str = "auto"      # pinned host memory budget per vGPU (auto: a share of the node's RAM; 0 = unlimited)
    host_memory_fraction: float = 0.5       # of the node's RAM, what vGPU containers may pin in total (buffers + spill)
    host_memory_total: str = ""             # the node's RAM (default: /proc/meminfo MemTotal)
    allow_latency_class: bool = False       # every container may take VGPU_TASK_PRIORITY=0
    latency_vgpus_per_gpu: int = 0          # vGPUs per GPU advertised as <resource>-latency (latency class granted)
    host_budget_bytes: int = -1             # resolved per-vGPU host budget (plugin/host_memory.py; -1 = not yet)
    gpu_concurrency: int = -1               # limited containers holding a GPU's time at once (0 = any, -1 = auto:
                                            # cross-socket pairs while the GPU is dispatch-bound and no bursty
                                            # serving pod is busy on it, profiles/r6k, r6a5)
    ledger: bool = True                     # run the node's GPU-time ledger daemon (vgpu-ledger; profiles/r4o)
    pod_resources_socket: str = "/var/lib/kubelet/pod-resources/kubelet.sock"  # kubelet PodResources v1
    active_oom_killer: bool = True          # the containers' memory backstop (limits file; reference ACTIVE_OOM_KILLER)
    numa_spread: str = "auto"               # co-tenant pods of a GPU on different CPU sockets: auto | on | off
    version_requested: bool = False
    extra: dict = field(default_factory=dict)

    @property
    def kubelet_socket(self):
        return os.path.join(self.device_plugin_path, "kubelet.sock")

    def validate(self):
        if self.partition_strategy not in (PARTITION_NONE, PARTITION_SINGLE, PARTITION_MIXED):
            raise ValueError(f"invalid --partition-strategy option: {self.partition_strategy}")
        if self.device_list_strategy not in (LIST_ENVVAR, LIST_AMD_RUNTIME, LIST_VOLUME_MOUNTS):
            raise ValueError(f"invalid --device-list-strategy option: {self.device_list_strategy}")
        if self.device_id_strategy not in (ID_UUID, ID_INDEX):
            raise ValueError(f"invalid --device-id-strategy option: {self.device_id_strategy}")
        if self.device_split_count < 1:
            raise ValueError(f"invalid --device-split-count option: {self.device_split_count}")
        if self.device_memory_scaling <= 0:
            raise ValueError(f"invalid --device-memory-scaling option: {self.device_memory_scaling}")
        if self.device_cores_scaling <= 0:
            raise ValueError(f"invalid --device-cores-scaling option: {self.device_cores_scaling}")
        if self.cu_mode not in CU_MODES:
            raise ValueError(f"invalid --cu-mode option: {self.cu_mode}")
        if self.placement not in PLACEMENTS:
            raise ValueError(f"invalid --placement option: {self.placement}")
        if self.duplicate_vgpus not in DUPLICATE_POLICIES:
            raise ValueError(f"invalid --duplicate-vgpus option: {self.duplicate_vgpus}")
        if self.numa_spread not in NUMA_SPREAD_MODES:
            raise ValueError(f"invalid --numa-spread option: {self.numa_spread}")
        if not -1 <= self.gpu_concurrency <= 64:
            raise ValueError(f"invalid --gpu-concurrency option: {self.gpu_concurrency}")
        from ..utils.sizes import parse_size
        if self.host_memory_per_vgpu != "auto":
            try:
                parse_size(self.host_memory_per_vgpu)
            except ValueError:
                raise ValueError(f"invalid --host-memory-per-vgpu option: {self.host_memory_per_vgpu}") from None
        if not 0.0 <= self.host_memory_fraction <= 1.0:
            raise ValueError(f"invalid --host-memory-fraction option: {self.host_memory_fraction}")
        if self.host_memory_total:
            try:
                parse_size(self.host_memory_total)
            except ValueError:
                raise ValueError(f"invalid --host-memory-total option: {self.host_memory_total}") from None
        if self.latency_vgpus_per_gpu < 0 or (self.latency_vgpus_per_gpu and
                                              self.latency_vgpus_per_gpu >= self.device_split_count):
            raise ValueError(f"invalid --latency-vgpus-per-gpu option: {self.latency_vgpus_per_gpu} (at most "
                             f"--device-split-count - 1 = {self.device_split_count - 1})")
        return self

    @property
    def host_memory_per_vgpu_bytes(self):
        """The explicit per-vGPU budget (0 = unlimited); "auto" is resolved against the node
        by host_memory.host_budget_per_vgpu."""
        from ..utils.sizes import parse_size
        return 0 if self.host_memory_per_vgpu == "auto" else parse_size(self.host_memory_per_vgpu)


# (flag, dest, type, env vars, help)
def concurrency_value(v):
    """--gpu-concurrency: an int (0..64) or "auto" (-1)."""
    return -1 if str(v).strip().lower() == "auto" else int(v)


_FLAGS = [
    ("--partition-strategy", "partition_strategy", str, ["PARTITION_STRATEGY", "MIG_STRATEGY"],
     "compute/memory partition strategy: none | single | mixed"),
    ("--fail-on-init-error", "fail_on_init_error", "bool", ["FAIL_ON_INIT_ERROR"],
     "fail the plugin if device discovery fails (false: wait forever, for non-GPU nodes)"),
    ("--pass-device-specs", "pass_device_specs", "bool", ["PASS_DEVICE_SPECS"],
     "pass /dev/kfd and /dev/dri nodes to the kubelet as DeviceSpecs"),
    ("--device-list-strategy", "device_list_strategy", str, ["DEVICE_LIST_STRATEGY"],
     "how visible devices reach the container: envvar | amd-container-runtime | volume-mounts"),
    ("--device-id-strategy", "device_id_strategy", str, ["DEVICE_ID_STRATEGY"], "uuid | index"),
    ("--driver-root", "driver_root", str, ["AMD_DRIVER_ROOT", "DRIVER_ROOT", "NVIDIA_DRIVER_ROOT"],
     "root of the host's /dev tree"),
    ("--device-split-count", "device_split_count", int, ["DEVICE_SPLIT_COUNT"], "vGPUs per physical GPU"),
    ("--device-memory-scaling", "device_memory_scaling", float, ["DEVICE_MEMORY_SCALING"],
     "memory oversubscription ratio (>1 spills to host memory)"),
    ("--device-cores-scaling", "device_cores_scaling", float, ["DEVICE_CORES_SCALING"],
     "compute oversubscription ratio (CU share = 100 * scaling / split)"),
    ("--enable-legacy-preferred", "enable_legacy_preferred", "bool", ["ENABLE_LEGACY_PREFERRED"],
     "preferred allocation for kubelets without GetPreferredAllocation"),
    ("--verbose", "verbose", int, ["VERBOSE"], "log verbosity"),
    ("--cu-mode", "cu_mode", str, ["CU_MODE"], "CU limit enforcement: auto (CU masks for shares >= 50 %% and while the GPU is not crowded, "
     "the GPU-time limiter for smaller shares on a crowded GPU) | spatial | "
     "temporal | both | off"),
    ("--backend", "backend", str, ["DEVICE_BACKEND"], "device backend: auto | amdsmi | sysfs | fake"),
    ("--fake-devices", "fake_devices", str, ["FAKE_DEVICES"], "JSON spec (or file) for the fake backend"),
    ("--resource-name", "resource_name", str, ["RESOURCE_NAME"], "extended resource name"),
    ("--device-plugin-path", "device_plugin_path", str, ["DEVICE_PLUGIN_PATH"], "kubelet device-plugin dir"),
    ("--vgpu-dir", "vgpu_dir", str, ["VGPU_DIR"], "host dir holding the shim (/usr/local/vgpu)"),
    ("--monitor-mode", "monitor_mode", "bool", ["VGPU_MONITOR_MODE"],
     "expose each container's region on a host path for the node monitor"),
    ("--pcibus-file", "pcibus_file", str, ["VGPU_PCIBUS_FILE", "PCIBUSFILE"], "write the GPU BDF list here"),
    ("--health-interval", "health_interval_s", float, ["HEALTH_INTERVAL"], "health poll period (s)"),
    ("--node-name", "node_name", str, ["NODE_NAME"], "this node (legacy-preferred / monitor mode)"),
    ("--placement", "placement", str, ["PLACEMENT_POLICY"],
     "GPU choice for a new pod: spread (the GPU with the most free vGPUs) | binpack (the fullest GPU with room)"),
    ("--duplicate-vgpus", "duplicate_vgpus", str, ["DUPLICATE_VGPUS"],
     "a container given two vGPUs of one GPU: split (default, as the reference: one HIP device per vGPU, each "
     "with its own quota; the shim virtualises the device ordinals, VGPU_DUPLICATE_SPLIT) | merge (one device with "
     "the summed quota and CU share; VGPU_DUPLICATE_MERGED and the amd-vgpu/merged-duplicates annotation tell the "
     "container) | reject (fail Allocate)"),
    ("--host-memory-per-vgpu", "host_memory_per_vgpu", str, ["HOST_MEMORY_PER_VGPU"],
     "pinned host memory (hipHostMalloc / hipHostRegister, and the host spill of oversubscribed vGPUs) per vGPU, "
     "e.g. 64g; auto (default) = --host-memory-fraction of the node's RAM divided among its vGPUs; "
     "0 = unlimited (tracked only)"),
    ("--host-memory-fraction", "host_memory_fraction", float, ["HOST_MEMORY_FRACTION"],
     "share of the node's RAM vGPU containers may pin in total (default 0.5); --device-memory-scaling whose "
     "host spill would not fit in it is refused at start; 0 = no node bound (neither the check nor an automatic "
     "per-vGPU budget: the reference's behaviour)"),
    ("--host-memory-total", "host_memory_total", str, ["HOST_MEMORY_TOTAL"],
     "the node's RAM for the budgets above (default: MemTotal from /proc/meminfo)"),
    ("--allow-latency-class", "allow_latency_class", "bool", ["ALLOW_LATENCY_CLASS"],
     "let every container take the latency class (VGPU_TASK_PRIORITY=0: high queue priority, never duty-cycled, "
     "reserves its CUs against background tenants); off by default: the class is granted by the plugin only"),
    ("--latency-vgpus-per-gpu", "latency_vgpus_per_gpu", int, ["LATENCY_VGPUS_PER_GPU"],
     "of each GPU's split vGPUs, this many are advertised as <resource>-latency (e.g. amd.com/gpu-latency), which "
     "grants the latency class; an operator bounds it per namespace with a ResourceQuota (default 0)"),
    ("--gpu-concurrency", "gpu_concurrency", concurrency_value, ["GPU_CONCURRENCY"],
     "containers on the GPU-time limiter that may hold a GPU at once, taking turns over the node-wide board, in "
     "pairs of different CPU sockets when --numa-spread places them (0 = no admission: every container whose credit "
     "allows runs; auto = pairs while the GPU's containers launch more than VGPU_PAIRS_ON_RATE (40k) kernels/s "
     "together - dispatch-bound pods, which three at once slow down - and no container that launches in bursts (a "
     "serving pod) is busy there, everybody at once otherwise; the default)"),
    ("--ledger", "ledger", "bool", ["VGPU_NODE_LEDGER"],
     "run the node GPU-time ledger (vgpu-ledger): one KFD occupancy sampler for every limited container of the "
     "node instead of one per container (n reads per period instead of n^2, one consistent snapshot), and "
     "exact GPU-time shares (VGPU_DEVICE_CU_SHARE) for the containers; on by default (12 and 16 pods: "
     "1.07-1.09x aggregate, slowest pod 0.91-1.01 of 1/N, profiles/r4o); --ledger=false: every container "
     "samples by itself"),
    ("--pod-resources-socket", "pod_resources_socket", str, ["POD_RESOURCES_SOCKET"],
     "kubelet PodResources socket: monitor mode attributes container directories to the pods holding their "
     "vGPUs through it, and a container's host files (limits, region, allow-list, board slot) are removed only "
     "once it lists the container's devices as free (missing socket: nothing is removed)"),
    ("--active-oom-killer", "active_oom_killer", "bool", ["ACTIVE_OOM_KILLER"],
     "the containers' memory backstop: kill a container's largest process when KFD-measured VRAM stays above "
     "its quota (plus a slack); written into the plugin-owned limits file, so a tenant cannot turn it off "
     "(default true, as the reference's ACTIVE_OOM_KILLER)"),
    ("--numa-spread", "numa_spread", str, ["NUMA_SPREAD"],
     "run the processes of vGPU k of a GPU on the CPUs of NUMA node order[k mod n] (the GPU's own node first, "
     "then the others): two launch-bound pods of one GPU whose threads share a CPU socket run no faster together "
     "than one alone, on two sockets up to twice as fast (profiles/r5d). The shim narrows a container's CPU "
     "affinity to that node when its allowed CPUs span more (VGPU_CPU_NODE; a tenant opts out with "
     "VGPU_CPU_SPREAD=0), and ListAndWatch advertises the node as the vGPU's topology. auto (default) = on for "
     "split > 1 on nodes with two or more CPU nodes | on | off"),
]


def build_parser():
    ap = argparse.ArgumentParser(prog="amd-vgpu-device-plugin",
                                 description="MI355X vGPU device plugin for Kubernetes")
    for flag, dest, typ, envs, help_ in _FLAGS:
        # The reference's flag names stay accepted, so its manifests work unchanged.
        names = [flag] + {"partition_strategy": ["--mig-strategy"], "driver_root": ["--nvidia-driver-root"]}.get(dest, [])
        if typ == "bool":
            ap.add_argument(*names, dest=dest, nargs="?", const="true", default=None,
                            help=f"{help_} (env {', '.join(envs)})")
        else:
            ap.add_argument(*names, dest=dest, type=typ, default=None, help=f"{help_} (env {', '.join(envs)})")
    ap.add_argument("--version", action="store_true")
    return ap


def parse_config(argv=None, environ=None):
    """Flags > env vars > defaults, then validate (reference: cli flag EnvVars + Before)."""
    environ = os.environ if environ is None else environ
    ns = build_parser().parse_args(argv)
    cfg = PluginConfig()
    for _flag, dest, typ, envs, _h in _FLAGS:
        val = getattr(ns, dest)
        if val is None:
            for e in envs:
                if e in environ and environ[e] != "":
                    val = environ[e]
                    break
        if val is None:
            continue
        if typ == "bool":
            val = _env_bool(val, getattr(cfg, dest))
        elif typ in (int, float, concurrency_value):
            val = typ(val)
        setattr(cfg, dest, val)
    cfg.disable_healthchecks = environ.get("DP_DISABLE_HEALTHCHECKS", "")
    if not cfg.device_plugin_path.endswith("/"):
        cfg.device_plugin_path += "/"
    cfg.version_requested = bool(ns.version)
    return cfg.validate()
