"""The plugin -> shim contract: what ``Allocate`` puts into a ContainerAllocateResponse.

Reference: ``server.go:459-522`` (visible devices, DeviceSpecs, annotations,
``CUDA_DEVICE_MEMORY_LIMIT_<i>``, ``CUDA_DEVICE_SM_LIMIT``, ``NVIDIA_DEVICE_MAP``,
``CUDA_DEVICE_MEMORY_SHARED_CACHE``, ``CUDA_OVERSUBSCRIBE``, and the mounts of the shim,
``/etc/ld.so.preload``, ``pciinfo.vgpu``, the validator and the license dir), plus
``apiEnvs``/``apiMounts``/``apiDeviceSpecs`` (:598-655). Env names are the VGPU_*
equivalents read by ``native/src/core/config.cpp``.

Differences from the reference, by design:
* visible devices go through ``ROCR_VISIBLE_DEVICES`` (ROCr accepts ``GPU-<uuid>``) and
  the device nodes (/dev/kfd, /dev/dri/renderD*, /dev/dri/card*) are always passed as
  DeviceSpecs by default — AMD has no container-runtime hook that would add them;
* CU share and CU range are per vdevice (``VGPU_DEVICE_CU_LIMIT_<i>``/``_RANGE_<i>``),
  not one value for the whole container (quirk ``server.go:492``);
* with memory oversubscription the HBM-resident cap (``VGPU_DEVICE_HBM_LIMIT_<i>``)
  is the tenant's physical share and the rest of the quota spills to host memory;
* the pciinfo mount is only emitted when the BDF file exists (the reference mounts an
  empty host path when ``PCIBUSFILE`` is unset, ``server.go:516``).
"""
import os
import uuid as _uuid

from ..utils.sizes import format_mib
from . import api
from .config import ID_INDEX, LIST_AMD_RUNTIME, LIST_ENVVAR, LIST_VOLUME_MOUNTS

VISIBLE_ENV = "ROCR_VISIBLE_DEVICES"
AMD_RUNTIME_ENV = "AMD_VISIBLE_DEVICES"
VOLUME_MOUNTS_ROOT = "/var/run/amd-container-devices"
VOLUME_MOUNTS_HOST = "/dev/null"
CONTAINER_SHIM = "/usr/local/vgpu/libvgpu_hip.so"
CONTAINER_PRELOAD = "/etc/ld.so.preload"
CONTAINER_PCIINFO = "/usr/local/vgpu/pciinfo.vgpu"
CONTAINER_VALIDATOR = "/usr/bin/vgpu-validate"
CONTAINER_ALLOWLIST_DIR = "/vgpu"
SHARED_HOST_DIR = "shared"
# Host-PID discovery lock shared by every vGPU container of the node (the reference's
# "unified lock" /tmp/vgpulock/lock, utils.c:30-36, which only serialised one container):
# processes of different containers that start together take turns probing KFD. The
# plugin creates the file (root-owned, 0644) and every container gets it read-only: a
# tenant can take the lock (flock works on a read-only descriptor) but cannot unlink or
# replace it, and the shim probes unlocked once its wait times out, so holding it forever
# only delays neighbours (native/src/core/kfd.cpp).
LOCK_HOST_DIR = "lock"
LOCK_FILE = "hostpid.lock"
CONTAINER_LOCK_DIR = "/usr/local/vgpu/lock"


# Node-wide board (native/include/vgpu/board.h): every container reads every slot (the
# directory is mounted read-only) and writes only its own (its slot file is mounted
# read-write on top). Task-priority classes act on it: a background container yields GPU
# time to busy containers of higher priority.
BOARD_HOST_DIR = "board"
CONTAINER_BOARD_DIR = "/usr/local/vgpu/board"


def ensure_board_dir(vgpu_dir):
    d = os.path.join(vgpu_dir, BOARD_HOST_DIR)
    os.makedirs(d, mode=0o755, exist_ok=True)
    return d


def board_slot(vgpu_dir, name):
    """Creates this container's slot file (world-writable: the container's processes may
    run as any user; only this container mounts it read-write). Returns its path, or None
    when there is no board directory. Removed with the container's other files once its
    pod is gone (gc_container_files), never by age: an idle container's slot is still the
    source of its bind mount when the container restarts."""
    d = os.path.join(vgpu_dir, BOARD_HOST_DIR)
    if not os.path.isdir(d):
        return None
    path = os.path.join(d, name + ".slot")
    try:
        fd = os.open(path, os.O_WRONLY | os.O_CREAT, 0o666)
        os.close(fd)
        os.chmod(path, 0o666)
    except OSError:
        return None
    return path


def ensure_lock_file(vgpu_dir):
    """Creates <vgpu_dir>/lock/hostpid.lock (0644) if missing; returns its path."""
    d = os.path.join(vgpu_dir, LOCK_HOST_DIR)
    os.makedirs(d, mode=0o755, exist_ok=True)
    path = os.path.join(d, LOCK_FILE)
    if not os.path.exists(path):
        fd = os.open(path, os.O_WRONLY | os.O_CREAT, 0o644)
        os.close(fd)
    os.chmod(path, 0o644)
    return path
ANN_REQUEST = "amd-vgpu/request"
ANN_USING = "amd-vgpu/using"
ANN_DUPLICATES = "amd-vgpu/merged-duplicates"
ANN_SPLIT = "amd-vgpu/split-duplicates"


ALLOWLIST_HOST_DIR = "allowlist"

# Plugin-owned limits (tamper resistance, native/include/vgpu/config.h load_ceiling): the
# container's contract, written by the plugin into a root-owned file mounted read-only at
# CONTAINER_LIMITS. The shim treats it as a ceiling over its environment and its shared
# region, both of which the tenant controls; its region is a file the plugin creates, mounted
# over its path (a bind-mounted file cannot be unlinked from inside the container), whose
# inode the limits file records.
LIMITS_HOST_DIR = "limits"
CONTAINER_LIMITS = "/vgpu/limits"
REGIONS_HOST_DIR = "regions"
CONTAINER_REGION_DIR = "/usr/local/vgpu/regions"
# Per-container host files (limits, region, allow-list, board slot) are the sources of the
# container's bind mounts, which the kubelet reuses from its checkpoint when a container
# restarts (it does not call Allocate again). They live as long as the pod that holds the
# container's devices: each Allocate records the device IDs in a manifest
# (<vgpu_dir>/containers/<name>.devices), and gc_container_files removes a container's
# files only when the kubelet's PodResources no longer lists those devices as held - never
# by age (except files older than the manifests themselves, LEGACY_GC_AGE_S), and never when
# PodResources cannot be asked.
MANIFEST_HOST_DIR = "containers"
CONTAINER_GC_GRACE_S = 600
# The env names the limits file carries (the shim reads it with the env parser).
LIMIT_KEYS = ("VGPU_DEVICE_MAP", "VGPU_DEVICE_MEMORY_LIMIT_", "VGPU_DEVICE_HBM_LIMIT_", "VGPU_DEVICE_CU_LIMIT_",
              "VGPU_DEVICE_CU_SHARE_", "VGPU_DEVICE_CU_RANGE_", "VGPU_HOST_MEMORY_LIMIT", "VGPU_OVERSUBSCRIBE",
              "VGPU_CU_MODE", "VGPU_SHARED_CACHE", "VGPU_ALLOWLIST", "VGPU_BOARD_DIR", "VGPU_BOARD_SLOT",
              "VGPU_GPU_CONCURRENCY")


def write_manifest(vgpu_dir, name, resource, ids):
    """Records which devices (kubelet IDs of ``resource``) container ``name``'s files serve."""
    d = os.path.join(vgpu_dir, MANIFEST_HOST_DIR)
    try:
        os.makedirs(d, exist_ok=True)
        tmp = os.path.join(d, name + ".devices.tmp")
        with open(tmp, "w") as f:
            f.write(f"resource={resource}\n" + "".join(f"{i}\n" for i in sorted(ids)))
        os.replace(tmp, os.path.join(d, name + ".devices"))
    except OSError:
        return None
    return os.path.join(d, name + ".devices")


def _read_manifest(path):
    try:
        with open(path) as f:
            lines = [x.strip() for x in f if x.strip()]
    except OSError:
        return None, None
    res = lines[0][len("resource="):] if lines and lines[0].startswith("resource=") else ""
    return res, frozenset(x for x in lines if not x.startswith("resource="))


def container_files(vgpu_dir, name):
    """Host files of container ``name`` (what Allocate created for it)."""
    return [os.path.join(vgpu_dir, LIMITS_HOST_DIR, "containers", name + ".env"),
            os.path.join(vgpu_dir, REGIONS_HOST_DIR, name + ".cache"),
            os.path.join(vgpu_dir, ALLOWLIST_HOST_DIR, "containers", name + ".list"),
            os.path.join(vgpu_dir, BOARD_HOST_DIR, name + ".slot")]


def gc_container_files(vgpu_dir, held, grace_s=CONTAINER_GC_GRACE_S, now=None):
    """Removes the host files of containers whose pods are gone. ``held``: {resource: set of
    frozensets of device IDs} that live containers hold (kubelet PodResources), or None when
    the service could not be asked - then nothing is removed. A manifest younger than
    ``grace_s`` is kept (its container may not be admitted yet). Returns the removed names."""
    import time
    if held is None:
        return []
    now = time.time() if now is None else now
    d = os.path.join(vgpu_dir, MANIFEST_HOST_DIR)
    removed = []
    try:
        names = [fn[:-len(".devices")] for fn in os.listdir(d) if fn.endswith(".devices")]
    except OSError:
        names = []
    for name in names:
        path = os.path.join(d, name + ".devices")
        try:
            if now - os.path.getmtime(path) < grace_s:
                continue
        except OSError:
            continue
        res, ids = _read_manifest(path)
        if res is None or not ids or ids in held.get(res, ()):
            continue
        for fp in container_files(vgpu_dir, name) + [path]:
            try:
                os.unlink(fp)
            except OSError:
                pass
        removed.append(name)
    return removed + _gc_legacy_container_files(vgpu_dir, now)


# Containers allocated by a plugin older than the manifests (round 4) have host files but no
# manifest, so PodResources cannot vouch for them either way. They are removed once their
# limits file is this old: far past any pod's restart of a node the plugin was upgraded on,
# and only when PodResources answered (the caller returns early otherwise).
LEGACY_GC_AGE_S = 30 * 24 * 3600


def _gc_legacy_container_files(vgpu_dir, now):
    d = os.path.join(vgpu_dir, LIMITS_HOST_DIR, "containers")
    try:
        names = [fn[:-len(".env")] for fn in os.listdir(d) if fn.endswith(".env")]
    except OSError:
        return []
    removed = []
    for name in names:
        if os.path.exists(os.path.join(vgpu_dir, MANIFEST_HOST_DIR, name + ".devices")):
            continue
        try:
            if now - os.path.getmtime(os.path.join(d, name + ".env")) < LEGACY_GC_AGE_S:
                continue
        except OSError:
            continue
        for fp in container_files(vgpu_dir, name):
            try:
                os.unlink(fp)
            except OSError:
                pass
        removed.append(name)
    return removed


def write_limits(vgpu_dir, name, values):
    """Writes <vgpu_dir>/limits/containers/<name>.env (root-owned, 0644) with ``values``;
    returns its path, or None when the host directory is not writable."""
    d = os.path.join(vgpu_dir, LIMITS_HOST_DIR, "containers")
    path = os.path.join(d, name + ".env")
    try:
        os.makedirs(d, exist_ok=True)
        tmp = path + ".tmp"
        with open(tmp, "w") as f:
            f.write("".join(f"{k}={v}\n" for k, v in values.items()))
        os.chmod(tmp, 0o644)
        os.replace(tmp, path)
    except OSError:
        return None
    return path


def create_region_file(host_dir, name):
    """Creates the empty region file <host_dir>/<name> (world-writable: the container's
    processes may run as any user) the shim initialises on first use. Returns (path, inode),
    or (None, 0) when the directory is not writable."""
    path = os.path.join(host_dir, name)
    try:
        os.makedirs(host_dir, exist_ok=True)
        fd = os.open(path, os.O_RDWR | os.O_CREAT | os.O_EXCL, 0o666)
        try:
            os.fchmod(fd, 0o666)
            ino = os.fstat(fd).st_ino
        finally:
            os.close(fd)
    except OSError:
        return None, 0
    return path, ino


def write_allowlist(vgpu_dir, name, uuids):
    """Writes <vgpu_dir>/allowlist/containers/<name>.list with ``uuids``; returns its path,
    or None if the host directory is not writable (removed with the container's other files,
    gc_container_files)."""
    d = os.path.join(vgpu_dir, ALLOWLIST_HOST_DIR, "containers")
    try:
        os.makedirs(d, exist_ok=True)
        path = os.path.join(d, name + ".list")
        with open(path, "w") as f:
            f.write("".join(u + "\n" for u in uuids))
    except OSError:
        return None
    return path


SHARED_GRACE_S = 300


def gc_shared_dirs(root, pods, grace_s=SHARED_GRACE_S, now=None, held=None):
    """Removes the monitor-mode host directories (<ns>_<pod>_<ctr>/<uuid>.cache) of pods
    that no longer exist on this node; the reference never removes them.

    Liveness comes from the pod list (``pods``: ``k8s.pod_summary`` dicts of this node),
    never from a directory's age or its region's process count: an idle notebook pod or a
    batch pod between runs keeps its directory however long it sleeps (its container's bind
    mount points there, and a missing directory would leave the next process of the
    container without its region). A directory is kept when a pod that is not Succeeded /
    Failed owns its tag - same namespace, name and container, and the UID in the
    ``.pod-uid`` marker when there is one (a re-created pod of the same name gets a fresh
    directory, so the old one goes). ``pods=None`` (no pod list) removes nothing; a
    directory younger than ``grace_s`` is never removed, nor one whose recorded device IDs
    (``.devices``) a live container holds according to the kubelet's PodResources
    (``held``: a set of frozensets of device IDs). Returns the removed tags."""
    import shutil
    import time
    from .k8s import POD_MARKER, TERMINAL_PHASES, pod_tag
    if pods is None:
        return []
    now = time.time() if now is None else now
    live = {}
    for p in pods:
        if p.get("phase") in TERMINAL_PHASES:
            continue
        for c in p.get("containers", []):
            live.setdefault(pod_tag(p, c["name"]), set()).add(p.get("uid", ""))
    removed = []
    try:
        tags = os.listdir(root)
    except OSError:
        return removed
    for tag in tags:
        d = os.path.join(root, tag)
        try:
            if not os.path.isdir(d) or now - os.path.getmtime(d) < grace_s:
                continue
            if held:
                from .podresources import read_devices
                ids = read_devices(d)
                if ids and ids in held:
                    continue
            uids = live.get(tag)
            if uids:
                try:
                    with open(os.path.join(d, POD_MARKER)) as f:
                        marker = f.read().strip()
                except OSError:
                    marker = ""
                if not marker or marker in uids:
                    continue
            shutil.rmtree(d, ignore_errors=True)
            removed.append(tag)
        except OSError:
            continue
    return removed


def duplicate_gpus(vdevs):
    """UUIDs of the physical GPUs that back more than one of ``vdevs`` (reference
    duplicate_devices, [nvml/util.c] "device index %d and %d are the same physical device")."""
    seen, dups = set(), []
    for v in vdevs:
        if v.uuid in seen and v.uuid not in dups:
            dups.append(v.uuid)
        seen.add(v.uuid)
    return dups


def device_ids(cfg, devices_by_uuid, uuids):
    if cfg.device_id_strategy == ID_INDEX:
        return [str(devices_by_uuid[u].index) for u in uuids if u in devices_by_uuid]
    return list(uuids)


def device_specs(cfg, devices):
    """/dev/kfd once, then render + card node of every device (permissions rw)."""
    specs, seen = [], set()
    for d in devices:
        for p in d.device_paths:
            if p in seen:
                continue
            seen.add(p)
            specs.append(api.DeviceSpec(container_path=p, host_path=os.path.join(cfg.driver_root, p.lstrip("/")),
                                        permissions="rw"))
    return specs


def visible_envs(cfg, ids):
    if cfg.device_list_strategy == LIST_ENVVAR:
        return {VISIBLE_ENV: ",".join(ids)}
    if cfg.device_list_strategy == LIST_AMD_RUNTIME:
        return {AMD_RUNTIME_ENV: ",".join(ids)}
    return {AMD_RUNTIME_ENV: VOLUME_MOUNTS_ROOT}


def build_container_response(cfg, vdevs, devices_by_uuid, request_ids=None, using_ids=None, pod_tag=None,
                             pod_uid=None, kubelet_ids=None, latency=False, resource=None):
    """ContainerAllocateResponse for one container holding vGPUs ``vdevs``. ``kubelet_ids``:
    the device IDs of the kubelet's request (monitor mode records them in the container's
    host directory, where the PodResources attribution finds them). ``latency``: the vGPUs
    come from the latency resource (--latency-vgpus-per-gpu), which grants the latency
    class and makes it the container's default."""
    resp = api.ContainerAllocateResponse()
    uuids = []
    for v in vdevs:
        if v.uuid not in uuids:
            uuids.append(v.uuid)
    ids = device_ids(cfg, devices_by_uuid, uuids)
    split = getattr(cfg, "duplicate_vgpus", "split") == "split" and len(uuids) < len(vdevs)
    # --duplicate-vgpus=split: one entry per vGPU, so frameworks that count devices from the
    # visible list (torch.cuda.device_count) see every vGPU; ROCr lists a GPU named twice once
    # (profiles/r4dup) and the shim presents the second one.
    vis_ids = device_ids(cfg, devices_by_uuid, [v.uuid for v in vdevs]) if split else ids
    resp.envs.update(visible_envs(cfg, vis_ids))
    if cfg.device_list_strategy == LIST_VOLUME_MOUNTS:
        for i in ids:
            resp.mounts.add(container_path=os.path.join(VOLUME_MOUNTS_ROOT, i), host_path=VOLUME_MOUNTS_HOST)
    if cfg.pass_device_specs:
        resp.devices.extend(device_specs(cfg, [devices_by_uuid[u] for u in uuids if u in devices_by_uuid]))
    if request_ids is not None:
        resp.annotations[ANN_REQUEST] = ",".join(request_ids)
        resp.annotations[ANN_USING] = ",".join(using_ids or request_ids)

    # Per-vGPU limits, indexed like the container's device ordinals (VGPU_DEVICE_MAP order).
    dmap = []
    for i, v in enumerate(vdevs):
        if v.memory:
            resp.envs[f"VGPU_DEVICE_MEMORY_LIMIT_{i}"] = format_mib(v.memory)
        if v.hbm_limit and v.hbm_limit < v.memory:
            resp.envs[f"VGPU_DEVICE_HBM_LIMIT_{i}"] = format_mib(v.hbm_limit)
        if v.cu_pct:
            resp.envs[f"VGPU_DEVICE_CU_LIMIT_{i}"] = str(v.cu_pct)
            # With the node ledger the limiter's charges are exact (one snapshot, adding up
            # to at most the GPU's busy time), so its grants take the exact share instead of
            # the rounded-up percent (profiles/r3v, r3w).
            if getattr(cfg, "ledger", False) and v.cu_share and v.cu_share != v.cu_pct:
                resp.envs[f"VGPU_DEVICE_CU_SHARE_{i}"] = f"{v.cu_share:g}"
            if v.cu_range:
                resp.envs[f"VGPU_DEVICE_CU_RANGE_{i}"] = f"{v.cu_range[0]}-{v.cu_range[1]}"
        dmap.append(f"{i}:{v.uuid}")
    resp.envs["VGPU_DEVICE_MAP"] = " ".join(dmap)
    nodes = [v.cpu_node for v in vdevs if getattr(v, "cpu_node", -1) >= 0]
    if nodes:
        # --numa-spread: the shim keeps the container's processes on this node's CPUs (the
        # first vGPU's, for a container holding several)
        resp.envs["VGPU_CPU_NODE"] = str(nodes[0])
    dups = duplicate_gpus(vdevs)
    if dups and getattr(cfg, "duplicate_vgpus", "split") == "split":
        # --duplicate-vgpus=split: one HIP device per vGPU, each with its own quota; the shim
        # virtualises the device ordinals (native/src/shim/vdev_hooks.cpp). Compute stays per
        # physical GPU, with the vGPUs' shares summed (docs/ABI.md "Duplicate vGPUs").
        resp.envs["VGPU_DUPLICATE_SPLIT"] = "1"
        resp.annotations[ANN_SPLIT] = ",".join(dups)
    elif dups:
        # --duplicate-vgpus=merge: the shim merges the vGPUs of one GPU into that device
        # (quotas and CU shares add up); the container is told, since it sees fewer
        # devices than it requested (docs/ABI.md "Duplicate vGPUs").
        resp.envs["VGPU_DUPLICATE_MERGED"] = ",".join(dups)
        resp.annotations[ANN_DUPLICATES] = ",".join(dups)
    host_per = getattr(cfg, "host_budget_bytes", -1)
    if host_per is None or host_per < 0:
        host_per = cfg.host_memory_per_vgpu_bytes if hasattr(cfg, "host_memory_per_vgpu_bytes") else 0
    if host_per:
        # Pinned host memory of the container (hipHostMalloc / hipHostRegister): one
        # budget per vGPU, summed (reference: class (b) host-alloc OOM checks).
        resp.envs["VGPU_HOST_MEMORY_LIMIT"] = format_mib(host_per * len(vdevs))
    # PCI addresses of the container's GPUs: in-container amd-smi lists only these
    # (reference: nvmlDeviceGetCount / GetHandleByIndex remapping, nvml/hook.c:438-527).
    # (split duplicates: one entry per vGPU, so amd-smi lists every vGPU)
    listed = [v.uuid for v in vdevs] if split else uuids
    bdfs = [devices_by_uuid[u].bdf for u in listed if u in devices_by_uuid and devices_by_uuid[u].bdf]
    if bdfs:
        resp.envs["VGPU_DEVICE_BDFS"] = ",".join(bdfs)
        # KFD gpu_ids of the same devices: compute partitions exposed as GPUs share a PCI
        # address, and amd-smi inside the container must list only this container's.
        gids = [str(devices_by_uuid[u].gpu_id or 0) for u in listed if u in devices_by_uuid and devices_by_uuid[u].bdf]
        if any(g != "0" for g in gids):
            resp.envs["VGPU_DEVICE_GPU_IDS"] = ",".join(gids)
    # Always explicit, so a container never depends on the shim's built-in default.
    resp.envs["VGPU_CU_MODE"] = cfg.cu_mode

    cache_name = f"{_uuid.uuid4()}.cache"
    region_inode = 0
    if cfg.monitor_mode and pod_tag:
        from .k8s import POD_MARKER
        host_dir = os.path.join(cfg.vgpu_dir, SHARED_HOST_DIR, pod_tag)
        os.makedirs(host_dir, exist_ok=True)
        if pod_uid:
            with open(os.path.join(host_dir, POD_MARKER), "w") as f:
                f.write(pod_uid + "\n")
        if kubelet_ids:
            from .podresources import write_devices
            write_devices(host_dir, kubelet_ids)
        resp.mounts.add(container_path=f"/{pod_tag}", host_path=host_dir, read_only=False)
        resp.envs["VGPU_SHARED_CACHE"] = f"/{pod_tag}/{cache_name}"
        region, region_inode = create_region_file(host_dir, cache_name)
        if region:
            # The region itself is mounted over its path: the directory stays writable for
            # the monitor's view, the file cannot be unlinked from inside the container.
            resp.mounts.add(container_path=f"/{pod_tag}/{cache_name}", host_path=region, read_only=False)
    else:
        regions = os.path.join(cfg.vgpu_dir, REGIONS_HOST_DIR)
        region, region_inode = create_region_file(regions, cache_name)
        if region:
            resp.mounts.add(container_path=f"{CONTAINER_REGION_DIR}/{cache_name}", host_path=region,
                            read_only=False)
            resp.envs["VGPU_SHARED_CACHE"] = f"{CONTAINER_REGION_DIR}/{cache_name}"
        else:
            resp.envs["VGPU_SHARED_CACHE"] = os.path.join(cfg.shared_cache_dir, cache_name)
    if cfg.device_memory_scaling > 1:
        resp.envs["VGPU_OVERSUBSCRIBE"] = "true"
    # Device authorisation (reference: vgpuvalidator against the licensed device pool):
    # every container gets its own allow-list holding exactly the GPUs it was allocated,
    # so a process that widens ROCR_VISIBLE_DEVICES inside the container gets no memory
    # on any other GPU. Falls back to the node-wide list when the host dir is read-only.
    resp.envs["VGPU_ALLOWLIST"] = CONTAINER_ALLOWLIST_DIR + "/allowlist"
    vdir = cfg.vgpu_dir
    if kubelet_ids and resource:
        write_manifest(vdir, cache_name.rsplit(".", 1)[0], resource, kubelet_ids)
    own_list = write_allowlist(vdir, cache_name.rsplit(".", 1)[0], uuids)

    resp.mounts.add(container_path=CONTAINER_SHIM, host_path=os.path.join(vdir, "libvgpu_hip.so"), read_only=True)
    resp.mounts.add(container_path=CONTAINER_PRELOAD, host_path=os.path.join(vdir, "ld.so.preload"), read_only=True)
    if cfg.pcibus_file and os.path.exists(cfg.pcibus_file):
        resp.mounts.add(container_path=CONTAINER_PCIINFO, host_path=cfg.pcibus_file, read_only=True)
    resp.mounts.add(container_path=CONTAINER_VALIDATOR, host_path=os.path.join(vdir, "vgpu-validate"),
                    read_only=True)
    if own_list:
        resp.mounts.add(container_path=CONTAINER_ALLOWLIST_DIR + "/allowlist", host_path=own_list, read_only=True)
    else:
        resp.mounts.add(container_path=CONTAINER_ALLOWLIST_DIR, host_path=os.path.join(vdir, "allowlist"),
                        read_only=True)
    slot = board_slot(vdir, cache_name.rsplit(".", 1)[0])
    if slot:
        resp.mounts.add(container_path=CONTAINER_BOARD_DIR, host_path=os.path.dirname(slot), read_only=True)
        resp.mounts.add(container_path=f"{CONTAINER_BOARD_DIR}/{os.path.basename(slot)}", host_path=slot,
                        read_only=False)
        resp.envs["VGPU_BOARD_DIR"] = CONTAINER_BOARD_DIR
        resp.envs["VGPU_BOARD_SLOT"] = os.path.basename(slot)
        if getattr(cfg, "gpu_concurrency", 0):
            resp.envs["VGPU_GPU_CONCURRENCY"] = "auto" if cfg.gpu_concurrency < 0 else str(cfg.gpu_concurrency)
    lock_file = os.path.join(vdir, LOCK_HOST_DIR, LOCK_FILE)
    if os.path.isfile(lock_file):
        resp.mounts.add(container_path=f"{CONTAINER_LOCK_DIR}/{LOCK_FILE}", host_path=lock_file, read_only=True)
        resp.envs["VGPU_LOCK_FILE"] = f"{CONTAINER_LOCK_DIR}/{LOCK_FILE}"
    # The ceiling: the contract's limits as written above, the region file's inode and the
    # lowest priority class the container may take (the latency class only when granted).
    envs = dict(resp.envs)
    limits = {k: v for k, v in envs.items() if k.startswith(LIMIT_KEYS)}
    if region_inode:
        limits["VGPU_REGION_INODE"] = str(region_inode)
    # The memory backstop (KFD-measured VRAM over the quota) is the plugin's to switch.
    limits["VGPU_ACTIVE_OOM_KILLER"] = "1" if getattr(cfg, "active_oom_killer", True) else "0"
    limits["VGPU_TASK_PRIORITY_MIN"] = "0" if latency or getattr(cfg, "allow_latency_class", False) else "1"
    limits_file = write_limits(vdir, cache_name.rsplit(".", 1)[0], limits)
    if limits_file:
        resp.mounts.add(container_path=CONTAINER_LIMITS, host_path=limits_file, read_only=True)
        resp.envs["VGPU_LIMITS_FILE"] = CONTAINER_LIMITS
    if latency:
        resp.envs.setdefault("VGPU_TASK_PRIORITY", "0")
    return resp


def build_partition_response(cfg, devices):
    """Whole-device response for partition resources (reference MIGAllocate :329-358):
    visible devices + device specs, no quota, no shim contract."""
    resp = api.ContainerAllocateResponse()
    by_uuid = {d.uuid: d for d in devices}
    ids = device_ids(cfg, by_uuid, [d.uuid for d in devices])
    resp.envs.update(visible_envs(cfg, ids))
    if cfg.device_list_strategy == LIST_VOLUME_MOUNTS:
        for i in ids:
            resp.mounts.add(container_path=os.path.join(VOLUME_MOUNTS_ROOT, i), host_path=VOLUME_MOUNTS_HOST)
    if cfg.pass_device_specs:
        resp.devices.extend(device_specs(cfg, devices))
    return resp


def response_to_env(resp):
    """(envs dict, [(container_path, host_path)]) — the view the launcher applies."""
    return dict(resp.envs), [(m.container_path, m.host_path) for m in resp.mounts]
