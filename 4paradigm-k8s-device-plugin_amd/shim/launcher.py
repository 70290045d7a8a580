"""Container-runtime emulator: runs a process under a vGPU Allocate contract.

In a cluster the kubelet hands the plugin's ``ContainerAllocateResponse`` (envs, mounts,
device specs) to the container runtime, which creates the container with those envs,
bind-mounts the shim over ``/usr/local/vgpu/libvgpu_hip.so`` and mounts an
``ld.so.preload`` that forces it into every process (reference ``server.go:486-522``).
Without a container runtime (CI, the gpurun box) this module applies the same contract
to a child process: envs are merged, the ``/etc/ld.so.preload`` mount becomes an
``LD_PRELOAD`` entry (appended to any preload already present, never replacing it), and
mounted host paths are substituted for container paths that appear in env values.

Also provides :func:`vgpu_env` to build a contract by hand for tests/benchmarks.
"""
import os
import subprocess
import sys
import tempfile
import uuid as _uuid

from ..utils.sizes import format_mib
from .native import shim_path

CONTAINER_SHIM = "/usr/local/vgpu/libvgpu_hip.so"
PRELOAD_FILE = "/etc/ld.so.preload"


def vgpu_env(mem_limit=None, cu_limit=None, cu_range=None, shared_cache=None, oversubscribe=False,
             device_map=None, cu_mode=None, per_device_mem=None, log_level=None, extra=None):
    """Builds the env half of a vGPU contract (the names the shim reads, §2.5 of SURVEY.md).

    mem_limit      bytes for every device (VGPU_DEVICE_MEMORY_LIMIT)
    per_device_mem list of bytes, one per visible device (VGPU_DEVICE_MEMORY_LIMIT_<i>)
    cu_limit       percent of CUs (VGPU_DEVICE_CU_LIMIT)
    cu_range       (begin, end) logical CU range for device 0 (VGPU_DEVICE_CU_RANGE_0)
    """
    env = {}
    if mem_limit is not None:
        env["VGPU_DEVICE_MEMORY_LIMIT"] = format_mib(mem_limit)
    for i, b in enumerate(per_device_mem or ()):
        env[f"VGPU_DEVICE_MEMORY_LIMIT_{i}"] = format_mib(b)
    if cu_limit is not None:
        env["VGPU_DEVICE_CU_LIMIT"] = str(int(cu_limit))
    if cu_range is not None:
        env["VGPU_DEVICE_CU_RANGE_0"] = f"{int(cu_range[0])}-{int(cu_range[1])}"
    if cu_mode:
        env["VGPU_CU_MODE"] = cu_mode
    if oversubscribe:
        env["VGPU_OVERSUBSCRIBE"] = "true"
    if device_map:
        env["VGPU_DEVICE_MAP"] = " ".join(f"{i}:{u}" for i, u in enumerate(device_map))
    if log_level is not None:
        env["VGPU_LOG_LEVEL"] = str(log_level)
    env["VGPU_SHARED_CACHE"] = shared_cache or os.path.join(tempfile.gettempdir(), f"vgpu-{_uuid.uuid4()}.cache")
    if extra:
        env.update(extra)
    return env


def _append_preload(env, lib):
    cur = env.get("LD_PRELOAD", "")
    parts = [p for p in cur.replace(" ", ":").split(":") if p]
    if lib not in parts:
        parts.append(lib)
    env["LD_PRELOAD"] = ":".join(parts)


def apply_contract(contract_envs, mounts=(), base_env=None, preload=True, shim=None):
    """Returns a process env for a container built from an Allocate response.

    ``mounts`` is a list of (container_path, host_path) pairs. ``shim`` overrides the
    library to preload (defaults to the in-tree libvgpu_hip.so).
    """
    env = dict(os.environ if base_env is None else base_env)
    remap = {c: h for c, h in mounts}
    for k, v in contract_envs.items():
        for c, h in remap.items():
            if c != "/" and (v == c or v.startswith(c.rstrip("/") + "/")):
                v = h + v[len(c):]
                break
        env[k] = v
    limits = env.get("VGPU_LIMITS_FILE")
    if limits and remap and os.path.isfile(limits):
        # The limits file names container paths (the region); inside a container the mounts
        # resolve them, here a copy with the host paths does.
        env["VGPU_LIMITS_FILE"] = _emulated_limits(limits, remap)
    if preload:
        lib = shim or remap.get(CONTAINER_SHIM)
        if not lib or not os.path.exists(lib):
            lib = shim_path()
        _append_preload(env, lib)
    return env


def _emulated_limits(path, remap):
    out = []
    for line in open(path).read().splitlines():
        k, sep, v = line.partition("=")
        for c, h in remap.items():
            if sep and c != "/" and (v == c or v.startswith(c.rstrip("/") + "/")):
                v = h + v[len(c):]
                break
        out.append(f"{k}{sep}{v}")
    dst = path + ".emulated"
    with open(dst, "w") as f:
        f.write("\n".join(out) + "\n")
    return dst


def run(cmd, contract_envs, mounts=(), base_env=None, preload=True, **kw):
    """Runs ``cmd`` as a 'container' under the contract; returns CompletedProcess."""
    env = apply_contract(contract_envs, mounts, base_env=base_env, preload=preload)
    return subprocess.run(cmd, env=env, **kw)


def popen(cmd, contract_envs, mounts=(), base_env=None, preload=True, **kw):
    env = apply_contract(contract_envs, mounts, base_env=base_env, preload=preload)
    return subprocess.Popen(cmd, env=env, **kw)


def python_cmd(*args):
    return [sys.executable, *args]


def cleanup_region(env):
    p = env.get("VGPU_SHARED_CACHE")
    if p and os.path.exists(p):
        try:
            os.unlink(p)
        except OSError:
            pass
