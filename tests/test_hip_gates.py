"""The HIP gate table (native/src/shim/hip_gates.def) against the runtime, and the gates
and lookup routing end to end on the CPU-only fake runtime.

Reference: the shim rate-limits every launch API and suspend-gates 41 copy / set / IPC /
pointer / advise hooks ([memory.c:598-611]), and routes runtime
lookups back into its hooks (dlsym [libvgpu.c:109-124], cuGetProcAddress
[cuda/hook.c:299-357]). Here the table is checked against ``nm -D libamdhip64.so`` so that
a new ROCm's launch or copy variant cannot slip through unnoticed, and every gated entry
point is called three ways - linked (global scope), ``dlsym`` on a libamdhip64 handle, and
``hipGetProcAddress`` fetched with ``dlsym`` (Triton's way, hence every torch.compile
tenant's) - while the container is suspended.
"""
import glob
import os
import re
import subprocess

import pytest

from amdvgpu.shim.native import LIB_DIR, shim_path

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEF = os.path.join(REPO, "native", "src", "shim", "hip_gates.def")
HARNESS = os.path.join(LIB_DIR, "fakerocm", "shim_harness")
TRAMPOLINE_KINDS = ("launch", "graph", "copy", "set", "suspend", "device")
ROCM_HIP = "/opt/rocm/lib/libamdhip64.so"

# Exported entry points that must be gated, by name pattern: every kernel launch and graph
# replay, every copy and set, and the reference's other suspend-gated families.
MUST_GATE = re.compile(
    r"^hip(.*Launch(Kernel|Cooperative|ByPtr|MultiKernel).*|GraphLaunch.*|Memcpy.*|DrvMemcpy.*|Memset.*"
    r"|MemAdvise.*|MemPrefetchAsync.*|Ipc(Get|Open|Close)MemHandle|PointerGetAttributes?|DrvPointerGetAttributes"
    r"|HostMalloc|HostAlloc|MallocHost|MemAllocHost|HostFree|FreeHost|HostRegister|HostUnregister|GetProcAddress)$")


def table():
    rows = []
    for line in open(DEF):
        line = line.split("#", 1)[0].split()
        if line:
            rows.append(tuple(line[:3]))   # (device rows carry argument positions too)
    return rows


def exports(lib):
    out = subprocess.run(["nm", "-D", "--defined-only", lib], capture_output=True, text=True, check=True).stdout
    syms = {}
    for line in out.splitlines():
        parts = line.split()
        if len(parts) == 3 and "@@" in parts[2]:
            name, ver = parts[2].split("@@")
            syms[name] = ver
    return syms


def runtimes():
    libs = [ROCM_HIP] if os.path.exists(ROCM_HIP) else []
    try:
        import torch
        libs += glob.glob(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so*"))[:1]
    except ImportError:
        pass
    return libs


@pytest.mark.parametrize("lib", runtimes())
def test_table_covers_every_launch_copy_and_set_export(lib):
    gated = {name for _k, name, _v in table()}
    missing = sorted(n for n in exports(lib) if MUST_GATE.match(n) and n not in gated)
    assert not missing, f"{lib} exports ungated entry points: {missing}"


def test_table_versions_match_the_runtime():
    if not os.path.exists(ROCM_HIP):
        pytest.skip("no ROCm HIP runtime")
    have = exports(ROCM_HIP)
    wrong = [(n, v, have.get(n)) for _k, n, v in table() if have.get(n) != v]
    assert not wrong, f"name, table version, runtime version: {wrong}"


def test_shim_exports_every_gate_with_its_version():
    have = exports(shim_path())
    wrong = [(n, v, have.get(n)) for _k, n, v in table() if have.get(n) != v]
    assert not wrong, wrong
    # the trampolines' common body and the dispatcher stay private
    assert not any(n.startswith("vgpu_gate") for n in have)


@pytest.fixture
def fake_env(tmp_path):
    kfd = tmp_path / "kfd"
    kfd.mkdir()
    e = {k: v for k, v in os.environ.items() if not k.startswith(("VGPU_", "FAKE_"))}
    e.update(FAKE_ROCR_GPUS="1", FAKE_KFD_ROOT=str(kfd), VGPU_KFD_ROOT=str(kfd),
             VGPU_SHARED_CACHE=str(tmp_path / "region.cache"), VGPU_LOCK_FILE=str(tmp_path / "lock" / "l"),
             VGPU_DEVICE_MEMORY_LIMIT="1g", LD_PRELOAD=shim_path())
    return e


def run_harness(env, *ops):
    import json
    p = subprocess.run([HARNESS, *ops], env=env, capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr[-3000:]
    return [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]


@pytest.mark.parametrize("mode", ["direct", "dlsym", "procaddr"])
def test_every_gate_is_routed_and_blocks_while_suspended(fake_env, mode):
    names = [n for k, n, _v in table() if k in TRAMPOLINE_KINDS]
    fake_env["FAKE_GATE_NAMES"] = ",".join(names)
    res = run_harness(fake_env, f"gates={mode}")[-1]
    assert res["n"] == len(names)
    assert res["unrouted"] == [] and res["ungated"] == [] and res["unreached"] == [], res


def test_routing_off_is_an_escape(fake_env):
    """Negative control: with the routing disabled (VGPU_HOOK_PROCADDR=0) the Triton path
    gets the runtime's own entry points, which the suspend gate never sees."""
    fake_env.update(VGPU_HOOK_PROCADDR="0", FAKE_GATE_NAMES="hipModuleLaunchKernel,hipDrvLaunchKernelEx,hipMemcpy")
    res = run_harness(fake_env, "gates=procaddr")[-1]
    assert set(res["unrouted"]) == {"hipModuleLaunchKernel", "hipDrvLaunchKernelEx", "hipMemcpy"}
    assert set(res["ungated"]) == set(res["unrouted"])


def test_pinned_host_memory_budget(fake_env):
    """VGPU_HOST_MEMORY_LIMIT bounds hipHostMalloc + hipHostRegister together (reference:
    class (b) OOM checks of cuMemAllocHost_v2 / cuMemHostAlloc / cuMemHostRegister_v2);
    frees and unregisters return the budget."""
    from amdvgpu.shim.region import Region
    fake_env["VGPU_HOST_MEMORY_LIMIT"] = "64m"
    out = run_harness(fake_env, "hostmalloc=40m", "hostregister=20m", "hostmalloc=8m", "hostfree",
                      "hostmalloc=8m", "hostunregister", "hostregister=24m", "sleep=0.1")
    got = [o.get("hostmalloc") or o.get("hostregister") for o in out if "hostmalloc" in o or "hostregister" in o]
    # 40 + 20 = 60 MiB; +8 over; after the free of the 40 MiB block +8 fits; after the
    # unregister of 20 MiB, 24 MiB fits (8 + 24 = 32)
    assert got == ["ok", "ok", "oom", "ok", "ok"], out
    with Region(fake_env["VGPU_SHARED_CACHE"]) as r:
        assert r.host() == {"limit": 64 << 20, "used": 0}  # the harness exited: its slot was released


def test_pinned_host_memory_freed_with_hipfree(fake_env):
    """hipFree releases hipHostMalloc'd memory too (CLR accepts it): the budget follows, so
    a tenant freeing pinned buffers that way is not refused later."""
    fake_env["VGPU_HOST_MEMORY_LIMIT"] = "64m"
    out = run_harness(fake_env, "hostmalloc=40m", "hostfree_hipfree", "hostmalloc=40m", "hostmalloc=40m")
    assert [o["hostmalloc"] for o in out if "hostmalloc" in o] == ["ok", "ok", "oom"], out


def test_pinned_host_memory_shared_by_the_container(fake_env):
    """Processes of one container share the host budget: the region holds the aggregate."""
    from amdvgpu.shim.region import Region
    fake_env["VGPU_HOST_MEMORY_LIMIT"] = "100m"
    import subprocess as sp
    first = sp.Popen([HARNESS, "hostmalloc=70m", "sleep=3"], env=fake_env, stdout=sp.PIPE, text=True)
    try:
        assert '"pid"' in first.stdout.readline() and '"ok"' in first.stdout.readline()
        out = run_harness(fake_env, "hostmalloc=40m", "hostmalloc=20m")
        assert [o["hostmalloc"] for o in out if "hostmalloc" in o] == ["oom", "ok"]
        with Region(fake_env["VGPU_SHARED_CACHE"]) as r:
            assert r.host()["used"] == 70 << 20
            assert sorted(p["host_used"] for p in r.procs()) == [70 << 20]
    finally:
        first.wait(timeout=30)
