"""ROCr entry points looked up on a library handle are routed into the shim.

Reference: libvgpu.so overrides dlsym and routes every hooked driver name back into its
hooks (dlsym@0x12bb6 [libvgpu.c:109-124], __dlsym_hook_section@0x12f0e), so a runtime that
dlopens the driver cannot step around the quota. On MI355X the primary interception layer
is ROCr (hsa_*): without routing, ``ctypes.CDLL("libhsa-runtime64.so.1")`` - or any
``dlsym(handle, "hsa_...")`` - reaches ROCr directly, with no quota, no CU mask and, for
``hsa_init``, no shim at all (missing 1).

These run a Python tenant that touches ROCr only through ctypes (the CPU-only fake ROCr,
native/tests/fake/fake_hsa.cpp), under the preloaded shim, and check that hsa_init
initialises the shim, pool and legacy region allocations past the quota are refused, a
queue gets the vGPU's CU mask, dlvsym is routed the same way, and the lookup functions
themselves cannot be fetched from the C library unrouted. A negative control turns the
routing off (VGPU_HOOK_DLSYM=0) and shows the escape.
"""
import json
import os
import subprocess
import sys

import pytest

from amdvgpu.shim.native import LIB_DIR, shim_path

FAKE_HSA = os.path.join(LIB_DIR, "fakerocm", "libhsa-runtime64.so.1")

TENANT = r"""
import ctypes, json, os, sys
from ctypes import CFUNCTYPE, POINTER, Structure, byref, c_char_p, c_int, c_uint32, c_uint64, c_void_p, c_size_t
sys.path.insert(0, os.environ["REPO"])

class DlInfo(Structure):
    _fields_ = [("dli_fname", c_char_p), ("dli_fbase", c_void_p), ("dli_sname", c_char_p), ("dli_saddr", c_void_p)]

libc = ctypes.CDLL(None)
libc.dladdr.argtypes = [c_void_p, POINTER(DlInfo)]
libc.dlvsym.restype = c_void_p
libc.dlvsym.argtypes = [c_void_p, c_char_p, c_char_p]

def owner(addr):
    info = DlInfo()
    if not addr or not libc.dladdr(c_void_p(addr), byref(info)) or not info.dli_fname:
        return "?"
    return os.path.basename(info.dli_fname.decode())

def addr(fn):
    return ctypes.cast(fn, c_void_p).value

hsa = ctypes.CDLL(os.environ["HSA_LIB"])          # RTLD_LOCAL, like a ctypes tenant
res = {"hsa_init_owner": owner(addr(hsa.hsa_init)),
       "pool_alloc_owner": owner(addr(hsa.hsa_amd_memory_pool_allocate)),
       "dlvsym_owner": owner(libc.dlvsym(c_void_p(hsa._handle), b"hsa_amd_memory_pool_allocate", b"ROCR_1")),
       "libc_dlsym_owner": owner(addr(ctypes.CDLL("libc.so.6").dlsym)),
       "libc_dlvsym_owner": owner(addr(ctypes.CDLL("libc.so.6").dlvsym))}
res["init"] = hsa.hsa_init()

AGENT_CB = CFUNCTYPE(c_int, c_uint64, c_void_p)
POOL_CB = CFUNCTYPE(c_int, c_uint64, c_void_p)
gpus, pools = [], []
def on_agent(a, _):
    t = c_uint32(0)
    hsa.hsa_agent_get_info(c_uint64(a), 17, byref(t))      # HSA_AGENT_INFO_DEVICE
    if t.value == 1:                                        # HSA_DEVICE_TYPE_GPU
        gpus.append(a)
    return 0
def on_pool(p, _):
    seg, flags, alloc_ok = c_uint32(0), c_uint32(0), ctypes.c_bool(False)
    hsa.hsa_amd_memory_pool_get_info(c_uint64(p), 0, byref(seg))        # SEGMENT
    hsa.hsa_amd_memory_pool_get_info(c_uint64(p), 1, byref(flags))      # GLOBAL_FLAGS
    hsa.hsa_amd_memory_pool_get_info(c_uint64(p), 5, byref(alloc_ok))   # RUNTIME_ALLOC_ALLOWED
    if seg.value == 0 and (flags.value & 4) and alloc_ok.value:       # global, coarse grained
        pools.append(p)
    return 0
regions = []
def on_region(g, _):
    seg, flags, alloc_ok = c_uint32(0), c_uint32(0), ctypes.c_bool(False)
    hsa.hsa_region_get_info(c_uint64(g), 0, byref(seg))        # HSA_REGION_INFO_SEGMENT
    hsa.hsa_region_get_info(c_uint64(g), 1, byref(flags))      # HSA_REGION_INFO_GLOBAL_FLAGS
    hsa.hsa_region_get_info(c_uint64(g), 5, byref(alloc_ok))   # HSA_REGION_INFO_RUNTIME_ALLOC_ALLOWED
    if seg.value == 0 and (flags.value & 4) and alloc_ok.value:
        regions.append(g)
    return 0
agent_cb, pool_cb, region_cb = AGENT_CB(on_agent), POOL_CB(on_pool), POOL_CB(on_region)
hsa.hsa_iterate_agents(agent_cb, None)
hsa.hsa_amd_agent_iterate_memory_pools(c_uint64(gpus[0]), pool_cb, None)
hsa.hsa_agent_iterate_regions(c_uint64(gpus[0]), region_cb, None)
pool = c_uint64(pools[0])
# the GPU's own memory: a GPU agent's region list also names the system regions it can reach
# (ROCr); in ROCr a region and the pool of the same memory share one handle
region = c_uint64([g for g in regions if g in pools][0])
MiB = 1 << 20
quota = int(os.environ["QUOTA_MIB"]) * MiB
allocs = []
def pool_alloc(n):
    p = c_void_p()
    st = hsa.hsa_amd_memory_pool_allocate(pool, c_size_t(n), c_uint32(0), byref(p))
    if st == 0:
        allocs.append(p.value)
    return st
def region_alloc(n):
    p = c_void_p()
    st = hsa.hsa_memory_allocate(region, c_size_t(n), byref(p))
    if st == 0:
        allocs.append(p.value)
    return st
res["pool_first"] = pool_alloc(quota * 3 // 4)
res["pool_over"] = pool_alloc(quota // 2)
res["region_over"] = region_alloc(quota // 2)
res["region_fits"] = region_alloc(quota // 8)
q = c_void_p()
res["queue"] = hsa.hsa_queue_create(c_uint64(gpus[0]), c_uint32(64), c_uint32(0), None, None, c_uint32(0),
                                    c_uint32(0), byref(q))
if os.environ.get("FAKE_INTROSPECT"):
    words = (c_uint32 * 8)()
    prio, dev = c_int(0), c_int(0)
    hsa.fake_rocr_queue_state(q, words, byref(prio), byref(dev))
    res["queue_cus"] = sum(bin(w).count("1") for w in words)
if os.path.exists(os.environ.get("VGPU_SHARED_CACHE", "")):
    from amdvgpu.shim.region import Region
    with Region(os.environ["VGPU_SHARED_CACHE"]) as r:
        res["region_procs"] = len(r.procs())
        res["charged"] = r.device(0)["used"]
for a in allocs:
    hsa.hsa_amd_memory_pool_free(c_void_p(a))
print("RESULT " + json.dumps(res), flush=True)
"""

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HSA_OUT_OF_RESOURCES = 0x1008


def run_tenant(env, timeout=120):
    p = subprocess.run([sys.executable, "-c", TENANT], env=env, capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stderr[-3000:]
    return json.loads([l for l in p.stdout.splitlines() if l.startswith("RESULT ")][0][7:])


@pytest.fixture
def fake_env(tmp_path):
    kfd = tmp_path / "kfd"
    kfd.mkdir()
    e = {k: v for k, v in os.environ.items() if not k.startswith(("VGPU_", "FAKE_"))}
    e.update(FAKE_ROCR_GPUS="1", FAKE_ROCR_HBM=str(8 << 30), FAKE_KFD_ROOT=str(kfd), VGPU_KFD_ROOT=str(kfd),
             VGPU_SHARED_CACHE=str(tmp_path / "region.cache"), VGPU_LOCK_FILE=str(tmp_path / "lock" / "l"),
             VGPU_DEVICE_MEMORY_LIMIT="1024m", VGPU_DEVICE_CU_LIMIT="25", VGPU_CU_MODE="spatial",
             LD_PRELOAD=shim_path(), HSA_LIB=FAKE_HSA, QUOTA_MIB="1024", FAKE_INTROSPECT="1", REPO=REPO)
    return e


def test_ctypes_tenant_is_held_to_the_quota_and_cu_mask(fake_env):
    r = run_tenant(fake_env)
    shim = os.path.basename(shim_path())
    # every lookup of a hooked name on the ROCr handle got the shim's definition
    assert r["hsa_init_owner"] == shim and r["pool_alloc_owner"] == shim and r["dlvsym_owner"] == shim, r
    # ... and so did the lookup functions fetched from the C library itself
    assert r["libc_dlsym_owner"] == shim and r["libc_dlvsym_owner"] == shim, r
    assert r["init"] == 0 and r["region_procs"] == 1, r        # hsa_init via ctypes started the shim
    assert r["pool_first"] == 0 and r["pool_over"] == HSA_OUT_OF_RESOURCES, r
    assert r["region_over"] == HSA_OUT_OF_RESOURCES and r["region_fits"] == 0, r   # legacy region API too
    assert r["charged"] == (1024 * 3 // 4 + 1024 // 8) << 20, r
    assert r["queue"] == 0 and r["queue_cus"] == 64, r         # 25 % of 256 CUs


def test_routing_off_is_an_escape(fake_env):
    """Negative control: with VGPU_HOOK_DLSYM=0 the ctypes tenant gets ROCr's own entry
    points - the shim never starts, nothing is charged, the queue keeps every CU."""
    fake_env["VGPU_HOOK_DLSYM"] = "0"
    r = run_tenant(fake_env)
    assert r["hsa_init_owner"] == "libhsa-runtime64.so.1", r
    assert r["pool_first"] == 0 and r["pool_over"] == 0 and r["region_over"] == 0, r
    assert r["queue_cus"] == 256 and "region_procs" not in r, r


def test_shim_routes_every_rocr_export():
    """The routing table (hsa_hooks.cpp kHsaHooked) names exactly the shim's ROCR_1 exports."""
    out = subprocess.run(["nm", "-D", "--defined-only", shim_path()], capture_output=True, text=True,
                         check=True).stdout
    exported = sorted(l.split()[2].split("@")[0] for l in out.splitlines() if l.endswith("@@ROCR_1"))
    src = open(os.path.join(REPO, "native", "src", "shim", "hsa_hooks.cpp")).read()
    table = src[src.index("kHsaHooked[] = {"):]
    table = table[:table.index("};")]
    import re
    assert sorted(re.findall(r'"(hsa_\w+)"', table)) == exported


@pytest.mark.gpu
def test_ctypes_rocr_tenant_is_held_to_the_quota_on_mi355x(tmp_path):
    """The same ctypes-only tenant on the real ROCr of an MI355X: hsa_init through ctypes
    starts the shim, and an hsa_amd_memory_pool_allocate (and a legacy hsa_memory_allocate)
    past the 8 GiB quota gets HSA_STATUS_ERROR_OUT_OF_RESOURCES."""
    lib = "/opt/rocm/lib/libhsa-runtime64.so.1"
    if not os.path.exists(lib):
        pytest.skip("no ROCm runtime")
    e = {k: v for k, v in os.environ.items() if not k.startswith("VGPU_")}
    e.update(VGPU_SHARED_CACHE=str(tmp_path / "region.cache"), VGPU_DEVICE_MEMORY_LIMIT="8192m",
             LD_PRELOAD=shim_path(), HSA_LIB=lib, QUOTA_MIB="8192", REPO=REPO)
    r = run_tenant(e, timeout=300)
    print(json.dumps(r))
    shim = os.path.basename(shim_path())
    assert r["hsa_init_owner"] == shim and r["pool_alloc_owner"] == shim and r["dlvsym_owner"] == shim, r
    assert r["init"] == 0 and r["region_procs"] == 1, r
    assert r["pool_first"] == 0 and r["pool_over"] == HSA_OUT_OF_RESOURCES, r
    assert r["region_over"] == HSA_OUT_OF_RESOURCES and r["region_fits"] == 0, r
    assert r["queue"] == 0, r
