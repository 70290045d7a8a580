"""Gate coverage on a real MI355X: entry points outside the classic launch / memcpy set,
reached the way applications reach them.

* hipMemcpy2D called through ctypes (dlsym on the runtime's handle: the shim's routing)
  stalls while the container is suspended (reference: every copy hook runs
  wait_status_self, [memory.c]);
* pinned host memory (hipHostMalloc through ctypes, and PyTorch's pin_memory) is held to
  VGPU_HOST_MEMORY_LIMIT and shows up in the region (reference: class (b) OOM checks of
  cuMemAllocHost_v2 / cuMemHostAlloc / cuMemHostRegister_v2).
"""
import time

import pytest

from amdvgpu.shim.launcher import vgpu_env
from amdvgpu.shim.region import Region
from conftest import child_results, run_child, spawn_child

pytestmark = pytest.mark.gpu
GiB = 1 << 30
MiB = 1 << 20

HIP = """
import ctypes, torch
torch.cuda.init()
hip = ctypes.CDLL("libamdhip64.so")          # the runtime torch loaded (dlsym on its handle)
"""


def test_suspended_memcpy2d_stalls(tmp_region):
    c = vgpu_env(mem_limit=8 * GiB, shared_cache=tmp_region)
    p = spawn_child(HIP + """
src = torch.ones(1024, 1024, device="cuda"); dst = torch.zeros_like(src)
pitch = 1024 * 4
def copy2d():
    rc = hip.hipMemcpy2D(ctypes.c_void_p(dst.data_ptr()), ctypes.c_size_t(pitch), ctypes.c_void_p(src.data_ptr()),
                         ctypes.c_size_t(pitch), ctypes.c_size_t(pitch), ctypes.c_size_t(1024), 3)
    assert rc == 0, rc
copy2d(); torch.cuda.synchronize()
emit(ready=True)
gaps = []; t = time.time()
for _ in range(200):
    copy2d()
    now = time.time(); gaps.append(now - t); t = now
    time.sleep(0.01)
torch.cuda.synchronize()
emit(max_gap=max(gaps), ok=bool(dst.eq(1).all()))
""", c)
    try:
        assert p.stdout.readline().startswith("RESULT"), p.stderr.read()[-3000:]
        with Region(tmp_region) as r:
            time.sleep(0.3)
            r.suspend_all()
            time.sleep(2.0)
            r.resume_all()
        out, err = p.communicate(timeout=120)
    finally:
        if p.poll() is None:
            p.kill()
    assert p.returncode == 0, err[-3000:]
    res = child_results(out)[0]
    assert res["ok"] and res["max_gap"] >= 1.5, res


def test_pinned_host_memory_limit(tmp_region):
    c = vgpu_env(mem_limit=8 * GiB, shared_cache=tmp_region, extra={"VGPU_HOST_MEMORY_LIMIT": "1g"})
    p = spawn_child(HIP + """
def host_malloc(n):
    ptr = ctypes.c_void_p()
    rc = hip.hipHostMalloc(ctypes.byref(ptr), ctypes.c_size_t(n), 0)
    return rc, ptr
rc1, a = host_malloc(600 << 20)
rc2, b = host_malloc(600 << 20)            # 1200 MiB > 1 GiB: refused
try:
    t = torch.empty(512 << 20, dtype=torch.uint8, pin_memory=True)   # caching allocator: 512 MiB block
    pinned = True
except RuntimeError:
    pinned = False
emit(rc1=rc1, rc2=rc2, torch_pinned=pinned)
time.sleep(2)
hip.hipHostFree(a)
rc3, c = host_malloc(300 << 20)
emit(rc3=rc3)
""", c)
    try:
        first = p.stdout.readline()
        assert first.startswith("RESULT"), p.stderr.read()[-3000:]
        with Region(tmp_region) as r:
            host = r.host()
            per_proc = [q["host_used"] for q in r.procs()]
        out, err = p.communicate(timeout=120)
    finally:
        if p.poll() is None:
            p.kill()
    assert p.returncode == 0, err[-3000:]
    res = child_results(first + out)
    assert res[0]["rc1"] == 0 and res[0]["rc2"] == 2  # hipErrorOutOfMemory
    assert res[0]["torch_pinned"] is False             # 600 + 512 MiB > 1 GiB
    assert res[1]["rc3"] == 0                          # the free returned the budget
    # charged where ROCr pins memory: the 600 MiB, plus whatever the runtime pinned for its
    # own staging buffers (pinned RAM all the same)
    assert host["limit"] == GiB and 600 * MiB <= host["used"] < 728 * MiB, host
    assert len(per_proc) == 1 and per_proc[0] == host["used"], (per_proc, host)


def test_unlimited_pinned_memory_is_tracked(tmp_region):
    c = vgpu_env(mem_limit=8 * GiB, shared_cache=tmp_region)
    res, _ = run_child("""
import torch
t = torch.empty(64 << 20, dtype=torch.uint8, pin_memory=True)
from amdvgpu.shim.region import Region
with Region(os.environ["VGPU_SHARED_CACHE"]) as r:
    emit(host=r.host())
""", c)
    assert res[0]["host"]["limit"] == 0 and res[0]["host"]["used"] >= 64 * MiB
