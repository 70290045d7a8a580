"""Quota escapes through stock ROCm APIs, on a real MI355X (the round-4 verdict's missing
items 1-3): each is held to the container's limits by the preloaded shim.

* SVM residency: ordinary memory registered with ``hsa_amd_svm_attributes_set`` and moved into
  HBM with ``hsa_amd_svm_prefetch_async`` passes no allocation entry point and ROCr's free
  memory does not show it (profiles/r4b); KFD's per-process counter does (profiles/r5b), so the
  OOM killer would act after the fact - the hook refuses it up front
  (native/src/shim/svm_hooks.cpp; reference: cuMemAllocManaged is accounted, [memory.c:216-223]).
* Pinned host memory through ROCr (a CPU-pool allocation, a memory lock) is held to
  VGPU_HOST_MEMORY_LIMIT (host_hooks.cpp; reference class (b)).
* A HIP runtime loaded with RTLD_DEEPBIND binds its ROCr imports past the preloaded shim
  unless the shim's dlopen hook intervenes (dlsym_hook.cpp; reference: dlsym [libvgpu.c:109-124]).
* The OOM killer is on without any tenant setting (reference: ACTIVE_OOM_KILLER unset = on).
"""
import json
import os
import signal
import subprocess
import time

import pytest

from amdvgpu.shim.launcher import apply_contract, vgpu_env
from amdvgpu.shim.native import LIB_DIR
from amdvgpu.shim.region import Region
from conftest import child_results, run_child, spawn_child

pytestmark = pytest.mark.gpu
GiB = 1 << 30
MiB = 1 << 20
OOR = 0x1008  # HSA_STATUS_ERROR_OUT_OF_RESOURCES
PROBE = os.path.join(LIB_DIR, "escape_probe")


def probe(contract, *args, timeout=120):
    p = subprocess.run([PROBE, *args], env=apply_contract(contract), capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, (p.returncode, p.stdout[-2000:], p.stderr[-3000:])
    r = json.loads(p.stdout.strip().splitlines()[-1])
    print(json.dumps(r))   # in the log when an assertion fails
    return r


def test_svm_prefetch_held_to_the_quota(tmp_region):
    """4 GiB quota: an 8 GiB SVM range prefetched into HBM is refused before the driver sees
    it; a 2 GiB one is admitted and charged (and its data survives the round trip); moved
    back to the CPU it is released."""
    r = probe(vgpu_env(mem_limit=4 * GiB, shared_cache=tmp_region), "svm", "8192", "2048")
    assert r["shim"] == 1 and r["big_attr"] == 0 and r["small_attr"] == 0, r
    assert r["big_prefetch"] == OOR, r
    assert r["small_prefetch"] == 0 and r["small_back"] == 0 and r["small_bad_words"] == 0, r
    base = r["usage_after_big"]               # the runtime's own footprint (context charge)
    assert r["usage_small_in_hbm"] - base >= 2 * GiB, r
    # released when moved back (the context re-sync may see the pages on their way out for a
    # period: read after it)
    assert r["usage_small_back_later"] - base < 256 * MiB, r


def test_svm_prefetch_without_the_shim_escapes():
    """Control: the same probe without the shim - the 8 GiB prefetch goes through (this is the
    escape the hook closes)."""
    p = subprocess.run([PROBE, "svm", "8192", "64"], capture_output=True, text=True, timeout=120,
                       env={k: v for k, v in os.environ.items() if k != "LD_PRELOAD"})
    assert p.returncode == 0, p.stderr[-2000:]
    r = json.loads(p.stdout.strip().splitlines()[-1])
    assert r["shim"] == 0 and r["big_prefetch"] == 0, r


def test_rocr_pinned_memory_held_to_the_host_budget(tmp_region):
    """1 GiB host budget, 600 MiB steps through ROCr directly: the first CPU-pool allocation is
    admitted, the second (1200 MiB) and a memory lock on top are refused; after the frees a
    600 MiB lock fits, and its unlock gives the budget back."""
    c = vgpu_env(mem_limit=8 * GiB, shared_cache=tmp_region, extra={"VGPU_HOST_MEMORY_LIMIT": "1g"})
    r = probe(c, "host", "600")
    assert r["pool_a"] == 0 and r["pool_b"] == OOR and r["lock_while_a"] == OOR, r
    assert r["host_after_a"] >= 600 * MiB, r
    assert r["lock"] == 0 and r["unlock"] == 0, r
    assert r["host_locked"] - r["host_after_free"] == 600 * MiB, r
    assert r["host_unlocked"] == r["host_after_free"], r


DEEPBIND = """
import ctypes, os
RTLD_DEEPBIND = 8
hip = ctypes.CDLL("libamdhip64.so", mode=os.RTLD_NOW | RTLD_DEEPBIND)   # before anything else loads HIP
p = ctypes.c_void_p()
free, total = ctypes.c_size_t(), ctypes.c_size_t()
rc_info = hip.hipMemGetInfo(ctypes.byref(free), ctypes.byref(total))
rc_small = hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(1 << 30))
q = ctypes.c_void_p()
rc_big = hip.hipMalloc(ctypes.byref(q), ctypes.c_size_t(3 << 30))
emit(rc_info=rc_info, total=total.value, rc_small=rc_small, rc_big=rc_big)
"""


def test_deepbind_loaded_hip_is_held_to_the_quota(tmp_region):
    """A tenant that loads HIP with RTLD_DEEPBIND first (its ROCr imports would bind to ROCr
    ahead of the preloaded shim): the quota still holds - 2 GiB total, 1 GiB fits, 3 GiB not."""
    res, _ = run_child(DEEPBIND, vgpu_env(mem_limit=2 * GiB, shared_cache=tmp_region))
    r = res[0]
    assert r["rc_info"] == 0 and r["total"] == 2 * GiB, r
    assert r["rc_small"] == 0 and r["rc_big"] == 2, r   # hipErrorOutOfMemory


def test_oom_killer_on_by_default(tmp_region):
    """No VGPU_ACTIVE_OOM_KILLER anywhere: a process whose measured VRAM exceeds a lowered
    quota (plus the slack) is killed, as with the reference's default."""
    c = vgpu_env(mem_limit=16 * GiB, shared_cache=tmp_region)
    p = spawn_child("""
import torch
x = torch.empty(6 << 30, dtype=torch.uint8, device="cuda")
x.fill_(1)
torch.cuda.synchronize()
emit(ready=True)
time.sleep(60)
""", c)
    try:
        assert p.stdout.readline().startswith("RESULT"), p.stderr.read()[-3000:]
        with Region(tmp_region) as r:
            deadline = time.time() + 10
            while r.device(0)["monitor_used"] < 6 * GiB and time.time() < deadline:
                time.sleep(0.1)
            r.set_memory_limit(0, 2 * GiB)
        p.wait(timeout=20)
    finally:
        if p.poll() is None:
            p.kill()
            pytest.fail("process over the lowered quota was not killed")
    assert p.returncode == -signal.SIGKILL
