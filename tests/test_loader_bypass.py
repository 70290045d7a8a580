"""Loader-level bypasses of the preloaded shim, on the CPU-only fake runtime.

RTLD_DEEPBIND puts a loaded object's own dependency scope ahead of the global one, where the
preloaded shim lives: a HIP runtime loaded that way would bind its ROCr imports straight to
ROCr (no quota), and a tenant module loaded that way would bind its HIP imports straight to
HIP. dlmopen(LM_ID_NEWLM) loads a second ROCr in a namespace the preload never reached. The
reference interposes the loader for the same reason (dlsym [libvgpu.c:109-124]); here
native/src/shim/dlsym_hook.cpp interposes dlopen / dlmopen as well.
"""
import json
import os
import subprocess
import sys

import pytest

from amdvgpu.shim.native import LIB_DIR, shim_path

GiB = 1 << 30
FAKE = os.path.join(LIB_DIR, "fakerocm")
RTLD_DEEPBIND = 8


@pytest.fixture
def env(tmp_path):
    kfd = tmp_path / "kfd"
    kfd.mkdir()
    e = {k: v for k, v in os.environ.items() if not k.startswith(("VGPU_", "FAKE_"))}
    e.update(FAKE_ROCR_GPUS="1", FAKE_ROCR_HBM=str(16 * GiB), FAKE_KFD_ROOT=str(kfd), VGPU_KFD_ROOT=str(kfd),
             VGPU_SHARED_CACHE=str(tmp_path / "r.cache"), VGPU_LOCK_FILE=str(tmp_path / "lock"),
             LD_PRELOAD=shim_path(), VGPU_DEVICE_MEMORY_LIMIT="2g")
    return e


def child(env, code):
    src = f"import ctypes, json, os, sys\nFAKE = {FAKE!r}\nDEEP = {RTLD_DEEPBIND}\n" + code
    p = subprocess.run([sys.executable, "-c", src], env=env, capture_output=True, text=True, timeout=60)
    assert p.returncode == 0, p.stderr[-3000:]
    return json.loads(p.stdout.strip().splitlines()[-1])


HIP_DIRECT = """
hip = ctypes.CDLL(os.path.join(FAKE, "libamdhip64.so"), mode=os.RTLD_NOW | DEEP)
hip.hipInit(0)
p = ctypes.c_void_p()
free, total = ctypes.c_size_t(), ctypes.c_size_t()
hip.hipMemGetInfo(ctypes.byref(free), ctypes.byref(total))
small = hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(1 << 30))
big = hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(3 << 30))
print(json.dumps(dict(total=total.value, small=small, big=big)))
"""

TENANT = """
t = ctypes.CDLL(os.path.join(FAKE, "libfaketenant.so"), mode=os.RTLD_NOW | DEEP)
t.tenant_total.restype = ctypes.c_ulonglong
total = t.tenant_total()
small = t.tenant_malloc(ctypes.c_ulonglong(1 << 30))
big = t.tenant_malloc(ctypes.c_ulonglong(3 << 30))
print(json.dumps(dict(total=total, small=small, big=big)))
"""


@pytest.mark.parametrize("code", [HIP_DIRECT, TENANT], ids=["deepbind-hip", "deepbind-tenant-module"])
def test_deepbind_load_is_held_to_the_quota(env, code):
    """The HIP runtime loaded with RTLD_DEEPBIND (the flag is dropped for it), or a tenant
    module that links HIP loaded that way (its and HIP's GOT entries for hooked names are
    rebound to the shim): the 2 GiB quota holds either way."""
    r = child(env, code)
    assert r == {"total": 2 * GiB, "small": 0, "big": 2}, r   # 2 = hipErrorOutOfMemory


@pytest.mark.parametrize("code", [HIP_DIRECT, TENANT], ids=["deepbind-hip", "deepbind-tenant-module"])
def test_deepbind_without_the_shim_escapes(env, code):
    """Control: the same loads with VGPU_HOOK_DLSYM=0 (the loader hooks off; no limits file)
    get the whole fake GPU - the escape the hooks close."""
    env["VGPU_HOOK_DLSYM"] = "0"
    r = child(env, code)
    assert r["total"] == 16 * GiB and r["big"] == 0, r


DLMOPEN = """
libc = ctypes.CDLL(None)
libc.dlmopen.restype = ctypes.c_void_p
libc.dlmopen.argtypes = [ctypes.c_long, ctypes.c_char_p, ctypes.c_int]
LM_ID_NEWLM = -1
h_hip = libc.dlmopen(LM_ID_NEWLM, os.path.join(FAKE, "libamdhip64.so").encode(), os.RTLD_NOW)
h_other = libc.dlmopen(LM_ID_NEWLM, b"libm.so.6", os.RTLD_NOW)
print(json.dumps(dict(hip=bool(h_hip), other=bool(h_other))))
"""


def test_dlmopen_of_the_rocm_runtime_is_refused(env):
    """A second link-map namespace holding a ROCm runtime (outside the preload) is refused in
    a vGPU container; dlmopen of anything else still works."""
    assert child(env, DLMOPEN) == {"hip": False, "other": True}


def test_dlmopen_only_logged_outside_a_vgpu_container(env):
    env.pop("VGPU_DEVICE_MEMORY_LIMIT")
    assert child(env, DLMOPEN) == {"hip": True, "other": True}


TENANT_AFTER_HIP = """
import threading, time
hip = ctypes.CDLL(os.path.join(FAKE, "libamdhip64.so"), mode=os.RTLD_NOW | os.RTLD_GLOBAL)  # torch's HIP
hip.hipInit(0)
t = ctypes.CDLL(os.path.join(FAKE, "libfaketenant.so"), mode=os.RTLD_NOW | DEEP)
t.tenant_total.restype = ctypes.c_ulonglong
me = ctypes.CDLL(None)
assert t.tenant_launch() == 0
me.vgpu_suspend_all()
threading.Timer(0.15, me.vgpu_resume_all).start()
t0 = time.time()
rc = t.tenant_launch()
blocked = time.time() - t0
print(json.dumps(dict(rc=rc, blocked=blocked, total=t.tenant_total(), big=t.tenant_malloc(ctypes.c_ulonglong(3 << 30)))))
"""


def test_deepbind_tenant_module_after_hip_is_gated(env):
    """The usual order: HIP is already loaded (torch imported) when a tenant module
    that links HIP is loaded with RTLD_DEEPBIND. Its hip* imports would bind to HIP ahead of the
    shim; they are rebound, so its launches pass the launch gate (held while the container is
    suspended) and its memory queries see the quota."""
    r = child(env, TENANT_AFTER_HIP)
    assert r["rc"] == 0 and r["blocked"] >= 0.12, r
    assert r["total"] == 2 * GiB and r["big"] == 2, r


def test_deepbind_tenant_module_after_hip_escapes_without_the_hooks(env):
    env["VGPU_HOOK_DLSYM"] = "0"
    r = child(env, TENANT_AFTER_HIP)
    assert r["rc"] == 0 and r["blocked"] < 0.1, r   # control: the launch skipped the gate


BARE_NAME = """
import shutil, tempfile
d = tempfile.mkdtemp()
# a loader library with RUNPATH=$ORIGIN next to the tenant module: its DEEPBIND dlopen of the
# bare name must still find the module (the caller's RUNPATH), with ROCm loaded
hip = ctypes.CDLL(os.path.join(FAKE, "libamdhip64.so"), mode=os.RTLD_NOW | os.RTLD_GLOBAL)
for f in ("libfaketenant.so", "libdeeploader.so"):
    shutil.copy(os.path.join(FAKE, f), d)
ld = ctypes.CDLL(os.path.join(d, "libdeeploader.so"))
ld.deep_open.restype = ctypes.c_void_p
h = ld.deep_open(b"libfaketenant.so", DEEP | 2)
print(json.dumps(dict(found=bool(h))))
"""


def test_deepbind_bare_name_uses_the_callers_runpath(env):
    assert child(env, BARE_NAME) == {"found": True}


NS_LOADER = """
libc = ctypes.CDLL(None)
libc.dlmopen.restype = ctypes.c_void_p
libc.dlmopen.argtypes = [ctypes.c_long, ctypes.c_char_p, ctypes.c_int]
libc.dlsym.restype = ctypes.c_void_p
libc.dlsym.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
h = libc.dlmopen(-1, b"libc.so.6", os.RTLD_NOW)   # a harmless library in a new namespace
got = {n: bool(libc.dlsym(h, n.encode())) for n in ("dlopen", "dlmopen", "dlsym", "printf")}
print(json.dumps(dict(ns=bool(h), **got)))
"""


def test_loader_of_another_namespace_is_not_handed_out(env):
    """dlmopen of a harmless library, then that namespace's own dlopen (which never
    saw the preload) to load ROCm there. The lookup of its loader entry points is refused in a
    vGPU container; its other symbols resolve."""
    assert child(env, NS_LOADER) == {"ns": True, "dlopen": False, "dlmopen": False, "dlsym": False, "printf": True}
    env.pop("VGPU_DEVICE_MEMORY_LIMIT")
    assert child(env, NS_LOADER) == {"ns": True, "dlopen": True, "dlmopen": True, "dlsym": True, "printf": True}
