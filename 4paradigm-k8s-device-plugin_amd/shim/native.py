"""Locating and building the native libraries.

All native artefacts are built in-tree into ``<pkg>/lib`` by ``make -C native`` (driven
by ``__graft_entry__.build()``), so they travel with the repository snapshot to a GPU
box and are never pip-installed. Missing artefacts raise: there is no Python fallback
for the data plane.
"""
import os
import subprocess

from .. import LIB_DIR, NATIVE_DIR

SHIM = "libvgpu_hip.so"
REGION = "libvgpu_region.so"
KERNELS = "libvgpu_kernels.so"
VGPUCTL = "vgpuctl"
LEDGER = "vgpu-ledger"
VALIDATE = "vgpu-validate"
CORE_TESTS = "vgpu_core_tests"


class NativeMissing(RuntimeError):
    pass


def lib_path(name):
    p = os.path.join(LIB_DIR, name)
    if not os.path.exists(p):
        raise NativeMissing(f"{p} is not built; run `make -C {NATIVE_DIR}` (or __graft_entry__.build())")
    return p


def shim_path():
    return lib_path(SHIM)


def ensure_built(targets=None, jobs=8, extra=None):
    """Runs make in native/ (incremental). Returns the make exit code."""
    cmd = ["make", "-C", NATIVE_DIR, f"-j{jobs}"]
    if extra:
        cmd += list(extra)
    if targets:
        cmd += list(targets)
    return subprocess.call(cmd)
