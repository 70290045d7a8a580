"""Native core unit tests (C++ runner) plus sanitizer builds, driven by pytest (no GPU)."""
import os
import subprocess

import pytest

from amdvgpu.shim.native import LIB_DIR, NATIVE_DIR


def _run(binary, timeout=300):
    p = subprocess.run([os.path.join(LIB_DIR, binary)], capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    assert "FAIL" not in p.stdout
    return p.stdout


def test_core_tests_pass():
    out = _run("vgpu_core_tests")
    assert out.count("PASS") >= 10


@pytest.mark.slow
@pytest.mark.parametrize("san", ["thread", "address"])
def test_core_tests_sanitized(san):
    rc = subprocess.call(["make", "-C", NATIVE_DIR, "-j8", f"SAN={san}"], stdout=subprocess.DEVNULL)
    assert rc == 0
    _run(f"vgpu_core_tests_{san}", timeout=600)


def test_shim_exports_versioned_symbols():
    """The shim must export the HSA entry points under ROCR_1 (what libamdhip64 imports)."""
    out = subprocess.run(["nm", "-D", "--defined-only", os.path.join(LIB_DIR, "libvgpu_hip.so")],
                         capture_output=True, text=True, check=True).stdout
    for sym in ("hsa_amd_memory_pool_allocate@@ROCR_1", "hsa_queue_create@@ROCR_1",
                "hsa_agent_get_info@@ROCR_1", "hipLaunchKernel@@hip_4.2", "hipGraphLaunch@@hip_4.3"):
        assert sym in out, sym
    # nothing else leaks: internal C++ symbols stay local
    assert "SharedRegion" not in out


def test_calibration_kernels_target_gfx950():
    """The calibration kernels are a gfx950 code object bundle (hipcc --offload-arch=gfx950)."""
    data = open(os.path.join(LIB_DIR, "libvgpu_kernels.so"), "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data


def test_shim_needs_only_old_glibc():
    """The preloaded shim must load in tenant images older than this build host: no C++
    runtime dependency (libstdc++/libgcc are static and local) and C library symbol
    versions no newer than glibc 2.17 (include/vgpu/glibc_compat.h,
    src/shim/glibc_shims.cpp); libdl/libpthread are linked for glibcs that keep the
    dl/pthread functions there."""
    import re
    import shutil
    import subprocess

    import pytest
    from amdvgpu.shim.native import shim_path
    if not shutil.which("readelf"):
        pytest.skip("readelf not available")
    lib = shim_path()
    dyn = subprocess.run(["readelf", "-d", lib], capture_output=True, text=True).stdout
    needed = re.findall(r"Shared library: \[([^\]]+)\]", dyn)
    assert not any(n.startswith(("libstdc++", "libgcc_s")) for n in needed), needed
    assert "libdl.so.2" in needed and "libpthread.so.0" in needed, needed
    ver = subprocess.run(["readelf", "-V", lib], capture_output=True, text=True).stdout
    needs = ver.split("Version needs", 1)[1] if "Version needs" in ver else ""
    names = re.findall(r"Name: (\S+)", needs)
    assert not [n for n in names if n.startswith(("GLIBCXX", "CXXABI", "GCC_"))], names
    glibc = [tuple(int(x) for x in n.split("_", 1)[1].split(".")) for n in names if n.startswith("GLIBC_")]
    assert glibc and max(glibc) <= (2, 17), sorted(glibc)
