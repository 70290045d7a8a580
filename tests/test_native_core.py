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
