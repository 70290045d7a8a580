"""``python -m amdvgpu`` entry points (no GPU)."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def amdvgpu(*args, **kw):
    return subprocess.run([sys.executable, "-m", "amdvgpu", *args], capture_output=True, text=True, cwd=REPO,
                          timeout=120, **kw)


def test_help_and_devices():
    assert "plugin" in amdvgpu("--help").stdout
    p = amdvgpu("devices", "--backend", "fake", "--fake", '{"n": 3}')
    assert p.returncode == 0, p.stderr
    devs = json.loads(p.stdout)
    assert len(devs) == 3 and devs[0]["cu_count"] == 256


def test_run_applies_contract(tmp_path):
    region = str(tmp_path / "r.cache")
    code = "import os; print(os.environ['VGPU_DEVICE_MEMORY_LIMIT'], os.environ['VGPU_DEVICE_CU_LIMIT'], " \
           "'libvgpu_hip.so' in os.environ['LD_PRELOAD'])"
    p = amdvgpu("run", "--memory", "16g", "--cu", "25", "--region", region, "--", sys.executable, "-c", code)
    assert p.returncode == 0, p.stderr
    assert p.stdout.split() == ["16384m", "25", "True"]


def test_region_commands(tmp_path):
    from amdvgpu.shim.region import Region
    path = str(tmp_path / "r.cache")
    r = Region(path, create=True)
    assert amdvgpu("region", path, "set-limit", "0", "4g").returncode == 0
    assert r.device(0)["mem_limit"] == 4 << 30
    p = amdvgpu("region", path, "show")
    assert json.loads(p.stdout)["devices"][0]["mem_limit"] == 4 << 30
    assert amdvgpu("region", path, "suspend").returncode == 0 and r.suspended
    r.close()


def test_plugin_version():
    p = amdvgpu("plugin", "--version")
    assert p.returncode == 0 and p.stdout.strip()
