"""Native CLI tools: vgpuctl (region control) and vgpu-validate (allow-list decode)."""
import json
import os
import subprocess

from amdvgpu.shim.native import LIB_DIR
from amdvgpu.shim.region import Region


def vgpuctl(*args):
    return subprocess.run([os.path.join(LIB_DIR, "vgpuctl"), *args], capture_output=True, text=True)


def test_vgpuctl_show_and_control(region_path):
    r = Region(region_path, create=True)
    r.set_memory_limit(0, 8 << 30)
    slot = r.register(os.getpid())
    r.charge(slot, 0, 1 << 30)
    p = vgpuctl(region_path, "show")
    assert p.returncode == 0, p.stderr
    snap = json.loads(p.stdout)
    assert snap["devices"][0]["mem_limit"] == 8 << 30 and snap["devices"][0]["used"] == 1 << 30
    assert snap["processes"][0]["pid"] == os.getpid()
    assert vgpuctl(region_path, "suspend").returncode == 0 and r.suspended
    assert vgpuctl(region_path, "resume").returncode == 0 and not r.suspended
    assert vgpuctl(region_path, "set-limit", "0", "16g").returncode == 0
    assert r.device(0)["mem_limit"] == 16 << 30
    assert vgpuctl(region_path, "set-cu", "0", "50").returncode == 0
    assert r.device(0)["cu_limit_pct"] == 50
    assert vgpuctl(region_path, "block").returncode == 0 and r.recent_kernel < 0
    assert vgpuctl(region_path, "unblock").returncode == 0 and r.recent_kernel == 2
    assert vgpuctl(region_path, "priority", "4").returncode == 0 and r.priority == 4
    assert vgpuctl(region_path, "set-host-limit", "2g").returncode == 0 and r.host()["limit"] == 2 << 30
    assert r.charge_host(slot, 1 << 20) == 0
    snap = json.loads(vgpuctl(region_path, "show").stdout)
    assert snap["host_limit"] == 2 << 30 and snap["host_used"] == 1 << 20
    assert snap["processes"][0]["host_used"] == 1 << 20
    assert vgpuctl(region_path, "bogus").returncode != 0
    assert vgpuctl(region_path + ".missing", "show").returncode != 0
    r.close()


def test_vgpu_validate_decode(tmp_path):
    f = tmp_path / "allow"
    f.write_text("GPU-ABCDEF0123456789\n9813000000000001\n")
    p = subprocess.run([os.path.join(LIB_DIR, "vgpu-validate"), "--decode", str(f)], capture_output=True, text=True)
    assert p.returncode == 0
    assert p.stdout.split() == ["GPU-abcdef0123456789", "GPU-9813000000000001"]


def test_vgpuctl_board_shows_the_live_containers(tmp_path):
    """vgpuctl board <dir>: the node board as JSON - each live container's class, CPU node,
    launch rate, steadiness and turn state per GPU (what the concurrency admission reads)."""
    import json
    board = tmp_path / "board"
    board.mkdir()
    # An empty board is an empty list; a slot of nonsense is ignored.
    (board / "junk.slot").write_text("not a slot")
    p = vgpuctl("board", str(board))
    assert p.returncode == 0, p.stderr
    assert json.loads(p.stdout) == {"containers": []}
    assert vgpuctl("board", str(tmp_path / "missing")).returncode != 0
