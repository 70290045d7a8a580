"""Node monitor over container regions (no GPU: regions filled through the same
admission path the shim uses)."""
import json
import os
import urllib.error
import urllib.request

import pytest

from amdvgpu.plugin.monitor import control, discover, render_metrics, serve
from amdvgpu.shim.region import Region


def make_region(root, tag, limit=8 << 30, used=3 << 30):
    d = os.path.join(root, tag)
    os.makedirs(d, exist_ok=True)
    p = os.path.join(d, "abc.cache")
    r = Region(p, create=True)
    r.set_memory_limit(0, limit)
    slot = r.register(os.getpid())
    assert r.charge(slot, 0, used, 0) == 0
    return r, slot


def test_metrics_and_control(tmp_path):
    root = str(tmp_path)
    r, slot = make_region(root, "pod1_main")
    assert list(discover(root)) == ["pod1_main"]
    text = render_metrics(root)
    assert 'vgpu_memory_limit_bytes{container="pod1_main",region="abc.cache",device="0"' in text
    assert f"vgpu_memory_used_bytes" in text and str(3 << 30) in text
    assert "vgpu_process_oom_events_total" in text
    assert 'vgpu_sampler_ticks_total{container="pod1_main",region="abc.cache"} 0' in text
    assert 'vgpu_sampler_other_refreshes_total{container="pod1_main",region="abc.cache"} 0' in text
    # pinned host memory: the budget and what the container's processes hold
    r.set_host_limit(8 << 30)
    assert r.charge_host(slot, 1 << 30) == 0 and r.charge_host(slot, 8 << 30) != 0
    text = render_metrics(root)
    assert f'vgpu_host_memory_limit_bytes{{container="pod1_main",region="abc.cache"}} {8 << 30}' in text
    assert f'vgpu_host_memory_used_bytes{{container="pod1_main",region="abc.cache"}} {1 << 30}' in text
    # quota enforcement through the region: a charge past the limit is refused
    assert r.charge(slot, 0, 6 << 30, 0) != 0
    assert control(root, "pod1_main", "suspend", {}) == 1
    assert r.suspended
    control(root, "pod1_main", "resume", {})
    assert not r.suspended
    control(root, "pod1_main", "limit", {"dev": "0", "bytes": str(16 << 30)})
    assert r.device(0)["mem_limit"] == 16 << 30
    control(root, "pod1_main", "block", {})
    assert r.recent_kernel < 0
    control(root, "pod1_main", "unblock", {})
    with pytest.raises(ValueError):
        control(root, "pod1_main", "cu", {"dev": "0", "pct": "150"})
    with pytest.raises(ValueError):
        control(root, "pod1_main", "limit", {"dev": "99", "bytes": "1"})
    control(root, "pod1_main", "priority", {"value": "3"})
    assert r.priority == 3
    r.close()


def test_http_endpoints(tmp_path):
    root = str(tmp_path)
    r, slot = make_region(root, "pod2_c")
    srv = serve(root, "127.0.0.1", 0)
    ctl = serve(root, "127.0.0.1", 0, control_enabled=True)
    port, cport = srv.server_address[1], ctl.server_address[1]
    try:
        body = urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics").read().decode()
        assert "vgpu_container_processes" in body
        snap = json.loads(urllib.request.urlopen(f"http://127.0.0.1:{port}/regions").read())
        assert snap["pod2_c"][0]["devices"][0]["used"] == 3 << 30
        # the metrics server never mutates a tenant
        req = urllib.request.Request(f"http://127.0.0.1:{port}/regions/pod2_c/suspend", method="POST", data=b"")
        with pytest.raises(urllib.error.HTTPError) as e:
            urllib.request.urlopen(req)
        assert e.value.code == 403 and not r.suspended
        req = urllib.request.Request(f"http://127.0.0.1:{cport}/regions/pod2_c/suspend", method="POST", data=b"")
        assert json.loads(urllib.request.urlopen(req).read())["regions"] == 1
        assert r.suspended
    finally:
        srv.shutdown()
        ctl.shutdown()
        r.close()


def test_control_token_and_bind_policy(tmp_path):
    root = str(tmp_path)
    r, slot = make_region(root, "pod3_c")
    with pytest.raises(ValueError):
        serve(root, "0.0.0.0", 0, control_enabled=True)          # beyond loopback without a token
    ctl = serve(root, "127.0.0.1", 0, control_enabled=True, token="s3cret")
    url = f"http://127.0.0.1:{ctl.server_address[1]}/regions/pod3_c/block"
    try:
        with pytest.raises(urllib.error.HTTPError) as e:
            urllib.request.urlopen(urllib.request.Request(url, method="POST", data=b""))
        assert e.value.code == 401 and r.recent_kernel >= 0
        req = urllib.request.Request(url, method="POST", data=b"", headers={"Authorization": "Bearer s3cret"})
        assert json.loads(urllib.request.urlopen(req).read())["regions"] == 1
        assert r.recent_kernel < 0
    finally:
        ctl.shutdown()
        r.close()


def test_board_metrics(tmp_path, monkeypatch):
    """The node board's containers become metrics labelled by region file: launch rate,
    steadiness, CPU node, and per GPU the turn held or waited for (`vgpuctl board` output)."""
    from amdvgpu.plugin import monitor
    assert monitor._board_json(str(tmp_path / "missing")) is None
    board = {"containers": [
        {"container": "c1", "priority": 1, "cpu_node": 1, "launches_per_s": 70000, "steady": True, "hostpids": [7],
         "gpus": [{"gpu_id": 4242, "holds_turn": True, "waiting_ms": None, "svm_vram": 0}]},
        {"container": "c2", "priority": 1, "cpu_node": 0, "launches_per_s": 900, "steady": False, "hostpids": [8],
         "gpus": [{"gpu_id": 4242, "holds_turn": False, "waiting_ms": 12.5, "svm_vram": 0}]}]}
    monkeypatch.setattr(monitor, "_board_json", lambda d: board)
    w = monitor.MetricsWriter()
    monitor.board_metrics(w, str(tmp_path))
    text = w.text()
    assert 'vgpu_board_launches_per_second{region="c1.cache"} 70000' in text
    assert 'vgpu_board_steady{region="c2.cache"} 0' in text
    assert 'vgpu_board_holds_turn{region="c1.cache",gpu_id="4242"} 1' in text
    assert 'vgpu_board_waiting_seconds{region="c2.cache",gpu_id="4242"} 0.0125' in text
