"""Allocate contract details, flag/env parsing, legacy checkpoint and monitor-mode matching."""
import base64
import json
import os
import tempfile

import pytest

from amdvgpu.plugin import api
from amdvgpu.plugin.config import PluginConfig, parse_config
from amdvgpu.plugin.contract import ANN_REQUEST, ANN_USING, build_container_response, response_to_env
from amdvgpu.plugin.devices import FakeBackend
from amdvgpu.plugin.k8s import PodMatcher, pod_summary
from amdvgpu.plugin.legacy import LegacyController
from amdvgpu.plugin.vdevice import device_to_vdevices


_VGPU_DIR = tempfile.mkdtemp(prefix="vgpu-host-")   # never the node's /usr/local/vgpu


def _setup(**kw):
    kw.setdefault("vgpu_dir", _VGPU_DIR)
    cfg = PluginConfig(**kw).validate()
    devs = FakeBackend(n=2).devices()
    vds = device_to_vdevices(devs, cfg.device_split_count, cfg.device_memory_scaling, cfg.device_cores_scaling)
    return cfg, devs, vds, {d.uuid: d for d in devs}


def test_oversubscription_contract():
    cfg, devs, vds, by = _setup(device_split_count=2, device_memory_scaling=1.8)
    envs = dict(build_container_response(cfg, [vds[0]], by).envs)
    total = devs[0].memory_total >> 20
    assert envs["VGPU_OVERSUBSCRIBE"] == "true"
    assert envs["VGPU_DEVICE_MEMORY_LIMIT_0"] == f"{int(total * 1.8 / 2)}m"
    assert envs["VGPU_DEVICE_HBM_LIMIT_0"] == f"{total // 2}m"


def test_index_strategy_and_runtime_list():
    cfg, devs, vds, by = _setup(device_id_strategy="index", device_list_strategy="amd-container-runtime")
    envs = dict(build_container_response(cfg, [vds[2]], by).envs)
    assert envs["AMD_VISIBLE_DEVICES"] == "1"
    assert "ROCR_VISIBLE_DEVICES" not in envs


def test_volume_mounts_strategy():
    cfg, devs, vds, by = _setup(device_list_strategy="volume-mounts")
    r = build_container_response(cfg, [vds[0]], by)
    assert any(m.container_path.startswith("/var/run/amd-container-devices/") for m in r.mounts)


def test_no_device_specs_when_disabled():
    cfg, devs, vds, by = _setup(pass_device_specs=False)
    assert len(build_container_response(cfg, [vds[0]], by).devices) == 0


def test_monitor_mode_host_path(tmp_path):
    cfg, devs, vds, by = _setup(monitor_mode=True, vgpu_dir=str(tmp_path))
    r = build_container_response(cfg, [vds[0]], by, pod_tag="mypod_main")
    envs, mounts = response_to_env(r)
    assert envs["VGPU_SHARED_CACHE"].startswith("/mypod_main/")
    assert ("/mypod_main", str(tmp_path / "shared" / "mypod_main")) in mounts
    assert (tmp_path / "shared" / "mypod_main").is_dir()


def test_temporal_mode_env():
    cfg, devs, vds, by = _setup(cu_mode="temporal")
    assert dict(build_container_response(cfg, [vds[0]], by).envs)["VGPU_CU_MODE"] == "temporal"


def test_pcibus_mount_only_when_present(tmp_path):
    f = tmp_path / "pci"
    cfg, devs, vds, by = _setup(pcibus_file=str(f))
    paths = [m.container_path for m in build_container_response(cfg, [vds[0]], by).mounts]
    assert "/usr/local/vgpu/pciinfo.vgpu" not in paths
    f.write_text("0000:05:00.0\n")
    paths = [m.container_path for m in build_container_response(cfg, [vds[0]], by).mounts]
    assert "/usr/local/vgpu/pciinfo.vgpu" in paths


def test_flags_env_fallback_and_validation():
    cfg = parse_config([], environ={"DEVICE_SPLIT_COUNT": "4", "DEVICE_MEMORY_SCALING": "1.5",
                                    "MIG_STRATEGY": "mixed", "PASS_DEVICE_SPECS": "false"})
    assert cfg.device_split_count == 4 and cfg.device_memory_scaling == 1.5
    assert cfg.partition_strategy == "mixed" and cfg.pass_device_specs is False
    cfg = parse_config(["--device-split-count", "8", "--mig-strategy", "single"], environ={"DEVICE_SPLIT_COUNT": "3"})
    assert cfg.device_split_count == 8 and cfg.partition_strategy == "single"
    for bad in (["--device-split-count", "0"], ["--device-memory-scaling", "0"], ["--device-cores-scaling", "-1"],
                ["--device-list-strategy", "x"], ["--device-id-strategy", "x"], ["--cu-mode", "x"],
                ["--partition-strategy", "x"]):
        with pytest.raises(ValueError):
            parse_config(bad, environ={})
    assert parse_config(["--fail-on-init-error=false"], environ={}).fail_on_init_error is False


def _checkpoint(tmp_path, entries):
    data = {"Data": {"PodDeviceEntries": entries, "RegisteredDevices": {"amd.com/gpu": []}}, "Checksum": 1}
    (tmp_path / "kubelet_internal_checkpoint").write_text(json.dumps(data))


def _alloc_resp(request, using):
    r = api.ContainerAllocateResponse()
    r.annotations[ANN_REQUEST] = ",".join(request)
    r.annotations[ANN_USING] = ",".join(using)
    return base64.b64encode(r.SerializeToString()).decode()


def test_legacy_checkpoint_acquire_release(tmp_path):
    ids = ["g-0", "g-1", "h-0", "h-1"]
    _checkpoint(tmp_path, [
        {"PodUID": "p1", "ContainerName": "c", "ResourceName": "amd.com/gpu", "DeviceIDs": ["g-0"],
         "AllocResp": _alloc_resp(["g-0"], ["h-0"])},
        {"PodUID": "p2", "ContainerName": "c", "ResourceName": "amd.com/gpu", "DeviceIDs": {"0": ["g-1"]},
         "AllocResp": _alloc_resp(["g-1"], ["h-1"])},
        {"PodUID": "p3", "ContainerName": "c", "ResourceName": "other/res", "DeviceIDs": ["x"],
         "AllocResp": _alloc_resp(["x"], ["g-0"])},
    ])
    lc = LegacyController(ids, "amd.com/gpu", str(tmp_path),
                          pod_lister=lambda: [{"uid": "p1", "phase": "Running"}, {"uid": "p2", "phase": "Succeeded"}])
    assert lc.update_from_checkpoint()
    assert lc.id_map["h-0"] == "g-0"     # live pod keeps its substitution
    assert lc.id_map["h-1"] == ""        # finished pod released
    assert lc.available(ids) == ["g-0", "g-1", "h-1"]
    lc.release_by_request(["g-0"])
    assert lc.id_map["h-0"] == ""


def test_legacy_missing_checkpoint(tmp_path):
    lc = LegacyController(["a"], "amd.com/gpu", str(tmp_path))
    assert lc.update_from_checkpoint() is False


def test_monitor_pod_matcher():
    pods = [
        pod_summary({"metadata": {"uid": "1", "name": "old", "creationTimestamp": "2024-01-01"},
                     "spec": {"containers": [{"name": "a", "resources": {"limits": {"amd.com/gpu": "2"}}}]},
                     "status": {"phase": "Running"}}),
        pod_summary({"metadata": {"uid": "2", "name": "new", "creationTimestamp": "2024-01-02"},
                     "spec": {"containers": [{"name": "side"}, {"name": "main", "resources": {
                         "limits": {"amd.com/gpu": "1"}}}]}, "status": {"phase": "Pending"}}),
    ]
    m = PodMatcher(lambda: pods)
    assert m.match([1]) == ["new_main"]
    with pytest.raises(LookupError):
        m.match([2])
    # Same pod name in two namespaces: distinct tags (distinct host dirs for the monitor).
    twin = [pod_summary({"metadata": {"uid": u, "name": "train", "namespace": ns, "creationTimestamp": t},
                         "spec": {"containers": [{"name": "main", "resources": {"limits": {"amd.com/gpu": "1"}}}]},
                         "status": {"phase": "Pending"}}) for u, ns, t in (("a", "team-a", "1"), ("b", "team-b", "2"))]
    assert PodMatcher(lambda: twin).match([1]) == ["team-a_train_main"]
    assert PodMatcher(lambda: twin[1:]).match([1]) == ["team-b_train_main"]


def _legacy_server(tmp_path, split=2):
    from amdvgpu.plugin.server import AllocationError, DevicePluginServer
    cfg = PluginConfig(device_plugin_path=str(tmp_path) + "/", device_split_count=split,
                       enable_legacy_preferred=True, vgpu_dir=str(tmp_path / "vgpu")).validate()
    devs = FakeBackend(n=1).devices()
    ids = [f"{devs[0].uuid}-{i}" for i in range(split)]
    srv = DevicePluginServer(cfg, "amd.com/gpu", "amd-gpu.sock", devs,
                             legacy=LegacyController(ids, "amd.com/gpu", str(tmp_path)))
    srv.initialize()
    return srv, ids, AllocationError


def _alloc_req(ids):
    return api.AllocateRequest(container_requests=[api.ContainerAllocateRequest(devicesIDs=ids)])


def test_legacy_allocate_refuses_when_pool_exhausted(tmp_path):
    """Reference server.go:436-439 ("no enough devices"): when the legacy pool has fewer
    free vGPUs than requested, Allocate fails instead of reusing the kubelet's IDs (which
    may belong to another container) or handing out fewer GPUs than asked for."""
    srv, ids, AllocationError = _legacy_server(tmp_path, split=3)
    _checkpoint(tmp_path, [])
    r1 = srv.Allocate(_alloc_req([ids[0]]), None)
    r2 = srv.Allocate(_alloc_req([ids[1]]), None)
    used = [dict(r.container_responses[0].annotations)[ANN_USING] for r in (r1, r2)]
    assert len(set(used)) == 2                       # no double booking
    # Live pods in the checkpoint hold every vGPU under other request IDs: a request for a
    # vGPU the kubelet believes free must be refused, not served with its own (taken) ID.
    entries = [{"PodUID": f"p{i}", "ContainerName": "c", "ResourceName": "amd.com/gpu", "DeviceIDs": [f"x-{i}"],
                "AllocResp": _alloc_resp([f"x-{i}"], [v])} for i, v in enumerate(ids)]
    _checkpoint(tmp_path, entries)
    srv2, ids2, _ = _legacy_server(tmp_path, split=3)
    srv2.legacy.pod_lister = lambda: [{"uid": f"p{i}", "phase": "Running"} for i in range(3)]
    with pytest.raises(AllocationError):
        srv2.Allocate(_alloc_req([ids2[0]]), None)
    # One of them ends: one vGPU free, two requested -> refused, never a short allocation.
    srv2.legacy.pod_lister = lambda: [{"uid": f"p{i}", "phase": "Running" if i else "Succeeded"} for i in range(3)]
    with pytest.raises(AllocationError):
        srv2.Allocate(_alloc_req(ids2[:2]), None)
    r = srv2.Allocate(_alloc_req([ids2[1]]), None)
    assert dict(r.container_responses[0].annotations)[ANN_USING] == ids2[0]


def test_legacy_allocate_refuses_without_checkpoint(tmp_path):
    """Reference server.go:410-412: an unreadable checkpoint fails the allocation."""
    srv, ids, AllocationError = _legacy_server(tmp_path)
    with pytest.raises(AllocationError):
        srv.Allocate(_alloc_req([ids[0]]), None)


def test_legacy_allocate_concurrent_calls_never_share_a_vgpu(tmp_path):
    """Allocate runs on the gRPC thread pool: concurrent legacy-mode calls must each get
    their own vGPUs (the read-available / acquire sequence is serialised)."""
    import threading

    srv, ids, _ = _legacy_server(tmp_path, split=8)
    _checkpoint(tmp_path, [])
    got, errors = [], []

    def one(i):
        try:
            resp = srv.Allocate(_alloc_req([ids[i]]), None)
            got.append(dict(resp.container_responses[0].annotations)[ANN_USING])
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    threads = [threading.Thread(target=one, args=(i,)) for i in range(8)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    assert not errors, errors
    assert len(got) == 8 and len(set(got)) == 8, got


def test_reference_flag_and_env_names_accepted():
    """The reference's manifests work unchanged: --mig-strategy / MIG_STRATEGY and
    --nvidia-driver-root / NVIDIA_DRIVER_ROOT map onto the MI355X flags."""
    from amdvgpu.plugin.config import parse_config
    c = parse_config(["--nvidia-driver-root=/run/driver", "--mig-strategy=single"], environ={})
    assert c.driver_root == "/run/driver" and c.partition_strategy == "single"
    c = parse_config([], environ={"NVIDIA_DRIVER_ROOT": "/x", "MIG_STRATEGY": "mixed"})
    assert c.driver_root == "/x" and c.partition_strategy == "mixed"


def _pod(uid, name, ctrs, phase="Pending", ns="ns", created="2024-01-01", init=()):
    return pod_summary({"metadata": {"uid": uid, "name": name, "namespace": ns, "creationTimestamp": created},
                        "spec": {"initContainers": [{"name": c, "resources": {"limits": {"amd.com/gpu": str(g)}}}
                                                    for c, g in init],
                                 "containers": [{"name": c, "resources": {"limits": {"amd.com/gpu": str(g)}}}
                                                for c, g in ctrs]},
                        "status": {"phase": phase}})


def test_monitor_matcher_allocates_containers_one_at_a_time(tmp_path):
    """A kubelet calls Allocate once per container: a pod with two GPU containers (and a
    GPU init container) is matched container by container, in allocation order; a
    restarted plugin picks up where the last one stopped through the .pod-uid markers."""
    root = tmp_path / "shared"
    pods = [_pod("u1", "two", [("a", 1), ("side", 0), ("b", 2)], init=[("prep", 1)])]
    m = PodMatcher(lambda: pods, shared_root=str(root))
    assert m.match([1]) == ["ns_two_prep"] and m.owner("ns_two_prep") == "u1"
    assert m.match([1]) == ["ns_two_a"]
    # the plugin restarts after the first two: the markers written by the contract tell
    (root / "ns_two_prep").mkdir(parents=True)
    (root / "ns_two_prep" / ".pod-uid").write_text("u1\n")
    (root / "ns_two_a").mkdir()
    (root / "ns_two_a" / ".pod-uid").write_text("u1\n")
    m2 = PodMatcher(lambda: pods, shared_root=str(root))
    assert m2.match([2]) == ["ns_two_b"]
    with pytest.raises(LookupError):
        m2.match([1])
    # a re-created pod of the same name (new UID) is not confused with the old markers
    again = [_pod("u2", "two", [("a", 1), ("side", 0), ("b", 2)], init=[("prep", 1)])]
    assert PodMatcher(lambda: again, shared_root=str(root)).match([1]) == ["ns_two_prep"]


def test_monitor_mode_shared_dirs_follow_the_pod_list(tmp_path):
    """Directories go when their pod is gone (or terminal, or re-created under the same
    name), never because they are old or their region is idle; no pod list, no GC."""
    import time

    from amdvgpu.plugin.contract import gc_shared_dirs
    root = tmp_path / "shared"
    now = time.time()
    old = now - 3 * 24 * 3600
    for tag, uid in (("ns_idle_main", "u-idle"), ("ns_gone_main", "u-gone"), ("ns_done_main", "u-done"),
                     ("ns_again_main", "u-old"), ("ns_fresh_main", "u-fresh")):
        (root / tag).mkdir(parents=True)
        (root / tag / ".pod-uid").write_text(uid + "\n")
        if tag != "ns_fresh_main":
            os.utime(root / tag, (old, old))
    pods = [_pod("u-idle", "idle", [("main", 1)], phase="Running"),
            _pod("u-done", "done", [("main", 1)], phase="Succeeded"),
            _pod("u-new", "again", [("main", 1)], phase="Running")]
    assert gc_shared_dirs(str(root), None, now=now) == []
    removed = gc_shared_dirs(str(root), pods, now=now)
    assert sorted(removed) == ["ns_again_main", "ns_done_main", "ns_gone_main"]
    assert sorted(os.listdir(root)) == ["ns_fresh_main", "ns_idle_main"]


def test_placement_duplicate_and_host_memory_flags():
    from amdvgpu.plugin.config import parse_config
    cfg = parse_config(["--placement", "binpack", "--duplicate-vgpus", "merge", "--host-memory-per-vgpu", "8g"],
                       environ={})
    assert (cfg.placement, cfg.duplicate_vgpus, cfg.host_memory_per_vgpu_bytes) == ("binpack", "merge", 8 << 30)
    cfg = parse_config([], environ={"PLACEMENT_POLICY": "binpack", "DUPLICATE_VGPUS": "merge",
                                    "HOST_MEMORY_PER_VGPU": "512m"})
    assert (cfg.placement, cfg.duplicate_vgpus, cfg.host_memory_per_vgpu_bytes) == ("binpack", "merge", 512 << 20)
    cfg = parse_config([], environ={})
    assert (cfg.placement, cfg.duplicate_vgpus, cfg.host_memory_per_vgpu_bytes) == ("spread", "split", 0)
    assert parse_config(["--duplicate-vgpus", "reject"], environ={}).duplicate_vgpus == "reject"
    assert parse_config(["--duplicate-vgpus", "split"], environ={}).duplicate_vgpus == "split"
    for bad in (["--placement", "random"], ["--duplicate-vgpus", "allow"], ["--host-memory-per-vgpu", "lots"]):
        with pytest.raises(ValueError):
            parse_config(bad, environ={})


def test_host_pid_lock_is_a_read_only_file_mount(tmp_path):
    """The node-wide host-PID lock is a plugin-created file mounted read-only (tenants can
    flock it but not unlink or replace it)."""
    from amdvgpu.plugin.contract import build_container_response, ensure_lock_file
    from amdvgpu.plugin.devices import FakeBackend
    from amdvgpu.plugin.vdevice import device_to_vdevices
    vdir = str(tmp_path / "vgpu")
    path = ensure_lock_file(vdir)
    assert os.stat(path).st_mode & 0o777 == 0o644
    assert os.stat(os.path.dirname(path)).st_mode & 0o777 == 0o755
    devs = FakeBackend(n=1).devices()
    cfg = PluginConfig(vgpu_dir=vdir).validate()
    resp = build_container_response(cfg, device_to_vdevices(devs, 2)[:1], {d.uuid: d for d in devs})
    mounts = {m.container_path: (m.host_path, m.read_only) for m in resp.mounts}
    assert mounts["/usr/local/vgpu/lock/hostpid.lock"] == (path, True)
    assert dict(resp.envs)["VGPU_LOCK_FILE"] == "/usr/local/vgpu/lock/hostpid.lock"


def test_board_slot_mounts(tmp_path):
    """Each container gets the board directory read-only and its own slot read-write."""
    from amdvgpu.plugin.contract import build_container_response, ensure_board_dir
    from amdvgpu.plugin.devices import FakeBackend
    from amdvgpu.plugin.vdevice import device_to_vdevices
    vdir = str(tmp_path / "vgpu")
    board = ensure_board_dir(vdir)
    devs = FakeBackend(n=1).devices()
    cfg = PluginConfig(vgpu_dir=vdir).validate()
    r1 = build_container_response(cfg, device_to_vdevices(devs, 2)[:1], {d.uuid: d for d in devs})
    r2 = build_container_response(cfg, device_to_vdevices(devs, 2)[1:2], {d.uuid: d for d in devs})
    slots = []
    for r in (r1, r2):
        envs = dict(r.envs)
        mounts = {m.container_path: (m.host_path, m.read_only) for m in r.mounts}
        assert envs["VGPU_BOARD_DIR"] == "/usr/local/vgpu/board"
        assert mounts["/usr/local/vgpu/board"] == (board, True)
        slot = envs["VGPU_BOARD_SLOT"]
        assert mounts[f"/usr/local/vgpu/board/{slot}"] == (os.path.join(board, slot), False)
        assert os.stat(os.path.join(board, slot)).st_mode & 0o777 == 0o666
        slots.append(slot)
    assert slots[0] != slots[1]
    # the container-side order matters: the directory is mounted before the file on top
    paths = [m.container_path for m in r1.mounts]
    assert paths.index("/usr/local/vgpu/board") < paths.index(f"/usr/local/vgpu/board/{slots[0]}")


def test_container_files_live_as_long_as_the_pod(tmp_path):
    """A container's host files (limits, region, allow-list, board slot) are the sources of
    its bind mounts, which the kubelet reuses when the container restarts: they are removed
    only when PodResources no longer lists the container's devices as held - however old they
    are - and never when PodResources cannot be asked (a week-old limits file or an
    idle hour-old region broke the restart)."""
    import time
    from amdvgpu.plugin.config import PluginConfig
    from amdvgpu.plugin.contract import build_container_response, container_files, gc_container_files
    from amdvgpu.plugin.devices import FakeBackend
    from amdvgpu.plugin.vdevice import device_to_vdevices
    from amdvgpu.plugin.contract import ensure_board_dir
    vdir = str(tmp_path / "vgpu")
    ensure_board_dir(vdir)
    cfg = PluginConfig(vgpu_dir=vdir, device_split_count=4).validate()
    devs = FakeBackend(n=1).devices()
    vds = device_to_vdevices(devs, 4, 1.0, 1.0)
    by_uuid = {d.uuid: d for d in devs}
    names = {}
    for ids in (["a-0"], ["a-1"], ["a-2"]):
        r = build_container_response(cfg, [vds[int(ids[0][-1])]], by_uuid, kubelet_ids=ids, resource="amd.com/gpu")
        names[ids[0]] = os.path.basename(dict(r.envs)["VGPU_SHARED_CACHE"]).rsplit(".", 1)[0]
    for n in names.values():
        assert all(os.path.exists(f) for f in container_files(vdir, n)), container_files(vdir, n)
    week = time.time() + 8 * 24 * 3600
    assert gc_container_files(vdir, None, now=week) == []                         # no PodResources: keep all
    assert gc_container_files(vdir, {"amd.com/gpu": set()}, now=time.time()) == []  # within the grace period
    held = {"amd.com/gpu": {frozenset(["a-0"]), frozenset(["a-2"])}}
    assert gc_container_files(vdir, held, now=week) == [names["a-1"]]
    assert not any(os.path.exists(f) for f in container_files(vdir, names["a-1"]))
    for k in ("a-0", "a-2"):
        assert all(os.path.exists(f) for f in container_files(vdir, names[k]))
    # the same IDs under another resource are not this container's
    assert sorted(gc_container_files(vdir, {"amd.com/gpu-latency": held["amd.com/gpu"]}, now=week)) == \
        sorted([names["a-0"], names["a-2"]])


def test_pre_manifest_container_files_go_once_they_are_a_month_old(tmp_path):
    """host files of containers allocated before manifests existed are removed
    once their limits file is 30 days old - never younger, never without PodResources."""
    import time
    from amdvgpu.plugin.contract import LEGACY_GC_AGE_S, container_files, gc_container_files
    vdir = tmp_path / "vgpu"
    files = [p for p in container_files(str(vdir), "old-ctr")]
    for p in files:
        os.makedirs(os.path.dirname(p), exist_ok=True)
        open(p, "w").close()
    now = time.time()
    assert gc_container_files(str(vdir), None, now=now + 2 * LEGACY_GC_AGE_S) == []
    assert gc_container_files(str(vdir), {}, now=now + LEGACY_GC_AGE_S / 2) == []
    assert all(os.path.exists(p) for p in files)
    assert gc_container_files(str(vdir), {}, now=now + LEGACY_GC_AGE_S + 60) == ["old-ctr"]
    assert not any(os.path.exists(p) for p in files)


def test_limits_file_carries_the_oom_killer(tmp_path):
    """The memory backstop is the plugin's: the limits file switches it (on by default)."""
    from amdvgpu.plugin.config import PluginConfig
    from amdvgpu.plugin.contract import build_container_response
    from amdvgpu.plugin.devices import FakeBackend
    from amdvgpu.plugin.vdevice import device_to_vdevices
    devs = FakeBackend(n=1).devices()
    vds = device_to_vdevices(devs, 2, 1.0, 1.0)
    for on, want in ((True, "1"), (False, "0")):
        cfg = PluginConfig(vgpu_dir=str(tmp_path / f"v{want}"), active_oom_killer=on).validate()
        r = build_container_response(cfg, vds[:1], {d.uuid: d for d in devs})
        mounts = {m.container_path: m.host_path for m in r.mounts}
        limits = dict(l.split("=", 1) for l in open(mounts["/vgpu/limits"]).read().splitlines())
        assert limits["VGPU_ACTIVE_OOM_KILLER"] == want
