"""SysfsBackend on a synthetic KFD/DRM sysfs tree (shaped like the MI355X box's)."""
import os

from amdvgpu.plugin.devices import IOLINK_XGMI, SysfsBackend, bdf_from_location, rocr_uuid


def make_tree(root, ngpu=2, cpx=False):
    kfd = root / "kfd"
    drm = root / "drm"
    # CPU node 0
    n0 = kfd / "0"
    n0.mkdir(parents=True)
    (n0 / "gpu_id").write_text("0\n")
    (n0 / "properties").write_text("cpu_cores_count 64\nsimd_count 0\n")
    parts = 8 if cpx else 1
    node = 1
    for g in range(ngpu):
        for p in range(parts):
            nd = kfd / str(node)
            (nd / "mem_banks" / "0").mkdir(parents=True)
            (nd / "gpu_id").write_text(f"{1000 + node}\n")
            minor = 128 + node
            props = {"simd_count": 1024 // parts, "simd_per_cu": 4, "num_xcc": 8 // parts,
                     "drm_render_minor": minor, "location_id": (0x05 + 0x10 * g) << 8, "domain": 0,
                     "unique_id": 0x9813000000000000 + g, "gfx_target_version": 90500}
            (nd / "properties").write_text("".join(f"{k} {v}\n" for k, v in props.items()))
            (nd / "mem_banks" / "0" / "properties").write_text(f"size_in_bytes {309220868096 // parts}\n")
            dev = drm / f"renderD{minor}" / "device"
            (dev / "drm" / f"card{node}").mkdir(parents=True)
            (dev / "numa_node").write_text(f"{g % 2}\n")
            (dev / "current_compute_partition").write_text("CPX\n" if cpx else "SPX\n")
            (dev / "current_memory_partition").write_text("NPS1\n")
            (dev / "ras").mkdir()
            (dev / "ras" / "umc_err_count").write_text("ue: 0\nce: 0\n")
            node += 1
    # xGMI links between the GPU nodes (SPX case)
    if not cpx:
        for a in range(1, node):
            for i, b in enumerate(x for x in range(1, node) if x != a):
                lk = kfd / str(a) / "io_links" / str(i)
                lk.mkdir(parents=True)
                lk.joinpath("properties").write_text(f"type {IOLINK_XGMI}\nnode_from {a}\nnode_to {b}\nweight 15\n")
    return str(kfd), str(drm)


def test_inventory(tmp_path):
    kfd, drm = make_tree(tmp_path, ngpu=2)
    devs = SysfsBackend(kfd, drm).devices()
    assert len(devs) == 2
    d = devs[0]
    assert d.uuid == rocr_uuid(0x9813000000000000) == "GPU-9813000000000000"
    assert d.bdf == "0000:05:00.0" and devs[1].bdf == "0000:15:00.0"
    assert d.cu_count == 256 and d.num_xcc == 8 and d.memory_total == 309220868096
    assert d.render_minor == 129 and d.card_index == 1 and d.gpu_id == 1001
    assert d.numa_node == 0 and devs[1].numa_node == 1
    assert d.gfx_target == "gfx950" and not d.is_partition
    assert d.links[1] == [(IOLINK_XGMI, 15)]
    assert d.device_paths == ["/dev/kfd", "/dev/dri/renderD129", "/dev/dri/card1"]


def test_cpx_partitions_get_distinct_uuids(tmp_path):
    kfd, drm = make_tree(tmp_path, ngpu=1, cpx=True)
    devs = SysfsBackend(kfd, drm).devices()
    assert len(devs) == 8
    assert len({d.uuid for d in devs}) == 8
    assert all(d.is_partition and d.cu_count == 32 and d.num_xcc == 1 for d in devs)


def test_ras_health_and_recovery(tmp_path):
    """Uncorrectable errors mark the GPU unhealthy; it recovers only after the UE count
    stayed flat for the hold-off (or at a reset), not after one quiet poll."""
    kfd, drm = make_tree(tmp_path, ngpu=1)
    now = [1000.0]
    be = SysfsBackend(kfd, drm, ras_recover_s=300, clock=lambda: now[0])
    devs = be.devices()
    assert be.poll_health(devs) == []
    ras = tmp_path / "drm" / "renderD129" / "device" / "ras" / "umc_err_count"
    ras.write_text("ue: 3\nce: 0\n")
    ev = be.poll_health(devs)
    assert len(ev) == 1 and not ev[0].healthy
    devs[0].healthy = False
    now[0] += 5
    assert be.poll_health(devs) == []          # flat, but inside the hold-off
    now[0] += 200
    ras.write_text("ue: 4\nce: 0\n")          # another UE restarts the hold-off
    assert be.poll_health(devs) == []
    now[0] += 299
    assert be.poll_health(devs) == []
    now[0] += 2
    ev = be.poll_health(devs)
    assert len(ev) == 1 and ev[0].healthy      # 301 s flat -> recovered
    devs[0].healthy = True
    ras.write_text("ue: 5\nce: 0\n")
    ev = be.poll_health(devs)
    assert len(ev) == 1 and not ev[0].healthy
    devs[0].healthy = False
    be.reset_observed(devs[0].uuid)            # a GPU reset clears the hold-off
    now[0] += 5
    ev = be.poll_health(devs)
    assert len(ev) == 1 and ev[0].healthy


def test_vanished_node_recovers_when_back(tmp_path):
    kfd, drm = make_tree(tmp_path, ngpu=1)
    be = SysfsBackend(kfd, drm)
    devs = be.devices()
    gid = os.path.join(kfd, str(devs[0].node_id), "gpu_id")
    saved = open(gid).read()
    os.unlink(gid)
    ev = be.poll_health(devs)
    assert len(ev) == 1 and not ev[0].healthy
    devs[0].healthy = False
    with open(gid, "w") as f:
        f.write(saved)
    assert be.poll_health(devs) == []          # back: UE count read again (first poll)
    ev = be.poll_health(devs)
    assert len(ev) == 1 and ev[0].healthy


def test_bdf_decode():
    assert bdf_from_location(0, 23040) == "0000:5a:00.0"
