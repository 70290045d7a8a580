"""--duplicate-vgpus=split (VGPU_DUPLICATE_SPLIT): two vGPUs of one physical GPU are two HIP
devices of the container, each with its own quota (VERDICT r5 Missing 3). On the CPU-only
fake runtime: one GPU agent, VGPU_DEVICE_MAP naming it twice (1 GiB and 2 GiB vGPUs).

Reference: duplicate vGPUs stay separate virtual devices with virtual PCI bus ids
(assigning_virtual_pcibusID [device.c:81-117], NVIDIA_DEVICE_MAP server.go:490,493).
"""
import pytest

from test_shim_fake import fake, run  # noqa: F401  (fixture)

GiB = 1 << 30
MiB = 1 << 20
UUID = "GPU-fa4e000000000000"


def _env(fake, split):  # noqa: F811
    return fake(gpus=1, VGPU_DEVICE_MAP=f"0:{UUID} 1:{UUID}", VGPU_DEVICE_MEMORY_LIMIT_0="1g",
                VGPU_DEVICE_MEMORY_LIMIT_1="2g", VGPU_DUPLICATE_SPLIT="1" if split else "0")


def _one(out, key):
    return [o for o in out if key in o]


def test_two_vgpus_of_one_gpu_are_two_devices(fake):  # noqa: F811
    out = run(_env(fake, True), "count", "props=0", "props=1", "dev=1", "meminfo", "malloc=1500m", "meminfo",
              "dev=0", "count", "malloc=1500m", "malloc=900m", "meminfo", "canpeer=0,1", "dev=2")
    counts = _one(out, "count")
    assert counts[0]["count"] == 2 and counts[0]["current"] == 0, counts
    props = _one(out, "props")
    assert [p["total"] for p in props] == [GiB, 2 * GiB] and [p["totalmem"] for p in props] == [GiB, 2 * GiB], props
    # an int attribute: a 2 GiB quota does not fit and saturates, as the MI355X runtime's own
    # answer for the whole GPU does (profiles/r6y)
    assert [p["attrmem"] for p in props] == [GiB, 2**31 - 1] and [p["rc3"] for p in props] == [0, 0], props
    info = _one(out, "free")
    assert info[0]["total"] == 2 * GiB and info[0]["free"] == 2 * GiB, info        # device 1: its own quota
    assert info[1]["free"] == 2 * GiB - 1500 * MiB, info
    assert [o["malloc"] for o in _one(out, "malloc")] == ["ok", "oom", "ok"], out  # device 0 holds 1 GiB only
    assert info[2]["total"] == GiB and info[2]["free"] == GiB - 900 * MiB, info
    assert counts[1]["current"] == 0
    peer = _one(out, "canpeer")[0]
    assert peer["canpeer"] == 1 and peer["rc"] == 0 and peer["enable"] == 0, peer   # one GPU's memory
    assert _one(out, "dev")[-1]["rc"] != 0   # no device 2


def test_split_holds_when_the_first_hip_call_takes_an_ordinal(fake):  # noqa: F811
    """A program whose first HIP call is hipSetDevice(1) (no hipGetDeviceCount before it): the
    split is decided after the shim has initialised, so device 1 exists and holds its quota."""
    e = dict(_env(fake, True), HARNESS_LAZY_INIT="1")   # no hipInit / agent scan up front
    out = run(e, "dev=1", "meminfo", "malloc=1500m", "count")
    assert _one(out, "dev")[0]["rc"] == 0, out
    assert _one(out, "free")[0]["total"] == 2 * GiB, out
    assert [o["malloc"] for o in _one(out, "malloc")] == ["ok"], out
    assert _one(out, "count")[0]["count"] == 2 and _one(out, "count")[0]["current"] == 1, out


def test_merge_keeps_one_device_with_the_summed_quota(fake):  # noqa: F811
    out = run(_env(fake, False), "count", "props=0", "meminfo", "dev=1")
    assert _one(out, "count")[0]["count"] == 1
    assert _one(out, "free")[0]["total"] == 3 * GiB
    assert _one(out, "dev")[-1]["rc"] != 0


def test_split_quota_is_shared_by_the_containers_processes(fake):  # noqa: F811
    """Two processes of the container on virtual device 1: its 2 GiB quota holds across them
    (a region slot), while the physical GPU keeps the summed 3 GiB as the guard."""
    import json
    import subprocess
    from test_shim_fake import HARNESS
    e = _env(fake, True)
    p = subprocess.Popen([HARNESS, "dev=1", "malloc=1500m", "mark=held", "sleep=2.0"], env=e, stdout=subprocess.PIPE,
                         text=True)
    for line in p.stdout:
        if '"mark"' in line:
            break
    out = run(e, "dev=1", "malloc=1g", "malloc=400m", "dev=0", "malloc=900m")
    p.stdout.read()
    assert p.wait(30) == 0
    assert [o["malloc"] for o in _one(out, "malloc")] == ["oom", "ok", "ok"], out


@pytest.mark.parametrize("split", [True, False])
def test_region_created_by_an_smi_process_first(fake, split):  # noqa: F811
    """torch counts devices through amdsmi before it initialises HIP, so a process that never
    initialises ROCr may create the container's region first, with the environment's raw
    per-vGPU limits. The first GPU process then writes the resolved ones: the merged GPU holds
    both vGPUs' quota (3 GiB), and with split each vGPU its own."""
    import subprocess
    import sys
    from test_rsmi_remap import CHILD, FAKE_RSMI
    e = _env(fake, split)
    p = subprocess.run([sys.executable, "-c", CHILD, FAKE_RSMI], env=e, capture_output=True, text=True, timeout=60)
    assert p.returncode == 0, p.stderr[-2000:]
    if split:
        out = run(e, "props=0", "props=1", "dev=1", "malloc=1500m", "dev=0", "malloc=1500m")
        assert [p["total"] for p in _one(out, "props")] == [GiB, 2 * GiB], out
        assert [o["malloc"] for o in _one(out, "malloc")] == ["ok", "oom"], out
    else:
        out = run(e, "meminfo", "malloc=2500m")
        assert _one(out, "free")[0]["total"] == 3 * GiB and _one(out, "malloc")[0]["malloc"] == "ok", out


def test_smi_lists_every_vgpu_with_split(tmp_path):
    """In-container rocm-smi / amd-smi list one device per vGPU with split (the plugin names
    the GPU once per vGPU in VGPU_DEVICE_BDFS), once per GPU with merge."""
    from test_rsmi_remap import run as rsmi_run
    two = rsmi_run(tmp_path, VGPU_DEVICE_BDFS="0000:05:00.0,0000:05:00.0", VGPU_DUPLICATE_SPLIT="1")
    assert two["n"] == 2 and [i for _st, i in two["ids"][:2]] == [0x1000, 0x1000], two
    one = rsmi_run(tmp_path, VGPU_DEVICE_BDFS="0000:05:00.0,0000:05:00.0")
    assert one["n"] == 1, one
