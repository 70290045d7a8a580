"""End-to-end on a real MI355X: plugin (sysfs backend) -> stub kubelet -> Allocate ->
'container' running stock PyTorch-ROCm under the returned contract,
plus oversubscription spill, SMI virtualisation and RCCL through the shim."""
import os
import threading
import time

import pytest

from amdvgpu.plugin.config import PluginConfig
from amdvgpu.plugin.devices import SysfsBackend
from amdvgpu.plugin.kubelet_stub import StubKubelet, run_pod
from amdvgpu.plugin.main import Supervisor
from amdvgpu.shim.launcher import vgpu_env
from conftest import CHILD_PRELUDE, run_child, spawn_child

pytestmark = pytest.mark.gpu

GiB = 1 << 30
MiB = 1 << 20


def test_sysfs_backend_sees_the_mi355x():
    devs = SysfsBackend().devices()
    assert len(devs) >= 1
    d = devs[0]
    assert d.cu_count == 256 and d.num_xcc == 8
    assert d.memory_total >= 280 * GiB
    assert d.render_minor >= 128
    assert d.uuid.startswith("GPU-")


def test_sysfs_uuid_matches_rocr(tmp_region):
    """The plugin's UUIDs (VGPU_DEVICE_MAP / ROCR_VISIBLE_DEVICES) are ROCr's UUIDs."""
    devs = SysfsBackend().devices()
    c = vgpu_env(mem_limit=8 * GiB, shared_cache=tmp_region, device_map=[devs[0].uuid])
    res, _ = run_child("""
import torch
from amdvgpu.shim.region import Region
torch.cuda.mem_get_info(0)
emit(uuid=Region(os.environ["VGPU_SHARED_CACHE"]).device(0)["uuid"])
""", c, extra_env={"ROCR_VISIBLE_DEVICES": devs[0].uuid})
    assert res[0]["uuid"].lower() == devs[0].uuid.lower()


@pytest.fixture
def plugin(tmp_path):
    pdir = str(tmp_path / "dp")
    os.makedirs(pdir)
    cfg = PluginConfig(device_plugin_path=pdir + "/", backend="sysfs", device_split_count=4,
                       shared_cache_dir=str(tmp_path), vgpu_dir=str(tmp_path / "vgpu")).validate()
    k = StubKubelet(pdir).start()
    sup = Supervisor(cfg, backend=SysfsBackend(), install_signals=False)
    stop = threading.Event()
    th = threading.Thread(target=sup.run, args=(stop,), daemon=True)
    th.start()
    k.wait_registered("amd.com/gpu", timeout=20)
    yield k
    stop.set()
    th.join(10)
    k.stop()


def test_slice_resnet50_in_allocated_vgpu(plugin):
    """4-way split: quota = HBM/4 (72 GiB), 25 % compute share; alone on the GPU the auto
    mode enforces it with the slot's CU mask (64 CUs), stock fp32 model runs."""
    code = CHILD_PRELUDE + """
import torch
from amdvgpu.models.aibench import Runner, get_case
from amdvgpu.ops import cu_census
free, total = torch.cuda.mem_get_info(0)
r = Runner(get_case("resnet50-inf"), "cuda:0", dtype=torch.float32)
for _ in range(3): r.step()
torch.cuda.synchronize()
t0 = time.time()
for _ in range(10): r.step()
torch.cuda.synchronize()
dt = (time.time() - t0) / 10
ncu = len(cu_census(nblocks=8192, spin_us=300))
from amdvgpu.shim.region import Region
emit(total=total, ms=dt * 1000, ips=50 / dt, ncu=ncu, mode=Region(os.environ["VGPU_SHARED_CACHE"]).device(0)["cu_mode"])
"""
    import sys
    ids, envs, proc = run_pod(plugin, "amd.com/gpu", 1, [sys.executable, "-c", code], capture_output=True,
                              text=True, timeout=600)
    assert proc.returncode == 0, proc.stderr[-3000:]
    import json
    r = [json.loads(l[7:]) for l in proc.stdout.splitlines() if l.startswith("RESULT ")][0]
    quota = int(envs["VGPU_DEVICE_MEMORY_LIMIT_0"].rstrip("m")) * MiB
    assert r["total"] == quota and 70 * GiB <= quota <= 73 * GiB
    assert envs["VGPU_CU_MODE"] == "auto" and envs["VGPU_DEVICE_CU_LIMIT_0"] == "25"
    assert r["ncu"] == 64 and r["mode"] == "spatial", r
    assert envs["VGPU_DEVICE_CU_RANGE_0"] in ("0-64", "64-128", "128-192", "192-256")
    print(f"slice: ResNet-V2-50 b=50 fp32 inference in a 1/4 vGPU (64 CUs): {r['ips']:.1f} img/s")


def test_readme_two_vgpu_pod_sees_two_devices(plugin):
    """The reference README's pod (two vGPUs, README.md:193-206) on a one-GPU node, through the
    plugin's default Allocate (--duplicate-vgpus=split): stock PyTorch sees two devices, each
    with its own 1/4 quota, runs on cuda:1 and copies between them (reference: duplicates as
    separate virtual devices, [device.c:81-155])."""
    code = CHILD_PRELUDE + """
import torch
n = torch.cuda.device_count()
totals = [torch.cuda.mem_get_info(d)[1] for d in range(n)]
torch.cuda.set_device(1)
a = torch.randn(512, 512, device="cuda:1")
s = (a @ a).sum().item()
ref = (a.cpu() @ a.cpu()).sum().item()
same = bool(torch.equal(a.to("cuda:0").cpu(), a.cpu()))
torch.cuda.synchronize()
emit(n=n, totals=totals, cur=torch.cuda.current_device(), close=abs(s - ref) <= 1e-3 * max(1.0, abs(ref)), same=same)
"""
    import json
    import sys
    # a container does not inherit the host job's device selection (the GPU box sets one)
    base = {k: v for k, v in os.environ.items()
            if k not in ("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "GPU_DEVICE_ORDINAL")}
    ids, envs, proc = run_pod(plugin, "amd.com/gpu", 2, [sys.executable, "-c", code], base_env=base,
                              capture_output=True, text=True, timeout=300)
    assert proc.returncode == 0, proc.stderr[-3000:]
    assert envs["VGPU_DUPLICATE_SPLIT"] == "1", envs
    r = [json.loads(l[7:]) for l in proc.stdout.splitlines() if l.startswith("RESULT ")][0]
    quota = int(envs["VGPU_DEVICE_MEMORY_LIMIT_0"].rstrip("m")) * MiB
    assert r["n"] == 2 and r["totals"] == [quota, quota], r
    assert r["cur"] == 1 and r["close"] and r["same"], r


def test_oversubscription_spills_past_hbm_share(tmp_region):
    c = vgpu_env(mem_limit=8 * GiB, shared_cache=tmp_region, oversubscribe=True,
                 extra={"VGPU_DEVICE_HBM_LIMIT_0": "2048m"})
    res, _ = run_child("""
import torch
from amdvgpu.shim.region import Region
from amdvgpu.ops import stream_copy
free, total = torch.cuda.mem_get_info(0)
a = torch.ones(1536 << 20, dtype=torch.uint8, device="cuda")     # resident
b = torch.full((1024 << 20,), 3, dtype=torch.uint8, device="cuda")  # crosses the share -> host
c = torch.full((1024 << 20,), 5, dtype=torch.uint8, device="cuda")  # host
torch.cuda.synchronize()
ok_ab = bool((a[:1 << 20] == 1).all()) and bool((b == 3).all()) and bool((c == 5).all())
r = Region(os.environ["VGPU_SHARED_CACHE"]).device(0)
# bandwidth of a kernel reading spilled memory
dst = torch.empty_like(c)
stream_copy(dst, c); torch.cuda.synchronize()
t0 = time.time()
for _ in range(5): stream_copy(dst, c)
torch.cuda.synchronize()
bw = 5 * c.numel() / (time.time() - t0) / 1e9
try:
    d = torch.empty(6 << 30, dtype=torch.uint8, device="cuda")
    over = False
except torch.OutOfMemoryError:
    over = True
emit(total=total, ok_ab=ok_ab, spilled=r["spilled"], used=r["used"], hbm=r["hbm_limit"], bw=bw, over=over,
     ok=bool((dst == 5).all()))
""", c)
    r = res[0]
    assert r["total"] == 8 * GiB
    assert r["ok_ab"]
    assert r["spilled"] >= 2 * GiB - 64 * MiB
    assert r["hbm"] == 2 * GiB
    assert r["ok"] and r["over"]
    print(f"spill read bandwidth {r['bw']:.1f} GB/s")


CONFIGURE = """
import torch
torch.cuda.mem_get_info(0)    # a GPU process of the container records the device (BDF) in the region
x = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
emit(ok=True)
time.sleep(30)
"""


AMDSMI_QUERY = """
try:
    import amdsmi
    amdsmi.amdsmi_init()
    h = amdsmi.amdsmi_get_processor_handles()[0]
    total = amdsmi.amdsmi_get_gpu_memory_total(h, amdsmi.AmdSmiMemoryType.VRAM)
    used = amdsmi.amdsmi_get_gpu_memory_usage(h, amdsmi.AmdSmiMemoryType.VRAM)
    emit(ok=True, total=total, used=used)
except Exception as e:
    emit(ok=False, err=repr(e)[:300])
"""


def test_amdsmi_reports_quota(tmp_region):
    """In-container amd-smi (Python amdsmi over ctypes) sees the vGPU quota while a GPU
    process of the same container is running."""
    c = vgpu_env(mem_limit=24 * GiB, shared_cache=tmp_region)
    holder = spawn_child(CONFIGURE, c)
    try:
        assert holder.stdout.readline().startswith("RESULT")
        res, _ = run_child(AMDSMI_QUERY, c)
        native = None
        if not res[0]["ok"]:  # is amdsmi usable at all here while a GPU process runs?
            native, _ = run_child(AMDSMI_QUERY, None)
    finally:
        holder.kill()
        holder.wait()
    r = res[0]
    if not r["ok"]:
        if native and native[0]["ok"]:
            pytest.fail(f"amdsmi works natively ({native[0]}) but not under the shim: {r['err']}")
        pytest.skip(f"amdsmi unavailable on this box: {r['err']} (native: {native and native[0]})")
    assert r["total"] == 24 * GiB
    assert GiB <= r["used"] <= 24 * GiB


def test_rccl_allreduce_through_shim(tmp_region):
    """RCCL inside a vGPU: the communicator's set-up allocations go through the quota and its
    kernels through the launch gates. One rank only - the test box has one GPU and RCCL
    refuses two ranks on one device. The inter-GPU path (an all-reduce between pods on
    different GPUs, against native) is bench.py's ``rccl_allreduce_between_pods`` on the
    driver's multi-GPU runs, rehearsed with gloo in tests/test_bench_contract.py."""
    c = vgpu_env(mem_limit=16 * GiB, shared_cache=tmp_region)
    res, _ = run_child("""
import torch, torch.distributed as dist
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29611")
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
x = torch.ones(1 << 24, device="cuda")
dist.all_reduce(x)
torch.cuda.synchronize()
emit(v=float(x[0]))
dist.destroy_process_group()
""", c)
    assert res[0]["v"] == 1.0


def test_temporal_mode_graph_launch(tmp_region):
    c = vgpu_env(cu_limit=50, cu_mode="temporal", shared_cache=tmp_region)
    res, _ = run_child("""
import torch
x = torch.zeros(1 << 20, device="cuda")
s = torch.cuda.Stream()
with torch.cuda.stream(s):
    x.add_(1)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    for _ in range(4): x.add_(1)
for _ in range(50): g.replay()
torch.cuda.synchronize()
emit(v=float(x[0]))
""", c)
    assert res[0]["v"] == 201.0


def test_rocm_smi_lib_reports_quota(tmp_region):
    """rocm_smi (ctypes over librocm_smi64, as the rocm-smi CLI does) sees the quota."""
    c = vgpu_env(mem_limit=24 * GiB, shared_cache=tmp_region)
    holder = spawn_child(CONFIGURE, c)
    try:
        assert holder.stdout.readline().startswith("RESULT")
        res, _ = run_child("""
import ctypes
lib = ctypes.CDLL("/opt/rocm/lib/librocm_smi64.so")
rc = lib.rsmi_init(ctypes.c_uint64(0))
if rc != 0:
    emit(ok=False, err=f"rsmi_init {rc}")
else:
    total, used = ctypes.c_uint64(), ctypes.c_uint64()
    rc = lib.rsmi_dev_memory_total_get(ctypes.c_uint32(0), ctypes.c_int(0), ctypes.byref(total))
    lib.rsmi_dev_memory_usage_get(ctypes.c_uint32(0), ctypes.c_int(0), ctypes.byref(used))
    emit(ok=rc == 0, total=total.value, used=used.value, err=f"rc {rc}")
""", c)
    finally:
        holder.kill()
        holder.wait()
    r = res[0]
    if not r["ok"]:
        pytest.skip(f"rocm_smi unavailable on this box: {r['err']}")
    assert r["total"] == 24 * GiB
    assert GiB <= r["used"] <= 24 * GiB


def test_amdsmi_native_diagnostic():
    """Diagnostic: does amdsmi initialise on this box without the shim?"""
    res, p = run_child("""
try:
    import amdsmi
    amdsmi.amdsmi_init()
    emit(ok=True, n=len(amdsmi.amdsmi_get_processor_handles()))
except Exception as e:
    emit(ok=False, err=repr(e)[:300])
""", None)
    print("amdsmi native:", res[0])


HOLD = """
import torch
x = torch.ones(256 << 20, dtype=torch.uint8, device="cuda"); torch.cuda.synchronize()
emit(ok=True)
time.sleep(40)
"""

AMDSMI_VIEW = """
try:
    import amdsmi
    amdsmi.amdsmi_init()
    hs = amdsmi.amdsmi_get_processor_handles()
    procs = [p["pid"] for h in hs for p in amdsmi.amdsmi_get_gpu_process_list(h)]
except Exception as e:
    emit(ok=False, err=repr(e)[:300])
    raise SystemExit(0)
rprocs = None
rn = None
try:
    import ctypes
    class P(ctypes.Structure):
        _fields_ = [("process_id", ctypes.c_uint32), ("pasid", ctypes.c_uint32), ("vram_usage", ctypes.c_uint64),
                    ("sdma_usage", ctypes.c_uint64), ("cu_occupancy", ctypes.c_uint32)]
    lib = ctypes.CDLL("/opt/rocm/lib/librocm_smi64.so")
    if lib.rsmi_init(ctypes.c_uint64(0)) == 0:
        n = ctypes.c_uint32(0)
        lib.rsmi_compute_process_info_get(None, ctypes.byref(n))
        arr = (P * max(n.value, 1))()
        m = ctypes.c_uint32(n.value)
        lib.rsmi_compute_process_info_get(arr, ctypes.byref(m))
        rprocs = [arr[k].process_id for k in range(m.value)]
        c = ctypes.c_uint32()
        if lib.rsmi_num_monitor_devices(ctypes.byref(c)) == 0:
            rn = c.value
except Exception as e:
    rprocs = repr(e)[:200]
emit(ok=True, n=len(hs), procs=procs, rprocs=rprocs, rn=rn)
"""


def test_amdsmi_shows_only_the_containers_gpus_and_processes(tmp_region):
    """In-container amd-smi (amdsmi over ctypes): the process list holds the container's
    processes only (a GPU process of another tenant on the same GPU is hidden) and the
    device list is the container's (reference: NVML count/handle remapping, nvml/hook.c
    :438-527). On the 1-GPU box the device filter is shown by a non-matching BDF list."""
    from amdvgpu.plugin.devices import SysfsBackend
    from amdvgpu.shim.region import Region
    dev = SysfsBackend().devices()[0]
    c = vgpu_env(mem_limit=24 * GiB, shared_cache=tmp_region, extra={"VGPU_DEVICE_BDFS": dev.bdf})
    foreign = spawn_child(HOLD, None)
    holder = spawn_child(HOLD, c)
    try:
        assert foreign.stdout.readline().startswith("RESULT")
        assert holder.stdout.readline().startswith("RESULT")
        time.sleep(1.0)
        with Region(tmp_region) as r:
            mine = {p["hostpid"] for p in r.procs()}
        native, _ = run_child(AMDSMI_VIEW, None)
        inside, _ = run_child(AMDSMI_VIEW, c)
        c_other = dict(c, VGPU_DEVICE_BDFS="0000:ff:1f.7")
        hidden, _ = run_child(AMDSMI_VIEW, c_other)
    finally:
        for p in (foreign, holder):
            p.kill()
            p.wait()
    if not native[0]["ok"]:
        pytest.skip(f"amdsmi unavailable on this box: {native[0]['err']}")
    n, i, h = native[0], inside[0], hidden[0]
    assert i["ok"] and h["ok"], (i, h)
    print("amdsmi native:", n, "inside:", i, "container hostpids:", mine)
    assert all(m > 0 for m in mine)
    assert len(n["procs"]) >= 2                     # both GPU processes are on the GPU
    assert set(i["procs"]) <= mine and mine & set(i["procs"]), (i, mine)
    assert i["n"] == n["n"] == 1 and h["n"] == 0
    if isinstance(n.get("rprocs"), list) and len(n["rprocs"]) >= 2:   # rocm_smi: same filtering
        assert set(i["rprocs"]) <= mine and mine & set(i["rprocs"]), (i, mine)
    if n.get("rn") is not None:                                        # rocm_smi device count
        assert n["rn"] == i["rn"] == 1 and h["rn"] == 0, (n, i, h)
