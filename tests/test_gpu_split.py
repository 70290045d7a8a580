"""--duplicate-vgpus=split on a real MI355X: a container holding two vGPUs of one GPU sees two
devices (VERDICT r5 Missing 3; reference: duplicate vGPUs as separate virtual devices,
[device.c:81-155]). Stock PyTorch: device_count, set_device(1), per-device memory info and
quota, kernels and a cross-device copy."""
import pytest

from amdvgpu.shim.launcher import vgpu_env
from conftest import run_child

pytestmark = pytest.mark.gpu
GiB = 1 << 30

SPLIT = """
import torch
uuid = os.environ["SPLIT_UUID"]
n = torch.cuda.device_count()
info = [torch.cuda.mem_get_info(d) for d in range(n)]
props = [torch.cuda.get_device_properties(d).total_memory for d in range(n)]
torch.cuda.set_device(1)
cur = torch.cuda.current_device()
a = torch.randn(1024, 1024, device="cuda:1")
b = (a @ a).sum().item()
ref = (a.cpu() @ a.cpu()).sum().item()
c = a.to("cuda:0")
same = bool(torch.equal(c.cpu(), a.cpu()))
big1 = torch.empty(5 << 30, dtype=torch.uint8, device="cuda:1")       # within device 1's 6 GiB
try:
    torch.empty(5 << 30, dtype=torch.uint8, device="cuda:0")          # device 0 holds 4 GiB
    oom0 = False
except torch.OutOfMemoryError:
    oom0 = True
x0 = torch.empty(3 << 30, dtype=torch.uint8, device="cuda:0")         # fits device 0
torch.cuda.synchronize()
import ctypes
hip = ctypes.CDLL("libamdhip64.so")
attr = []
for d in range(n):
    v = ctypes.c_int(-1)
    rc = hip.hipDeviceGetAttribute(ctypes.byref(v), 84, d)   # hipDeviceAttributeTotalGlobalMem
    attr.append([rc, v.value])
emit(n=n, totals=[t for _f, t in info], props=props, cur=cur, close=abs(b - ref) <= 1e-3 * max(1.0, abs(ref)),
     same=same, oom0=oom0, dev_of=[str(big1.device), str(x0.device)], attr=attr)
"""


def _gpu():
    from amdvgpu.plugin.devices import SysfsBackend
    devs = SysfsBackend().devices()
    assert devs, "no GPU in sysfs"
    return devs[0]


def test_two_vgpus_of_one_gpu_are_two_torch_devices(tmp_region):
    g = _gpu()
    # As the plugin's contract for --duplicate-vgpus=split (contract.py): the GPU named once per
    # vGPU in the visible list and the BDF list. (HIP_VISIBLE_DEVICES, which the GPU box sets,
    # is widened to match: torch prefers it over ROCR_VISIBLE_DEVICES.)
    c = vgpu_env(shared_cache=tmp_region, device_map=[g.uuid, g.uuid], per_device_mem=[4 * GiB, 6 * GiB],
                 extra={"VGPU_DUPLICATE_SPLIT": "1", "SPLIT_UUID": g.uuid, "ROCR_VISIBLE_DEVICES": f"{g.uuid},{g.uuid}",
                        "HIP_VISIBLE_DEVICES": "0,1", "VGPU_DEVICE_BDFS": f"{g.bdf},{g.bdf}"})
    res, p = run_child(SPLIT, c, timeout=300, check=False)
    assert res, p.stderr[-3000:]
    r = res[0]
    assert r["n"] == 2, r
    assert r["totals"] == [4 * GiB, 6 * GiB] and r["props"] == [4 * GiB, 6 * GiB], r
    assert r["cur"] == 1 and r["close"] and r["same"], r
    assert r["oom0"], r                      # device 0's own quota holds
    assert r["dev_of"] == ["cuda:1", "cuda:0"], r
    # the int attribute: each device's own quota, saturated (4 and 6 GiB exceed an int)
    assert r["attr"] == [[0, 2**31 - 1], [0, 2**31 - 1]], r


# hipDeviceAttributeTotalGlobalMem (84) of every device the process sees, as its first HIP call
ATTR = """
import ctypes
hip = ctypes.CDLL("libamdhip64.so")
out = []
for d in range(int(os.environ.get("ATTR_DEVICES", "1"))):
    v = ctypes.c_int(-1)
    rc = hip.hipDeviceGetAttribute(ctypes.byref(v), 84, d)
    out.append([rc, v.value])
emit(attr=out)
"""


def test_total_global_mem_attribute_of_split_vgpus(tmp_region):
    """The int TotalGlobalMem attribute per virtual device: a vGPU's own quota when it fits an
    int (1 GiB), saturated otherwise (the runtime's own answer for the whole GPU is printed)."""
    g = _gpu()
    native, _ = run_child(ATTR, None)
    c = vgpu_env(shared_cache=tmp_region, device_map=[g.uuid, g.uuid], per_device_mem=[1 << 30, 6 * GiB],
                 extra={"VGPU_DUPLICATE_SPLIT": "1", "ROCR_VISIBLE_DEVICES": f"{g.uuid},{g.uuid}",
                        "HIP_VISIBLE_DEVICES": "0,1", "VGPU_DEVICE_BDFS": f"{g.bdf},{g.bdf}", "ATTR_DEVICES": "2"})
    res, p = run_child(ATTR, c, timeout=300, check=False)
    assert res, p.stderr[-3000:]
    print("TotalGlobalMem attribute, native:", native[0]["attr"], "split:", res[0]["attr"])
    assert native[0]["attr"][0][0] == 0, native
    assert res[0]["attr"] == [[0, 1 << 30], [0, 2**31 - 1]], res
