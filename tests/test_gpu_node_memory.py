"""Virtual device memory across containers on a real MI355X (VERDICT r5 Missing 2, item 2).

Container A is an oversubscribed vGPU whose buffer past its HBM share spilled to an SVM range
and was promoted into HBM when the share freed up. ROCr's free-memory figure does not show
SVM pages in VRAM (profiles/r4b), so container B - another tenant of the GPU - would read
them as free. With the node board (both containers' VGPU_BOARD_DIR):

* B's torch.cuda.mem_get_info free is ROCr's figure less A's promoted bytes;
* B allocating more than that, within its quota, succeeds - A's migrator demotes its promoted
  spill back to host memory when B is refused (or the driver evicts the SVM pages itself) -
  and A's data is intact afterwards.
"""
import json
import os
import time

import pytest

from amdvgpu.shim.launcher import vgpu_env
from conftest import run_child, spawn_child, child_results

pytestmark = pytest.mark.gpu
GiB = 1 << 30
MiB = 1 << 20

A_CODE = """
import torch
from amdvgpu.shim.region import Region
torch.zeros(1, device="cuda")                                           # the shim attaches its region
reg = Region(os.environ["VGPU_SHARED_CACHE"])
x = torch.empty(20 << 30, dtype=torch.uint8, device="cuda")            # most of the 24 GiB share
y = torch.full((8 << 30,), 7, dtype=torch.uint8, device="cuda")         # past it: spilled (SVM)
torch.cuda.synchronize()
spilled0 = reg.device(0)["spilled"]
del x
torch.cuda.empty_cache()                                                 # the share frees up
t0 = time.time()
while reg.device(0)["spilled"] and time.time() - t0 < 30:
    time.sleep(0.1)
promoted = spilled0 - reg.device(0)["spilled"]
hostpid = [p["hostpid"] for p in reg.procs() if p["pid"] == os.getpid()][0]
def kfd_vram():   # KFD's count of this process's VRAM (SVM pages included on MI355X, profiles/r5b)
    import glob
    for f in glob.glob(f"/sys/class/kfd/kfd/proc/{hostpid}/vram_*"):
        return int(open(f).read())
    return -1
emit(phase="promoted", spilled0=spilled0, promoted=promoted, promote_s=round(time.time() - t0, 2), vram=kfd_vram())
open(os.environ["A_READY"], "w").close()
t0 = time.time()
while not os.path.exists(os.environ["A_DONE"]) and time.time() - t0 < 120:
    time.sleep(0.1)
vram_after = kfd_vram()
ok = bool((y == 7).all().item())
emit(phase="after", spilled=reg.device(0)["spilled"], intact=ok, vram=vram_after)
"""

NATIVE_FREE = """
import torch
emit(free=torch.cuda.mem_get_info(0)[0])
"""

B_CODE = """
import torch
time.sleep(1.5)                                  # the sampler has read the board
free, total = torch.cuda.mem_get_info(0)
import ctypes
shim = ctypes.CDLL(None)
shim.vgpu_get_current_device_hidden_vram.restype = ctypes.c_uint64
hidden = shim.vgpu_get_current_device_hidden_vram()
want = free + (7 << 30)                          # needs 7 of A's 8 GiB: more than B sees free, within its quota
t0 = time.time()
try:
    z = torch.empty(want, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    ok = True
except torch.OutOfMemoryError as e:
    ok = False
emit(free=free, total=total, want=want, ok=ok, alloc_s=round(time.time() - t0, 2), hidden=hidden)
"""


def test_promoted_spill_is_seen_and_given_back_across_containers(tmp_path):
    board = tmp_path / "board"
    board.mkdir()
    common = {"VGPU_BOARD_DIR": str(board), "A_READY": str(tmp_path / "a.ready"), "A_DONE": str(tmp_path / "a.done")}
    a = vgpu_env(mem_limit=48 * GiB, shared_cache=str(tmp_path / "a.cache"), oversubscribe=True,
                 extra={**common, "VGPU_BOARD_SLOT": "a.slot", "VGPU_DEVICE_HBM_LIMIT_0": "24576m",
                        "VGPU_SPILL_POLICY": "first-come", "VGPU_SPILL_RESERVE": "1g"})
    pa = spawn_child(A_CODE, a)
    try:
        t0 = time.time()
        while not os.path.exists(common["A_READY"]) and pa.poll() is None and time.time() - t0 < 120:
            time.sleep(0.1)
        assert os.path.exists(common["A_READY"]), pa.stderr.read()[-3000:] if pa.poll() is not None else "A not ready"
        (native,), _ = run_child(NATIVE_FREE, None, preload=False, timeout=120)
        b = vgpu_env(mem_limit=300 * GiB, shared_cache=str(tmp_path / "b.cache"), log_level=2,
                     extra={**common, "VGPU_BOARD_SLOT": "b.slot"})
        (rb,), pb = run_child(B_CODE, b, timeout=120, check=False)
    finally:
        open(common["A_DONE"], "w").close()
        out, err = pa.communicate(timeout=120)
    ra = child_results(out)
    print("A log:", [l for l in err.splitlines() if "vGPU" in l][-6:])
    print("B log:", [l for l in pb.stderr.splitlines() if "vGPU" in l][-6:])
    promoted = [r for r in ra if r.get("phase") == "promoted"][0]
    after = [r for r in ra if r.get("phase") == "after"][0]
    print(json.dumps({"a": ra, "native_free": native["free"], "b": rb}))
    assert promoted["promoted"] >= 8 * GiB, promoted
    # B takes A's promoted 8 GiB off ROCr's free figure (B's and the probe's own runtime
    # footprints differ by up to ~1 GiB between runs)
    assert rb["hidden"] == 8 * GiB, rb
    assert 7 * GiB <= native["free"] - rb["free"] <= 9 * GiB + 512 * MiB, (native, rb)
    assert rb["ok"], rb                            # served: A's spill gave the HBM back
    assert after["intact"], after                  # A's data survived the move
