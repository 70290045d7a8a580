"""Data-plane tests on a real MI355X: stock PyTorch-ROCm processes run as vGPU 'containers'
under the interception shim (SURVEY.md §4 tier 3).

Each test starts child processes with the Allocate-contract env + preload (the shim has to
be in the process from the start, like /etc/ld.so.preload in a pod) and asserts on what
the children observe.
"""
import os
import time

import pytest

from amdvgpu.shim.launcher import vgpu_env
from conftest import child_results, run_child, spawn_child

pytestmark = pytest.mark.gpu

GiB = 1 << 30
MiB = 1 << 20


def test_mem_get_info_reports_quota(tmp_region):
    c = vgpu_env(mem_limit=72 * GiB, shared_cache=tmp_region)
    res, _ = run_child("""
import torch
free, total = torch.cuda.mem_get_info(0)
p = torch.cuda.get_device_properties(0)
x = torch.empty(4 << 30, dtype=torch.uint8, device="cuda")
free2, total2 = torch.cuda.mem_get_info(0)
emit(free=free, total=total, props_total=p.total_memory, free2=free2, total2=total2)
""", c)
    r = res[0]
    assert r["total"] == 72 * GiB
    assert r["props_total"] == 72 * GiB
    assert r["free"] <= 72 * GiB
    assert r["free"] - r["free2"] >= 4 * GiB  # the 4 GiB tensor is charged


def test_oom_at_quota(tmp_region):
    c = vgpu_env(mem_limit=2 * GiB, shared_cache=tmp_region)
    res, _ = run_child("""
import torch
ok = []
try:
    a = torch.empty(1536 << 20, dtype=torch.uint8, device="cuda")
    ok.append(1)
    b = torch.empty(1024 << 20, dtype=torch.uint8, device="cuda")
    ok.append(2)
    emit(oom=False, ok=ok)
except torch.OutOfMemoryError as e:
    emit(oom=True, ok=ok, msg=str(e)[:200])
""", c)
    assert res[0]["oom"] is True
    assert res[0]["ok"] == [1]


def test_native_process_is_unlimited():
    res, _ = run_child("""
import torch
free, total = torch.cuda.mem_get_info(0)
emit(total=total)
""", None)
    assert res[0]["total"] > 250 * GiB


def test_multiprocess_shared_quota(tmp_region):
    """Two processes of one container share one quota (reference: shared region)."""
    c = vgpu_env(mem_limit=6 * GiB, shared_cache=tmp_region)
    holder = spawn_child("""
import torch
x = torch.empty(4 << 30, dtype=torch.uint8, device="cuda")
torch.cuda.synchronize()
emit(held=True)
sys.stdout.flush()
time.sleep(60)
""", c)
    # wait until the holder has allocated
    line = holder.stdout.readline()
    assert line.startswith("RESULT"), line + holder.stderr.read()
    try:
        res, _ = run_child("""
import torch
from amdvgpu.shim.region import Region
free, total = torch.cuda.mem_get_info(0)
try:
    y = torch.empty(3 << 30, dtype=torch.uint8, device="cuda")
    big = False
except torch.OutOfMemoryError:
    big = True
z = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
r = Region(os.environ["VGPU_SHARED_CACHE"])
emit(free=free, total=total, oom_3g=big, procs=len(r.procs()), used=r.device(0)["used"])
""", c)
    finally:
        holder.kill()
        holder.wait()
    r = res[0]
    assert r["total"] == 6 * GiB
    assert r["free"] <= 2 * GiB + 64 * MiB
    assert r["oom_3g"] is True
    assert r["procs"] == 2
    assert r["used"] >= 5 * GiB


def test_dead_process_reclaim(tmp_region):
    """A SIGKILLed process's charges are reclaimed when the quota is hit."""
    c = vgpu_env(mem_limit=4 * GiB, shared_cache=tmp_region)
    p = spawn_child("""
import torch
x = torch.empty(3 << 30, dtype=torch.uint8, device="cuda")
torch.cuda.synchronize()
emit(held=True)
time.sleep(120)
""", c)
    assert p.stdout.readline().startswith("RESULT")
    p.kill()
    p.wait()
    res, _ = run_child("""
import torch
y = torch.empty(3 << 30, dtype=torch.uint8, device="cuda")
emit(ok=True)
""", c)
    assert res[0]["ok"]


@pytest.mark.parametrize("pct,expect", [(25, 64), (50, 128)])
def test_cu_mask_confinement(tmp_region, pct, expect):
    c = vgpu_env(cu_limit=pct, cu_mode="spatial", shared_cache=tmp_region)
    res, _ = run_child("""
import torch
from amdvgpu.ops import cu_census
locs = cu_census(nblocks=8192, spin_us=300)
xcc = sorted({l[0] for l in locs})
per_xcc = {x: sum(1 for l in locs if l[0] == x) for x in xcc}
emit(n=len(locs), xcc=xcc, per_xcc=per_xcc)
""", c)
    r = res[0]
    assert r["n"] == expect, r
    assert len(r["xcc"]) == 8
    assert len(set(r["per_xcc"].values())) == 1  # XCD-balanced


def test_cu_unmasked_uses_whole_chip():
    res, _ = run_child("""
import torch
from amdvgpu.ops import cu_census
emit(n=len(cu_census(nblocks=8192, spin_us=300)))
""", None)
    assert res[0]["n"] == 256


def test_disjoint_cu_ranges(tmp_region):
    """Two co-resident vGPUs with plugin-assigned ranges get disjoint physical CUs."""
    from amdvgpu.shim.region import cu_partition_range
    seen = []
    for slot in range(2):
        b, e = cu_partition_range(256, 8, 2, slot)
        c = vgpu_env(cu_limit=50, cu_range=(b, e), shared_cache=tmp_region + f".{slot}")
        res, _ = run_child("""
from amdvgpu.ops import cu_census
emit(locs=sorted(cu_census(nblocks=8192, spin_us=300)))
""", c)
        seen.append({tuple(x) for x in res[0]["locs"]})
        os.unlink(tmp_region + f".{slot}")
    assert len(seen[0]) == 128 and len(seen[1]) == 128
    assert not (seen[0] & seen[1])


def test_suspend_resume_blocks_launches(tmp_region):
    c = vgpu_env(mem_limit=8 * GiB, shared_cache=tmp_region)
    p = spawn_child("""
import torch
x = torch.ones(1 << 20, device="cuda")
torch.cuda.synchronize()
emit(ready=True)
t0 = time.time()
for i in range(200):
    x.add_(1)
    torch.cuda.synchronize()
    time.sleep(0.01)
emit(elapsed=time.time() - t0, val=float(x[0]))
""", c)
    assert p.stdout.readline().startswith("RESULT")
    from amdvgpu.shim.region import Region
    r = Region(tmp_region)
    r.suspend_all()
    time.sleep(3.0)
    assert r.suspended
    r.resume_all()
    out, err = p.communicate(timeout=120)
    assert p.returncode == 0, err[-3000:]
    res = child_results(out)[0]
    assert res["val"] == 201.0
    assert res["elapsed"] >= 4.0  # ~2 s of work + ~3 s suspended
    procs = r.procs()
    r.close()
    assert not procs  # the exited process released its slot


def test_hip_graph_replay_under_shim(tmp_region):
    c = vgpu_env(mem_limit=16 * GiB, shared_cache=tmp_region)
    res, _ = run_child("""
import torch
x = torch.zeros(1 << 20, device="cuda")
s = torch.cuda.Stream()
with torch.cuda.stream(s):
    for _ in range(3): x.add_(1)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    x.add_(1)
for _ in range(10): g.replay()
torch.cuda.synchronize()
emit(v=float(x[0]))
""", c)
    assert res[0]["v"] == 13.0  # 3 eager + 10 replays (capture itself does not execute)


def test_se_exclusive_layout_for_four_tenants(tmp_region):
    """SE-major logical CU layout: each of 4 co-resident vGPUs owns one whole shader
    engine on every XCD (no shared SE dispatcher between tenants)."""
    from amdvgpu.shim.region import cu_partition_range
    code = """
from amdvgpu.ops import cu_census
emit(locs=sorted(cu_census(nblocks=8192, spin_us=300)))
"""
    for slot in (0, 3):
        b, e = cu_partition_range(256, 8, 4, slot)
        c = vgpu_env(cu_limit=25, cu_range=(b, e), cu_mode="spatial", shared_cache=tmp_region + f".{slot}")
        res, _ = run_child(code, c)
        os.unlink(tmp_region + f".{slot}")
        locs = [tuple(x) for x in res[0]["locs"]]
        assert len(locs) == 64
        assert {l[1] for l in locs} == {slot}, sorted({(l[0], l[1]) for l in locs})
        assert len({l[0] for l in locs}) == 8


@pytest.mark.parametrize("kind", ["managed", "malloc", "pitch", "3d", "ext", "async", "vmm"])
def test_hip_allocations_are_accounted(tmp_region, kind):
    """A plain HIP program (linked normally against libamdhip64) under a 2 GiB quota, for
    every HIP device allocation API (malloc, managed, pitch, 3D, ext flags, stream-ordered
    async pool, VMM handles): 3/4 of the quota's free memory fits, +1/2 is refused,
    after freeing the first block 1/2 fits again (a stream's queue memory is charged to
    the quota as context, so "free" is measured after setup)."""
    import json
    import subprocess
    from amdvgpu.shim.launcher import apply_contract
    from amdvgpu.shim.native import LIB_DIR
    c = vgpu_env(mem_limit=2 * GiB, shared_cache=tmp_region)
    p = subprocess.run([os.path.join(LIB_DIR, "hip_alloc_probe"), kind], env=apply_contract(c),
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr[-2000:]
    r = json.loads(p.stdout.strip().splitlines()[-1])
    assert r["r1"] == 0 and r["r2"] != 0 and r["f1"] == 0 and r["r3"] == 0, r
    assert r["total"] == 2 * GiB


def test_allowlist_authorisation(tmp_region, tmp_path):
    """VGPU_ALLOWLIST: a GPU whose UUID is not listed gets no device memory at all - not
    through the pool API, not through the legacy region API HIP also uses while it brings the
    device up - so HIP drops the device ("No HIP GPUs are available" with one GPU) or, if the
    device came up, the first allocation fails."""
    from amdvgpu.plugin.devices import SysfsBackend
    uuid = SysfsBackend().devices()[0].uuid
    code = """
import torch
try:
    x = torch.empty(1 << 20, device="cuda"); ok = True
except torch.OutOfMemoryError:
    ok = False
except RuntimeError as e:   # the device did not come up: no memory for HIP's own buffers either
    ok = "No HIP GPUs" not in str(e)
emit(ok=ok)
"""
    allow = tmp_path / "allowlist"
    allow.write_text(uuid + "\n")
    c = vgpu_env(mem_limit=8 * GiB, shared_cache=tmp_region, extra={"VGPU_ALLOWLIST": str(allow)})
    assert run_child(code, c)[0][0]["ok"] is True
    allow.write_text("GPU-0000000000000000\n")
    os.unlink(tmp_region)
    assert run_child(code, c)[0][0]["ok"] is False
