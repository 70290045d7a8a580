"""Spilled buffers and inter-process sharing on a real MI355X (the round-4 verdict's weak item
3): a buffer an oversubscribed vGPU placed in host memory is shared with a second process the
way PyTorch shares CUDA tensors (torch.multiprocessing: hipIpcGetMemHandle in the producer,
hipIpcOpenMemHandle in the consumer) - what RCCL does with its transport buffers too.

Reference: cuIpcGetMemHandle / cuIpcOpenMemHandle are suspend-gated pass-throughs
([memory.c:374-388]); its UVM spill (cuMemAllocManaged) can be exported. Here a spill is
either pinned host memory (a ROCr allocation: exportable) or an SVM range (not a ROCr
allocation); the spill policy keeps allocations below VGPU_SPILL_LARGE pinned
(docs/DESIGN.md §4), so small, share-able buffers stay exportable.
"""
import pytest

from amdvgpu.shim.launcher import vgpu_env
from conftest import REPO, run_child

pytestmark = pytest.mark.gpu
GiB = 1 << 30
MiB = 1 << 20

SHARE = """
import torch, torch.multiprocessing as mp
from amdvgpu.shim.region import Region
sys.path.insert(0, os.path.join({repo!r}, "tests"))
from ipc_helpers import sum_consumer as consumer

if True:
    ctx = mp.get_context("spawn")
    a = torch.ones({resident} << 20, dtype=torch.uint8, device="cuda")      # fills the HBM share
    b = torch.full(({spill} << 20,), 2, dtype=torch.uint8, device="cuda")   # past it: spilled
    torch.cuda.synchronize()
    r = Region(os.environ["VGPU_SHARED_CACHE"]).device(0)
    q, out = ctx.Queue(), ctx.Queue()
    p = ctx.Process(target=consumer, args=(q, out))
    p.start()
    try:
        q.put(b)
        got = out.get(timeout=75)
        err = got if isinstance(got, str) else ""
        got = None if err else got
    except Exception as e:
        got, err = None, repr(e)[:300]
    p.join(timeout=10)
    if p.is_alive():
        p.terminate()
    emit(spilled=r["spilled"], got=got, want=float(2 * ({spill} << 20)), err=err, exitcode=p.exitcode)
"""


@pytest.mark.parametrize("backing", ["auto", "pinned"])
def test_small_spilled_buffer_shared_with_another_process(tmp_region, backing):
    """A 64 MiB buffer past a 1 GiB HBM share (below VGPU_SPILL_LARGE, so a pinned spill
    under the default policy) is shared through CUDA IPC with a second process, which reads
    the producer's data."""
    _share(tmp_region, backing, expect_ok=True)


def test_svm_spilled_buffer_cannot_be_exported(tmp_region):
    """What the policy avoids: the same buffer as an SVM range (VGPU_SPILL_BACKING=svm) is no
    ROCr allocation, so the producer's export fails - cleanly, as an error in the producer,
    not a hang or a fault."""
    _share(tmp_region, "svm", expect_ok=False)


RCCL_ONE_RANK = """
import torch, torch.distributed as dist
from amdvgpu.shim.region import Region
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str({port}))
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
a = torch.ones({resident} << 20, dtype=torch.uint8, device="cuda")      # fills the HBM share
x = torch.full(({spill} << 18,), 3.0, device="cuda")                     # past it: spilled
torch.cuda.synchronize()
r = Region(os.environ["VGPU_SHARED_CACHE"]).device(0)
spilled_before = r["spilled"]
dist.all_reduce(x)          # RCCL's own buffers are allocated past the share too
y = torch.full((1 << 20,), 1.0, device="cuda")
dist.all_reduce(y)
torch.cuda.synchronize()
ok = bool((x == 3.0).all().item()) and bool((y == 1.0).all().item())
dist.destroy_process_group()
emit(ok=ok, spilled=spilled_before, spilled_after=Region(os.environ["VGPU_SHARED_CACHE"]).device(0)["spilled"])
"""


def test_rccl_all_reduce_in_a_full_oversubscribed_pod(tmp_region):
    """A one-rank RCCL all-reduce in an oversubscribed pod whose HBM share is already full:
    the tensor and RCCL's own buffers are placed past the share (spilled, default policy),
    and the collective completes with the right data."""
    import random
    c = vgpu_env(mem_limit=8 * GiB, shared_cache=tmp_region, oversubscribe=True,
                 extra={"VGPU_DEVICE_HBM_LIMIT_0": "1024m", "VGPU_SPILL_POLICY": "first-come"})
    res, p = run_child(RCCL_ONE_RANK.format(resident=1024, spill=64, port=random.randint(20000, 40000)), c,
                       timeout=130, check=False)
    assert res, p.stderr[-3000:]
    r = res[0]
    assert r["ok"], r
    assert r["spilled"] >= 64 * MiB, r


def _share(tmp_region, backing, expect_ok):
    c = vgpu_env(mem_limit=8 * GiB, shared_cache=tmp_region, oversubscribe=True,
                 extra={"VGPU_DEVICE_HBM_LIMIT_0": "1024m", "VGPU_SPILL_POLICY": "first-come",
                        "VGPU_SPILL_BACKING": backing})
    res, p = run_child(SHARE.format(resident=1024, spill=64, repo=REPO), c, timeout=130, check=False)
    assert res, p.stderr[-3000:]
    r = res[0]
    assert r["spilled"] >= 64 * MiB, r
    if expect_ok:
        assert r["got"] == r["want"], r
    else:
        assert r["got"] is None and r["err"], r
