"""Compute-limit and accounting behaviour on a real MI355X (round-2 data-plane work).

* temporal (GPU-time credit) limiter accuracy, one tenant and two concurrent tenants;
* auto mode: spatial CU masks for shares >= 50 % and for smaller shares while the GPU is not
  crowded (at most one other busy process), the temporal limiter otherwise;
* live control: ``set_cu_limit`` re-masks a running process's queues; the external launch
  block stalls a tenant in every cu mode; the launch counter counts;
* host-PID discovery for several processes starting together inside a PID namespace;
* continuous context accounting (a scratch-hungry kernel is charged);
* IPC: a tensor shared between two processes of one container is charged once.

Reference behaviour: rate_limiter / utilization_watcher
([multiprocess_utilization_watcher.c:53-216]), set_current_device_sm_limit_scale
([multiprocess_memory_limit.c:787-789]), set_task_pid ([utils.c:188-255]), context and
module charges ([context.c:49-86], [export_table.c:85-113]), cuIpc* ([memory.c:374-388]).
"""
import json
import os
import subprocess
import sys
import time

import pytest

from amdvgpu.shim.launcher import apply_contract, cleanup_region, vgpu_env
from amdvgpu.shim.region import Region
from conftest import CHILD_PRELUDE, child_results, run_child, spawn_child

pytestmark = pytest.mark.gpu

GiB = 1 << 30
MiB = 1 << 20

SPIN_RATE = """
import torch
from amdvgpu.ops import spin
spin(2048, 200); torch.cuda.synchronize()
n = 0
t0 = time.perf_counter()
while time.perf_counter() - t0 < {secs}:
    spin(2048, 500)
    n += 1
    if n % 16 == 0:
        torch.cuda.synchronize()
torch.cuda.synchronize()
emit(rate=n / (time.perf_counter() - t0))
"""


RESNET_RATE = """
import torch
from amdvgpu.models.aibench import Runner, get_case
torch.backends.cudnn.benchmark = True
r = Runner(get_case("resnet50-inf"), "cuda:0", dtype=torch.float32, batch={batch})
for _ in range(5): r.step()
torch.cuda.synchronize()
open(os.environ["VGPU_TEST_READY"], "w").close()
while not os.path.exists(os.environ["VGPU_TEST_GO"]):
    time.sleep(0.002)
reg = None
def mine():
    return sum(p["throttle_ns"] for p in reg.procs() if p["pid"] == os.getpid())
if os.environ.get("VGPU_SHARED_CACHE"):
    from amdvgpu.shim.region import Region
    reg = Region(os.environ["VGPU_SHARED_CACHE"])
    d0 = reg.device(0)
    th0 = mine()
n = 0
t0 = time.perf_counter()
while time.perf_counter() - t0 < {secs}:
    r.step()
    n += 1
    if n % 8 == 0:
        torch.cuda.synchronize()
torch.cuda.synchronize()
el = time.perf_counter() - t0
rate = n / el
busy = throttle = None
if reg is not None:
    d1 = reg.device(0)
    busy = (d1["charged_ns"] - d0["charged_ns"]) / max(1, d1["wall_ns"] - d0["wall_ns"])
    throttle = (mine() - th0) / (el * 1e9)
emit(rate=rate, busy=busy, throttle=throttle)
"""


def _spin_rates(contracts, secs=3.0):
    """Runs one spinning tenant per contract concurrently; returns their launch rates."""
    ps = [spawn_child(SPIN_RATE.format(secs=secs), c) for c in contracts]
    out = []
    for p in ps:
        o, e = p.communicate(timeout=300)
        assert p.returncode == 0, e[-3000:]
        out.append(child_results(o)[0]["rate"])
    return out


def _resnet_rates(contracts, tmp_path, secs=4.0, batch=None, full=False):
    """Stock fp32 ResNet-50 inference tenants, released together after warm-up. Returns
    each one's rate, or with ``full`` its result (rate and charged GPU-time fraction)."""
    os.makedirs(tmp_path, exist_ok=True)
    go = str(tmp_path / "go")
    ps = []
    for i, c in enumerate(contracts):
        ready = str(tmp_path / f"ready{i}")
        ps.append((spawn_child(RESNET_RATE.format(secs=secs, batch=batch), c,
                               extra_env={"VGPU_TEST_READY": ready, "VGPU_TEST_GO": go}), ready))
    deadline = time.time() + 240
    while not all(os.path.exists(r) for _, r in ps):
        if time.time() > deadline or any(p.poll() is not None for p, _ in ps):
            errs = [p.communicate()[1][-2000:] for p, _ in ps if p.poll() is not None]
            raise AssertionError(f"tenant failed to start: {errs}")
        time.sleep(0.05)
    open(go, "w").close()
    out = []
    for p, _ in ps:
        o, e = p.communicate(timeout=300)
        assert p.returncode == 0, e[-3000:]
        res = child_results(o)[0]
        out.append(res if full else res["rate"])
    return out


@pytest.fixture(scope="module")
def native_spin_rate():
    return _spin_rates([None])[0]


@pytest.mark.parametrize("limit", [25, 50])
def test_temporal_accuracy_single_tenant(native_spin_rate, limit):
    c = vgpu_env(cu_limit=limit, cu_mode="temporal")
    try:
        got = _spin_rates([c])[0]
    finally:
        cleanup_region(c)
    achieved = 100.0 * got / native_spin_rate
    assert abs(achieved - limit) <= 5.0, f"limit {limit}%: achieved {achieved:.1f}%"


def test_temporal_limit_through_the_node_ledger(native_spin_rate, tmp_path):
    """The node ledger on real KFD (opt-in, `--ledger`): with vgpu-ledger running over the
    board, two spinning tenants at 25 % (temporal) charge themselves from the ledger -
    almost no occupancy reads of their own - and are held well below their solo rate. Two
    spin kernels co-run without slowing each other, so a processor-sharing charge gives
    each more than its share (32.6 % for 25 %, profiles/r3x): the bound is the limit
    binding, not its accuracy (test_temporal_accuracy_two_tenants_stock_resnet)."""
    import subprocess as sp
    from amdvgpu.plugin.ledger import read_board
    from amdvgpu.shim.native import LEDGER, lib_path
    board = tmp_path / "board"
    board.mkdir()
    cs = [vgpu_env(cu_limit=25, cu_mode="temporal", extra={"VGPU_BOARD_DIR": str(board),
                                                          "VGPU_BOARD_SLOT": f"t{i}.slot"}) for i in range(2)]
    d = sp.Popen([lib_path(LEDGER), "--dir", str(board)])
    try:
        got = _spin_rates(cs, secs=4.0)
        leds = read_board(str(board))
        stats = []
        for c in cs:
            with Region(c["VGPU_SHARED_CACHE"]) as r:
                stats.append((r.samples, r.other_refreshes))
    finally:
        d.terminate()
        d.wait(timeout=10)
        for c in cs:
            cleanup_region(c)
    achieved = [100.0 * g / native_spin_rate for g in got]
    print(json.dumps({"achieved_pct": achieved, "sampler": stats, "ledgers": {k: v["samples"] for k, v in leds.items()}}))
    assert len(leds) == 1 and next(iter(leds.values()))["samples"] > 500, leds
    assert all(refr < 0.2 * smp for smp, refr in stats), stats
    assert all(15.0 <= a <= 40.0 for a in achieved), achieved


def test_temporal_accuracy_two_tenants_stock_resnet(tmp_path):
    """Two stock fp32 ResNet-50 tenants at 25 % each, concurrently: each gets 25 % of the
    GPU's solo throughput (charged by its share of the resident waves while they overlap).
    A saturating workload is required for that equivalence: two low-occupancy kernels that
    co-run without slowing each other down are each charged half the time while running
    at full speed (profiles/r2e/README.md)."""
    native = _resnet_rates([None], tmp_path / "n")[0] if (tmp_path / "n").mkdir() is None else 0
    cs = [vgpu_env(cu_limit=25, cu_mode="temporal", mem_limit=64 * GiB) for _ in range(2)]
    (tmp_path / "t").mkdir()
    try:
        got = _resnet_rates(cs, tmp_path / "t")
    finally:
        for c in cs:
            cleanup_region(c)
    achieved = [100.0 * g / native for g in got]
    assert all(abs(a - 25) <= 5.0 for a in achieved), achieved


def test_lone_pod_under_the_gpu_time_limiter(tmp_path):
    """Round-3 verdict, weak 3: alone on the GPU, a stock ResNet-50 b=50 pod in a 25 %
    temporal vGPU gets >= 0.95 of its entitlement (native throughput x 0.25) while charged
    25 +- 3 % of the GPU's time. The solo credit window (VGPU_LIMITER_SOLO_WINDOW_MS, 160 ms
    by default while no other process keeps the GPU busy) gives it fewer, longer on-periods:
    each one pays the GPU's warm-up after an idle gap once."""
    native = _resnet_rates([None], tmp_path / "n", secs=6.0, full=True)[0]["rate"]
    c = vgpu_env(cu_limit=25, cu_mode="temporal", mem_limit=32 * GiB)
    try:
        r = _resnet_rates([c], tmp_path / "v", secs=8.0, full=True)[0]
    finally:
        cleanup_region(c)
    ratio = r["rate"] / (native * 0.25)
    print(f"lone 25 % temporal: {r['rate']:.1f} steps/s vs native {native:.1f}: {ratio:.3f} of entitlement, "
          f"charged {100 * r['busy']:.1f} % GPU time, throttled {100 * r['throttle']:.1f} %")
    assert abs(100 * r["busy"] - 25.0) <= 3.0, r
    assert ratio >= 0.95, (ratio, r, native)


def test_temporal_four_light_tenants(tmp_path):
    """Small-batch inference (ResNet-50 b=4, launch-bound: the GPU idles between kernels)
    at 25 %, four tenants at once, judged against what the hardware and the host give four
    such tenants without any compute limit (`unlimited x4`, measured in the same window).

    Alone, the tenant is charged its 25 % of the GPU's time, which buys it ~33-35 % of its
    native throughput (it keeps the GPU only ~75 % busy by itself). Four at once share the
    GPU's instants and the host: unlimited, the four together reach only ~120-130 % of one
    native tenant (profiles/r4a), so each can get at most a quarter of that whatever the
    limiter does. The bar is therefore physical:
      * alone: charged 25 +- 5 % of the GPU's time;
      * together: nobody is charged more than 25 + 3 %;
      * each gets >= min(alone, unlimited-together / 4) - 5 points;
      * the four together get >= 0.9 x min(4 x alone, unlimited-together).
    Each tenant's throttle time (launches blocked at the gate) is printed: near zero
    together means the limiter was not what held the tenants back."""
    for d in ("n", "u", "s", "t"):
        (tmp_path / d).mkdir()
    native = _resnet_rates([None], tmp_path / "n", batch=4)[0]
    free = [vgpu_env(mem_limit=32 * GiB) for _ in range(4)]
    solo = vgpu_env(cu_limit=25, cu_mode="temporal", mem_limit=32 * GiB)
    cs = [vgpu_env(cu_limit=25, cu_mode="temporal", mem_limit=32 * GiB) for _ in range(4)]
    try:
        unlimited = _resnet_rates(free, tmp_path / "u", secs=6.0, batch=4)
        one = _resnet_rates([solo], tmp_path / "s", secs=6.0, batch=4, full=True)[0]
        four = _resnet_rates(cs, tmp_path / "t", secs=6.0, batch=4, full=True)
    finally:
        for c in free + [solo] + cs:
            cleanup_region(c)
    alone = 100.0 * one["rate"] / native
    ceiling = 100.0 * sum(unlimited) / native          # four unlimited tenants together
    together = [100.0 * r["rate"] / native for r in four]
    busy = [100.0 * r["busy"] for r in four]
    throttle = [100.0 * r["throttle"] for r in four]
    print(json.dumps({"native": native, "alone_pct": alone, "unlimited_together_pct": ceiling,
                      "together_pct": together, "busy_pct": busy, "throttle_pct": throttle,
                      "alone_busy_pct": 100.0 * one["busy"], "alone_throttle_pct": 100.0 * one["throttle"]}))
    assert abs(100.0 * one["busy"] - 25.0) <= 5.0, one
    assert all(b <= 25.0 + 3.0 for b in busy), busy
    floor = min(alone, ceiling / 4) - 5.0
    assert all(t >= floor for t in together), (floor, together, alone, ceiling)
    assert sum(together) >= 0.9 * min(4 * alone, ceiling), (sum(together), alone, ceiling)


LATENCY_SPIN = """
import torch
from amdvgpu.ops import spin
spin(2048, 200); torch.cuda.synchronize()
open(os.environ["VGPU_TEST_READY"], "w").close()
t0 = time.perf_counter()
while not os.path.exists(os.environ["VGPU_TEST_GO"]) and time.perf_counter() - t0 < 120:
    spin(2048, 500)
    torch.cuda.synchronize()
emit(ok=True)
"""


BG_RATE = """
import torch
from amdvgpu.ops import spin
open(os.environ["VGPU_TEST_STARTED"], "w").close()
n = 0
t0 = time.perf_counter()        # before any launch: a held tenant would never get past a warm-up
while time.perf_counter() - t0 < {secs}:
    spin(2048, 500)
    n += 1
    if n % 16 == 0:
        torch.cuda.synchronize()
torch.cuda.synchronize()
emit(rate=n / (time.perf_counter() - t0))
"""


def _background_rate_next_to(neighbour_prio, tmp_path, secs=5.0):
    """A background tenant (priority 2, GPU-time limiter at 50 %) spins for `secs` next to a
    neighbour container of priority `neighbour_prio` that keeps the GPU busy. The neighbour
    stops 2 s after the window: a tenant held at its launch gate for the whole window is let
    go then, ends its loop at once, and its rate counts what it launched while held."""
    board = tmp_path / "board"
    board.mkdir()
    ready, stop = str(tmp_path / "ready"), str(tmp_path / "stop")
    nb = vgpu_env(mem_limit=16 * GiB, extra={"VGPU_BOARD_DIR": str(board), "VGPU_BOARD_SLOT": "svc.slot",
                                             "VGPU_TASK_PRIORITY": str(neighbour_prio)})
    bg = vgpu_env(mem_limit=16 * GiB, cu_limit=50, cu_mode="temporal",
                  extra={"VGPU_BOARD_DIR": str(board), "VGPU_BOARD_SLOT": "batch.slot", "VGPU_TASK_PRIORITY": "2"})
    svc = spawn_child(LATENCY_SPIN, nb, extra_env={"VGPU_TEST_READY": ready, "VGPU_TEST_GO": stop})
    try:
        deadline = time.time() + 240
        while not os.path.exists(ready):
            assert time.time() < deadline and svc.poll() is None, "neighbour failed to start"
            time.sleep(0.05)
        time.sleep(1.0)  # on the board, busy
        started = str(tmp_path / "started")
        p = spawn_child(BG_RATE.format(secs=secs), bg, extra_env={"VGPU_TEST_STARTED": started})
        t_end = time.time() + 240
        while p.poll() is None and not os.path.exists(started) and time.time() < t_end:
            time.sleep(0.05)
        try:
            p.wait(timeout=secs + 2.0)            # the window (and the context's set-up) + 2 s
        except subprocess.TimeoutExpired:
            pass
        open(stop, "w").close()                  # the neighbour stops: a held tenant is let go
        o, e = p.communicate(timeout=120)
        assert p.returncode == 0, e[-3000:]
        rate = child_results(o)[0]["rate"]
        with Region(bg["VGPU_SHARED_CACHE"]) as r:   # the limiter's side, for a failure's message
            d = r.device(0)
            diag = {"samples": r.samples, "other_refreshes": r.other_refreshes, "charged_ns": d["charged_ns"],
                    "wall_ns": d["wall_ns"], "preempt": d["preempt"], "cu_mode": d["cu_mode"],
                    "hostpids": [p["hostpid"] for p in r.procs()]}
    finally:
        open(stop, "w").close()
        _, svc_err = svc.communicate(timeout=120)
        cleanup_region(nb)
        cleanup_region(bg)
    # the neighbour kept the GPU busy throughout (a neighbour that died early - killed, say -
    # leaves the background tenant alone at its 50 %)
    diag["neighbour_rc"] = svc.returncode
    if svc.returncode != 0:
        diag["neighbour_err"] = svc_err[-1500:]
    return rate, diag


def test_background_class_yields_to_a_busy_latency_class(tmp_path):
    """VGPU_TASK_PRIORITY=2 (background) earns no GPU time while a container of a better
    class keeps the GPU busy (the board, vgpu/board.h), and runs at its share next to an
    equal-class neighbour. This is what cuts the inference service's P99 next to
    background trainers (profiles/r3d, r3j)."""
    (tmp_path / "eq").mkdir()
    (tmp_path / "lat").mkdir()
    equal, d_eq = _background_rate_next_to(2, tmp_path / "eq")
    behind, d_lat = _background_rate_next_to(0, tmp_path / "lat")
    print(json.dumps({"next_to_equal": equal, "next_to_latency": behind, "limiter": [d_eq, d_lat]}))
    assert equal > 0, equal
    assert behind < 0.3 * equal, (equal, behind, d_eq, d_lat)


IDLE_ON_BOARD = """
import torch
from amdvgpu.ops import spin
spin(64, 100); torch.cuda.synchronize()
open(os.environ["VGPU_TEST_READY"], "w").close()
t0 = time.perf_counter()
while not os.path.exists(os.environ["VGPU_TEST_GO"]) and time.perf_counter() - t0 < 120:
    time.sleep(0.05)
"""

BURST = """
import torch
from amdvgpu.ops import spin
from amdvgpu.shim.region import Region
spin(64, 100); torch.cuda.synchronize()
time.sleep(1.5)  # crowd and board assessed by the lease holder
t0 = time.perf_counter()
for _ in range(200):
    spin(64, 500)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
emit(enqueue_s=t1 - t0, total_s=t2 - t0, depth_cap=Region(os.environ["VGPU_SHARED_CACHE"]).device(0)["depth_cap"])
"""


@pytest.mark.parametrize("depth", [0, 2])
def test_background_depth_bound_next_to_a_latency_class(tmp_path, depth):
    """VGPU_PREEMPT_DEPTH: with a latency-class container on the board (idle) and the GPU
    crowded by an equal-class neighbour, a background container's launches wait on its HSA
    queues' read index - 200 async 0.5 ms kernels take about as long to enqueue as to run.
    Without the bound they are all queued at once."""
    board = tmp_path / "board"
    board.mkdir()
    ready, go = str(tmp_path / "ready"), str(tmp_path / "go")
    ex = {"VGPU_BOARD_DIR": str(board)}
    lat = vgpu_env(mem_limit=8 * GiB, extra=dict(ex, VGPU_BOARD_SLOT="svc.slot", VGPU_TASK_PRIORITY="0"))
    peer = vgpu_env(mem_limit=8 * GiB, extra=dict(ex, VGPU_BOARD_SLOT="peer.slot", VGPU_TASK_PRIORITY="2"))
    bg = vgpu_env(mem_limit=8 * GiB, extra=dict(ex, VGPU_BOARD_SLOT="batch.slot", VGPU_TASK_PRIORITY="2",
                                                   VGPU_PREEMPT_DEPTH=str(depth)))
    svc = spawn_child(IDLE_ON_BOARD, lat, extra_env={"VGPU_TEST_READY": ready, "VGPU_TEST_GO": go})
    busy = spawn_child(LATENCY_SPIN, peer, extra_env={"VGPU_TEST_READY": ready + ".peer", "VGPU_TEST_GO": go})
    try:
        deadline = time.time() + 240
        while not (os.path.exists(ready) and os.path.exists(ready + ".peer")):
            assert time.time() < deadline and svc.poll() is None and busy.poll() is None, "neighbours failed"
            time.sleep(0.05)
        res, _ = run_child(BURST, bg, timeout=240)
    finally:
        open(go, "w").close()
        svc.communicate(timeout=120)
        busy.communicate(timeout=120)
        for c in (lat, peer, bg):
            cleanup_region(c)
    r = res[0]
    print(json.dumps(r))
    if depth:
        assert r["depth_cap"] == depth and r["enqueue_s"] > 0.8 * r["total_s"], r
    else:
        assert r["depth_cap"] == 0 and r["enqueue_s"] < 0.3 * r["total_s"], r


CENSUS = """
import torch
from amdvgpu.ops import cu_census
from amdvgpu.shim.region import Region
time.sleep(1.5)   # the lease holder assesses the GPU's crowd every 120 ms
n = len(cu_census(nblocks=8192, spin_us=300))
d = Region(os.environ["VGPU_SHARED_CACHE"]).device(0)
emit(n=n, mode=d["cu_mode"], crowd=d["crowd"])
"""

NEIGHBOUR = """
import torch
from amdvgpu.ops import spin
spin(256, 200); torch.cuda.synchronize()
emit(ready=True)
go = os.environ["VGPU_TEST_GO"]
while not os.path.exists(go):
    for _ in range(8):
        spin(256, 2000)
    torch.cuda.synchronize()
"""


@pytest.mark.parametrize("pct,neighbours,mode,ncu", [(50, 0, "spatial", 128), (25, 0, "spatial", 64),
                                                      (25, 2, "temporal", 256)])
def test_auto_mode_picks_enforcement(tmp_region, tmp_path, pct, neighbours, mode, ncu):
    """Default (auto) mode: a 1/2 share is always a CU mask; a 1/4 share keeps its CU mask
    while at most one other process keeps the GPU busy and is time-limited on all CUs when
    the GPU is crowded (masked tenants beyond two stall each other in the dispatchers)."""
    go = str(tmp_path / "go")
    others = [spawn_child(NEIGHBOUR, None, extra_env={"VGPU_TEST_GO": go}) for _ in range(neighbours)]
    try:
        for o in others:
            assert o.stdout.readline().startswith("RESULT")
        c = vgpu_env(cu_limit=pct, shared_cache=tmp_region)
        res, _ = run_child(CENSUS, c)
    finally:
        open(go, "w").close()
        for o in others:
            o.communicate(timeout=60)
    assert res[0]["n"] == ncu and res[0]["mode"] == mode, res
    assert res[0]["crowd"] == neighbours or pct >= 50, res


SLICE_HOLDER = """
import torch
from amdvgpu.ops import cu_census
time.sleep(1.5)
emit(cus=sorted(cu_census(nblocks=8192, spin_us=300)))
t0 = time.perf_counter()
while not os.path.exists(os.environ["VGPU_TEST_GO"]) and time.perf_counter() - t0 < 120:
    time.sleep(0.05)
"""

BG_CENSUS = """
import torch
from amdvgpu.ops import cu_census
time.sleep(1.5)   # the lease holder reads the board and re-masks the queues
emit(cus=sorted(cu_census(nblocks=8192, spin_us=300)))
"""


def test_background_class_keeps_off_the_latency_slice(tmp_path):
    """A latency-class container (priority 0, 25 %: its 64-CU slice) publishes its slice on
    the board; a background container (priority 2) on the same GPU runs its kernels on the
    other 192 CUs only - the real-hardware check of the board's CU reservation."""
    board = tmp_path / "board"
    board.mkdir()
    go = str(tmp_path / "go")
    lat = vgpu_env(mem_limit=16 * GiB, cu_limit=25, extra={"VGPU_BOARD_DIR": str(board), "VGPU_BOARD_SLOT": "svc.slot",
                                                           "VGPU_TASK_PRIORITY": "0"})
    bg = vgpu_env(mem_limit=16 * GiB, extra={"VGPU_BOARD_DIR": str(board), "VGPU_BOARD_SLOT": "batch.slot",
                                             "VGPU_TASK_PRIORITY": "2"})
    svc = spawn_child(SLICE_HOLDER, lat, extra_env={"VGPU_TEST_GO": go})
    try:
        line = svc.stdout.readline()
        assert line.startswith("RESULT"), svc.stderr.read()[-3000:]
        mine = {tuple(c) for c in json.loads(line[7:])["cus"]}
        res, _ = run_child(BG_CENSUS, bg)
    finally:
        open(go, "w").close()
        svc.communicate(timeout=60)
        cleanup_region(lat)
        cleanup_region(bg)
    theirs = {tuple(c) for c in res[0]["cus"]}
    assert len(mine) == 64, len(mine)
    assert len(theirs) == 192 and not (mine & theirs), (len(theirs), sorted(mine & theirs)[:8])


LIVE = """
import torch
from amdvgpu.ops import cu_census, spin
from amdvgpu.shim.region import Region
emit(n=len(cu_census(nblocks=8192, spin_us=300)))
go = os.environ["VGPU_TEST_GO"]
while not os.path.exists(go):
    spin(64, 50); torch.cuda.synchronize(); time.sleep(0.01)
emit(n=len(cu_census(nblocks=8192, spin_us=300)),
     mode=Region(os.environ["VGPU_SHARED_CACHE"]).device(0)["cu_mode"])
"""


@pytest.mark.parametrize("cu_mode,after_n,after_mode", [("spatial", 64, "spatial"), ("auto", 64, "spatial")])
def test_live_cu_limit_change(tmp_region, tmp_path, cu_mode, after_n, after_mode):
    """vgpuctl set-cu 50 -> 25 on a running container re-masks its existing queues
    (reference: set_current_device_sm_limit_scale feeds the running limiter)."""
    go = str(tmp_path / "go")
    c = vgpu_env(cu_limit=50, cu_mode=cu_mode, shared_cache=tmp_region, extra={"VGPU_TEST_GO": go})
    p = spawn_child(LIVE, c)
    first = json.loads(p.stdout.readline()[7:])
    assert first["n"] == 128, first
    with Region(tmp_region) as r:
        assert r.set_cu_limit(0, 25) == 0
    open(go, "w").close()
    out, err = p.communicate(timeout=120)
    assert p.returncode == 0, err[-3000:]
    second = child_results(out)[0]
    assert second["n"] == after_n and second["mode"] == after_mode, second


BLOCKABLE = """
import torch
from amdvgpu.ops import spin
x = torch.ones(1 << 20, device="cuda"); torch.cuda.synchronize()
emit(ready=True)
gaps = []
last = time.time()
for i in range(300):
    x.add_(1)
    torch.cuda.synchronize()
    now = time.time(); gaps.append(now - last); last = now
    time.sleep(0.005)
emit(max_gap=max(gaps), val=float(x[0]))
"""


@pytest.mark.parametrize("cu_mode", ["spatial", "off"])
def test_launch_block_in_every_mode(tmp_region, cu_mode):
    """recent_kernel < 0 (vgpuctl block / monitor POST /block) stalls launches even when
    no temporal limiter runs (reference rate_limiter checks it before the SM limit)."""
    c = vgpu_env(cu_limit=50, cu_mode=cu_mode, mem_limit=8 * GiB, shared_cache=tmp_region)
    p = spawn_child(BLOCKABLE, c)
    assert p.stdout.readline().startswith("RESULT")
    with Region(tmp_region) as r:
        time.sleep(0.3)
        r.recent_kernel = -1
        time.sleep(2.0)
        r.recent_kernel = 2
        out, err = p.communicate(timeout=120)
        procs_after = r.procs()
    assert p.returncode == 0, err[-3000:]
    res = child_results(out)[0]
    assert res["val"] == 301.0
    assert res["max_gap"] >= 1.5, res
    assert not procs_after


def test_launch_counter_and_hostpids_for_simultaneous_starters(tmp_region):
    """Four processes of one container start together: each resolves its host PID (the
    gpurun box runs in a PID namespace with foreign KFD processes coming and going) and
    counts its launches in the region."""
    c = vgpu_env(mem_limit=32 * GiB, shared_cache=tmp_region)
    code = """
import torch
x = torch.ones(1 << 20, device="cuda")
for _ in range(50): x.add_(1)
torch.cuda.synchronize()
emit(ok=True)
time.sleep(4)
"""
    ps = [spawn_child(code, c) for _ in range(4)]
    try:
        for p in ps:
            assert p.stdout.readline().startswith("RESULT")
        time.sleep(1.5)  # maintenance-thread retries, if the first attempt lost the race
        with Region(tmp_region) as r:
            procs = r.procs()
        alive = [os.path.isdir(f"/sys/class/kfd/kfd/proc/{p['hostpid']}") for p in procs]
    finally:
        for p in ps:
            p.wait(60)
    assert len(procs) == 4
    hostpids = [p["hostpid"] for p in procs]
    assert all(h > 0 for h in hostpids) and len(set(hostpids)) == 4, procs
    assert all(alive), list(zip(hostpids, alive))
    assert all(p["launches"] >= 50 for p in procs), [p["launches"] for p in procs]


def test_scratch_is_charged_as_context(tmp_region):
    """ROCr's scratch backing store for a kernel with a 16 KiB/lane private segment never
    passes the allocation hooks; the maintenance thread re-syncs the process's context
    charge from KFD's VRAM counter, so it counts against the quota."""
    c = vgpu_env(mem_limit=64 * GiB, shared_cache=tmp_region)
    res, _ = run_child("""
import torch
from amdvgpu.ops import scratch_hog
from amdvgpu.shim.region import Region
x = torch.ones(1 << 20, device="cuda"); torch.cuda.synchronize(); time.sleep(0.5)
r = Region(os.environ["VGPU_SHARED_CACHE"])
def ctx():
    return r.procs()[0]["used_kind"][0]["context"]
before = ctx()
free0, _ = torch.cuda.mem_get_info(0)
y = scratch_hog(nblocks=8192)
torch.cuda.synchronize()
time.sleep(0.6)
after = ctx()
free1, _ = torch.cuda.mem_get_info(0)
emit(before=before, after=after, free0=free0, free1=free1, hostpid=r.procs()[0]["hostpid"])
""", c)
    r = res[0]
    assert r["hostpid"] > 0
    assert r["after"] - r["before"] >= 256 * MiB, r
    assert r["free0"] - r["free1"] >= 256 * MiB, r


IPC_PRODUCER = """
import torch, torch.multiprocessing as mp
from amdvgpu.shim.region import Region

def consumer(q, res):
    t = q.get()
    res.put(float(t[:1024].sum()))
    time.sleep(2.0)   # keep the mapping while the parent inspects the region

if __name__ == "__main__":
    ctx = mp.get_context("spawn")
    q, res = ctx.Queue(), ctx.Queue()
    x = torch.full((1 << 28,), 2.0, device="cuda")   # 1 GiB
    torch.cuda.synchronize()
    p = ctx.Process(target=consumer, args=(q, res))
    p.start()
    q.put(x)
    s = res.get(timeout=120)
    time.sleep(0.8)   # both maintenance threads re-sync context charges
    r = Region(os.environ["VGPU_SHARED_CACHE"])
    gid = r.device(0)["gpu_id"]
    def vram(hp):
        try:
            return int(open(f"/sys/class/kfd/kfd/proc/{hp}/vram_{gid}").read())
        except OSError:
            return -1
    emit(sum=s, used=r.device(0)["used"], procs=[{"pid": pr["pid"], "hostpid": pr["hostpid"],
                                                  "data": pr["used_kind"][0]["data"],
                                                  "context": pr["used_kind"][0]["context"],
                                                  "kfd_vram": vram(pr["hostpid"])} for pr in r.procs()])
    p.join(60)
"""


def test_ipc_tensor_is_charged_once(tmp_region, tmp_path):
    """torch.multiprocessing shares a 1 GiB CUDA tensor (hipIpcGetMemHandle →
    hsa_amd_ipc_memory_attach in the consumer): it works across the two processes of
    the container and is charged to the exporter only."""
    c = vgpu_env(mem_limit=16 * GiB, shared_cache=tmp_region)
    script = tmp_path / "ipc.py"
    script.write_text(CHILD_PRELUDE + IPC_PRODUCER)
    p = subprocess.run([sys.executable, str(script)], env=apply_contract(c), capture_output=True, text=True,
                       timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    r = child_results(p.stdout)[0]
    assert r["sum"] == 2048.0
    assert len(r["procs"]) == 2
    gib_data = [pr["data"] for pr in r["procs"]]
    ctx = [pr["context"] for pr in r["procs"]]
    print("ipc:", r)
    assert max(gib_data) >= GiB and min(gib_data) < 256 * MiB, r   # only the exporter holds data
    assert max(ctx) < GiB, r                                        # no second charge as context
    assert r["used"] < 2 * GiB, r
    # Each process's charge matches KFD's own count of its VRAM (the import is not in it).
    for pr in r["procs"]:
        assert abs(pr["data"] + pr["context"] - pr["kfd_vram"]) < 64 * MiB, pr


SPILL = """
import torch
from amdvgpu.shim.region import Region
x = torch.ones(1 << 20, device="cuda"); x.add_(1); torch.cuda.synchronize()
time.sleep(1.0)   # let the context charge (runtime-internal memory) settle first
r = Region(os.environ["VGPU_SHARED_CACHE"])
big = [torch.ones(1 << 30, dtype=torch.uint8, device="cuda") for _ in range(10)]    # 10 x 1 GiB ("large")
torch.cuda.synchronize()
after_big = r.device(0)["spilled"]
small = [torch.full((32 << 20,), 7, dtype=torch.uint8, device="cuda") for _ in range(64)]   # 64 x 32 MiB
torch.cuda.synchronize()
after_small = r.device(0)["spilled"]
ok = all(bool(t[:4096].eq(1).all()) for t in big) and all(bool(t[:4096].eq(7).all()) for t in small)
emit(after_big=after_big, after_small=after_small, ok=ok)
"""


@pytest.mark.parametrize("policy", ["large-first", "first-come"])
def test_spill_placement_policy(tmp_region, policy):
    """Virtual device memory with an 8 GiB HBM share: first-come fills HBM with seven
    1 GiB buffers and spills the later small (hot) allocations; large-first spills large
    buffers once they would eat into the share's reserve (3 GiB here), so the 2 GiB of
    small ones still find HBM."""
    c = vgpu_env(mem_limit=16 * GiB, shared_cache=tmp_region, oversubscribe=True,
                 extra={"VGPU_DEVICE_HBM_LIMIT_0": "8192m", "VGPU_SPILL_POLICY": policy,
                        "VGPU_SPILL_RESERVE": "3g"})
    res, _ = run_child(SPILL, c)
    r = res[0]
    assert r["ok"], r
    small_spilled = r["after_small"] - r["after_big"]
    if policy == "large-first":
        assert r["after_big"] >= 2 * GiB and small_spilled == 0, r
    else:
        assert small_spilled >= 256 * MiB, r


SPILL_PROMOTE = """
import ctypes, torch
lib = ctypes.CDLL(None)
lib.vgpu_get_current_device_spilled.restype = ctypes.c_uint64
def spilled():
    return lib.vgpu_get_current_device_spilled()
def read_gbps(t, reps=5):
    torch.cuda.synchronize(); t0 = time.time()
    for _ in range(reps):
        t.max()
    torch.cuda.synchronize()
    return round(t.numel() * t.element_size() * reps / (time.time() - t0) / 1e9, 1)
x = torch.ones(1 << 20, device="cuda"); x.add_(1); torch.cuda.synchronize()
time.sleep(1.0)   # the context charge settles first
mode = os.environ["SPILL_MODE"]
if mode == "own":
    a = torch.empty(3 << 30, dtype=torch.uint8, device="cuda")           # 3 GiB: (nearly) fills the share
torch.cuda.synchronize()
s_pre = spilled()                                                         # 0: everything so far is in HBM
n = int(os.environ["SPILL_ELEMS"])
b = torch.full((n,), 7, dtype=torch.int32, device="cuda")                 # spilled
torch.cuda.synchronize()
s0 = spilled()
ok0 = int(b.sum(dtype=torch.int64)) == 7 * n
gbps0 = read_gbps(b)
if mode == "own":
    del a
    torch.cuda.empty_cache()                                              # hipFree: HBM share frees up
else:
    open(os.environ["SPILL_GO"], "w").close()                             # the neighbour frees its HBM
t0 = time.time()
while spilled() and time.time() - t0 < float(os.environ.get("SPILL_WAIT", "20")):
    time.sleep(0.02)
t_promote = round(time.time() - t0, 3)
s1 = spilled()
b.add_(1); torch.cuda.synchronize()
ok1 = int(b.sum(dtype=torch.int64)) == 8 * n
gbps1 = read_gbps(b)
emit(spilled_pre=s_pre, spilled_before=s0, spilled_after=s1, ok_before=ok0, ok_after=ok1, gbps_spilled=gbps0,
     gbps_promoted=gbps1, promote_s=t_promote, bytes=4 * n)
"""

HBM_HOG = """
import torch
keep = int(os.environ["HOG_KEEP"])
held = []
while True:
    free, _ = torch.cuda.mem_get_info()
    if free <= keep + (64 << 20):
        break
    held.append(torch.empty(min(free - keep, 16 << 30), dtype=torch.uint8, device="cuda"))
open(os.environ["HOG_READY"], "w").close()
t0 = time.time()
while not os.path.exists(os.environ["SPILL_GO"]) and time.time() - t0 < 120:
    time.sleep(0.02)
del held
torch.cuda.empty_cache()
emit(freed=True)
time.sleep(2.0)
"""


@pytest.mark.parametrize("neighbour", ["own-buffer", "other-tenant"])
def test_spill_is_promoted_after_hbm_frees_up(tmp_region, tmp_path, neighbour):
    """Virtual device memory that moves (round-3 verdict, missing 2): a buffer that spilled to
    host memory - past the tenant's 4 GiB HBM share behind its own 3 GiB buffer, or (large-
    first) because another tenant holds nearly all of the GPU's HBM - is an SVM range the GPU
    reads in place; once the HBM frees up, the shim migrates it into HBM at the same address:
    the spill counter returns to 0, the data are intact, the buffer keeps working, and reading
    it runs at HBM speed instead of over the host link."""
    import torch
    if neighbour == "own-buffer":
        c = vgpu_env(mem_limit=16 * GiB, shared_cache=tmp_region, oversubscribe=True,
                     extra={"VGPU_DEVICE_HBM_LIMIT_0": "4096m", "VGPU_SPILL_POLICY": "first-come"})
        env = {"SPILL_MODE": "own", "SPILL_ELEMS": str(1 << 28)}                       # 1 GiB
        res, _ = run_child(SPILL_PROMOTE, c, extra_env=env)
    else:
        ready, go = tmp_path / "ready", tmp_path / "go"
        hog = spawn_child(HBM_HOG, None, extra_env={"HOG_KEEP": str(3 * GiB), "HOG_READY": str(ready),
                                                   "SPILL_GO": str(go)})
        try:
            t0 = time.time()
            while not ready.exists():
                assert hog.poll() is None and time.time() - t0 < 120, hog.communicate()[1][-3000:]
                time.sleep(0.1)
            c = vgpu_env(mem_limit=16 * GiB, shared_cache=tmp_region, oversubscribe=True,
                         extra={"VGPU_DEVICE_HBM_LIMIT_0": "8192m", "VGPU_SPILL_POLICY": "large-first",
                                "VGPU_SPILL_RESERVE": "1g"})
            env = {"SPILL_MODE": "neighbour", "SPILL_ELEMS": str(1 << 29), "SPILL_GO": str(go)}   # 2 GiB
            res, _ = run_child(SPILL_PROMOTE, c, extra_env=env)
        finally:
            go.touch()
            hog.wait(timeout=60)
    r = res[0]
    print("spill promotion:", r)
    assert r["spilled_pre"] == 0 and r["spilled_before"] >= r["bytes"], r   # the buffer itself spilled
    assert r["ok_before"] and r["ok_after"], r
    assert r["spilled_after"] == 0, r
    assert r["gbps_promoted"] > 3 * r["gbps_spilled"], r


def test_pinned_spill_backing_stays_in_host_memory(tmp_region):
    """VGPU_SPILL_BACKING=pinned keeps the round-3 spill: a pinned host-pool allocation the
    GPU reads in place, correct, and never moved (it stays spilled after HBM frees up)."""
    c = vgpu_env(mem_limit=16 * GiB, shared_cache=tmp_region, oversubscribe=True,
                 extra={"VGPU_DEVICE_HBM_LIMIT_0": "4096m", "VGPU_SPILL_POLICY": "first-come",
                        "VGPU_SPILL_BACKING": "pinned"})
    res, _ = run_child(SPILL_PROMOTE, c, extra_env={"SPILL_MODE": "own", "SPILL_ELEMS": str(1 << 28),
                                                    "SPILL_WAIT": "2"})
    r = res[0]
    print("pinned spill:", r)
    assert r["spilled_pre"] == 0 and r["spilled_before"] >= r["bytes"], r
    assert r["ok_before"] and r["ok_after"], r
    assert r["spilled_after"] >= r["bytes"], r   # still in host memory: a pinned spill never moves


CU_PROPS = """
import torch
p = torch.cuda.get_device_properties(0)
a = torch.randn(2048, 2048, device="cuda"); b = torch.randn(2048, 2048, device="cuda")
c = a @ b
conv = torch.nn.Conv2d(64, 64, 3, padding=1).cuda()
y = conv(torch.randn(8, 64, 56, 56, device="cuda"))
torch.cuda.synchronize()
ok = bool(torch.allclose(c[:64, :64].cpu(), (a[:64].cpu() @ b[:, :64].cpu()), atol=1e-2, rtol=1e-3))
emit(cus=p.multi_processor_count, ok=ok, conv_finite=bool(torch.isfinite(y).all()))
"""


@pytest.mark.parametrize("mode,pct,want", [("spatial", 25, 64), ("temporal", 25, 256), ("auto", 25, 64),
                                           ("auto", 7, 256)])
def test_runtime_sees_the_spatial_slice_cu_count(tmp_region, mode, pct, want):
    """Reference: cuDeviceGetAttribute virtualisation [device.c:130-134]. A 25 % vGPU with
    a CU slice (spatial, or auto whichever enforcement is on) reports 64 CUs to HIP
    (multiProcessorCount), so stock libraries size grids for the slice; stock GEMM / conv
    still compute correctly. Explicitly temporal vGPUs keep 256, and so does a thin share in
    auto mode (7 %: a 16-CU slice is time-sliced on every CU, VGPU_AUTO_MIN_SLICE_CUS)."""
    c = vgpu_env(mem_limit=24 * GiB, cu_limit=pct, cu_mode=mode, shared_cache=tmp_region)
    res, _ = run_child(CU_PROPS, c)
    r = res[0]
    assert r["cus"] == want, r
    assert r["ok"] and r["conv_finite"], r
