"""bench.py's multi-rank orchestration, rehearsed on CPU with gloo (world_size 2, 4 and
8): the driver launches it under torch.distributed.run exactly like this on an 8-GPU
node. Each rank runs its own plugin + stub kubelet (NodeHarness) for its GPU; the ranks'
sockets, region files, allow-lists and lock files must never collide."""
import json
import os
import socket
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port(span=16):
    """A free MASTER_PORT whose next `span` ports are free too: bench.py puts its workers'
    process groups (one per mode, the node point, the RCCL probes) on MASTER_PORT+1, +2, ..."""
    for _ in range(200):
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        p = s.getsockname()[1]
        s.close()
        if p + span >= 65536:
            continue
        ok = True
        for q in range(p + 1, p + span + 1):
            t = socket.socket()
            try:
                t.bind(("127.0.0.1", q))
            except OSError:
                ok = False
            finally:
                t.close()
            if not ok:
                break
        if ok:
            return p
    raise RuntimeError("no free port range")


@pytest.mark.slow
@pytest.mark.parametrize("world", [2, 4, 8])
def test_bench_multi_rank_cpu_rehearsal(world, tmp_path):
    port = free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(REPO, "bench.py"),
           "--gpus", str(world), "--steps", "2", "--warmup", "1", "--sweep-seconds", "1", "--cpu-rehearsal"]
    env = dict(os.environ, OMP_NUM_THREADS="1", VGPU_BENCH_CONTRACT_DIR=str(tmp_path))
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=900, env=env, cwd=REPO)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout  # only rank 0 prints
    r = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in r, k
    assert r["n_gpus"] == world and r["steps"] == 2 and r["warmup"] == 1
    assert r["config"]["global_batch"] == 50 * world and r["config"]["model"] == "ResNet-V2-50"
    assert "overhead_pct_quota_only" in r and "entitlement_ratio" in r and "parity_split2_mem1.8" in r
    assert r["dtype"] == "fp32" and r["config"]["vgpu"]["cu_limit_pct"] == 25
    rc = r["rccl_allreduce_between_pods"]
    assert rc["native"]["ok"] and rc["vgpu"]["ok"] and "vgpu_vs_native_busbw" in rc, rc
    node = r["node"]  # BASELINE config 5: every vGPU of every GPU busy at once
    assert node["vgpus"] == 4 * world and node["gpus_measured"] == world and not node["failures"], node
    assert node["aggregate"] > 0 and "min_pod_vs_entitlement" in node and "aggregate_vs_native" in node
    ranks = [json.load(open(tmp_path / f"rank{i}.json")) for i in range(world)]
    assert sorted(x["local_rank"] for x in ranks) == list(range(world))
    assert len({x["uuid"] for x in ranks}) == world  # one GPU per rank
    pods = [(x["uuid"], pod) for x in ranks for pod in x["pods"].values()]
    assert len(pods) == 3 * world  # vgpu, quota, parity
    for uuid, pod in pods:
        assert pod["ROCR_VISIBLE_DEVICES"] == uuid and pod["VGPU_DEVICE_MAP"] == f"0:{uuid}"
    for key in ("VGPU_SHARED_CACHE", "VGPU_ALLOWLIST", "node_dir"):
        vals = [pod[key] for _u, pod in pods]
        assert None not in vals and len(set(vals)) == len(vals), key
    locks = {x["uuid"]: {pod["VGPU_LOCK_FILE"] for pod in x["pods"].values()} for x in ranks}
    assert len({lf for s in locks.values() for lf in s}) == 3 * world  # one per plugin instance


@pytest.mark.slow
def test_node_point_survives_a_failing_rank(tmp_path):
    """A rank whose pods fail in the node point reaches the cross-rank barrier anyway: the
    job completes, rank 0 prints its line, and the node entry lists the failure instead of
    the whole run hanging until the driver's limit."""
    port = free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(REPO, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--sweep-seconds", "1", "--modes", "native",
           "--rccl-probe", "0", "--cpu-rehearsal"]
    env = dict(os.environ, OMP_NUM_THREADS="1", VGPU_BENCH_FAIL_NODE_RANK="1")
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=REPO)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    r = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][0])
    node = r["node"]
    assert node["gpus_measured"] == 1 and len(node["failures"]) == 1 and node["vgpus"] == 8, node


@pytest.mark.slow
def test_bench_self_launches_its_ranks(tmp_path):
    """``python bench.py --gpus N`` with no launcher (how the driver may call it on an 8-GPU
    node) starts the N ranks itself: the line says n_gpus N, every rank ran its own pods
    and the node point covers all N GPUs."""
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "4", "--steps", "2", "--warmup", "1",
           "--sweep-seconds", "1", "--cpu-rehearsal"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(OMP_NUM_THREADS="1", VGPU_BENCH_CONTRACT_DIR=str(tmp_path))
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=900, env=env, cwd=REPO)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout
    r = json.loads(lines[0])
    assert r["n_gpus"] == 4 and r["config"]["global_batch"] == 200 and r["steps"] == 2 and r["warmup"] == 1
    assert r["node"]["vgpus"] == 16 and r["node"]["gpus_measured"] == 4, r["node"]
    assert r["rccl_allreduce_between_pods"]["vgpu"]["ok"]
    ranks = [json.load(open(tmp_path / f"rank{i}.json")) for i in range(4)]
    assert sorted(x["local_rank"] for x in ranks) == [0, 1, 2, 3] and len({x["uuid"] for x in ranks}) == 4


@pytest.mark.parametrize("fake", [True, False])
def test_bench_refuses_more_gpus_than_visible(fake):
    """--gpus N beyond the GPUs this job can see exits non-zero with a message, instead of
    quietly measuring fewer GPUs under an n_gpus it did not run (this container has no GPU:
    the sysfs inventory is empty; the rehearsal fakes a 1-GPU node)."""
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    if fake:
        cmd.append("--cpu-rehearsal")
        env["VGPU_BENCH_FAKE_GPUS"] = "1"
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=120, env=env, cwd=REPO)
    assert p.returncode != 0 and "refusing" in p.stderr, p.stderr
    assert not [l for l in p.stdout.splitlines() if l.startswith("{")]


def test_visible_devices_honours_rocr_visible_devices(monkeypatch):
    sys.path.insert(0, REPO)
    import bench
    from amdvgpu.plugin.devices import FakeBackend
    be = FakeBackend(n=4)
    uu = [d.uuid for d in be.devices()]
    monkeypatch.delenv("HIP_VISIBLE_DEVICES", raising=False)
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", f"2,{uu[0]}")
    # FakeBackend devices have no render node: all usable, then narrowed by the variable
    assert [d.uuid for d in bench.visible_devices(be, cpu=False)] == [uu[2], uu[0]]
    monkeypatch.delenv("ROCR_VISIBLE_DEVICES")
    assert len(bench.visible_devices(be, cpu=False)) == 4


def test_sweep_respects_the_time_budget(monkeypatch):
    """The driver kills bench.py at its own limit: sweep points that would not finish within
    --time-budget are skipped and reported, and max_vgpus_per_gpu only counts measured points."""
    sys.path.insert(0, REPO)
    import bench
    from amdvgpu.plugin.devices import FakeBackend

    clock = [1000.0]
    monkeypatch.setattr(bench, "now", lambda: clock[0])
    monkeypatch.setattr(bench, "T_START", 1000.0)

    def fake_run(args, envs, label, deadline=None):
        n = len(envs)
        clock[0] += 10.0 * n  # start-up grows with the pods
        per = 4000.0 / n
        return [{"items_per_step": 50, "steps": int(per * 6 / 50), "t0": 0.0, "t1": 6.0} for _ in envs]

    monkeypatch.setattr(bench, "run_concurrent", fake_run)
    args = bench.parse(["--time-budget", "200", "--sweep-seconds", "6"])
    backend = FakeBackend(n=1)
    rows, best = bench.sweep(args, backend, backend.devices()[0].uuid, [1, 2, 4, 8, 12])
    measured = [r["tenants"] for r in rows if "skipped" not in r]
    skipped = [r["tenants"] for r in rows if "skipped" in r]
    # 1 + 2 + 4 pods take 70 s; 8 pods are estimated at 80 s (150 < 200: run), 12 at 120 s.
    assert measured == [1, 2, 4, 8] and skipped == [12], rows
    assert best == 8


def test_common_window_rates_pods_while_all_run():
    """Concurrent pods are rated over the window in which all of them run. A pod whose own
    window runs on after the others stop has the GPU to itself there; its own-window rate
    flatters it and the common window does not."""
    sys.path.insert(0, REPO)
    import bench

    # two pods at 10 items/s while both run (steps of 1 s, 10 items); pod b runs 2 s longer
    # alone at twice the rate (steps of 0.5 s)
    a = {"items_per_step": 10, "steps": 6, "t0": 0.0, "t1": 6.0, "step_done": [1.0 * i for i in range(1, 7)]}
    b_done = [1.0 * i for i in range(1, 7)] + [6.5, 7.0, 7.5, 8.0]
    b = {"items_per_step": 10, "steps": 10, "t0": 0.0, "t1": 8.0, "step_done": b_done}
    rates, w = bench.common_window([a, b])
    assert w == pytest.approx(6.0) and rates == pytest.approx([10.0, 10.0])
    # own windows: b looks 25 % faster
    assert b["items_per_step"] * b["steps"] / (b["t1"] - b["t0"]) == pytest.approx(12.5)
    # a step straddling the window's edge counts in proportion
    c = {"items_per_step": 10, "steps": 3, "t0": 0.5, "t1": 6.5, "step_done": [2.5, 4.5, 6.5]}
    rates, w = bench.common_window([a, c])
    assert w == pytest.approx(5.5)  # 0.5 .. 6.0
    assert rates[0] == pytest.approx(55.0 / 5.5) and rates[1] == pytest.approx((10 + 10 + 7.5) / 5.5)
    # no per-step marks (older workers) or a window too short to rate: None
    assert bench.common_window([dict(a, step_done=[]), b]) is None
    late = {"items_per_step": 10, "steps": 1, "t0": 5.5, "t1": 6.0, "step_done": [6.0]}
    assert bench.common_window([a, late]) is None
