"""bench.py's multi-rank orchestration, rehearsed on CPU with gloo (world_size 2): the
driver launches it under torch.distributed.run exactly like this on an 8-GPU node."""
import json
import os
import socket
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.slow
def test_bench_two_ranks_cpu_rehearsal():
    port = free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(REPO, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--cpu-rehearsal"]
    env = dict(os.environ, OMP_NUM_THREADS="2")
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=REPO)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout  # only rank 0 prints
    r = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in r, k
    assert r["n_gpus"] == 2 and r["steps"] == 2 and r["warmup"] == 1
    assert r["config"]["global_batch"] == 100 and r["config"]["model"] == "ResNet-V2-50"
    assert "overhead_pct_quota_only" in r and "entitlement_ratio" in r and "parity_split2_mem1.8" in r
    assert r["dtype"] == "fp32" and r["config"]["vgpu"]["cu_limit_pct"] == 25
    rc = r["rccl_allreduce_between_pods"]
    assert rc["native"]["ok"] and rc["vgpu"]["ok"] and "vgpu_vs_native_busbw" in rc, rc
