"""Regression bar for the shim's per-call cost on the hot paths (benchmarks/hook_overhead.py).

Every launch / copy / set entry point goes through a generated trampoline
(native/src/shim/hip_gates.def). These bars keep that cost from creeping up unnoticed.

Launches are measured from C++ (native/tests/hip_launch_probe.hip: empty kernels in
batches of 256, hipPointerGetAttributes for the gate alone, 4-byte hipMemsetAsync): the
PyTorch-level figure (~4 us per `x.add_(1)`, mostly the interpreter and the dispatcher)
moved by +-10 % between native runs on one box (round 3: 4.04-4.43 us native), which made
a 10 % bar on it a coin toss (GPUTEST r4a: 4.04 vs 4.84). The C++ probe's figures are
stable to a few percent. Bars: a vGPU may cost at most 10 % + 0.2 us per launch, 100 ns per
gated host-only call, 15 % + 0.3 us per small set; and (PyTorch-level) 10 % + 1 us per
graph replay, 15 % + 10 us per allocation pair, 15 % + 0.3 us per small copy.
"""
import json
import os
import subprocess
import sys
import tempfile

import pytest

from amdvgpu.shim.launcher import apply_contract, cleanup_region, vgpu_env
from amdvgpu.shim.native import lib_path

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "benchmarks", "hook_overhead.py")

# metric: (relative tolerance, absolute slack in the metric's unit)
PROBE_BARS = {"launch_us": (0.10, 0.2), "gate_ns": (0.0, 100.0), "memset_us": (0.15, 0.3)}
TORCH_BARS = {"graph_replay_us": (0.10, 1.0), "malloc_free_us": (0.15, 10.0), "memcpy_us": (0.15, 0.3)}


def _probe(contract):
    env = apply_contract(contract) if contract else dict(os.environ)
    out = subprocess.run([lib_path("hip_launch_probe"), "50000", "500000"], env=env, capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    return json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])


def _torch(contract, iters=10000):
    env = apply_contract(contract) if contract else dict(os.environ)
    fd, out = tempfile.mkstemp(suffix=".json")
    os.close(fd)
    try:
        subprocess.run([sys.executable, BENCH, "--worker", "--iters", str(iters), "--out", out], env=env, check=True,
                       timeout=300)
        return json.load(open(out))
    finally:
        os.unlink(out)


def _best(measure, rounds=3):
    best = {"native": {}, "vgpu": {}}
    for _ in range(rounds):  # interleaved, best of N: the box's clocks and neighbours drift
        for mode in best:
            c = vgpu_env(mem_limit=64 << 30) if mode == "vgpu" else None
            try:
                r = measure(c)
            finally:
                if c:
                    cleanup_region(c)
            for k, v in r.items():
                best[mode][k] = min(v, best[mode].get(k, float("inf")))
    return best


def _over(best, bars):
    return {k: (round(best["native"][k], 3), round(best["vgpu"][k], 3)) for k, (rel, slack) in bars.items()
            if best["vgpu"][k] > best["native"][k] * (1 + rel) + slack}


def test_launch_and_gate_cost_within_bars():
    best = _best(_probe)
    print(json.dumps(best))
    over = _over(best, PROBE_BARS)
    assert not over, f"native vs vGPU per call over the bar: {over}"


def test_graph_alloc_copy_cost_within_bars():
    best = _best(_torch)
    print(json.dumps(best))
    over = _over(best, TORCH_BARS)
    assert not over, f"native vs vGPU us/call over the bar: {over}"
