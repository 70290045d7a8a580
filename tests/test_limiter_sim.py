"""Many-pod closed loop of the GPU-time limiter on the CPU (native/tests/limiter_sim.cpp,
profiles/r2ak): the shim's accounting functions against a GPU model with independent
per-pod samplers."""
import json
import os
import subprocess

from amdvgpu.shim.native import LIB_DIR

SIM = os.path.join(LIB_DIR, "vgpu_limiter_sim")


def sim(*args):
    p = subprocess.run([SIM, *map(str, args)], capture_output=True, text=True, timeout=120, check=True)
    return json.loads(p.stdout)


def test_fair_gpu_twelve_pods_share_equally():
    r = sim(12, 4500, 3, 1)           # the plugin's rounded-up 9 %, the stretched period
    assert r["aggregate"] > 0.99 and r["slowest_vs_1_over_n"] > 0.99, r


def test_binding_shares_equalise_unfair_arbitration():
    r = sim(12, 4500, 3, 1, 1.3, 8)   # shares sum to 96 %: every credit binds
    assert r["slowest_vs_1_over_n"] > 0.93 and r["fastest_vs_1_over_n"] < 1.02, r
    r = sim(12, 4500, 3, 1, 1.3)      # rounded-up 9 % (108 %): only the favoured pods are capped
    assert 0.88 < r["slowest_vs_1_over_n"] < 0.93, r
