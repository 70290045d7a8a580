"""Pair turns for dispatch-bound pods, on a real MI355X (profiles/r6f, r6k).

Three or more processes with launches in flight each dispatch at about a quarter of the rate
two reach: the command processor, not the host (profiles/r6f). The concurrency admission
(VGPU_GPU_CONCURRENCY, the node board) lets two containers of a crowded GPU hold it at a time,
one per CPU socket. Four split-4 pods (50 % of the GPU's time each) from a real Allocate each
run the C++ tiny-kernel probe (native/tests/cotenancy_probe.hip: 2 us kernels, a wait every
8), first all at once, then with pair turns. The pairs must beat all-at-once
clearly, and no pod may starve (the round-6 bug where one socket's pods kept both places,
profiles/r6k/starve).
"""
import json
import os
import subprocess
import time

import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu

PROBE = os.path.join(REPO, "4paradigm-k8s-device-plugin_amd", "lib", "cotenancy_probe")


def _four_pods(tmp_path, conc):
    from amdvgpu.plugin.devices import SysfsBackend
    from amdvgpu.plugin.kubelet_stub import NodeHarness
    from amdvgpu.shim.launcher import apply_contract
    backend = SysfsBackend()
    uuid = backend.devices()[0].uuid
    # Cores scaling 2: each split-4 vGPU is entitled to 50 % of the GPU's time, so a pod that
    # holds its turn (2 us kernels at ~200k/s: ~40 % busy) runs on the admission alone, not
    # into its GPU-time share.
    with NodeHarness(backend, device_split_count=4, device_cores_scaling=2.0, cu_mode="temporal",
                     gpu_concurrency=conc, workdir=str(tmp_path / f"node{conc}")) as node:
        procs = []
        for vid in node.vgpu_ids(uuid)[:4]:
            env = apply_contract(*node.pod([vid]))
            # HIP's own wait: a crowded GPU's polled waits (sync_hooks.cpp) would cap a pod that
            # waits every 8 tiny kernels at ~40k kernels/s whatever the admission does
            env.update(VGPU_SYNC_WAIT="native", VGPU_STATS="1")
            procs.append(subprocess.Popen([PROBE, "procs", "1", "4", "2", "4", "spin", "none"], env=env,
                                          stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
        outs = []
        for p in procs:
            out, err = p.communicate(timeout=90)
            assert p.returncode == 0, err[-2000:]
            outs.append(json.loads(out.strip().splitlines()[-1]))
            print("\n".join(l for l in err.splitlines() if "turns=" in l))
    return [o["per_tenant"][0]["kps"] for o in outs]


def test_pair_turns_lift_dispatch_bound_pods(tmp_path):
    assert os.path.exists(PROBE), "make -C native first"
    t0 = time.time()
    together = _four_pods(tmp_path, 0)
    pairs = _four_pods(tmp_path, 2)
    print(json.dumps({"all_at_once_kps": [round(x) for x in together], "pairs_kps": [round(x) for x in pairs],
                      "seconds": round(time.time() - t0, 1)}))
    assert sum(pairs) >= 1.4 * sum(together), (pairs, together)
    assert min(pairs) >= 0.25 * max(pairs), pairs      # everybody gets turns
