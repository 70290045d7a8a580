#!/usr/bin/env python3
"""Dispatch-bound pods: N split-N vGPUs from a real Allocate, each running the C++ tiny-kernel
probe (native/tests/cotenancy_probe.hip: back-to-back spin kernels, a wait every 8), started
together. Reports kernels/s per pod and in all, with the admission statistics of each pod
(VGPU_STATS). Knobs: the plugin's --gpu-concurrency, the pods' VGPU_SYNC_WAIT.

    python3 benchmarks/tiny_pods.py --pods 4 --conc 0 --sync-wait auto --seconds 4
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
PROBE = os.path.join(REPO, "4paradigm-k8s-device-plugin_amd", "lib", "cotenancy_probe")


def run(pods, conc, sync_wait, seconds, spin_us, cu_mode):
    from amdvgpu.plugin.devices import SysfsBackend
    from amdvgpu.plugin.kubelet_stub import NodeHarness
    from amdvgpu.shim.launcher import apply_contract
    backend = SysfsBackend()
    uuid = backend.devices()[0].uuid
    with NodeHarness(backend, device_split_count=pods, cu_mode=cu_mode, gpu_concurrency=conc,
                     workdir=tempfile.mkdtemp(prefix="tiny-")) as node:
        procs = []
        for vid in node.vgpu_ids(uuid)[:pods]:
            env = apply_contract(*node.pod([vid]))
            env["VGPU_STATS"] = "1"
            if sync_wait:
                env["VGPU_SYNC_WAIT"] = sync_wait
            procs.append(subprocess.Popen([PROBE, "procs", "1", str(seconds), str(spin_us), "4", "spin", "none"],
                                          env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
        res = []
        for p in procs:
            out, err = p.communicate(timeout=seconds + 90)
            if p.returncode != 0:
                raise SystemExit(f"pod failed: {err[-2000:]}")
            t = json.loads(out.strip().splitlines()[-1])["per_tenant"][0]
            stats = [l for l in err.splitlines() if l.startswith("[vGPU stats") and "kernel launches=" in l]
            res.append({"kps": round(t["kps"]), "wait_us": round(t["wait_us"], 1), "launch_us": round(t["launch_us"], 2),
                        "stats": stats[-1][:300] if stats else None})
    return {"pods": pods, "conc": conc, "sync_wait": sync_wait or "default", "spin_us": spin_us,
            "aggregate_kps": sum(r["kps"] for r in res), "per_pod": res}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pods", type=int, default=4)
    ap.add_argument("--conc", type=lambda v: -1 if v == "auto" else int(v), default=0)
    ap.add_argument("--sync-wait", default="", help="VGPU_SYNC_WAIT for the pods (default: the shim's auto)")
    ap.add_argument("--seconds", type=float, default=4.0)
    ap.add_argument("--spin-us", type=float, default=2.0)
    ap.add_argument("--cu-mode", default="temporal")
    a = ap.parse_args()
    print(json.dumps(run(a.pods, a.conc, a.sync_wait, a.seconds, a.spin_us, a.cu_mode)), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
