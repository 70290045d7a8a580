#!/usr/bin/env python3
"""Virtual device memory (BASELINE.json config 4): one vGPU whose quota exceeds the
MI355X's 288 GiB of HBM, with a workload whose own working set exceeds it.

The plugin (NodeHarness: split 1, --device-memory-scaling 1.12) allocates the vGPU:
quota 322 GiB, HBM share 288 GiB (VGPU_DEVICE_HBM_LIMIT_0), VGPU_OVERSUBSCRIBE=true. The
tenant trains the ai-benchmark LSTM (test 5.2: batch 10, 1024 x 300, stock nn.LSTM, fp32)
on a device-resident dataset: ``--dataset-gib`` of sequences allocated up front in 1 GiB
chunks, every training step reading its batch from a different chunk (round-robin over the
whole dataset). No ballast: every byte is the workload's data. The shim serves what does
not fit in HBM from pinned host memory (the reference switches *all* allocations to CUDA
managed memory instead).

Modes:
* resident      the same vGPU, dataset small enough to stay in HBM (the no-spill baseline);
* vdm           dataset of --dataset-gib (> HBM), default placement (large-first);
* policy study  at a reduced HBM share (--study-hbm-gib, default 160) so that first-come
                never fills the physical HBM: large-first vs first-come on the same data.

    python benchmarks/oversubscribe.py [--dataset-gib 300] [--steps 10] [--json-out F] [--md-out F]
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
GiB = 1 << 30


def worker(case, dataset_gib, steps, warmup, out):
    import torch
    from amdvgpu.models.aibench import Runner, get_case
    from amdvgpu.shim.region import Region
    torch.backends.cudnn.benchmark = True
    free, total = torch.cuda.mem_get_info(0)
    t0 = time.perf_counter()
    chunks = []
    for _ in range(dataset_gib):
        chunks.append(torch.empty(GiB // 4, dtype=torch.float32, device="cuda").normal_())
    torch.cuda.synchronize()
    fill_s = time.perf_counter() - t0
    r = Runner(get_case(case), "cuda:0", dtype=torch.float32)
    per = r.x.numel()
    per_chunk = (GiB // 4) // per

    def batch(i):
        c = chunks[(i * 37) % len(chunks)]
        k = (i // len(chunks)) % per_chunk
        return c[k * per:(k + 1) * per].view_as(r.x)

    for i in range(warmup):
        r.x = batch(i)
        r.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        r.x = batch(warmup + i)
        loss = r.step().item()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1000 / steps
    dev = Region(os.environ["VGPU_SHARED_CACHE"]).device(0)
    json.dump({"case": case, "quota_seen": total, "dataset_gib": dataset_gib, "fill_s": fill_s, "ms_per_batch": ms,
               "throughput": r.batch * 1000 / ms, "loss": loss, "spilled": dev["spilled"], "used": dev["used"],
               "hbm_limit": dev["hbm_limit"]}, open(out, "w"))


def run(env, case, dataset_gib, steps, warmup):
    fd, out = tempfile.mkstemp(suffix=".json")
    os.close(fd)
    try:
        subprocess.check_call([sys.executable, os.path.abspath(__file__), "--worker", "--case", case, "--dataset-gib",
                               str(dataset_gib), "--steps", str(steps), "--warmup", str(warmup), "--out", out],
                              env=env)
        return json.load(open(out))
    finally:
        os.unlink(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dataset-gib", type=int, default=300)
    ap.add_argument("--resident-gib", type=int, default=16)
    ap.add_argument("--study-hbm-gib", type=int, default=160)
    ap.add_argument("--study-dataset-gib", type=int, default=200)
    ap.add_argument("--memory-scaling", type=float, default=1.12)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--modes", default="resident,vdm,large-first,first-come")
    ap.add_argument("--case", default="lstm-train", help="config-4 workload (resident / vdm rows)")
    ap.add_argument("--study-cases", default="lstm-train,resnet50-train", help="workloads of the policy study")
    ap.add_argument("--worker", action="store_true")
    ap.add_argument("--out")
    ap.add_argument("--json-out")
    ap.add_argument("--md-out")
    a = ap.parse_args()
    if a.worker:
        return worker(a.case, a.dataset_gib, a.steps, a.warmup, a.out)
    from amdvgpu.plugin.devices import SysfsBackend
    from amdvgpu.plugin.kubelet_stub import NodeHarness
    from amdvgpu.shim.launcher import apply_contract
    backend = SysfsBackend()
    uuid = backend.devices()[0].uuid
    rows = []
    with NodeHarness(backend, device_split_count=1, device_memory_scaling=a.memory_scaling) as node:
        plan = [(m, a.case) for m in a.modes.split(",") if m in ("resident", "vdm")]
        plan += [(m, c) for c in a.study_cases.split(",") for m in ("resident", "large-first", "first-come")
                 if m in a.modes.split(",") and (m != "resident" or c != a.case)]
        for mode, case in plan:
            envs, mounts = node.pod(node.vgpu_ids(uuid)[:1])
            env = apply_contract(envs, mounts)
            data = {"resident": a.resident_gib, "vdm": a.dataset_gib}.get(mode, a.study_dataset_gib)
            if mode in ("large-first", "first-come"):
                env["VGPU_DEVICE_HBM_LIMIT_0"] = f"{a.study_hbm_gib * 1024}m"
                env["VGPU_SPILL_POLICY"] = mode
            steps = a.steps if mode != "first-come" else max(2, a.steps // 5)
            r = run(env, case, data, steps, a.warmup if mode != "first-come" else 1)
            r.update(mode=mode, quota_mib=int(envs["VGPU_DEVICE_MEMORY_LIMIT_0"].rstrip("m")),
                     contract_hbm_mib=int(envs.get("VGPU_DEVICE_HBM_LIMIT_0", "0").rstrip("m") or 0),
                     policy=env.get("VGPU_SPILL_POLICY", "large-first"))
            rows.append(r)
            print(json.dumps(r), flush=True)
    base = {r["case"]: r["ms_per_batch"] for r in rows if r["mode"] == "resident"}
    md = ["# Virtual device memory: stock fp32 training on a device-resident dataset (quota 322 GiB > 288 GiB HBM)",
          "", "| case | mode | policy | HBM share GiB | dataset GiB | spilled GiB | ms/batch | vs resident |",
          "|---|---|---|---|---|---|---|---|"]
    for r in rows:
        rel = f"{r['ms_per_batch'] / base[r['case']]:.2f}x" if r["case"] in base else "-"
        md.append(f"| {r['case']} | {r['mode']} | {r['policy']} | {r['hbm_limit'] / GiB:.0f} | {r['dataset_gib']} | "
                  f"{r['spilled'] / GiB:.1f} | {r['ms_per_batch']:.1f} | {rel} |")
    print("\n".join(md))
    if a.json_out:
        json.dump(rows, open(a.json_out, "w"), indent=1)
    if a.md_out:
        open(a.md_out, "w").write("\n".join(md) + "\n")


if __name__ == "__main__":
    main()
