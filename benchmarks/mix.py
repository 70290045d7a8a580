#!/usr/bin/env python3
"""Heterogeneous tenants on one MI355X: isolation and inference latency next to trainers.

Every sweep before this one ran N copies of one model. Here different ai-benchmark cases
share one GPU, each in its own vGPU of a split-N plugin (default --cu-mode auto), the way
a real node is shared: a small-batch inference service next to training jobs.

For every pod the benchmark reports
  * its throughput when alone in its vGPU ("solo at share": the same contract, so the
    same CU share / quota, with the GPU otherwise idle) and when all pods run together;
    ``vs_entitlement`` = together / solo-at-share (>= 0.9 means the neighbours did not
    take what the pod is entitled to);
  * for latency pods (``:lat``), the P50 / P99 step latency (one synchronised step per
    request), alone and together.
Optionally a second concurrent run with task priorities (``--priority``: e.g.
``resnet50-inf:1:lat=0,vgg16-train=2``) shows what VGPU_TASK_PRIORITY buys the latency pod.

Pods are given as CASE[:BATCH][:lat], e.g. the default
    resnet50-inf:1:lat vgg16-train lstm-train deeplab-inf
Every contract comes from an Allocate of the plugin (NodeHarness, sysfs backend).

    python benchmarks/mix.py [--pods ...] [--seconds 8] [--priority SPEC] [--json-out F] [--md-out F]
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

DEFAULT_PODS = ["resnet50-inf:1:lat", "vgg16-train", "lstm-train", "deeplab-inf"]


def parse_pod(spec):
    parts = spec.split(":")
    case, batch, lat = parts[0], None, False
    for p in parts[1:]:
        if p == "lat":
            lat = True
        elif p:
            batch = int(p)
    return {"spec": spec, "case": case, "batch": batch, "latency": lat}


def worker(a):
    import torch
    from amdvgpu.models.aibench import Runner, get_case
    torch.backends.cudnn.benchmark = True
    case = get_case(a.case)
    r = Runner(case, "cuda:0", batch=a.batch or None)
    for _ in range(a.warmup):
        r.step()
    torch.cuda.synchronize()
    open(a.out + ".ready", "w").close()
    while not os.path.exists(a.go):
        time.sleep(0.005)
    lat = []
    n = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < a.seconds:
        s = time.perf_counter()
        r.step()
        n += 1
        if a.latency:
            torch.cuda.synchronize()
            lat.append(time.perf_counter() - s)
        elif n % 2 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    res = {"steps": n, "items": r.batch * n, "t0": t0, "t1": t1, "throughput": r.batch * n / (t1 - t0)}
    if lat:
        lat.sort()
        res["p50_ms"] = 1000 * lat[len(lat) // 2]
        res["p99_ms"] = 1000 * lat[min(len(lat) - 1, int(len(lat) * 0.99))]
        res["mean_ms"] = 1000 * sum(lat) / len(lat)
    json.dump(res, open(a.out, "w"))
    return 0


def run_pods(node, uuid, pods, ids, seconds, warmup, priorities=None):
    """Starts one worker per pod (pods[i] in vGPU ids[i]), releases them together."""
    from amdvgpu.shim.launcher import apply_contract
    tmp = tempfile.mkdtemp(prefix="mix-")
    go = os.path.join(tmp, "go")
    procs, outs = [], []
    for i, (pod, vid) in enumerate(zip(pods, ids)):
        envs, mounts = node.pod([vid])
        env = apply_contract(envs, mounts)
        if priorities and priorities.get(pod["spec"]) is not None:
            env["VGPU_TASK_PRIORITY"] = str(priorities[pod["spec"]])
        out = os.path.join(tmp, f"p{i}.json")
        cmd = [sys.executable, os.path.abspath(__file__), "--worker", "--case", pod["case"], "--batch",
               str(pod["batch"] or 0), "--seconds", str(seconds), "--warmup", str(warmup), "--out", out, "--go", go]
        if pod["latency"]:
            cmd.append("--latency")
        procs.append(subprocess.Popen(cmd, env=env))
        outs.append(out)
    try:
        deadline = time.time() + 900
        while not all(os.path.exists(o + ".ready") for o in outs):
            if any(p.poll() not in (None, 0) for p in procs) or time.time() > deadline:
                raise SystemExit("a pod failed before the start barrier")
            time.sleep(0.05)
        open(go, "w").close()
        for p in procs:
            if p.wait(timeout=900) != 0:
                raise SystemExit("a pod failed")
        return [json.load(open(o)) for o in outs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--pods", nargs="+", default=DEFAULT_PODS)
    ap.add_argument("--split", type=int, default=0, help="vGPUs per GPU (default: one per pod)")
    ap.add_argument("--cu-mode", default="auto")
    ap.add_argument("--seconds", type=float, default=8.0)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--priority", default="", help="SPEC=PRIO,...: a second concurrent run with these priorities")
    ap.add_argument("--json-out")
    ap.add_argument("--md-out")
    ap.add_argument("--worker", action="store_true")
    ap.add_argument("--case")
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--latency", action="store_true")
    ap.add_argument("--out")
    ap.add_argument("--go")
    a = ap.parse_args()
    if a.worker:
        return worker(a)
    from amdvgpu.plugin.devices import SysfsBackend
    from amdvgpu.plugin.kubelet_stub import NodeHarness
    pods = [parse_pod(s) for s in a.pods]
    backend = SysfsBackend()
    uuid = backend.devices()[0].uuid
    split = a.split or len(pods)
    prio = {}
    for item in filter(None, a.priority.split(",")):
        k, _, v = item.rpartition("=")
        prio[k] = int(v)
    out = {"pods": [p["spec"] for p in pods], "split": split, "cu_mode": a.cu_mode, "seconds": a.seconds,
           "solo": [], "together": None, "together_priority": None, "priorities": prio or None}
    with NodeHarness(backend, device_split_count=split, cu_mode=a.cu_mode) as node:
        ids = node.vgpu_ids(uuid)[:len(pods)]
        for pod, vid in zip(pods, ids):
            t = time.time()
            out["solo"].append(run_pods(node, uuid, [pod], [vid], a.seconds, a.warmup)[0])
            print(f"[mix] solo {pod['spec']}: {out['solo'][-1]['throughput']:.1f}/s ({time.time() - t:.0f} s)",
                  file=sys.stderr, flush=True)
        out["together"] = run_pods(node, uuid, pods, ids, a.seconds, a.warmup)
        if prio:
            out["together_priority"] = run_pods(node, uuid, pods, ids, a.seconds, a.warmup, prio)
    rows = []
    for i, pod in enumerate(pods):
        solo, tog = out["solo"][i], out["together"][i]
        row = {"pod": pod["spec"], "solo": round(solo["throughput"], 2), "together": round(tog["throughput"], 2),
               "vs_entitlement": round(tog["throughput"] / solo["throughput"], 3)}
        if pod["latency"]:
            row.update(solo_p50_ms=round(solo["p50_ms"], 3), solo_p99_ms=round(solo["p99_ms"], 3),
                       p50_ms=round(tog["p50_ms"], 3), p99_ms=round(tog["p99_ms"], 3))
        if out["together_priority"]:
            tp = out["together_priority"][i]
            row["prio"] = prio.get(pod["spec"], 1)
            row["together_prio"] = round(tp["throughput"], 2)
            row["vs_entitlement_prio"] = round(tp["throughput"] / solo["throughput"], 3)
            if pod["latency"]:
                row.update(prio_p50_ms=round(tp["p50_ms"], 3), prio_p99_ms=round(tp["p99_ms"], 3))
        rows.append(row)
    out["rows"] = rows
    out["min_vs_entitlement"] = min(r["vs_entitlement"] for r in rows)
    md = [f"# heterogeneous pods on one MI355X (split {split}, --cu-mode {a.cu_mode}, {a.seconds:.0f} s windows)", "",
          "| pod | solo at share | together | vs entitlement | P50 / P99 ms solo | P50 / P99 ms together |"
          + (" priority | together (prio) | vs entitlement (prio) | P50 / P99 ms (prio) |" if prio else ""),
          "|---|---|---|---|---|---|" + ("---|---|---|---|" if prio else "")]
    for r in rows:
        lat_s = f"{r['solo_p50_ms']:.2f} / {r['solo_p99_ms']:.2f}" if "p50_ms" in r else "-"
        lat_t = f"{r['p50_ms']:.2f} / {r['p99_ms']:.2f}" if "p50_ms" in r else "-"
        line = f"| {r['pod']} | {r['solo']:.1f} | {r['together']:.1f} | {r['vs_entitlement']:.2f} | {lat_s} | {lat_t} |"
        if prio:
            lat_p = f"{r['prio_p50_ms']:.2f} / {r['prio_p99_ms']:.2f}" if "prio_p50_ms" in r else "-"
            line += f" {r['prio']} | {r['together_prio']:.1f} | {r['vs_entitlement_prio']:.2f} | {lat_p} |"
        md.append(line)
    text = "\n".join(md)
    print(text)
    print(json.dumps({k: v for k, v in out.items() if k in ("pods", "split", "min_vs_entitlement", "rows")}))
    if a.json_out:
        json.dump(out, open(a.json_out, "w"), indent=1)
    if a.md_out:
        open(a.md_out, "w").write(text + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
