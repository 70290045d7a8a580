#!/usr/bin/env python3
"""Heterogeneous tenants on one MI355X: isolation and inference latency next to trainers.

Every sweep before this one ran N copies of one model. Here different ai-benchmark cases
share one GPU, each in its own vGPU of a split-N plugin (default --cu-mode auto), the way
a real node is shared: a small-batch inference service next to training jobs.

For every pod the benchmark reports
  * its throughput alone in its vGPU, under both enforcements auto mode uses: "solo
    spatial" (the GPU otherwise idle: its CU slice, all the time) and "solo temporal"
    (its share of the GPU's time on all CUs: what it is entitled to on a crowded GPU);
  * its throughput when all pods run together; ``vs_entitlement`` = together / solo
    temporal (>= 0.9: the neighbours did not take GPU time that is the pod's);
  * for latency pods (``:lat``), the P50 / P99 request latency alone and together.
    Requests arrive as a Poisson stream (``:rate=R`` per second, default 100; latency
    counts from arrival, queueing included), so the pod idles between bursts as a service
    does.
Optionally a further concurrent run with task priorities (``--priority``: e.g.
``resnet50-inf:1:lat=0,vgg16-train=2``) shows what VGPU_TASK_PRIORITY buys the latency pod:
priority 0 keeps its CU slice however crowded the GPU, priority >= 2 (background) yields
GPU time while a higher-priority pod is busy (the node-wide board, vgpu/board.h).

Pods are given as CASE[:BATCH][:lat][:rate=R][:nolimit] (nolimit: the pod has no compute
share, memory quota only), e.g. the default
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
    case, batch, lat, rate, nolimit = parts[0], None, False, 100.0, False
    for p in parts[1:]:
        if p == "lat":
            lat = True
        elif p == "nolimit":
            nolimit = True
        elif p.startswith("rate="):
            rate = float(p[5:])
        elif p:
            batch = int(p)
    return {"spec": spec, "case": case, "batch": batch, "latency": lat, "rate": rate, "nolimit": nolimit}


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
    import random
    rng = random.Random(1234)
    lat, gpu = [], []
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 0
    t0 = time.perf_counter()
    arrival = t0
    while time.perf_counter() - t0 < a.seconds:
        if a.latency:
            # Poisson arrivals; a request that arrived while the previous one ran waits.
            arrival += rng.expovariate(a.rate)
            now = time.perf_counter()
            if arrival > now:
                time.sleep(arrival - now)
            ev0.record()
            r.step()
            ev1.record()
            torch.cuda.synchronize()
            lat.append(time.perf_counter() - arrival)
            gpu.append(ev0.elapsed_time(ev1))  # the request on the GPU: its kernels and the gaps between them
        else:
            r.step()
            if n % 2 == 1:
                torch.cuda.synchronize()
        n += 1
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    res = {"steps": n, "items": r.batch * n, "t0": t0, "t1": t1, "throughput": r.batch * n / (t1 - t0)}
    if lat:
        lat.sort()
        res["p50_ms"] = 1000 * lat[len(lat) // 2]
        res["p99_ms"] = 1000 * lat[min(len(lat) - 1, int(len(lat) * 0.99))]
        res["mean_ms"] = 1000 * sum(lat) / len(lat)
        gpu.sort()
        res["gpu_p50_ms"] = gpu[len(gpu) // 2]
        res["gpu_p99_ms"] = gpu[min(len(gpu) - 1, int(len(gpu) * 0.99))]
    json.dump(res, open(a.out, "w"))
    return 0


def run_pods(node, uuid, pods, ids, seconds, warmup, priorities=None, pod_env=None, bg_env=None, trace=None):
    """Starts one worker per pod (pods[i] in vGPU ids[i]), releases them together.
    ``bg_env`` is added to the pods whose priority is background (>= 2)."""
    from amdvgpu.shim.launcher import apply_contract
    tmp = tempfile.mkdtemp(prefix="mix-")
    go = os.path.join(tmp, "go")
    procs, outs = [], []
    for i, (pod, vid) in enumerate(zip(pods, ids)):
        envs, mounts = node.pod([vid])
        env = apply_contract(envs, mounts)
        if pod["nolimit"]:  # no compute share (memory quota only): the whole GPU, unless a class rule applies
            for k in [k for k in env if k.startswith("VGPU_DEVICE_CU_LIMIT") or k.startswith("VGPU_DEVICE_CU_RANGE")]:
                del env[k]
        if priorities and priorities.get(pod["spec"]) is not None:
            env["VGPU_TASK_PRIORITY"] = str(priorities[pod["spec"]])
            if priorities[pod["spec"]] >= 2:
                env.update(bg_env or {})
        env.update(pod_env or {})
        out = os.path.join(tmp, f"p{i}.json")
        cmd = [sys.executable, os.path.abspath(__file__), "--worker", "--case", pod["case"], "--batch",
               str(pod["batch"] or 0), "--seconds", str(seconds), "--warmup", str(warmup), "--out", out, "--go", go]
        if pod["latency"]:
            cmd += ["--latency", "--rate", str(pod["rate"])]
            if trace:  # kernel trace of the latency pod (rocprofv3 starts the worker as its child)
                os.makedirs(trace, exist_ok=True)
                cmd = ["rocprofv3", "--kernel-trace", "--stats", "--output-format", "csv", "-d", trace, "-o", "lat",
                       "--"] + cmd
        procs.append(subprocess.Popen(cmd, env=env))
        outs.append(out)
    try:
        deadline = time.time() + 900
        while not all(os.path.exists(o + ".ready") for o in outs):
            if any(p.poll() not in (None, 0) for p in procs) or time.time() > deadline:
                raise SystemExit("a pod failed before the start barrier")
            time.sleep(0.05)
        open(go, "w").close()
        end = time.time() + seconds + 240  # the timed window, then the pods' exit (a profiler may hang there)
        for p in procs:
            if p.wait(timeout=max(1.0, end - time.time())) != 0:
                raise SystemExit("a pod failed")
        return [json.load(open(o)) for o in outs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()


def ab_compare(a, pods, backend, uuid, split, prio):
    """ABAB runs of all pods together, without (A) and with (B) the priorities."""
    from amdvgpu.plugin.kubelet_stub import NodeHarness
    runs = []
    # The operator grants the latency class here (--allow-latency-class): the pods choose theirs.
    with NodeHarness(backend, device_split_count=split, cu_mode=a.cu_mode, allow_latency_class=True,
                     **({} if a.gpu_concurrency is None else {"gpu_concurrency": a.gpu_concurrency})) as node:
        ids = node.vgpu_ids(uuid)[:len(pods)]
        arms = ([] if a.skip_default else [("default", None, None)]) + [("priority", prio, None)]
        for bg in a.bg_env:
            arms.append(("priority+" + " ".join(f"{k}={v}" for k, v in bg.items()), prio, bg))
        for i in range(a.ab):
            for label, pr, bg in arms:
                trace = os.path.join(a.trace_latency, f"{label}_{i}") if a.trace_latency else None
                res = run_pods(node, uuid, pods, ids, a.seconds, a.warmup, pr, bg_env=bg, trace=trace)
                row = {"run": i, "label": label}
                for pod, r in zip(pods, res):
                    row[pod["spec"]] = {k: round(v, 3) for k, v in r.items()
                                        if k in ("throughput", "p50_ms", "p99_ms", "mean_ms")}
                runs.append(row)
                print(json.dumps(row), flush=True)
    md = [f"# default vs priority classes, ABAB x{a.ab} ({a.seconds:.0f} s windows, split {split}"
          + "".join(f"; bg env {bg}" for bg in a.bg_env) + ")", "",
          "| run | " + " | ".join(p["spec"] + (" P50 / P99 ms (on the GPU P50 / P99)" if p["latency"] else " /s")
                                  for p in pods) + " |",
          "|---|" + "---|" * len(pods)]
    for r in runs:
        cells = []
        for p in pods:
            v = r[p["spec"]]
            cells.append(f"{v['p50_ms']:.2f} / {v['p99_ms']:.2f} ({v.get('gpu_p50_ms', 0):.2f} / {v.get('gpu_p99_ms', 0):.2f})"
                         if p["latency"] else f"{v['throughput']:.1f}")
        md.append(f"| {r['label']} #{r['run']} | " + " | ".join(cells) + " |")
    for label, _, _ in arms:
        sel = [r for r in runs if r["label"] == label]
        cells = []
        for p in pods:
            if p["latency"]:
                vals = sorted(r[p["spec"]]["p99_ms"] for r in sel)
                cells.append(f"median P99 {vals[len(vals) // 2]:.2f}")
            else:
                vals = sorted(r[p["spec"]]["throughput"] for r in sel)
                cells.append(f"median {vals[len(vals) // 2]:.1f}")
        md.append(f"| **{label}** | " + " | ".join(cells) + " |")
    text = "\n".join(md)
    print(text)
    if a.json_out:
        json.dump({"pods": [p["spec"] for p in pods], "priorities": prio, "bg_env": a.bg_env, "runs": runs}, open(a.json_out, "w"), indent=1)
    if a.md_out:
        open(a.md_out, "w").write(text + "\n")
    return 0


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--pods", nargs="+", default=DEFAULT_PODS)
    ap.add_argument("--split", type=int, default=0, help="vGPUs per GPU (default: one per pod)")
    ap.add_argument("--cu-mode", default="auto")
    ap.add_argument("--seconds", type=float, default=8.0)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--priority", default="", help="SPEC=PRIO,...: a second concurrent run with these priorities")
    ap.add_argument("--ab", type=int, default=0,
                    help="skip the solo runs; alternate N times between the default and the --priority run "
                         "(ABAB...) and report each run's latency-pod P50 / P99 and pod throughputs")
    ap.add_argument("--bg-env", action="append", default=[],
                    help="K=V,...: with --ab, one more arm where the background pods (priority >= 2) also get "
                         "this env (repeatable: one arm each)")
    ap.add_argument("--skip-default", action="store_true", help="with --ab: no arm without priorities")
    ap.add_argument("--trace-latency", default="", help="with --ab: rocprofv3 kernel trace of the latency pods "
                                                          "under DIR/<arm>_<run>")
    ap.add_argument("--gpu-concurrency", type=lambda v: -1 if v == "auto" else int(v), default=None,
                    help="the plugin's --gpu-concurrency for every pod (default: the plugin's own, auto)")
    ap.add_argument("--json-out")
    ap.add_argument("--md-out")
    ap.add_argument("--worker", action="store_true")
    ap.add_argument("--case")
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--latency", action="store_true")
    ap.add_argument("--rate", type=float, default=100.0)
    ap.add_argument("--out")
    ap.add_argument("--go")
    a = ap.parse_args()
    a.bg_env = [dict(kv.split("=", 1) for kv in spec.split(",") if kv) for spec in a.bg_env]
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
           "solo": [], "solo_spatial": [], "together": None, "together_priority": None, "priorities": prio or None}
    if a.ab:
        return ab_compare(a, pods, backend, uuid, split, prio)
    # The operator grants the latency class here (--allow-latency-class): the pods choose theirs.
    with NodeHarness(backend, device_split_count=split, cu_mode=a.cu_mode, allow_latency_class=True,
                     **({} if a.gpu_concurrency is None else {"gpu_concurrency": a.gpu_concurrency})) as node:
        ids = node.vgpu_ids(uuid)[:len(pods)]
        for pod, vid in zip(pods, ids):
            t = time.time()
            out["solo_spatial"].append(run_pods(node, uuid, [pod], [vid], a.seconds, a.warmup)[0])
            out["solo"].append(run_pods(node, uuid, [pod], [vid], a.seconds, a.warmup,
                                        pod_env={"VGPU_CU_MODE": "temporal"})[0])
            print(f"[mix] solo {pod['spec']}: {out['solo_spatial'][-1]['throughput']:.1f}/s spatial, "
                  f"{out['solo'][-1]['throughput']:.1f}/s temporal ({time.time() - t:.0f} s)",
                  file=sys.stderr, flush=True)
        out["together"] = run_pods(node, uuid, pods, ids, a.seconds, a.warmup)
        if prio:
            out["together_priority"] = run_pods(node, uuid, pods, ids, a.seconds, a.warmup, prio)
    rows = []
    for i, pod in enumerate(pods):
        solo, tog, sp = out["solo"][i], out["together"][i], out["solo_spatial"][i]
        row = {"pod": pod["spec"], "solo_spatial": round(sp["throughput"], 2), "solo": round(solo["throughput"], 2),
               "together": round(tog["throughput"], 2),
               "vs_entitlement": round(tog["throughput"] / solo["throughput"], 3)}
        if pod["latency"]:
            row.update(solo_spatial_p99_ms=round(sp["p99_ms"], 3), solo_p50_ms=round(solo["p50_ms"], 3),
                       solo_p99_ms=round(solo["p99_ms"], 3), p50_ms=round(tog["p50_ms"], 3),
                       p99_ms=round(tog["p99_ms"], 3))
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
          "| pod | solo spatial | solo temporal (entitlement) | together | vs entitlement | P99 ms solo spatial | "
          "P50 / P99 ms solo temporal | P50 / P99 ms together |"
          + (" priority | together (prio) | vs entitlement (prio) | P50 / P99 ms (prio) |" if prio else ""),
          "|---|---|---|---|---|---|---|---|" + ("---|---|---|---|" if prio else "")]
    for r in rows:
        lat_sp = f"{r['solo_spatial_p99_ms']:.2f}" if "p50_ms" in r else "-"
        lat_s = f"{r['solo_p50_ms']:.2f} / {r['solo_p99_ms']:.2f}" if "p50_ms" in r else "-"
        lat_t = f"{r['p50_ms']:.2f} / {r['p99_ms']:.2f}" if "p50_ms" in r else "-"
        line = (f"| {r['pod']} | {r['solo_spatial']:.1f} | {r['solo']:.1f} | {r['together']:.1f} | "
                f"{r['vs_entitlement']:.2f} | {lat_sp} | {lat_s} | {lat_t} |")
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
