#!/usr/bin/env python3
"""Does --numa-spread cost a CPU-heavy tenant?

The shim's NUMA spread (native/src/shim/numa_spread.cpp) narrows a shared-pool container's
processes to its vGPU's CPU socket before main(). Launch-bound pods gain from it
(profiles/r5k); this measures what a pod that needs the CPU pays: stock ResNet-50 training
fed by a PyTorch DataLoader whose workers decode JPEGs on the CPU (PIL decode, random crop +
resize, flip - an ImageNet-style input pipeline; normalisation on the GPU), in a quota-only
vGPU with VGPU_CPU_NODE set, spread on vs off, alternating (ABAB...) in fresh processes.

Reported per run: images/s of the whole training loop, the CPUs the tenant may use (affinity)
and its cgroup CPU quota, the CPU seconds per second its loader workers burned, and once the
GPU-only rate (the same model on a resident batch) so the reader sees whether the loader is
the bound.

    python3 benchmarks/dataloader_spread.py --workers 8 --repeats 2 --json-out r.json

Synthetic data: random-content JPEGs encoded once per process; random-init weights.
"""
import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def _gpu_node():
    try:
        from amdvgpu.plugin.devices import SysfsBackend
        bdf = SysfsBackend().devices()[0].bdf
        return max(0, int(open(f"/sys/bus/pci/devices/{bdf}/numa_node").read()))
    except Exception:  # noqa: BLE001
        return 0


def _cpu_quota():
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        return None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        return None


class Jpegs:
    """An endless dataset of ImageNet-like samples decoded from JPEG bytes on the CPU."""

    def __init__(self, n_blobs, width, height, crop, seed=0):
        import io

        import numpy as np
        from PIL import Image
        rng = np.random.default_rng(seed)
        self.blobs, self.crop = [], crop
        for _ in range(n_blobs):
            # smooth random content (a photo-like spectrum, not white noise) + some noise
            small = rng.integers(0, 256, (height // 16, width // 16, 3), dtype=np.uint8)
            img = Image.fromarray(small).resize((width, height), Image.BICUBIC)
            arr = np.asarray(img, dtype=np.int16) + rng.integers(-12, 13, (height, width, 3), dtype=np.int16)
            buf = io.BytesIO()
            Image.fromarray(np.clip(arr, 0, 255).astype(np.uint8)).save(buf, format="JPEG", quality=90)
            self.blobs.append(buf.getvalue())

    def __len__(self):
        return 1 << 30

    def __getitem__(self, i):
        import io
        import random

        import numpy as np
        import torch
        from PIL import Image
        img = Image.open(io.BytesIO(self.blobs[i % len(self.blobs)])).convert("RGB")
        w, h = img.size
        s = random.uniform(0.35, 1.0)
        cw, ch = int(w * s), int(h * s)
        x0, y0 = random.randint(0, w - cw), random.randint(0, h - ch)
        img = img.resize((self.crop, self.crop), Image.BILINEAR, box=(x0, y0, x0 + cw, y0 + ch))
        if random.random() < 0.5:
            img = img.transpose(Image.FLIP_LEFT_RIGHT)
        t = torch.from_numpy(np.array(img, dtype=np.uint8)).permute(2, 0, 1)
        return t, i % 1000


def child(a):
    import psutil
    import torch
    from torch.utils.data import DataLoader

    from amdvgpu.models.aibench import Runner, get_case
    me = psutil.Process()
    r = Runner(get_case("resnet50-train"), "cuda:0", batch=a.batch)
    mean = torch.tensor([0.485, 0.456, 0.406], device="cuda:0").view(1, 3, 1, 1) * 255
    std = torch.tensor([0.229, 0.224, 0.225], device="cuda:0").view(1, 3, 1, 1) * 255
    r.x = torch.randn(a.batch, 3, a.crop, a.crop, device="cuda:0").contiguous(memory_format=torch.channels_last)
    out = {"spread": os.environ.get("VGPU_CPU_SPREAD"), "affinity": len(os.sched_getaffinity(0)),
           "cgroup_cpus": _cpu_quota()}
    if a.gpu_only:
        for _ in range(5):
            r.step()
        torch.cuda.synchronize()
        n, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < a.seconds / 2:
            r.step()
            n += 1
        torch.cuda.synchronize()
        out["gpu_only_img_s"] = round(n * a.batch / (time.perf_counter() - t0), 1)
    ds = Jpegs(32, a.width, a.height, a.crop)
    dl = DataLoader(ds, batch_size=a.batch, num_workers=a.workers, pin_memory=True, persistent_workers=True,
                    prefetch_factor=4, shuffle=False)
    it = iter(dl)

    def step():
        xb, yb = next(it)
        x = ((xb.to("cuda:0", non_blocking=True).float() - mean) / std).contiguous(memory_format=torch.channels_last)
        r.x, r.y = x, yb.to("cuda:0", non_blocking=True)
        r.step()

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    kids = me.children(recursive=True)
    out["worker_affinity"] = sorted({len(k.cpu_affinity()) for k in kids}) if kids else []
    c0 = sum(sum(k.cpu_times()[:2]) for k in kids)
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < a.seconds:
        step()
        n += 1
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    c1 = sum(sum(k.cpu_times()[:2]) for k in kids)
    out.update(img_s=round(n * a.batch / dt, 1), steps=n, loader_cpus_busy=round((c1 - c0) / dt, 2))
    print("RESULT " + json.dumps(out), flush=True)
    del it, dl
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--crop", type=int, default=224)
    ap.add_argument("--width", type=int, default=800)
    ap.add_argument("--height", type=int, default=600)
    ap.add_argument("--seconds", type=float, default=15.0)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--repeats", type=int, default=2)
    ap.add_argument("--child", action="store_true")
    ap.add_argument("--gpu-only", action="store_true")
    ap.add_argument("--json-out", default="")
    a = ap.parse_args()
    if a.child:
        return child(a)
    from amdvgpu.shim.launcher import apply_contract, cleanup_region, vgpu_env
    node = _gpu_node()
    base = [sys.executable, os.path.abspath(__file__), "--child", "--workers", str(a.workers), "--batch", str(a.batch),
            "--crop", str(a.crop), "--width", str(a.width), "--height", str(a.height), "--seconds", str(a.seconds),
            "--warmup", str(a.warmup)]
    runs = []
    order = [m for _ in range(a.repeats) for m in ("1", "0")]
    for k, spread in enumerate(order):
        env = apply_contract(vgpu_env(mem_limit=64 << 30, extra={"VGPU_CPU_NODE": str(node), "VGPU_CPU_SPREAD": spread}))
        cmd = base + (["--gpu-only"] if k < 2 else [])
        t0 = time.time()
        p = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, text=True, timeout=900)
        cleanup_region(env)
        lines = [ln for ln in p.stdout.splitlines() if ln.startswith("RESULT ")]
        if p.returncode != 0 or not lines:
            print(f"run {k} (spread={spread}) failed rc={p.returncode}", file=sys.stderr)
            return 1
        res = json.loads(lines[-1][len("RESULT "):])
        res["wall_s"] = round(time.time() - t0, 1)
        runs.append(res)
        print(json.dumps(res), flush=True)

    def med(spread):
        xs = sorted(r["img_s"] for r in runs if r["spread"] == spread)
        return xs[len(xs) // 2] if len(xs) % 2 else (xs[len(xs) // 2 - 1] + xs[len(xs) // 2]) / 2
    summary = {"gpu_numa_node": node, "workers": a.workers, "batch": a.batch,
               "jpeg": f"{a.width}x{a.height}", "crop": a.crop,
               "spread_img_s": med("1"), "nospread_img_s": med("0"),
               "spread_vs_nospread": round(med("1") / med("0"), 4), "runs": runs}
    print(json.dumps({k: v for k, v in summary.items() if k != "runs"}), flush=True)
    if a.json_out:
        with open(a.json_out, "w") as f:
            json.dump(summary, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
