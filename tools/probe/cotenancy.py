#!/usr/bin/env python3
"""Do two launch-bound processes' kernels ever run at the same time on one MI355X?

Round 4 measured two unmasked LSTM inference processes at 1.00x aggregate (profiles/r4h)
where round 2 had 1.78x, and asserted "the box" without evidence. This probe runs N stock
PyTorch tenants of one case side by side (no shim, no mask), each timing its own steps, for
a rocprofv3 kernel trace of all of them; --analyze then reads the per-process kernel traces
and reports, over the window in which all of them run:

    busy        fraction of the window each process has a kernel executing
    both        fraction in which kernels of every process execute at once (true overlap)
    any         fraction in which some kernel executes (the GPU's busy time)
    gap_us      each process's gaps between consecutive kernels (median / p90 / p99): how
                long its queue stays empty while the other one runs
    long_gap_share  the share of the window each process spends in gaps of >= 100 us

If `both` stays ~0 while each process's gaps are as long as the other's bursts, the GPU
time-slices the processes' queues (the hardware scheduler switching between process
contexts) rather than running their kernels concurrently.

    python3 tools/probe/cotenancy.py --case lstm-inf --procs 2 --seconds 4 --trace OUT
    python3 tools/probe/cotenancy.py --analyze OUT

--trace runs every tenant under its own rocprofv3 (--kernel-trace, csv, OUT/t<i>): the
launcher itself never loads the GPU runtime, and each tenant's trace lands in a directory of
its own (rocprofv3's timestamps share one clock across the processes of a host).
"""
import argparse
import csv
import glob
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)


def _cpu_limit():
    """The CPUs this process may use: (affinity count, cgroup cpu.max quota in CPUs or None)."""
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        quota = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return len(os.sched_getaffinity(0)), quota


def _numa_nodes():
    """NUMA node -> the CPUs of it this process may use."""
    allowed = os.sched_getaffinity(0)
    out = {}
    for d in glob.glob("/sys/devices/system/node/node[0-9]*"):
        try:
            cpus = set()
            for part in open(os.path.join(d, "cpulist")).read().strip().split(","):
                lo, _, hi = part.partition("-")
                if lo:
                    cpus.update(range(int(lo), int(hi or lo) + 1))
            out[int(os.path.basename(d)[4:])] = sorted(cpus & allowed)
        except (OSError, ValueError):
            pass
    return out


def _gpu_node():
    """The NUMA node of the GPU this job sees (sysfs backend), -1 if unknown."""
    try:
        from amdvgpu.plugin.devices import SysfsBackend
        bdf = SysfsBackend().devices()[0].bdf
        return int(open(f"/sys/bus/pci/devices/{bdf}/numa_node").read())
    except Exception:  # noqa: BLE001
        return -1


def _where():
    """The CPU the calling thread ran on last, and that CPU's NUMA node."""
    try:
        st = open("/proc/thread-self/stat").read()
        cpu = int(st[st.rindex(")") + 2:].split()[36])
    except (OSError, ValueError, IndexError):
        return -1, -1
    node = next((n for n, cs in _numa_nodes().items() if cpu in cs), -1)
    return cpu, node


def _bind_memory(node):
    """set_mempolicy(MPOL_BIND, {node}) for this process (before the runtime allocates)."""
    import ctypes
    libc = ctypes.CDLL(None, use_errno=True)
    mask = ctypes.c_ulong(1 << node)
    if libc.syscall(238, 2, ctypes.byref(mask), ctypes.c_ulong(64 + 1)) != 0:   # SYS_set_mempolicy, MPOL_BIND
        raise OSError(ctypes.get_errno(), "set_mempolicy")


def tenant(case, seconds, go, batch, cpus, mem_node=-1):
    if cpus:
        os.sched_setaffinity(0, {int(c) for c in cpus.split(",")})
    if mem_node >= 0:
        _bind_memory(mem_node)
    import resource

    import torch
    from amdvgpu.models.aibench import Runner, get_case
    torch.backends.cudnn.benchmark = True
    r = Runner(get_case(case), "cuda:0", dtype=torch.float32, batch=batch or None)
    for _ in range(5):
        r.step()
    torch.cuda.synchronize()
    open(go + f".ready.{os.getpid()}", "w").close()
    while not os.path.exists(go):
        time.sleep(0.001)
    ru0, c0 = resource.getrusage(resource.RUSAGE_SELF), time.thread_time()
    n, t0 = 0, time.perf_counter()
    seen = {}   # NUMA nodes the main thread ran on, sampled every 8 steps
    while time.perf_counter() - t0 < seconds:
        r.step()
        n += 1
        if n % 4 == 0:
            torch.cuda.synchronize()
        if n % 8 == 0:
            node = _where()[1]
            seen[node] = seen.get(node, 0) + 1
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    ru1, c1 = resource.getrusage(resource.RUSAGE_SELF), time.thread_time()
    aff, quota = _cpu_limit()
    print(json.dumps({"pid": os.getpid(), "case": case, "steps": n, "ms_per_step": round(dt * 1e3 / n, 3),
                      "items_per_s": round(n * r.items_per_step / dt, 1),
                      # CPU seconds per second of the window: all threads, and the main thread
                      "cpus_busy": round((ru1.ru_utime + ru1.ru_stime - ru0.ru_utime - ru0.ru_stime) / dt, 3),
                      "main_thread_busy": round((c1 - c0) / dt, 3),
                      "invol_ctx": ru1.ru_nivcsw - ru0.ru_nivcsw, "affinity": aff, "cgroup_cpus": quota,
                      "cpu_last": _where()[0], "numa_seen": seen}),
          flush=True)


def burner(go, seconds):
    """A CPU-only neighbour: spins one core for the window (no GPU)."""
    while not os.path.exists(go):
        time.sleep(0.001)
    t0 = time.perf_counter()
    x = 0
    while time.perf_counter() - t0 < seconds:
        x += 1


def launch(a):
    go = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"cotenancy-go-{os.getpid()}")
    args = [sys.executable, os.path.abspath(__file__), "--tenant", "--case", a.case, "--seconds", str(a.seconds),
            "--go", go] + (["--batch", str(a.batch)] if a.batch else [])
    allowed = sorted(os.sched_getaffinity(0))
    nodes, gnode = _numa_nodes(), _gpu_node()
    local = nodes.get(gnode, [])
    remote = [c for n, cs in sorted(nodes.items()) if n != gnode for c in cs]

    def cpus_of(i):
        """Tenant i's CPUs: --placement local / remote = disjoint slices of the GPU's NUMA node
        / of the other nodes; split = even tenants local, odd ones remote; none = --pin K of
        all allowed CPUs (or unpinned)."""
        k = max(1, a.pin or 4)
        if a.cpu_lists:   # explicit: "64-67;96-99" = tenant 0 on 64-67, tenant 1 on 96-99
            spec = a.cpu_lists.split(";")[i % len(a.cpu_lists.split(";"))]
            out = []
            for part in spec.split(","):
                lo, _, hi = part.partition("-")
                out += list(range(int(lo), int(hi or lo) + 1))
            return out
        if a.placement == "local":
            pool, j = local, i
        elif a.placement == "remote":
            pool, j = remote, i
        elif a.placement == "split":
            pool, j = (local if i % 2 == 0 else remote), i // 2
        elif a.pin:
            pool, j = allowed, i
        else:
            return []
        return pool[j * k:(j + 1) * k]

    def mem_of(i):
        """--mem local / remote / split: tenant i's host memory bound to that NUMA node."""
        if a.mem == "none" or gnode < 0:
            return -1
        other = next((n for n in sorted(nodes) if n != gnode), gnode)
        if a.mem == "local":
            return gnode
        if a.mem == "remote":
            return other
        return gnode if i % 2 == 0 else other

    def cmd(i):
        c = list(args)
        cs = cpus_of(i)
        if cs:
            c += ["--cpus", ",".join(str(x) for x in cs)]
        if mem_of(i) >= 0:
            c += ["--mem-node", str(mem_of(i))]
        if not a.trace:
            return c
        prof = ["rocprofv3", "--kernel-trace"] + (["--hip-trace"] if a.hip_stats else []) + \
            (["--hsa-trace"] if a.hsa_stats else []) + (["--stats"] if a.hip_stats or a.hsa_stats else [])
        return prof + ["--output-format", "csv", "-d", os.path.join(a.trace, f"t{i}"), "-o", f"t{i}", "--"] + c
    def env_of(i):
        env = dict(os.environ)
        if a.shim:   # each tenant a quota-only vGPU of its own (the shim preloaded, no limits)
            from amdvgpu.shim.launcher import apply_contract, vgpu_env
            env = apply_contract(vgpu_env(mem_limit=64 << 30))
        env.update(dict(kv.split("=", 1) for kv in a.env))
        return env
    procs = [subprocess.Popen(cmd(i), stdout=subprocess.PIPE, text=True, env=env_of(i)) for i in range(a.procs)]
    burners = [subprocess.Popen([sys.executable, os.path.abspath(__file__), "--burner", "--go", go,
                                 "--seconds", str(a.seconds)]) for _ in range(a.burners)]
    deadline = time.time() + 600
    while len(glob.glob(go + ".ready.*")) < a.procs and time.time() < deadline:
        if any(p.poll() not in (None, 0) for p in procs):
            break
        time.sleep(0.05)
    open(go, "w").close()

    def result(p):   # the tenant's line (rocprofv3 prints its own lines around it)
        lines = [ln for ln in p.communicate(timeout=600)[0].splitlines() if ln.startswith('{"pid"')]
        return json.loads(lines[-1])
    outs = [result(p) for p in procs]
    for b in burners:
        b.wait(timeout=600)
    for f in glob.glob(go + "*"):
        os.unlink(f)
    agg = sum(o["items_per_s"] for o in outs)
    aff, quota = _cpu_limit()
    print(json.dumps({"case": a.case, "procs": a.procs, "burners": a.burners, "pin": a.pin,
                      "placement": a.placement, "mem": a.mem, "shim": a.shim, "env": a.env, "gpu_numa_node": gnode,
                      "numa_cpus": {n: len(cs) for n, cs in nodes.items()},
                      "aggregate_items_per_s": round(agg, 1), "affinity": aff, "cgroup_cpus": quota,
                      "tenants": outs}), flush=True)
    return 0 if all(p.returncode == 0 for p in procs) else 1


def hip_stats(d, api="hip"):
    """Per tenant: the HIP (or HSA) API calls that took the most time (rocprofv3
    --hip-trace / --hsa-trace --stats)."""
    out = {}
    for f in glob.glob(os.path.join(d, "**", f"*{api}_api_stats.csv"), recursive=True):
        rows = []
        with open(f) as fh:
            for row in csv.DictReader(fh):
                try:
                    rows.append((row["Name"], int(row["Calls"]), float(row["TotalDurationNs"]) / 1e6,
                                 float(row["AverageNs"]) / 1e3))
                except (KeyError, ValueError):
                    continue
        rows.sort(key=lambda r: -r[2])
        out[_tenant_of_path(d, f)] = [{"api": n, "calls": c, "total_ms": round(t, 1), "avg_us": round(av, 2)}
                                      for n, c, t, av in rows[:10]]
    return out


def merge(iv):
    out = []
    for s, e in sorted(iv):
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def clip(iv, lo, hi):
    return [[max(s, lo), min(e, hi)] for s, e in iv if e > lo and s < hi]


def length(iv):
    return sum(e - s for s, e in iv)


def intersect(a, b):
    out, i, j = [], 0, 0
    while i < len(a) and j < len(b):
        s, e = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if s < e:
            out.append([s, e])
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return out


def pct(xs, q):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(q * len(xs)))] if xs else 0


def _tenant_of_path(d, f):
    # --trace puts tenant i's files under d/t<i>/...
    return os.path.relpath(f, d).split(os.sep)[0]


def analyze(d):
    per = {}
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                pid = _tenant_of_path(d, f)
                try:
                    s, e = int(row["Start_Timestamp"]), int(row["End_Timestamp"])
                except (KeyError, ValueError):
                    continue
                per.setdefault(str(pid), []).append((s, e))
    # tenants only: the launcher itself runs no kernels
    per = {p: merge(iv) for p, iv in per.items() if len(iv) > 100}
    if not per:
        return {"error": f"no kernel traces under {d}"}
    lo = max(iv[0][0] for iv in per.values())
    hi = min(iv[-1][1] for iv in per.values())
    span = hi - lo
    lo, hi = lo + span // 10, hi - span // 10   # the steady middle of the common window
    win = hi - lo
    res = {"window_ms": round(win / 1e6, 1), "procs": {}}
    clipped = {p: clip(iv, lo, hi) for p, iv in per.items()}
    both = None
    for p, iv in clipped.items():
        gaps = [b[0] - a[1] for a, b in zip(iv, iv[1:])]
        res["procs"][p] = {"busy": round(length(iv) / win, 4), "kernels": len(iv),
                           "gap_us_median": round(pct(gaps, 0.5) / 1e3, 1), "gap_us_p90": round(pct(gaps, 0.9) / 1e3, 1),
                           "gap_us_p99": round(pct(gaps, 0.99) / 1e3, 1),
                           # idle time in gaps of 100 us or more (where another queue could run)
                           "long_gap_share": round(sum(g for g in gaps if g >= 100_000) / win, 4),
                           "kernel_us_median": round(pct([e - s for s, e in iv], 0.5) / 1e3, 1)}
        both = iv if both is None else intersect(both, iv)
    res["both"] = round(length(both) / win, 4) if len(clipped) > 1 else None
    res["any"] = round(length(merge([x for iv in clipped.values() for x in iv])) / win, 4)
    for api in ("hip", "hsa"):
        hs = hip_stats(d, api)
        if hs:
            res[f"{api}_api"] = hs
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", default="lstm-inf")
    ap.add_argument("--procs", type=int, default=2)
    ap.add_argument("--seconds", type=float, default=4.0)
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--tenant", action="store_true")
    ap.add_argument("--go")
    ap.add_argument("--analyze")
    ap.add_argument("--trace", default="", help="rocprofv3 kernel trace of every tenant under this directory")
    ap.add_argument("--hip-stats", action="store_true", help="with --trace: HIP API trace and stats too")
    ap.add_argument("--hsa-stats", action="store_true", help="with --trace: HSA API trace and stats too")
    ap.add_argument("--pin", type=int, default=0, help="pin tenant i to K CPUs of its own")
    ap.add_argument("--burners", type=int, default=0, help="CPU-only processes spinning during the window")
    ap.add_argument("--placement", default="none", choices=["none", "local", "remote", "split"],
                    help="pin the tenants (--pin CPUs each, default 4) to the GPU's NUMA node, the others, or both")
    ap.add_argument("--mem", default="none", choices=["none", "local", "remote", "split"],
                    help="bind each tenant's host memory to the GPU's NUMA node, another one, or alternate")
    ap.add_argument("--mem-node", type=int, default=-1)
    ap.add_argument("--cpu-lists", default="", help='explicit CPUs per tenant, e.g. "64-67;96-99"')
    ap.add_argument("--l3", action="store_true", help="print the L3 (CCD) domains of the allowed CPUs and exit")
    ap.add_argument("--burner", action="store_true")
    ap.add_argument("--shim", action="store_true", help="run every tenant in a quota-only vGPU")
    ap.add_argument("--env", action="append", default=[], help="KEY=VALUE for every tenant")
    ap.add_argument("--cpus", default="")
    a = ap.parse_args()
    if a.l3:
        doms = {}
        for c in sorted(os.sched_getaffinity(0)):
            try:
                doms.setdefault(open(f"/sys/devices/system/cpu/cpu{c}/cache/index3/shared_cpu_list").read().strip(),
                                None)
            except OSError:
                pass
        print(json.dumps({"l3_domains": list(doms), "numa": {n: f"{cs[0]}..{cs[-1]} ({len(cs)})"
                                                             for n, cs in _numa_nodes().items()},
                          "gpu_node": _gpu_node()}))
        return 0
    if a.analyze:
        print(json.dumps(analyze(a.analyze)))
        return 0
    if a.tenant:
        return tenant(a.case, a.seconds, a.go, a.batch, a.cpus, a.mem_node)
    if a.burner:
        return burner(a.go, a.seconds)
    return launch(a)


if __name__ == "__main__":
    sys.exit(main())
