"""The co-tenancy probe's trace analysis (tools/probe/cotenancy.py --analyze), on synthetic
rocprofv3 kernel traces: time-sliced tenants show no overlap and gaps as long as the other's
bursts; concurrent tenants show their overlap."""
import csv
import importlib.util
import os

from conftest import REPO

spec = importlib.util.spec_from_file_location("cotenancy", os.path.join(REPO, "tools", "probe", "cotenancy.py"))
cot = importlib.util.module_from_spec(spec)
spec.loader.exec_module(cot)


def _trace(d, name, kernels):
    os.makedirs(d / name / "host", exist_ok=True)
    with open(d / name / "host" / f"{name}_kernel_trace.csv", "w", newline="") as f:
        w = csv.DictWriter(f, ["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        w.writeheader()
        for s, e in kernels:
            w.writerow({"Kernel_Name": "k", "Start_Timestamp": s, "End_Timestamp": e})


def test_time_sliced_tenants(tmp_path):
    # t0 runs 1 ms bursts of 10 kernels, t1 runs in t0's gaps: never both at once
    us = 1000
    a, b = [], []
    for burst in range(200):
        base = burst * 2000 * us
        a += [(base + i * 100 * us, base + (i + 1) * 100 * us - 5 * us) for i in range(10)]
        b += [(base + 1000 * us + i * 100 * us, base + 1000 * us + (i + 1) * 100 * us - 5 * us) for i in range(10)]
    _trace(tmp_path, "t0", a)
    _trace(tmp_path, "t1", b)
    r = cot.analyze(str(tmp_path))
    assert set(r["procs"]) == {"t0", "t1"}
    assert r["both"] == 0.0
    assert 0.45 < r["procs"]["t0"]["busy"] < 0.5
    assert r["procs"]["t0"]["gap_us_p99"] >= 1000   # the other tenant's burst
    assert 0.45 < r["procs"]["t0"]["long_gap_share"] < 0.55
    assert r["any"] > 0.9


def test_concurrent_tenants(tmp_path):
    us = 1000
    a = [(i * 100 * us, (i + 1) * 100 * us - 10 * us) for i in range(2000)]
    b = [(s + 20 * us, e + 20 * us) for s, e in a]
    _trace(tmp_path, "t0", a)
    _trace(tmp_path, "t1", b)
    r = cot.analyze(str(tmp_path))
    assert r["both"] > 0.6
