"""rocm_smi device virtualisation on the CPU: a fake librocm_smi64 (native/tests/fake/
fake_rsmi.cpp, four GPUs whose answers encode their node index) driven over ctypes — as
the rocm-smi CLI does — with the shim preloaded. The container sees only its GPUs, in
node order, under its own indices (reference: NVML count / handle-by-index remapping,
nvml/hook.c:438-527)."""
import json
import os
import subprocess
import sys

import pytest

from amdvgpu.shim.native import LIB_DIR, shim_path

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FAKE_RSMI = os.path.join(LIB_DIR, "fakerocm", "smi", "librocm_smi64.so")

CHILD = r"""
import ctypes, json, sys
lib = ctypes.CDLL(sys.argv[1])
lib.rsmi_init(ctypes.c_uint64(0))
n = ctypes.c_uint32()
lib.rsmi_num_monitor_devices(ctypes.byref(n))
ids = []
for i in range(n.value + 1):
    v = ctypes.c_uint16()
    st = lib.rsmi_dev_id_get(ctypes.c_uint32(i), ctypes.byref(v))
    ids.append([st, v.value])
w = ctypes.c_uint64()
lib.rsmi_topo_get_link_weight(ctypes.c_uint32(0), ctypes.c_uint32(1), ctypes.byref(w))
name = ctypes.create_string_buffer(32)
lib.rsmi_dev_name_get(ctypes.c_uint32(1), name, ctypes.c_size_t(32))
g = (ctypes.c_uint32 * 8)()
gn = ctypes.c_uint32(8)
lib.rsmi_compute_process_gpus_get(ctypes.c_uint32(1), g, ctypes.byref(gn))
tot = ctypes.c_uint64()
lib.rsmi_dev_memory_total_get(ctypes.c_uint32(1), 0, ctypes.byref(tot))
print(json.dumps({"n": n.value, "ids": ids, "w01": w.value, "name1": name.value.decode(),
                  "gpus": list(g)[:gn.value], "mem1_gib": tot.value >> 30}))
"""


def run(tmp_path, **env):
    e = {k: v for k, v in os.environ.items() if not k.startswith("VGPU_")}
    e.update(LD_PRELOAD=shim_path(), VGPU_SHARED_CACHE=str(tmp_path / "region.cache"), **env)
    p = subprocess.run([sys.executable, "-c", CHILD, FAKE_RSMI], env=e, capture_output=True, text=True, timeout=60)
    assert p.returncode == 0, p.stderr[-2000:]
    return json.loads(p.stdout.strip().splitlines()[-1])


def test_generated_wrappers_are_current():
    p = subprocess.run([sys.executable, os.path.join(REPO, "native", "tools", "gen_rsmi_remap.py"), "--check"],
                       capture_output=True, text=True)
    assert p.returncode == 0, p.stderr


def test_container_sees_only_its_gpus_under_its_own_indices(tmp_path):
    # The container holds node GPUs 2 and 0 (listed in that order by the plugin).
    r = run(tmp_path, VGPU_DEVICE_BDFS="0000:25:00.0,0000:05:00.0")
    assert r["n"] == 2
    assert r["ids"] == [[0, 0x1000], [0, 0x1002], [1, 0]]   # index 2 does not exist (INVALID_ARGS)
    assert r["w01"] == 2                                     # container 0 -> 1 is node 0 -> 2
    assert r["name1"] == "fake-gpu-2"
    assert r["gpus"] == [0, 1]                               # node GPUs 1 and 3 are hidden
    assert r["mem1_gib"] == 3


@pytest.mark.parametrize("env", [{}, {"VGPU_DEVICE_BDFS": "0000:25:00.0", "VGPU_HOOK_SMI": "0"}])
def test_nothing_hidden_without_a_device_list_or_with_smi_hooks_off(tmp_path, env):
    r = run(tmp_path, **env)
    assert r["n"] == 4 and [v for _, v in r["ids"][:4]] == [0x1000, 0x1001, 0x1002, 0x1003]
    assert r["w01"] == 1 and r["gpus"] == [0, 1, 2, 3]
