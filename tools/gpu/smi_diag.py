"""Diagnose SMI library initialisation under the shim (run on the GPU box)."""
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from amdvgpu.shim.launcher import apply_contract, vgpu_env  # noqa: E402

CODE = r'''
import ctypes, json, os
out = {}
try:
    lib = ctypes.CDLL("/opt/rocm/lib/librocm_smi64.so")
    out["rsmi_init"] = lib.rsmi_init(ctypes.c_uint64(0))
    t = ctypes.c_uint64()
    out["rsmi_total_rc"] = lib.rsmi_dev_memory_total_get(ctypes.c_uint32(0), ctypes.c_int(0), ctypes.byref(t))
    out["rsmi_total"] = t.value
except Exception as e:
    out["rsmi_err"] = repr(e)
try:
    import amdsmi
    amdsmi.amdsmi_init()
    h = amdsmi.amdsmi_get_processor_handles()[0]
    out["amdsmi_total"] = amdsmi.amdsmi_get_gpu_memory_total(h, amdsmi.AmdSmiMemoryType.VRAM)
except Exception as e:
    out["amdsmi_err"] = repr(e)[:200]
print(json.dumps(out))
'''

cases = {
    "native": None,
    "shim": {},
    "shim-no-dlsym": {"VGPU_HOOK_DLSYM": "0"},
    "shim-no-smi": {"VGPU_HOOK_SMI": "0"},
    "shim-disabled": {"VGPU_DISABLE": "1"},
}
for name, extra in cases.items():
    if extra is None:
        env = dict(os.environ)
    else:
        env = apply_contract(vgpu_env(mem_limit=24 << 30, extra=extra))
    p = subprocess.run([sys.executable, "-c", CODE], env=env, capture_output=True, text=True, timeout=120)
    print(name, p.stdout.strip(), p.stderr.strip()[-300:])
