"""What bench.py's rank setup sees on a box: the KFD sysfs inventory, which render nodes
this process may open, the *_VISIBLE_DEVICES variables, and bench.visible_devices()."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
import bench  # noqa: E402
from amdvgpu.plugin.devices import SysfsBackend  # noqa: E402

be = SysfsBackend()
devs = be.devices()
print(json.dumps({
    "sysfs": [{"uuid": d.uuid, "bdf": d.bdf, "render": d.render_minor, "numa": d.numa_node,
               "openable": os.access(f"/dev/dri/renderD{d.render_minor}", os.R_OK | os.W_OK)} for d in devs],
    "env": {k: os.environ.get(k) for k in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES")},
    "visible": [d.uuid for d in bench.visible_devices(be, cpu=False)],
}))
