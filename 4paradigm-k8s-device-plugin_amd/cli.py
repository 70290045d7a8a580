"""``python -m amdvgpu <command>`` — one entry point for the node and for debugging.

    plugin   [flags]                     run the device plugin (same flags as plugin.main)
    monitor  [--root DIR] [--port N]     Prometheus metrics + control API over regions
    run      [--memory 16g] [--cu 25] [--cu-range 0-64] [--oversubscribe] -- CMD...
                                         run CMD as a vGPU 'container' under the shim
    region   PATH [show|suspend|resume|set-limit DEV SIZE|set-cu DEV PCT|reclaim]
    devices  [--backend auto|sysfs|amdsmi|fake]   print the discovered GPUs as JSON
"""
import argparse
import json
import sys


def _run(argv):
    from .shim.launcher import cleanup_region, run, vgpu_env
    from .utils.sizes import parse_size
    ap = argparse.ArgumentParser(prog="amdvgpu run")
    ap.add_argument("--memory", default=None, help="HBM quota, e.g. 16g")
    ap.add_argument("--hbm", default=None, help="HBM-resident share (with --oversubscribe)")
    ap.add_argument("--cu", type=int, default=None, help="CU share in percent")
    ap.add_argument("--cu-range", default=None, help="logical CU range b-e")
    ap.add_argument("--cu-mode", default=None, choices=["auto", "spatial", "temporal", "both", "off"])
    ap.add_argument("--oversubscribe", action="store_true")
    ap.add_argument("--region", default=None, help="shared region file (default: a fresh /tmp file)")
    ap.add_argument("--keep-region", action="store_true")
    ap.add_argument("cmd", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    cmd = a.cmd[1:] if a.cmd and a.cmd[0] == "--" else a.cmd
    if not cmd:
        ap.error("no command given")
    extra = {}
    if a.hbm:
        extra["VGPU_DEVICE_HBM_LIMIT_0"] = f"{parse_size(a.hbm) >> 20}m"
    rng = tuple(int(x) for x in a.cu_range.split("-")) if a.cu_range else None
    c = vgpu_env(mem_limit=parse_size(a.memory) if a.memory else None, cu_limit=a.cu, cu_range=rng,
                 cu_mode=a.cu_mode, oversubscribe=a.oversubscribe, shared_cache=a.region, extra=extra)
    try:
        return run(cmd, c).returncode
    finally:
        if not a.keep_region and not a.region:
            cleanup_region(c)


def _region(argv):
    from .shim.region import Region
    from .utils.sizes import parse_size
    if not argv:
        print("usage: amdvgpu region PATH [show|suspend|resume|set-limit DEV SIZE|set-cu DEV PCT|reclaim]")
        return 2
    r = Region(argv[0])
    op = argv[1] if len(argv) > 1 else "show"
    if op == "show":
        print(json.dumps(r.snapshot(), indent=1))
    elif op == "suspend":
        r.suspend_all()
    elif op == "resume":
        r.resume_all()
    elif op == "set-limit":
        r.set_memory_limit(int(argv[2]), parse_size(argv[3]))
    elif op == "set-cu":
        r.set_cu_limit(int(argv[2]), int(argv[3]))
    elif op == "reclaim":
        print(r.reclaim())
    else:
        print(f"unknown region op {op}", file=sys.stderr)
        return 2
    return 0


def _devices(argv):
    from .plugin.devices import detect_backend
    ap = argparse.ArgumentParser(prog="amdvgpu devices")
    ap.add_argument("--backend", default="auto")
    ap.add_argument("--fake", default=None)
    a = ap.parse_args(argv)
    be = detect_backend(a.backend, a.fake)
    devs = be.devices() if be else []
    print(json.dumps([d.to_dict() for d in devs], indent=1))
    return 0


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv or argv[0] in ("-h", "--help"):
        print(__doc__)
        return 0
    cmd, rest = argv[0], argv[1:]
    if cmd == "plugin":
        from .plugin.main import main as plugin_main
        return plugin_main(rest)
    if cmd == "monitor":
        from .plugin.monitor import main as monitor_main
        return monitor_main(rest)
    if cmd == "run":
        return _run(rest)
    if cmd == "region":
        return _region(rest)
    if cmd == "devices":
        return _devices(rest)
    print(f"unknown command {cmd!r}\n{__doc__}", file=sys.stderr)
    return 2
