"""Node-side vGPU monitor: Prometheus metrics + control API over the containers' regions.

Reference: with ``VGPU_MONITOR_MODE`` each container's shared region lives on a host path
``/usr/local/vgpu/shared/<ns>_<pod>_<ctr>/<uuid>.cache`` (``server.go:494-501``) so that an
*external* monitor can mmap it and drive the control API exported by libvgpu.so
(``suspend_all``, ``resume_all``, ``set_current_device_sm_limit_scale``,
``set_current_device_memory_limit``, ``recent_kernel``, ``priority``).
That monitor is not part of the reference; this is the in-tree one.

* ``GET /metrics``  Prometheus text: per container/device memory limit, usage, spill,
  monitored usage, CU limit/mask width, utilisation, token bucket, per process
  launches / throttle / suspend seconds / OOM events, suspend state;
* ``GET /regions``  JSON snapshot of every region;
* the node GPU-time ledger (``<root>/../board/ledger.<gpu_id>``, ``plugin/ledger.py``):
  snapshots, reads, period and age per GPU, GPU time charged per host process;
* ``vgpu_container_info`` names the pod and container a directory belongs to: from the
  kubelet's PodResources (``--pod-resources-socket``, the device IDs the kubelet gave the
  container) when reachable, else the tag the plugin chose at Allocate
  (``plugin/podresources.py``);
* ``POST /regions/<pod_ctr>/{suspend,resume,block,unblock,reclaim}`` and
  ``POST /regions/<pod_ctr>/limit?dev=0&bytes=N`` / ``cu?dev=0&pct=P`` / ``priority?value=N``.

    python -m amdvgpu.plugin.monitor --root /usr/local/vgpu/shared --port 9394
"""
import argparse
import hmac
import ipaddress
import glob
import json
import logging
import os
import threading
import urllib.parse
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

from ..shim.region import Region

log = logging.getLogger("amdvgpu.monitor")


def discover(root):
    """{container tag: [region paths]} under ``root/<ns>_<pod>_<ctr>/*.cache``."""
    out = {}
    for p in sorted(glob.glob(os.path.join(root, "*", "*.cache"))):
        out.setdefault(os.path.basename(os.path.dirname(p)), []).append(p)
    return out


def _esc(v):
    return str(v).replace("\\", "\\\\").replace('"', '\\"').replace("\n", " ")


def _labels(**kw):
    return "{" + ",".join(f'{k}="{_esc(v)}"' for k, v in kw.items()) + "}"


class MetricsWriter:
    def __init__(self):
        self.lines = []
        self._seen = set()

    def metric(self, name, mtype, help_, labels, value):
        if name not in self._seen:
            self._seen.add(name)
            self.lines.append(f"# HELP {name} {help_}")
            self.lines.append(f"# TYPE {name} {mtype}")
        self.lines.append(f"{name}{_labels(**labels)} {value}")

    def text(self):
        return "\n".join(self.lines) + "\n"


def owners(root, pod_resources_socket=None, resources=("amd.com/gpu",)):
    """{tag: owner} (``podresources.attribute``), PodResources consulted when reachable."""
    from .podresources import attribute, list_pod_resources
    pods = list_pod_resources(pod_resources_socket, timeout=1.0) if pod_resources_socket else None
    return attribute(root, pods, set(resources))


def ledger_metrics(w, board_dir):
    """The node GPU-time ledger (``plugin/ledger.py``): per GPU the daemon's sampling and
    per process the GPU time it charged."""
    from .ledger import monotonic_ns, read_board
    now = monotonic_ns()
    for gpu_id, led in sorted(read_board(board_dir).items()):
        lb = {"gpu_id": gpu_id}
        w.metric("vgpu_ledger_samples_total", "counter", "node ledger: occupancy snapshots of the GPU", lb,
                 led["samples"])
        w.metric("vgpu_ledger_reads_total", "counter", "node ledger: KFD cu_occupancy reads", lb, led["reads"])
        w.metric("vgpu_ledger_period_seconds", "gauge", "node ledger: current sampling period", lb,
                 led["period_ns"] / 1e9)
        w.metric("vgpu_ledger_age_seconds", "gauge", "node ledger: time since the last snapshot (stale past 0.05)",
                 lb, max(0, now - led["heartbeat_ns"]) / 1e9)
        for p in led["procs"]:
            w.metric("vgpu_ledger_process_charged_seconds_total", "counter",
                     "node ledger: processor-sharing GPU time charged to a host process", dict(lb, hostpid=p["pid"]),
                     p["charged_ns"] / 1e9)


def _board_json(board_dir):
    """The node board's live containers, as ``vgpuctl board`` reads them (None when the tool or
    the board is missing)."""
    import subprocess
    from ..shim import native
    if not os.path.isdir(board_dir):
        return None
    try:
        p = subprocess.run([native.lib_path(native.VGPUCTL), "board", board_dir], capture_output=True, text=True,
                           timeout=10)
        return json.loads(p.stdout) if p.returncode == 0 else None
    except (native.NativeMissing, OSError, ValueError, subprocess.TimeoutExpired):
        return None


def board_metrics(w, board_dir):
    """The node board (``native/include/vgpu/board.h``): per container its launch rate, whether
    it launches steadily (batch) or in bursts (serving), its CPU node, and per GPU whether it
    holds a turn of the concurrency admission or waits for one (``--gpu-concurrency``).
    Labelled by region file, like the container metrics."""
    data = _board_json(board_dir) or {}
    for c in data.get("containers", []):
        lb = {"region": c["container"] + ".cache"}
        w.metric("vgpu_board_launches_per_second", "gauge", "node board: the container's kernel launches per second",
                 lb, c["launches_per_s"])
        if c.get("steady") is not None:
            w.metric("vgpu_board_steady", "gauge", "node board: 1 launches steadily (batch), 0 in bursts (serving)",
                     lb, int(c["steady"]))
        w.metric("vgpu_board_cpu_node", "gauge", "node board: the CPU node of the container's processes (-1 = none)",
                 lb, c["cpu_node"])
        for g in c.get("gpus", []):
            gl = dict(lb, gpu_id=g["gpu_id"])
            w.metric("vgpu_board_holds_turn", "gauge", "node board: 1 while the container holds a turn on the GPU",
                     gl, int(g["holds_turn"]))
            if g.get("waiting_ms") is not None:
                w.metric("vgpu_board_waiting_seconds", "gauge", "node board: how long the container has waited for "
                         "its turn", gl, g["waiting_ms"] / 1e3)


def render_metrics(root, pod_resources_socket=None, resources=("amd.com/gpu",), board_dir=None):
    w = MetricsWriter()
    board_dir = board_dir or os.path.join(os.path.dirname(os.path.normpath(root)), "board")
    ledger_metrics(w, board_dir)
    board_metrics(w, board_dir)
    regions = discover(root)
    w.metric("vgpu_monitor_regions", "gauge", "container regions found", {}, sum(len(v) for v in regions.values()))
    who = owners(root, pod_resources_socket, resources)
    for tag in sorted(regions):
        o = who.get(tag)
        if o:
            w.metric("vgpu_container_info", "gauge",
                     "pod and container of a container directory (source: podresources = the kubelet's device "
                     "assignment, allocate = the plugin's Allocate-time match; mismatch = the two disagree)",
                     {"container": tag, "namespace": o["namespace"], "pod": o["pod"], "pod_container": o["container"],
                      "source": o["source"], "mismatch": str(bool(o.get("mismatch"))).lower()}, 1)
    for tag, paths in regions.items():
        for path in paths:
            try:
                with Region(path) as r:
                    snap = r.snapshot()
            except OSError as e:
                log.warning("skip region %s: %s", path, e)
                continue
            base = {"container": tag, "region": os.path.basename(path)}
            w.metric("vgpu_container_suspended", "gauge", "1 while every gate of the container blocks", base,
                     int(snap["suspended"]))
            w.metric("vgpu_container_priority", "gauge", "task priority", base, snap["priority"])
            w.metric("vgpu_container_processes", "gauge", "processes attached to the region", base,
                     len(snap["procs"]))
            host = snap.get("host") or {}
            w.metric("vgpu_host_memory_limit_bytes", "gauge", "pinned host memory budget (0 = unlimited)", base,
                     host.get("limit", 0))
            w.metric("vgpu_host_memory_used_bytes", "gauge", "pinned host memory (hipHostMalloc / hipHostRegister)",
                     base, host.get("used", 0))
            w.metric("vgpu_sampler_ticks_total", "counter", "temporal limiter: occupancy samples taken", base,
                     snap["samples"])
            w.metric("vgpu_sampler_other_refreshes_total", "counter",
                     "temporal limiter: samples that re-read the other processes' occupancy", base,
                     snap["other_refreshes"])
            for d in snap["devices"]:
                if not d["configured"] and not d["mem_limit"]:
                    continue
                lb = dict(base, device=d["index"], uuid=d["uuid"])
                w.metric("vgpu_memory_limit_bytes", "gauge", "device memory quota (0 = unlimited)", lb,
                         d["mem_limit"])
                w.metric("vgpu_memory_used_bytes", "gauge", "bytes charged to the container", lb, d["used"])
                w.metric("vgpu_memory_spilled_bytes", "gauge", "bytes served from host memory", lb, d["spilled"])
                w.metric("vgpu_memory_monitored_bytes", "gauge", "KFD-measured VRAM of the container's processes",
                         lb, d["monitor_used"])
                w.metric("vgpu_cu_limit_percent", "gauge", "CU share (0 = unlimited)", lb, d["cu_limit_pct"])
                w.metric("vgpu_cu_mask_count", "gauge", "CUs in the spatial mask", lb, d["cu_mask_count"])
                w.metric("vgpu_cu_mode", "gauge", "effective enforcement: 0 off, 1 CU mask, 2 GPU-time limiter, 3 both",
                         lb, {"off": 0, "spatial": 1, "temporal": 2, "both": 3}.get(d["cu_mode"], -1))
                w.metric("vgpu_gpu_crowd", "gauge", "auto mode: other busy processes on the GPU (-1 = not assessed)",
                         lb, d.get("crowd", -1))
                w.metric("vgpu_utilization_percent", "gauge", "smoothed GPU-time share charged to the container",
                         lb, d["util_pct"])
                w.metric("vgpu_compute_credit_seconds", "gauge", "temporal limiter: remaining GPU-time credit", lb,
                         d["credit_ns"] / 1e9)
                w.metric("vgpu_compute_charged_seconds_total", "counter", "GPU time charged to the container", lb,
                         d["charged_ns"] / 1e9)
                w.metric("vgpu_preempted", "gauge", "background class: launches held while a better class is busy",
                         lb, int(d.get("preempt", False)))
                w.metric("vgpu_inflight_cap", "gauge",
                         "background class: AQL packets in flight allowed per process (0 = unbounded)", lb,
                         d.get("depth_cap", 0))
            for p in snap["procs"]:
                lp = dict(base, pid=p["pid"], hostpid=p["hostpid"])
                w.metric("vgpu_process_launches_total", "counter", "kernel launches through the gates", lp,
                         p["launches"])
                w.metric("vgpu_process_throttle_seconds_total", "counter", "time blocked by the rate limiter", lp,
                         p["throttle_ns"] / 1e9)
                w.metric("vgpu_process_suspend_seconds_total", "counter", "time blocked while suspended", lp,
                         p["suspend_ns"] / 1e9)
                w.metric("vgpu_process_oom_events_total", "counter", "allocations refused at the quota", lp,
                         p["oom_events"])
                for dev, used in enumerate(p["used"]):
                    if used:
                        w.metric("vgpu_process_memory_used_bytes", "gauge", "bytes charged to the process",
                                 dict(lp, device=dev), used)
    return w.text()


def control(root, tag, action, params):
    paths = discover(root).get(tag)
    if not paths:
        raise KeyError(tag)
    done = 0
    for path in paths:
        with Region(path) as r:
            if action == "suspend":
                r.suspend_all()
            elif action == "resume":
                r.resume_all()
            elif action == "block":
                r.recent_kernel = -1
            elif action == "unblock":
                r.recent_kernel = 2
            elif action == "reclaim":
                r.reclaim()
            elif action == "limit":
                nbytes = int(params["bytes"])
                if nbytes < 0 or r.set_memory_limit(int(params.get("dev", 0)), nbytes) != 0:
                    raise ValueError(f"invalid device or size: {params}")
            elif action == "cu":
                if r.set_cu_limit(int(params.get("dev", 0)), int(params["pct"])) != 0:
                    raise ValueError(f"invalid device or CU share (0-100): {params}")
            elif action == "priority":
                r.priority = int(params["value"])
            else:
                raise ValueError(action)
            done += 1
    return done


def make_handler(root, control_enabled=False, token=None, pod_resources_socket=None):
    """HTTP handler. The metrics side (GET /metrics, /regions, /healthz) is read-only and
    meant for Prometheus on the pod IP. The control side (POST /regions/<tag>/<action>)
    changes tenants' quotas, CU shares and run state, so it is only served by a handler
    built with ``control_enabled`` (the control server, loopback by default) and, when a
    ``token`` is configured, only to requests carrying ``Authorization: Bearer <token>``."""

    class Handler(BaseHTTPRequestHandler):
        def _send(self, code, body, ctype="text/plain; version=0.0.4"):
            data = body.encode()
            self.send_response(code)
            self.send_header("Content-Type", ctype)
            self.send_header("Content-Length", str(len(data)))
            self.end_headers()
            self.wfile.write(data)

        def do_GET(self):
            u = urllib.parse.urlparse(self.path)
            if u.path == "/metrics":
                return self._send(200, render_metrics(root, pod_resources_socket))
            if u.path == "/regions":
                snaps = {}
                for tag, paths in discover(root).items():
                    snaps[tag] = []
                    for p in paths:
                        try:
                            with Region(p) as r:
                                snaps[tag].append(r.snapshot())
                        except OSError:
                            pass
                return self._send(200, json.dumps(snaps), "application/json")
            if u.path == "/healthz":
                return self._send(200, "ok\n")
            return self._send(404, "not found\n")

        def do_POST(self):
            if not control_enabled:
                return self._send(403, "control endpoints are served on the control address only\n")
            if token is not None:
                got = self.headers.get("Authorization", "")
                if not hmac.compare_digest(got.encode(), f"Bearer {token}".encode()):
                    return self._send(401, "unauthorized\n")
            u = urllib.parse.urlparse(self.path)
            parts = u.path.strip("/").split("/")
            if len(parts) != 3 or parts[0] != "regions":
                return self._send(404, "not found\n")
            params = dict(urllib.parse.parse_qsl(u.query))
            try:
                n = control(root, parts[1], parts[2], params)
            except KeyError:
                return self._send(404, "unknown container\n")
            except (ValueError, TypeError) as e:
                return self._send(400, f"bad request: {e}\n")
            log.info("control %s %s %s by %s", parts[1], parts[2], params, self.client_address[0])
            return self._send(200, json.dumps({"regions": n}), "application/json")

        def log_message(self, fmt, *args):
            log.debug(fmt, *args)

    return Handler


def _is_loopback(host):
    try:
        return ipaddress.ip_address(host).is_loopback
    except ValueError:
        return host == "localhost"


def serve(root, host="0.0.0.0", port=9394, control_enabled=False, token=None):
    """Starts a server thread. A control server on a non-loopback address needs a token."""
    if control_enabled and token is None and not _is_loopback(host):
        raise ValueError("the control server listens beyond loopback only with a token (--control-token-file)")
    srv = ThreadingHTTPServer((host, port), make_handler(root, control_enabled, token))
    th = threading.Thread(target=srv.serve_forever, daemon=True)
    th.start()
    return srv


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--root", default="/usr/local/vgpu/shared")
    ap.add_argument("--host", default="0.0.0.0", help="metrics address (read-only endpoints)")
    ap.add_argument("--port", type=int, default=9394)
    ap.add_argument("--enable-control", action="store_true",
                    help="serve the mutating control endpoints (off by default)")
    ap.add_argument("--control-host", default="127.0.0.1", help="control address (loopback unless a token is set)")
    ap.add_argument("--control-port", type=int, default=9395)
    ap.add_argument("--control-token-file", default=None, help="file holding the bearer token for control calls")
    ap.add_argument("--pod-resources-socket", default="/var/lib/kubelet/pod-resources/kubelet.sock",
                    help="kubelet PodResources socket (pod attribution); ignored when absent")
    a = ap.parse_args(argv)
    token = open(a.control_token_file).read().strip() if a.control_token_file else None
    if a.enable_control:
        serve(a.root, a.control_host, a.control_port, control_enabled=True, token=token)
        log.info("control endpoints on %s:%d%s", a.control_host, a.control_port, " (token)" if token else "")
    srv = ThreadingHTTPServer((a.host, a.port), make_handler(a.root, pod_resources_socket=a.pod_resources_socket))
    srv.serve_forever()


if __name__ == "__main__":
    main()
