"""Plugin entry point: flags -> discovery -> supervisor restart loop.

Reference: ``main.go`` — ``start`` (:163-293): write the GPU PCI bus-ID list to
``$PCIBUSFILE`` (from ``lspci`` filtered on "NVIDIA", :164-185), init NVML and block
forever on failure when ``--fail-on-init-error=false`` (:186-199), start the fsnotify
and signal watchers, then the ``restart:`` loop: stop old plugins, rebuild them via the
strategy, start those with devices; restart on a plugin start error, on
``kubelet.sock`` re-creation or SIGHUP; exit on other signals (:212-291).

Here the BDF list comes from the device backend (no lspci, no vendor-string filter).

    python -m amdvgpu.plugin.main [flags]      (see --help; every flag has an env var)
"""
import logging
import os
import queue
import signal
import sys
import threading
import time

from .. import __version__
from ..utils.log import get_logger
from .config import parse_config
from .contract import ensure_board_dir, ensure_lock_file
from .devices import FakeBackend, detect_backend
from .legacy import LegacyController
from .strategy import plugins_for
from .watchers import FSWatcher, OSWatcher

log = logging.getLogger("amdvgpu")


def write_pcibus_file(path, devices):
    bdfs = sorted({d.bdf for d in devices if d.bdf})
    with open(path, "w") as f:
        f.write("".join(b + "\n" for b in bdfs))


class LedgerDaemon:
    """The node's GPU-time ledger (native/src/tools/vgpu_ledger.cpp, vgpu/ledger.h): one
    KFD occupancy sampler for every limited container, writing <board>/ledger.<gpu_id>.
    Restarted if it exits; the containers fall back to sampling by themselves whenever its
    ledger goes stale, so a missing binary only costs the saving."""

    def __init__(self, board_dir):
        self.board_dir = board_dir
        self.proc = None
        self.starts = 0
        self._next_try = 0.0

    def poll(self):
        if self.proc is not None and self.proc.poll() is None:
            return
        if time.monotonic() < self._next_try:
            return
        self._next_try = time.monotonic() + 5.0
        import subprocess
        from ..shim.native import LEDGER, NativeMissing, lib_path
        try:
            exe = lib_path(LEDGER)
        except NativeMissing as e:
            if self.starts == 0:
                log.warning("no ledger daemon (%s); containers sample the GPU by themselves", e)
            self.starts += 1
            return
        if self.proc is not None:
            log.warning("vgpu-ledger exited with %s; restarting", self.proc.returncode)
        self.proc = subprocess.Popen([exe, "--dir", self.board_dir], stdin=subprocess.DEVNULL)
        self.starts += 1

    def stop(self):
        if self.proc is not None and self.proc.poll() is None:
            self.proc.terminate()
            try:
                self.proc.wait(timeout=5)
            except Exception:
                self.proc.kill()
        self.proc = None


class Supervisor:
    def __init__(self, cfg, backend=None, install_signals=True, pod_lister=None):
        self.cfg = cfg
        self.backend = backend
        self.install_signals = install_signals
        self.pod_lister = pod_lister
        self.events = queue.Queue()
        self.plugins = []
        self.restarts = 0
        self.started = threading.Event()
        self._fs = None
        self._os = None
        self.ledger = None

    def init_backend(self):
        if self.backend is not None:
            return True
        try:
            if self.cfg.backend == "fake" or self.cfg.fake_devices:
                self.backend = FakeBackend.from_spec(self.cfg.fake_devices or "{}")
            else:
                self.backend = detect_backend(self.cfg.backend)
        except Exception as e:
            log.error("failed to initialise the device backend: %s", e)
            self.backend = None
        return self.backend is not None

    def _legacy_factory(self, ids):
        return LegacyController(ids, self.cfg.resource_name, self.cfg.device_plugin_path, self.pod_lister)

    def start_plugins(self):
        for p in self.plugins:
            p.stop()
        devices = self.backend.devices()
        matcher = None
        if self.cfg.monitor_mode and self.pod_lister is not None:
            from .k8s import PodMatcher
            matcher = PodMatcher(self.pod_lister, shared_root=os.path.join(self.cfg.vgpu_dir, "shared"))
        self.plugins = plugins_for(self.cfg, devices, self.backend, self._legacy_factory, matcher)
        started = 0
        for p in self.plugins:
            if not p.devices:
                continue
            try:
                p.start()
            except Exception as e:
                log.error("could not contact kubelet, retrying (%s). Is the device plugin feature enabled?", e)
                return False
            started += 1
        if started == 0:
            log.info("no devices found; waiting indefinitely")
        self.restarts += 1
        self.started.set()
        return True

    def stop(self):
        for p in self.plugins:
            p.stop()
        self.plugins = []

    def run(self, stop_event=None):
        cfg = self.cfg
        if not self.init_backend():
            if cfg.fail_on_init_error:
                return 1
            log.error("no usable GPU backend; if this is not a GPU node use a nodeSelector/toleration")
            (stop_event or threading.Event()).wait()
            return 0
        if cfg.pcibus_file:
            try:
                write_pcibus_file(cfg.pcibus_file, self.backend.devices())
            except OSError as e:
                log.warning("cannot write %s: %s", cfg.pcibus_file, e)
        os.makedirs(cfg.device_plugin_path, exist_ok=True)
        try:
            ensure_lock_file(cfg.vgpu_dir)
            board = ensure_board_dir(cfg.vgpu_dir)
            if cfg.ledger:
                self.ledger = LedgerDaemon(board)
                self.ledger.poll()
        except OSError as e:
            log.warning("cannot create the host-PID lock file / board under %s: %s", cfg.vgpu_dir, e)
        self._fs = FSWatcher(cfg.device_plugin_path.rstrip("/"), self.events)
        if self.install_signals and threading.current_thread() is threading.main_thread():
            self._os = OSWatcher(self.events)
        try:
            return self._loop(stop_event)
        finally:
            self.stop()
            if self.ledger:
                self.ledger.stop()
            self._fs.close()
            if self._os:
                self._os.close()

    def _loop(self, stop_event):
        kubelet_sock = os.path.normpath(self.cfg.kubelet_socket)
        need_restart = True
        retry_at = 0.0
        while True:
            # A failed start (kubelet not up yet) is retried every second, but events keep
            # being read meanwhile, so signals and a stop request still end the plugin.
            if need_restart and time.monotonic() >= retry_at:
                need_restart = False
                if not self.start_plugins():
                    need_restart = True
                    retry_at = time.monotonic() + 1.0
            if self.ledger:
                self.ledger.poll()
            try:
                ev = self.events.get(timeout=0.2)
            except queue.Empty:
                if stop_event is not None and stop_event.is_set():
                    return 0
                fatal = [p.fatal for p in self.plugins if p.fatal]
                if fatal:
                    log.error("fatal: %s", fatal[0])
                    return 1
                continue
            if isinstance(ev, tuple) and ev[0] == "signal":
                if ev[1] == signal.SIGHUP:
                    log.info("received SIGHUP, restarting")
                    need_restart, retry_at = True, 0.0
                    continue
                log.info("received signal %d, shutting down", ev[1])
                return 0
            if os.path.normpath(ev.name) == kubelet_sock and ev.op == "create":
                log.info("inotify: %s created, restarting", kubelet_sock)
                need_restart, retry_at = True, 0.0


def main(argv=None):
    cfg = parse_config(argv)
    if cfg.version_requested:
        print(__version__)
        return 0
    get_logger("amdvgpu", cfg.verbose)
    log.info("amd-vgpu-device-plugin %s: split=%d memory-scaling=%.2f cores-scaling=%.2f strategy=%s cu-mode=%s",
             __version__, cfg.device_split_count, cfg.device_memory_scaling, cfg.device_cores_scaling,
             cfg.partition_strategy, cfg.cu_mode)
    pod_lister = None
    if (cfg.monitor_mode or cfg.enable_legacy_preferred) and cfg.node_name:
        from .k8s import PodClient
        pod_lister = PodClient(cfg.node_name).pods_on_node
    return Supervisor(cfg, pod_lister=pod_lister).run()


if __name__ == "__main__":
    sys.exit(main())
