"""kubelet device-plugin gRPC server (one instance per advertised resource).

Reference: ``server.go`` — ``NvidiaDevicePlugin`` (:62-76), ``initialize``/``cleanup``
(:98-128), ``Start``/``Stop`` (:132-168), ``Serve`` with a crash-restart budget of 5 per
hour and a 5 s self-dial (:171-218), ``Register`` (:221-243),
``GetDevicePluginOptions`` (:246-251), ``ListAndWatch`` (:254-268),
``GetPreferredAllocation`` (:271-326), ``MIGAllocate``/``Allocate`` (:329-533),
``PreStartContainer`` (:536-538), ``apiDevices`` (:583-596).

Fixed reference quirks: devices recover from Unhealthy when the
backend reports recovery (``server.go:262``); ``Register`` and
``GetDevicePluginOptions`` advertise the same options (:234 vs :248); the
legacy-preferred ``acquire`` runs once per container (:456 and :484); monitor mode
looks only at this node's pending pods and never indexes out of range (:376-392).
"""
import collections
import logging
import os
import threading
import time
from concurrent import futures

import grpc

from ..parallel.topology import allocate_vdevices
from . import api
from .contract import (SHARED_HOST_DIR, build_container_response, build_partition_response, duplicate_gpus,
                       gc_container_files, gc_shared_dirs)
from .vdevice import assign_cpu_nodes, device_to_vdevices, vdevices_by_ids

log = logging.getLogger("amdvgpu.plugin")

RESTART_BUDGET = 5          # gRPC server restarts allowed ...
RESTART_WINDOW_S = 3600.0   # ... per hour (reference server.go:180-207)
DIAL_TIMEOUT_S = 5.0
WATCHDOG_PERIOD_S = 5.0


class AllocationError(Exception):
    pass


class DevicePluginServer:
    """Serves one resource (``amd.com/gpu`` vGPUs, or one partition resource)."""

    def __init__(self, cfg, resource_name, socket_name, devices, backend=None, partition_resource=False,
                 legacy=None, pod_matcher=None, vdev_filter=None, latency=False):
        self.cfg = cfg
        self.resource_name = resource_name
        self.socket = os.path.join(cfg.device_plugin_path, socket_name)
        self.devices = list(devices)
        self.backend = backend
        self.partition_resource = partition_resource
        self.legacy = legacy
        self.pod_matcher = pod_matcher
        self.vdev_filter = vdev_filter   # which of each GPU's vGPUs this resource serves (None = all)
        self.latency = latency           # the latency resource: grants VGPU_TASK_PRIORITY=0
        self._cond = threading.Condition()
        # Allocate runs on the gRPC thread pool; with the legacy controller its
        # read-available / choose / acquire sequence must not interleave with another call's.
        self._alloc_mu = threading.Lock()
        self._version = 0
        self._stopped = threading.Event()
        self._server = None
        self._health_thread = None
        self._watchdog_thread = None
        self._restarts = []
        self.fatal = None            # set when the restart budget is exhausted
        self.watchdog_period_s = WATCHDOG_PERIOD_S
        self.vdevices = []
        # (request ids, using ids) of recent Allocate calls, for observability; bounded so a
        # long-lived plugin does not grow with every container start.
        self.allocations = collections.deque(maxlen=1024)

    # ------------------------------------------------------------------ lifecycle
    def initialize(self):
        if self.partition_resource:
            self.vdevices = device_to_vdevices(self.devices, 1)
        else:
            self.vdevices = device_to_vdevices(self.devices, self.cfg.device_split_count,
                                               self.cfg.device_memory_scaling, self.cfg.device_cores_scaling)
            if self.vdev_filter is not None:
                self.vdevices = [v for v in self.vdevices if self.vdev_filter(v)]
            spread = getattr(self.cfg, "numa_spread", "off")
            if spread == "on" or (spread == "auto" and self.cfg.device_split_count > 1):
                nodes = self.backend.cpu_numa_nodes() if hasattr(self.backend, "cpu_numa_nodes") else []
                assign_cpu_nodes(self.vdevices, nodes)
                if any(v.cpu_node >= 0 for v in self.vdevices):
                    log.info("numa spread: the vGPUs of each GPU alternate over CPU nodes %s", nodes)
        self._by_uuid = {d.uuid: d for d in self.devices}
        self._stopped.clear()

    def start(self):
        self.initialize()
        self.serve()
        try:
            self.register()
        except Exception as e:
            log.error("could not register with kubelet at %s: %s", self.cfg.kubelet_socket, e)
            self.stop()
            raise
        log.info("registered device plugin for %s with kubelet (%d vGPUs on %d devices)", self.resource_name,
                 len(self.vdevices), len(self.devices))
        self._health_thread = threading.Thread(target=self._health_loop, name=f"health-{self.resource_name}",
                                               daemon=True)
        self._health_thread.start()
        self._watchdog_thread = threading.Thread(target=self._watchdog, name=f"watchdog-{self.resource_name}",
                                                 daemon=True)
        self._watchdog_thread.start()

    def stop(self):
        self._stopped.set()
        with self._cond:
            self._version += 1
            self._cond.notify_all()
        if self._server is not None:
            self._server.stop(grace=0.5).wait(2.0)
            self._server = None
        try:
            os.unlink(self.socket)
        except FileNotFoundError:
            pass

    def serve(self):
        """Listen on the unix socket, then confirm readiness by dialing it (<= 5 s)."""
        try:
            os.unlink(self.socket)
        except FileNotFoundError:
            pass
        os.makedirs(os.path.dirname(self.socket), exist_ok=True)
        server = grpc.server(futures.ThreadPoolExecutor(max_workers=8, thread_name_prefix="dp-grpc"))
        server.add_generic_rpc_handlers((api.service_handler("DevicePlugin", self),))
        if server.add_insecure_port(api.unix_target(self.socket)) == 0:
            raise OSError(f"cannot bind {self.socket}")
        server.start()
        self._server = server
        ch = grpc.insecure_channel(api.unix_target(self.socket))
        try:
            grpc.channel_ready_future(ch).result(timeout=DIAL_TIMEOUT_S)
        finally:
            ch.close()

    def restart_server(self):
        """Crash-restart with the reference's budget (5 per hour, then fatal)."""
        now = time.monotonic()
        self._restarts = [t for t in self._restarts if now - t < RESTART_WINDOW_S] + [now]
        if len(self._restarts) > RESTART_BUDGET:
            raise RuntimeError(f"gRPC server for {self.resource_name} crashed more than {RESTART_BUDGET} "
                               f"times in an hour")
        if self._server is not None:
            self._server.stop(0)
            self._server = None
        self.serve()

    def _serving(self):
        if not os.path.exists(self.socket):
            return False
        ch = grpc.insecure_channel(api.unix_target(self.socket))
        try:
            grpc.channel_ready_future(ch).result(timeout=2.0)
            return True
        except grpc.FutureTimeoutError:
            return False
        finally:
            ch.close()

    def _watchdog(self):
        """The Go server's crash-restart goroutine (server.go:180-207): if the socket
        stops answering (deleted, server died), serve again and re-register, at most
        RESTART_BUDGET times per hour; past that the plugin is marked fatal and the
        supervisor exits (the DaemonSet restarts the pod, like log.Fatal)."""
        unregistered = False  # served again, but the kubelet has not heard of it yet
        while not self._stopped.wait(self.watchdog_period_s):
            if self._serving():
                if not unregistered:
                    continue
            else:
                log.error("device plugin socket %s is not serving; restarting the gRPC server", self.socket)
                try:
                    self.restart_server()
                except RuntimeError as e:
                    self.fatal = str(e)
                    log.error("%s", e)
                    return
                except Exception as e:
                    log.warning("gRPC server restart failed: %r", e)
                    continue
            try:
                self.register()
                unregistered = False
            except Exception as e:  # kubelet slow or away: retried next tick (a restarted kubelet
                # also triggers the supervisor's inotify restart)
                unregistered = True
                log.warning("re-register after restart failed: %r; retrying", e)

    def options(self):
        return api.DevicePluginOptions(pre_start_required=False,
                                       get_preferred_allocation_available=not self.partition_resource)

    def register(self):
        ch = grpc.insecure_channel(api.unix_target(self.cfg.kubelet_socket))
        try:
            grpc.channel_ready_future(ch).result(timeout=DIAL_TIMEOUT_S)
            stub = api.registration_stub(ch)
            stub.Register(api.RegisterRequest(version=api.VERSION, endpoint=os.path.basename(self.socket),
                                              resource_name=self.resource_name, options=self.options()),
                          timeout=DIAL_TIMEOUT_S)
        finally:
            ch.close()

    # ------------------------------------------------------------------ health
    def set_health(self, uuid, healthy, reason=""):
        changed = False
        for d in self.devices:
            if d.uuid == uuid and d.healthy != healthy:
                d.healthy = healthy
                changed = True
        if changed:
            log.warning("device %s is now %s (%s)", uuid, api.HEALTHY if healthy else api.UNHEALTHY, reason)
            with self._cond:
                self._version += 1
                self._cond.notify_all()
        return changed

    def _health_loop(self):
        mode = (self.cfg.disable_healthchecks or "").lower()
        if mode == "all" or self.backend is None:
            return
        while not self._stopped.wait(self.cfg.health_interval_s):
            try:
                events = self.backend.poll_health(self.devices)
            except Exception as e:  # a flaky backend must not kill the plugin
                log.warning("health poll failed: %s", e)
                continue
            for ev in events:
                if mode in ("xids", "events") and not ev.healthy and "RAS" not in ev.reason:
                    continue
                self.set_health(ev.uuid, ev.healthy, ev.reason)

    # ------------------------------------------------------------------ gRPC API
    def api_devices(self):
        out = []
        for v in self.vdevices:
            d = api.Device(ID=v.id, health=api.HEALTHY if v.dev.healthy else api.UNHEALTHY)
            # The GPU's own PCIe NUMA node: what a topology-aware kubelet aligns an exclusive-CPU
            # pod's CPUs and memory with. The --numa-spread CPU node is a placement inside the
            # shared pool and travels in the contract only (VGPU_CPU_NODE); the shim keeps an
            # exclusive cpuset whole (native/src/shim/numa_spread.cpp).
            if v.dev.numa_node >= 0:
                d.topology.nodes.add(ID=v.dev.numa_node)
            out.append(d)
        return out

    def GetDevicePluginOptions(self, request, context):
        return self.options()

    def ListAndWatch(self, request, context):
        with self._cond:
            seen = self._version
        yield api.ListAndWatchResponse(devices=self.api_devices())
        while not self._stopped.is_set():
            with self._cond:
                self._cond.wait_for(lambda: self._version != seen or self._stopped.is_set(), timeout=1.0)
                changed = self._version != seen
                seen = self._version
            if context is not None and not context.is_active():
                return
            if self._stopped.is_set():
                return
            if changed:
                yield api.ListAndWatchResponse(devices=self.api_devices())

    def GetPreferredAllocation(self, request, context):
        resp = api.PreferredAllocationResponse()
        for req in request.container_requests:
            ids = allocate_vdevices(self.vdevices, list(req.available_deviceIDs), list(req.must_include_deviceIDs),
                                    req.allocation_size, placement=self.cfg.placement)
            resp.container_responses.add(deviceIDs=ids)
        return resp

    def _fail(self, context, msg):
        if context is not None:
            context.abort(grpc.StatusCode.INVALID_ARGUMENT, msg)
        raise AllocationError(msg)

    def Allocate(self, request, context):
        if self.legacy is None:
            return self._allocate(request, context)
        with self._alloc_mu:
            return self._allocate(request, context)

    def _held_by_resource(self):
        """{resource: set of device-ID frozensets} that live containers hold (kubelet
        PodResources), or None when the service cannot be reached."""
        from .podresources import list_pod_resources
        pods = list_pod_resources(self.cfg.pod_resources_socket, timeout=1.0)
        if pods is None:
            return None
        held = {}
        for p in pods:
            for c in p["containers"]:
                for res, ids in c["devices"].items():
                    if ids:
                        held.setdefault(res, set()).add(frozenset(ids))
        return held

    def _held_device_sets(self):
        """Device-ID sets of this resource that live containers hold, or None (see above)."""
        held = self._held_by_resource()
        return None if held is None else held.get(self.resource_name, set())

    def _allocate(self, request, context):
        resp = api.AllocateResponse()
        if self.partition_resource:
            for req in request.container_requests:
                try:
                    vds = vdevices_by_ids(self.vdevices, list(req.devicesIDs))
                except KeyError as e:
                    self._fail(context, f"invalid allocation request for '{self.resource_name}': {e}")
                resp.container_responses.append(build_partition_response(self.cfg, [v.dev for v in vds]))
            return resp

        # Host files of containers whose pods are gone (never by age: a restarted container
        # re-mounts them from the kubelet's checkpointed response).
        removed = gc_container_files(self.cfg.vgpu_dir, self._held_by_resource())
        if removed:
            log.info("removed the host files of %d departed container(s)", len(removed))
        tags = [None] * len(request.container_requests)
        if self.cfg.monitor_mode and self.pod_matcher is not None:
            try:
                tags = self.pod_matcher.match([len(r.devicesIDs) for r in request.container_requests])
            except Exception as e:
                log.warning("monitor mode: pod match failed: %s", e)
            # Directories of pods that are gone, judged from the pod list just fetched.
            gc_shared_dirs(os.path.join(self.cfg.vgpu_dir, SHARED_HOST_DIR), getattr(self.pod_matcher, "last_pods", None),
                           held=self._held_device_sets())
        if self.legacy is not None and not self.legacy.update_from_checkpoint():
            # Reference server.go:410-412: without the checkpoint the controller cannot know
            # which vGPUs other containers hold, so it refuses instead of double-booking.
            self._fail(context, f"legacy preferred allocation for '{self.resource_name}': "
                                "cannot read the kubelet checkpoint")
        for i, req in enumerate(request.container_requests):
            requested = list(req.devicesIDs)
            using = requested
            if self.legacy is not None:
                self.legacy.release_by_request(requested)
                avail = self.legacy.available([v.id for v in self.vdevices])
                using = allocate_vdevices(self.vdevices, avail, [], len(requested),
                                          placement=self.cfg.placement) if len(avail) >= len(requested) else []
                if len(using) < len(requested):
                    # Reference server.go:436-439 ("no enough devices"): never fall back to
                    # the kubelet's IDs, which may belong to another container's vGPUs.
                    self._fail(context, f"no enough devices for '{self.resource_name}': requested "
                                        f"{len(requested)}, {len(avail)} free")
                self.legacy.acquire(requested, using)
            try:
                vds = vdevices_by_ids(self.vdevices, using)
            except KeyError as e:
                self._fail(context, f"invalid allocation request for '{self.resource_name}': {e}")
            dups = duplicate_gpus(vds)
            if dups and self.cfg.duplicate_vgpus == "reject":
                # Reference [device.c:81-155] keeps duplicates as separate virtual devices
                # (virtual PCI ids, cooperative launch off); so does the default =split (the shim
                # virtualises the device ordinals, vdev_hooks.cpp). =reject refuses them.
                self._fail(context, f"allocation for '{self.resource_name}' holds several vGPUs of one GPU "
                                    f"({', '.join(dups)}), refused by --duplicate-vgpus=reject "
                                    f"(plugin flag --duplicate-vgpus=split presents them as separate devices, "
                                    f"=merge as one merged device)")
            unhealthy = [v.id for v in vds if not v.dev.healthy]
            if unhealthy:
                log.warning("allocating unhealthy vGPUs %s", unhealthy)
            cr = build_container_response(self.cfg, vds, self._by_uuid,
                                          request_ids=requested if self.legacy is not None else None,
                                          using_ids=using, pod_tag=tags[i] if i < len(tags) else None,
                                          pod_uid=self.pod_matcher.owner(tags[i]) if (
                                              self.pod_matcher is not None and i < len(tags) and tags[i]) else None,
                                          kubelet_ids=requested, latency=self.latency,
                                          resource=self.resource_name)
            resp.container_responses.append(cr)
            self.allocations.append((requested, using))
            if self.cfg.verbose > 5:
                log.debug("allocate request %s -> %s", requested, using)
        return resp

    def PreStartContainer(self, request, context):
        return api.PreStartContainerResponse()
