"""Stub kubelet: the other end of the device-plugin API, for tests and the GPU slice.

Implements what the real kubelet does with a device plugin (``Registration.Register``
on ``kubelet.sock``, then dialling the plugin's endpoint for ``ListAndWatch`` /
``GetPreferredAllocation`` / ``Allocate``), plus pod emulation: ``run_pod`` allocates
vGPUs for a container and starts a process under the returned contract through the
container-runtime emulator (``shim/launcher.py``). This is BASELINE.json config 1 and
the SURVEY.md §7.3 end-to-end slice; the reference has no equivalent.

    python -m amdvgpu.plugin.kubelet_stub --plugin-dir DIR [--gpus 1] -- python train.py
"""
import argparse
import os
import sys
import threading
import time
from concurrent import futures

import grpc

from . import api


class StubKubelet:
    def __init__(self, plugin_dir):
        self.plugin_dir = plugin_dir
        self.socket = os.path.join(plugin_dir, "kubelet.sock")
        self.registrations = []
        self._registered = threading.Condition()
        self.devices = {}          # resource -> {id: health}
        self.topologies = {}       # resource -> {id: [numa node, ...]}
        self._streams = {}
        self._server = None
        self.allocated = set()

    # ----------------------------------------------------------------- Registration service
    def Register(self, request, context):
        if request.version not in api.SUPPORTED_VERSIONS:
            context.abort(grpc.StatusCode.INVALID_ARGUMENT, f"unsupported version {request.version}")
        with self._registered:
            self.registrations.append(request)
            self._registered.notify_all()
        threading.Thread(target=self._watch, args=(request.resource_name, request.endpoint), daemon=True).start()
        return api.Empty()

    def start(self):
        os.makedirs(self.plugin_dir, exist_ok=True)
        try:
            os.unlink(self.socket)
        except FileNotFoundError:
            pass
        s = grpc.server(futures.ThreadPoolExecutor(max_workers=4))
        s.add_generic_rpc_handlers((api.service_handler("Registration", self),))
        s.add_insecure_port(api.unix_target(self.socket))
        s.start()
        self._server = s
        return self

    def stop(self):
        for ch, _ in self._streams.values():
            ch.close()
        self._streams.clear()
        if self._server:
            self._server.stop(0).wait(2)
            self._server = None

    def restart(self):
        """Kubelet restart: the socket is re-created, plugins must re-register."""
        self.stop()
        with self._registered:
            self.registrations.clear()
        self.devices.clear()
        return self.start()

    def wait_registered(self, resource=None, timeout=10.0, count=1):
        def ok():
            regs = [r for r in self.registrations if resource is None or r.resource_name == resource]
            return len(regs) >= count
        with self._registered:
            if not self._registered.wait_for(ok, timeout=timeout):
                raise TimeoutError(f"no registration for {resource} within {timeout}s")
        return [r for r in self.registrations if resource is None or r.resource_name == resource][-1]

    # ----------------------------------------------------------------- plugin client side
    def _channel(self, endpoint):
        return grpc.insecure_channel(api.unix_target(os.path.join(self.plugin_dir, endpoint)))

    def _watch(self, resource, endpoint):
        ch = self._channel(endpoint)
        stub = api.device_plugin_stub(ch)
        self._streams[resource] = (ch, stub)
        try:
            for resp in stub.ListAndWatch(api.Empty()):
                self.devices[resource] = {d.ID: d.health for d in resp.devices}
                self.topologies[resource] = {d.ID: [n.ID for n in d.topology.nodes] for d in resp.devices}
        except grpc.RpcError:
            pass

    def stub_for(self, resource):
        reg = next(r for r in reversed(self.registrations) if r.resource_name == resource)
        return api.device_plugin_stub(self._channel(reg.endpoint))

    def topology(self, resource):
        """NUMA nodes of each advertised device (its TopologyInfo), as last listed."""
        return dict(self.topologies.get(resource, {}))

    def wait_devices(self, resource, timeout=10.0, predicate=None):
        t0 = time.time()
        while time.time() - t0 < timeout:
            devs = self.devices.get(resource)
            if devs and (predicate is None or predicate(devs)):
                return devs
            time.sleep(0.05)
        raise TimeoutError(f"no device list for {resource}")

    def allocate(self, resource, count):
        """kubelet device-manager flow: pick healthy free devices (preferred allocation
        when the plugin supports it), then Allocate. Returns (ids, ContainerAllocateResponse)."""
        stub = self.stub_for(resource)
        opts = stub.GetDevicePluginOptions(api.Empty())
        devs = self.wait_devices(resource)
        free = [i for i, h in devs.items() if h == api.HEALTHY and i not in self.allocated]
        if len(free) < count:
            raise RuntimeError(f"insufficient {resource}: want {count}, free {len(free)}")
        ids = free[:count]
        if opts.get_preferred_allocation_available:
            pref = stub.GetPreferredAllocation(api.PreferredAllocationRequest(container_requests=[
                api.ContainerPreferredAllocationRequest(available_deviceIDs=free, allocation_size=count)]))
            got = list(pref.container_responses[0].deviceIDs)
            if len(got) == count:
                ids = got
        resp = stub.Allocate(api.AllocateRequest(container_requests=[api.ContainerAllocateRequest(devicesIDs=ids)]))
        self.allocated.update(ids)
        return ids, resp.container_responses[0]

    def allocate_ids(self, resource, ids):
        """Allocate exactly ``ids`` (a pod pinned to given vGPUs, e.g. a benchmark rank's
        own GPU). Returns the ContainerAllocateResponse."""
        stub = self.stub_for(resource)
        devs = self.wait_devices(resource)
        missing = [i for i in ids if i not in devs]
        if missing:
            raise RuntimeError(f"unknown {resource} devices {missing}")
        resp = stub.Allocate(api.AllocateRequest(container_requests=[api.ContainerAllocateRequest(
            devicesIDs=list(ids))]))
        self.allocated.update(ids)
        return resp.container_responses[0]

    def release(self, ids):
        self.allocated.difference_update(ids)


class NodeHarness:
    """A device plugin (``main.Supervisor``) registered with a stub kubelet in a private
    directory: the node side of a pod's life, for benchmarks and GPU tests. ``pod(ids)``
    returns the (envs, mounts) the kubelet would hand to the container runtime for a
    container holding vGPUs ``ids``; ``launcher.apply_contract`` turns them into a
    process environment.

        with NodeHarness(SysfsBackend(), device_split_count=4) as node:
            envs, mounts = node.pod([f"{uuid}-0"])
    """

    def __init__(self, backend, resource="amd.com/gpu", workdir=None, **cfg_kw):
        import tempfile
        self.backend = backend
        self.resource = resource
        self._own_dir = workdir is None
        self.dir = workdir or tempfile.mkdtemp(prefix="vgpu-node-")
        self.cfg_kw = cfg_kw
        self.kubelet = None
        self._sup = None
        self._stop = None
        self._thread = None

    def __enter__(self):
        from .config import PluginConfig
        from .main import Supervisor
        pdir = os.path.join(self.dir, "device-plugins")
        os.makedirs(pdir, exist_ok=True)
        kw = dict(device_plugin_path=pdir + "/", shared_cache_dir=self.dir, vgpu_dir=os.path.join(self.dir, "vgpu"),
                  resource_name=self.resource)
        kw.update(self.cfg_kw)
        cfg = PluginConfig(**kw).validate()
        self.kubelet = StubKubelet(pdir).start()
        self._sup = Supervisor(cfg, backend=self.backend, install_signals=False)
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._sup.run, args=(self._stop,), daemon=True)
        self._thread.start()
        self.kubelet.wait_registered(self.resource, timeout=30)
        self.kubelet.wait_devices(self.resource, timeout=30)
        return self

    def __exit__(self, *exc):
        if self._stop:
            self._stop.set()
        if self._thread:
            self._thread.join(10)
        if self.kubelet:
            self.kubelet.stop()
        if self._own_dir:
            import shutil
            shutil.rmtree(self.dir, ignore_errors=True)

    def vgpu_ids(self, uuid):
        """The advertised vGPU IDs of physical GPU ``uuid``, in slot order."""
        ids = [i for i in self.kubelet.devices.get(self.resource, {}) if i.rsplit("-", 1)[0] == uuid]
        return sorted(ids, key=lambda i: int(i.rsplit("-", 1)[1]))

    def pod(self, ids):
        from .contract import response_to_env
        return response_to_env(self.kubelet.allocate_ids(self.resource, ids))


def run_pod(kubelet, resource, count, cmd, **kw):
    """Allocate ``count`` vGPUs and run ``cmd`` under the contract (container emulation)."""
    from ..shim.launcher import run
    from .contract import response_to_env
    ids, resp = kubelet.allocate(resource, count)
    envs, mounts = response_to_env(resp)
    try:
        return ids, envs, run(cmd, envs, mounts, **kw)
    finally:
        kubelet.release(ids)


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--plugin-dir", required=True)
    ap.add_argument("--resource", default="amd.com/gpu")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--wait", type=float, default=30.0)
    ap.add_argument("cmd", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    k = StubKubelet(a.plugin_dir).start()
    try:
        k.wait_registered(a.resource, timeout=a.wait)
        cmd = a.cmd[1:] if a.cmd and a.cmd[0] == "--" else a.cmd
        ids, envs, proc = run_pod(k, a.resource, a.gpus, cmd)
        print(f"pod ran on {ids} rc={proc.returncode}", file=sys.stderr)
        return proc.returncode
    finally:
        k.stop()


if __name__ == "__main__":
    sys.exit(main())
