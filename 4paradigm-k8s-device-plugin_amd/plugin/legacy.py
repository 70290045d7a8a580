"""Legacy preferred-allocation controller ("vdevice-controller").

Reference: ``vdevice-controller.go`` — for kubelets without GetPreferredAllocation the
plugin keeps ``idMap[vdeviceID] -> requestedID`` (:33-57), rebuilds it from the kubelet's
device-manager checkpoint (``kubelet_internal_checkpoint``, JSON
``{Data: {PodDeviceEntries: [{PodUID, ContainerName, ResourceName, DeviceIDs,
AllocResp}], RegisteredDevices}, Checksum}``, vendor ``checkpoint.go:33-85``) by
unmarshalling each ``AllocResp`` and reading the request/using annotations, acquires for
pods that are Pending/Running and releases the rest (:60-111), and substitutes the
kubelet-chosen IDs in ``Allocate`` with preferred ones (:231-286).

Checkpoint checksum verification is skipped (the kubelet computes it over a Go-specific
deep-print of the struct; reading is all the plugin does). The pod phase lookup goes
through a ``pod_lister`` callable (``k8s.PodClient.pods_on_node``), so tests inject
fakes; with no lister every checkpointed pod is treated as live.
"""
import base64
import json
import logging
import os
import threading

from . import api
from .contract import ANN_REQUEST, ANN_USING

CHECKPOINT_NAME = "kubelet_internal_checkpoint"
log = logging.getLogger("amdvgpu.legacy")


def read_checkpoint(path):
    """Returns the list of PodDevicesEntry dicts (AllocResp decoded to bytes)."""
    with open(path) as f:
        data = json.load(f)
    entries = (data.get("Data") or {}).get("PodDeviceEntries") or []
    out = []
    for e in entries:
        raw = e.get("AllocResp") or ""
        try:
            blob = base64.b64decode(raw) if isinstance(raw, str) else bytes(raw)
        except Exception:
            blob = b""
        ids = e.get("DeviceIDs")
        if isinstance(ids, dict):  # newer kubelets: {numa_node: [ids]}
            ids = [i for v in ids.values() for i in v]
        out.append({"PodUID": e.get("PodUID", ""), "ContainerName": e.get("ContainerName", ""),
                    "ResourceName": e.get("ResourceName", ""), "DeviceIDs": ids or [], "AllocResp": blob})
    return out


class LegacyController:
    def __init__(self, device_ids, resource_name, plugin_path, pod_lister=None):
        self._mu = threading.Lock()
        self.id_map = {i: "" for i in device_ids}
        self.resource_name = resource_name
        self.checkpoint = os.path.join(plugin_path, CHECKPOINT_NAME)
        self.pod_lister = pod_lister

    def update_from_checkpoint(self):
        try:
            entries = read_checkpoint(self.checkpoint)
        except (OSError, ValueError) as e:
            log.error("read checkpoint error: %s", e)
            return False
        phases = None
        if self.pod_lister is not None:
            try:
                phases = {p["uid"]: p.get("phase", "") for p in self.pod_lister()}
            except Exception as e:
                log.warning("pod list failed: %s", e)
        for e in entries:
            if e["ResourceName"] != self.resource_name:
                continue
            try:
                resp = api.ContainerAllocateResponse.FromString(e["AllocResp"])
            except Exception:
                log.error("unmarshal container allocate response failed")
                continue
            req_s, use_s = resp.annotations.get(ANN_REQUEST, ""), resp.annotations.get(ANN_USING, "")
            if not req_s and not use_s:
                continue
            request, using = req_s.split(","), use_s.split(",")
            live = phases is None or phases.get(e["PodUID"]) in ("Pending", "Running")
            if live:
                self.acquire(request, using)
            else:
                self.release(using)
        return True

    def available(self, order=None):
        with self._mu:
            ids = [k for k, v in self.id_map.items() if v == ""]
        if order:
            pos = {k: i for i, k in enumerate(order)}
            ids.sort(key=lambda k: pos.get(k, len(pos)))
        return ids

    def acquire(self, request, using):
        with self._mu:
            for i, v in enumerate(using):
                if v not in self.id_map:
                    log.error("device %s unknown", v)
                    continue
                self.id_map[v] = request[i] if i < len(request) else "mismatched"

    def release(self, using):
        with self._mu:
            for v in using:
                if v in self.id_map:
                    self.id_map[v] = ""
                else:
                    log.error("device %s unknown", v)

    def release_by_request(self, request):
        req = set(request)
        with self._mu:
            for k, v in self.id_map.items():
                if v and v in req:
                    log.warning("device %s[%s] lost", k, v)
                    self.id_map[k] = ""
