"""Minimal in-cluster Kubernetes API client (pods on this node) for monitor mode and the
legacy-preferred controller.

Reference: client-go usage in ``server.go:365-406`` (monitor mode: ``Pods("").List`` of
**all** namespaces on every Allocate, then pick the pending pod whose per-container
``nvidia.com/gpu`` requests match) and ``vdevice-controller.go:162-223`` (node-scoped pod
informer via ``spec.nodeName=$NODE_NAME``). Here both use one node-scoped list
(fieldSelector ``spec.nodeName``) over HTTPS with the pod's service-account token; no
client-go equivalent is needed. ``PodClient`` is injectable, tests use fakes.
"""
import json
import os
import ssl
import urllib.parse
import urllib.request

SA_DIR = "/var/run/secrets/kubernetes.io/serviceaccount"


class PodClient:
    def __init__(self, node_name, host=None, port=None, token_path=None, ca_path=None, timeout=5.0):
        self.node_name = node_name
        host = host or os.environ.get("KUBERNETES_SERVICE_HOST", "kubernetes.default.svc")
        port = port or os.environ.get("KUBERNETES_SERVICE_PORT", "443")
        self.base = f"https://{host}:{port}"
        self.token_path = token_path or os.path.join(SA_DIR, "token")
        self.ca_path = ca_path or os.path.join(SA_DIR, "ca.crt")
        self.timeout = timeout

    def _get(self, path, params):
        url = self.base + path + "?" + urllib.parse.urlencode(params)
        req = urllib.request.Request(url)
        with open(self.token_path) as f:
            req.add_header("Authorization", "Bearer " + f.read().strip())
        ctx = ssl.create_default_context(cafile=self.ca_path if os.path.exists(self.ca_path) else None)
        with urllib.request.urlopen(req, timeout=self.timeout, context=ctx) as r:
            return json.loads(r.read())

    def pods_on_node(self):
        data = self._get("/api/v1/pods", {"fieldSelector": f"spec.nodeName={self.node_name}"})
        return [pod_summary(p) for p in data.get("items", [])]


def pod_summary(p, resource="amd.com/gpu"):
    meta, spec, status = p.get("metadata", {}), p.get("spec", {}), p.get("status", {})
    ctrs = []
    for c in spec.get("containers", []):
        lim = (c.get("resources", {}).get("limits") or {}).get(resource, "0")
        ctrs.append({"name": c.get("name", ""), "gpus": int(lim or 0)})
    return {"uid": meta.get("uid", ""), "name": meta.get("name", ""), "namespace": meta.get("namespace", ""),
            "phase": status.get("phase", ""), "containers": ctrs,
            "created": meta.get("creationTimestamp", "")}


class PodMatcher:
    """Monitor mode: find the pending pod being allocated and name its containers.

    The kubelet's Allocate carries only device IDs; the reference recovers the pod by
    matching per-container GPU counts against pending pods (server.go:381-405). Matching
    is over containers *with* GPUs, in order; the oldest matching pending pod wins.
    Returns one "<namespace>_<pod>_<container>" tag per container request (the
    reference's "<pod>_<container>" would give two same-named pods of different namespaces
    one host directory, so the monitor would control both as one container). Kubernetes
    names never contain "_", so the tag is unambiguous.
    """

    def __init__(self, list_pods):
        self.list_pods = list_pods

    def match(self, request_sizes):
        pods = [p for p in self.list_pods() if p.get("phase") == "Pending"]
        pods.sort(key=lambda p: p.get("created", ""))
        for p in pods:
            gpu_ctrs = [c for c in p["containers"] if c["gpus"] > 0]
            if [c["gpus"] for c in gpu_ctrs] == list(request_sizes):
                prefix = f"{p['namespace']}_" if p.get("namespace") else ""
                return [f"{prefix}{p['name']}_{c['name']}" for c in gpu_ctrs]
        raise LookupError(f"no pending pod requests {request_sizes} GPUs per container")
