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
    """Pod fields the plugin uses. Containers are listed in the order the kubelet
    allocates their devices: init containers first, then the app containers."""
    meta, spec, status = p.get("metadata", {}), p.get("spec", {}), p.get("status", {})
    ctrs = []
    for c in list(spec.get("initContainers") or []) + list(spec.get("containers") or []):
        lim = (c.get("resources", {}).get("limits") or {}).get(resource, "0")
        ctrs.append({"name": c.get("name", ""), "gpus": int(lim or 0)})
    return {"uid": meta.get("uid", ""), "name": meta.get("name", ""), "namespace": meta.get("namespace", ""),
            "phase": status.get("phase", ""), "containers": ctrs,
            "created": meta.get("creationTimestamp", "")}


POD_MARKER = ".pod-uid"
TERMINAL_PHASES = ("Succeeded", "Failed")


def pod_tag(pod, container):
    """"<namespace>_<pod>_<container>" (Kubernetes names never contain "_")."""
    prefix = f"{pod['namespace']}_" if pod.get("namespace") else ""
    return f"{prefix}{pod['name']}_{container}"


class PodMatcher:
    """Monitor mode: find the pod and container an ``Allocate`` is for, and name it.

    The kubelet's Allocate carries only device IDs. The reference lists every pod of the
    cluster and picks the first pending pod whose per-container GPU counts equal the
    *whole* request (server.go:381-405) - but a kubelet calls Allocate once per container,
    so a pod with two GPU containers never matches. Here the request is matched against
    the next not-yet-allocated GPU containers of the pending pods on this node, in the
    order the kubelet allocates them (init containers, then containers), oldest pod first.
    A container counts as allocated once a previous Allocate took it - remembered here and,
    across plugin restarts, by the ``.pod-uid`` marker the contract writes into the
    container's host directory (a directory left by a deleted pod of the same name has
    another UID and does not count).

    Returns one "<namespace>_<pod>_<container>" tag per container request (the
    reference's "<pod>_<container>" would give two same-named pods of different namespaces
    one host directory, so the monitor would control both as one container); ``owner(tag)``
    is the pod UID the tag was matched to.
    """

    def __init__(self, list_pods, shared_root=None):
        self.list_pods = list_pods
        self.shared_root = shared_root
        self._owner = {}        # tag -> pod uid of the current allocation
        self.last_pods = None   # the pod list of the last successful match (for GC)

    def owner(self, tag):
        return self._owner.get(tag)

    def _allocated(self, uid, tag):
        if self._owner.get(tag) == uid:
            return True
        if self.shared_root:
            try:
                with open(os.path.join(self.shared_root, tag, POD_MARKER)) as f:
                    return f.read().strip() == uid
            except OSError:
                return False
        return False

    def match(self, request_sizes):
        self.last_pods = None
        pods = self.list_pods()
        self.last_pods = pods
        pending = sorted((p for p in pods if p.get("phase") == "Pending"), key=lambda p: p.get("created", ""))
        want = list(request_sizes)
        for p in pending:
            todo = [c for c in p["containers"] if c["gpus"] > 0 and not self._allocated(p["uid"], pod_tag(p, c["name"]))]
            if [c["gpus"] for c in todo[:len(want)]] == want:
                tags = [pod_tag(p, c["name"]) for c in todo[:len(want)]]
                for t in tags:
                    self._owner[t] = p["uid"]
                return tags
        raise LookupError(f"no pending pod has unallocated containers requesting {want} GPUs")
