"""Kubernetes API-server adapter: run the controllers against a real cluster
(the reference is a controller-runtime operator, ``cmd/manager/main.go:181-196``, ``pkg/client``).

:class:`KubeClient` speaks the API server's REST protocol (list / get / create / replace /
status subresource / merge patch / delete / chunked ``?watch=1`` streams) with bearer-token or
client-certificate auth from in-cluster service-account files or a kubeconfig.

:class:`KubeStore` is the informer: a :class:`~ome_amd.store.store.Store` whose cache is filled by
an initial LIST per watched kind and kept current by a WATCH thread per kind (resourceVersion
resume, ``410 Gone`` -> relist); reads come from the cache, writes go to the API server first and
the returned object (with the server's resourceVersion) is written into the cache.  The in-process
controllers and watchers therefore run unchanged: they see the cluster's objects and their
events.  Admission runs in the API server (our hooks are served as AdmissionReview webhooks by
:func:`admission_review`), not in the store.
"""
from __future__ import annotations

import base64
import copy
import json
import logging
import os
import ssl
import tempfile
import threading
import time
import urllib.error
import urllib.parse
import urllib.request

from ome_amd.store.store import (CLUSTER_SCOPED, NO_STATUS_SUBRESOURCE, AlreadyExists, APIError, Conflict,
                                 Forbidden, Invalid, NotFound, Store, WatchEvent, gk, group_of)

log = logging.getLogger("ome_amd.kube")

# (group, kind) -> plural; everything not listed falls back to API discovery, then kind+"s"
PLURALS = {
    ("", "Node"): "nodes", ("", "Namespace"): "namespaces", ("", "ConfigMap"): "configmaps",
    ("", "Secret"): "secrets", ("", "Service"): "services", ("", "Pod"): "pods", ("", "Event"): "events",
    ("", "ServiceAccount"): "serviceaccounts", ("", "PersistentVolumeClaim"): "persistentvolumeclaims",
    ("", "PersistentVolume"): "persistentvolumes", ("apps", "Deployment"): "deployments",
    ("batch", "Job"): "jobs", ("autoscaling", "HorizontalPodAutoscaler"): "horizontalpodautoscalers",
    ("policy", "PodDisruptionBudget"): "poddisruptionbudgets", ("networking.k8s.io", "Ingress"): "ingresses",
    ("rbac.authorization.k8s.io", "Role"): "roles", ("rbac.authorization.k8s.io", "RoleBinding"): "rolebindings",
    ("rbac.authorization.k8s.io", "ClusterRole"): "clusterroles",
    ("rbac.authorization.k8s.io", "ClusterRoleBinding"): "clusterrolebindings",
    ("leaderworkerset.x-k8s.io", "LeaderWorkerSet"): "leaderworkersets", ("serving.knative.dev", "Service"): "services",
    ("keda.sh", "ScaledObject"): "scaledobjects", ("gateway.networking.k8s.io", "HTTPRoute"): "httproutes",
    ("networking.istio.io", "VirtualService"): "virtualservices", ("networking.istio.io", "Sidecar"): "sidecars",
    ("ray.io", "RayCluster"): "rayclusters", ("ome.io", "InferenceService"): "inferenceservices",
    ("ome.io", "BaseModel"): "basemodels", ("ome.io", "ClusterBaseModel"): "clusterbasemodels",
    ("ome.io", "ServingRuntime"): "servingruntimes", ("ome.io", "ClusterServingRuntime"): "clusterservingruntimes",
    ("ome.io", "FineTunedWeight"): "finetunedweights", ("ome.io", "AcceleratorClass"): "acceleratorclasses",
    ("ome.io", "BenchmarkJob"): "benchmarkjobs",
}
_ERR = {404: NotFound, 409: Conflict, 422: Invalid, 403: Forbidden, 400: Invalid}


# ------------------------------------------------------------------ client
class KubeClient:
    def __init__(self, server: str, token: str | None = None, ca_file: str | None = None,
                 cert_file: str | None = None, key_file: str | None = None, insecure: bool = False,
                 timeout: float = 30.0):
        self.server = server.rstrip("/")
        self.token, self.timeout = token, timeout
        self.ctx = None
        if self.server.startswith("https"):
            self.ctx = ssl.create_default_context(cafile=ca_file) if ca_file else ssl.create_default_context()
            if insecure:
                self.ctx.check_hostname = False
                self.ctx.verify_mode = ssl.CERT_NONE
            if cert_file:
                self.ctx.load_cert_chain(cert_file, key_file)
        self._plural_cache: dict[tuple[str, str, str], tuple[str, bool]] = {}

    # ---- construction
    @classmethod
    def in_cluster(cls) -> "KubeClient":
        sa = "/var/run/secrets/kubernetes.io/serviceaccount"
        host, port = os.environ["KUBERNETES_SERVICE_HOST"], os.environ.get("KUBERNETES_SERVICE_PORT", "443")
        return cls(f"https://{host}:{port}", open(f"{sa}/token").read().strip(), f"{sa}/ca.crt")

    @classmethod
    def from_kubeconfig(cls, path: str | None = None, context: str | None = None) -> "KubeClient":
        import yaml

        path = os.path.expanduser(path or os.environ.get("KUBECONFIG", "~/.kube/config"))
        cfg = yaml.safe_load(open(path))
        ctx_name = context or cfg.get("current-context")
        ctx = next(c["context"] for c in cfg["contexts"] if c["name"] == ctx_name)
        cl = next(c["cluster"] for c in cfg["clusters"] if c["name"] == ctx["cluster"])
        user = next((u["user"] for u in cfg.get("users", []) if u["name"] == ctx.get("user")), {})

        def materialise(data_key, file_key, src):
            if src.get(file_key):
                return os.path.expanduser(src[file_key])
            if src.get(data_key):
                f = tempfile.NamedTemporaryFile(delete=False, suffix=".pem")
                f.write(base64.b64decode(src[data_key]))
                f.close()
                return f.name
            return None

        token = user.get("token")
        if not token and user.get("tokenFile"):
            token = open(os.path.expanduser(user["tokenFile"])).read().strip()
        return cls(cl["server"], token, materialise("certificate-authority-data", "certificate-authority", cl),
                   materialise("client-certificate-data", "client-certificate", user),
                   materialise("client-key-data", "client-key", user), bool(cl.get("insecure-skip-tls-verify")))

    # ---- paths
    def resource(self, api_version: str, kind: str) -> tuple[str, bool]:
        g = group_of(api_version)
        key = (api_version, g, kind)
        got = self._plural_cache.get(key)
        if got:
            return got
        plural = PLURALS.get((g, kind))
        namespaced = (g, kind) not in CLUSTER_SCOPED
        if plural is None:
            try:
                base = "/api/v1" if api_version == "v1" else f"/apis/{api_version}"
                _, body = self.request("GET", base)
                for r in body.get("resources", []):
                    if r.get("kind") == kind and "/" not in r["name"]:
                        plural, namespaced = r["name"], bool(r.get("namespaced"))
                        break
            except APIError:
                pass
            plural = plural or kind.lower() + "s"
        self._plural_cache[key] = (plural, namespaced)
        return plural, namespaced

    def path(self, api_version: str, kind: str, namespace: str | None = None, name: str | None = None,
             sub: str | None = None) -> str:
        plural, namespaced = self.resource(api_version, kind)
        base = "/api/v1" if api_version == "v1" else f"/apis/{api_version}"
        p = base + (f"/namespaces/{namespace or 'default'}" if namespaced and namespace is not None else "")
        p += f"/{plural}" + (f"/{name}" if name else "") + (f"/{sub}" if sub else "")
        return p

    # ---- HTTP
    def _open(self, method: str, path: str, body: dict | None = None, content_type: str = "application/json",
              timeout: float | None = None):
        data = json.dumps(body).encode() if body is not None else None
        h = {"Accept": "application/json"}
        if data is not None:
            h["Content-Type"] = content_type
        if self.token:
            h["Authorization"] = f"Bearer {self.token}"
        req = urllib.request.Request(self.server + path, data=data, method=method, headers=h)
        try:
            return urllib.request.urlopen(req, timeout=timeout or self.timeout, context=self.ctx)
        except urllib.error.HTTPError as e:
            raw = e.read()
            try:
                msg = json.loads(raw).get("message", raw.decode()[:300])
            except ValueError:
                msg = raw.decode(errors="replace")[:300]
            if e.code == 409 and "already exists" in msg:
                raise AlreadyExists(msg) from e
            raise _ERR.get(e.code, APIError)(f"{method} {path}: {e.code} {msg}") from e

    def request(self, method: str, path: str, body: dict | None = None,
                content_type: str = "application/json") -> tuple[int, dict]:
        with self._open(method, path, body, content_type) as r:
            raw = r.read()
            return r.status, (json.loads(raw) if raw else {})

    def watch(self, path: str, resource_version: str, timeout_s: int = 300):
        """Yield (type, object) from a chunked watch stream until the server closes it."""
        q = urllib.parse.urlencode({"watch": "1", "resourceVersion": resource_version,
                                    "allowWatchBookmarks": "true", "timeoutSeconds": str(timeout_s)})
        with self._open("GET", f"{path}?{q}", timeout=timeout_s + 30) as r:
            for line in r:
                line = line.strip()
                if line:
                    ev = json.loads(line)
                    yield ev["type"], ev["object"]


# ------------------------------------------------------------------ informer-backed store
class KubeStore(Store):
    def __init__(self, client: KubeClient, kinds: list[tuple[str, str]], namespace: str | None = None,
                 start_watches: bool = True):
        super().__init__()
        self.client, self.kinds, self.namespace = client, list(kinds), namespace
        self._stop = threading.Event()
        self._threads: list[threading.Thread] = []
        self._kind_rv: dict[tuple[str, str], str] = {}
        for av, kind in self.kinds:
            self._relist(av, kind)
        if start_watches:
            for av, kind in self.kinds:
                t = threading.Thread(target=self._watch_loop, args=(av, kind), daemon=True, name=f"watch-{kind}")
                t.start()
                self._threads.append(t)

    def close(self) -> None:
        self._stop.set()

    # ---- cache maintenance
    def _apply_cache(self, typ: str, obj: dict, notify: bool = True) -> None:
        key = self._okey(obj)
        with self._lock:
            cur = self._objs.get(key)
            rv = obj["metadata"].get("resourceVersion")
            if typ == "DELETED":
                if cur is None:
                    return
                del self._objs[key]
            else:
                if cur is not None and cur["metadata"].get("resourceVersion") == rv:
                    return                       # our own write, already cached
                typ = "MODIFIED" if cur is not None else "ADDED"
                self._objs[key] = copy.deepcopy(obj)
        if notify:
            self._notify([WatchEvent(typ, copy.deepcopy(obj))])

    def _list_path(self, av, kind):
        _, namespaced = self.client.resource(av, kind)
        return self.client.path(av, kind, self.namespace if namespaced else None)

    def _relist(self, av: str, kind: str) -> None:
        _, body = self.client.request("GET", self._list_path(av, kind))
        seen = set()
        for o in body.get("items", []):
            o.setdefault("apiVersion", av)
            o.setdefault("kind", kind)
            seen.add(self._okey(o))
            self._apply_cache("ADDED", o)
        g = group_of(av)
        with self._lock:
            gone = [(k, o) for k, o in self._objs.items() if k[0] == g and k[1] == kind and k not in seen]
        for _, o in gone:
            self._apply_cache("DELETED", o)
        self._kind_rv[(av, kind)] = (body.get("metadata") or {}).get("resourceVersion", "0")

    def _watch_loop(self, av: str, kind: str) -> None:
        backoff = 0.2
        while not self._stop.is_set():
            try:
                for typ, obj in self.client.watch(self._list_path(av, kind), self._kind_rv[(av, kind)]):
                    if self._stop.is_set():
                        return
                    rv = (obj.get("metadata") or {}).get("resourceVersion")
                    if typ == "BOOKMARK":
                        self._kind_rv[(av, kind)] = rv or self._kind_rv[(av, kind)]
                        continue
                    if typ == "ERROR":
                        if obj.get("code") == 410:     # resourceVersion too old: relist
                            self._relist(av, kind)
                        break
                    obj.setdefault("apiVersion", av)
                    obj.setdefault("kind", kind)
                    self._apply_cache(typ, obj)
                    if rv:
                        self._kind_rv[(av, kind)] = rv
                backoff = 0.2
            except NotFound:
                time.sleep(5.0)
            except (APIError, OSError, ValueError) as e:
                if self._stop.is_set():
                    return
                log.warning("watch %s/%s: %s (retrying)", av, kind, e)
                time.sleep(backoff)
                backoff = min(10.0, backoff * 2)
                try:
                    self._relist(av, kind)
                except (APIError, OSError):
                    pass

    # ---- writes go to the API server first
    def _remote(self, method: str, obj: dict, sub: str | None = None, name: bool = True) -> dict:
        av, kind = obj.get("apiVersion", "v1"), obj["kind"]
        m = obj.get("metadata", {})
        _, namespaced = self.client.resource(av, kind)
        ns = (m.get("namespace") or "default") if namespaced else None
        path = self.client.path(av, kind, ns, m["name"] if name else None, sub)
        _, out = self.client.request(method, path, obj)
        out.setdefault("apiVersion", av)
        out.setdefault("kind", kind)
        return out

    def create(self, obj: dict, dry_run: bool = False) -> dict:
        obj = copy.deepcopy(obj)
        obj.setdefault("apiVersion", "v1")
        m = obj.setdefault("metadata", {})
        g, k = gk(obj)
        if self.namespaced(g, k):
            m.setdefault("namespace", "default")
        if dry_run:
            return obj
        out = self._remote("POST", obj, name=False)
        self._apply_cache("ADDED", out)
        return copy.deepcopy(out)

    def update(self, obj: dict, status_only: bool = False) -> dict:
        obj = copy.deepcopy(obj)
        if not obj["metadata"].get("resourceVersion"):
            cur = self.get(obj.get("apiVersion", "v1"), obj["kind"], obj["metadata"]["name"],
                           obj["metadata"].get("namespace"))
            obj["metadata"]["resourceVersion"] = cur["metadata"]["resourceVersion"]
        sub = "status" if status_only and gk(obj) not in NO_STATUS_SUBRESOURCE else None
        out = self._remote("PUT", obj, sub)
        if out["metadata"].get("deletionTimestamp") and not out["metadata"].get("finalizers"):
            self._apply_cache("DELETED", out)
        else:
            self._apply_cache("MODIFIED", out)
        return copy.deepcopy(out)

    def patch(self, api_version: str, kind: str, name: str, patch: dict, namespace: str | None = None,
              status: bool = False) -> dict:
        _, namespaced = self.client.resource(api_version, kind)
        path = self.client.path(api_version, kind, (namespace or "default") if namespaced else None, name,
                                "status" if status else None)
        _, out = self.client.request("PATCH", path, patch, "application/merge-patch+json")
        out.setdefault("apiVersion", api_version)
        out.setdefault("kind", kind)
        self._apply_cache("MODIFIED", out)
        return copy.deepcopy(out)

    def delete(self, api_version: str, kind: str, name: str, namespace: str | None = None,
               ignore_missing: bool = False) -> dict | None:
        cur = self.try_get(api_version, kind, name, namespace)
        _, namespaced = self.client.resource(api_version, kind)
        path = self.client.path(api_version, kind, (namespace or "default") if namespaced else None, name)
        try:
            _, out = self.client.request("DELETE", path, {"propagationPolicy": "Background"})
        except NotFound:
            if ignore_missing:
                if cur is not None:
                    self._apply_cache("DELETED", cur)
                return None
            raise
        if out.get("kind") == kind and (out.get("metadata") or {}).get("deletionTimestamp") and \
                (out["metadata"].get("finalizers")):
            out.setdefault("apiVersion", api_version)
            self._apply_cache("MODIFIED", out)
            return out
        if cur is not None:
            self._apply_cache("DELETED", cur)
        return cur


# ------------------------------------------------------------------ admission webhook server side
def admission_review(store: Store, review: dict) -> dict:
    """``admission.k8s.io/v1`` AdmissionReview -> response: run the store's mutating hooks (JSON
    patch of the changed top-level fields / metadata maps) and validating hooks (deny with the
    hook's message) on the request object."""
    req = review.get("request") or {}
    uid = req.get("uid", "")
    obj, old = req.get("object"), req.get("oldObject")
    op = req.get("operation", "CREATE")
    resp: dict = {"uid": uid, "allowed": True}
    try:
        kind = obj["kind"]
        new = copy.deepcopy(obj)
        for kinds, hook in store.mutating:
            if kinds is None or kind in kinds:
                r = hook(op, new, old, store)
                if r is not None:
                    new = r
        for kinds, hook in store.validating:
            if kinds is None or kind in kinds:
                hook(op, new, old, store)
        ops = []
        for f in sorted(set(obj) | set(new)):
            if f == "metadata":
                for mf in ("labels", "annotations", "finalizers"):
                    a, b = (obj.get("metadata") or {}).get(mf), (new.get("metadata") or {}).get(mf)
                    if a != b:
                        ops.append({"op": "add" if a is None else "replace", "path": f"/metadata/{mf}", "value": b})
            elif f not in new:
                ops.append({"op": "remove", "path": f"/{f}"})
            elif obj.get(f) != new.get(f):
                ops.append({"op": "add" if f not in obj else "replace", "path": f"/{f}", "value": new[f]})
        if ops:
            resp["patchType"] = "JSONPatch"
            resp["patch"] = base64.b64encode(json.dumps(ops).encode()).decode()
    except (Invalid, Forbidden) as e:
        resp = {"uid": uid, "allowed": False, "status": {"code": e.code, "message": str(e)}}
    return {"apiVersion": "admission.k8s.io/v1", "kind": "AdmissionReview", "response": resp}


#: kinds the manager's controllers read or own
MANAGER_KINDS = [
    ("v1", "Node"), ("v1", "Namespace"), ("v1", "ConfigMap"), ("v1", "Secret"), ("v1", "Service"), ("v1", "Pod"),
    ("v1", "ServiceAccount"), ("apps/v1", "Deployment"), ("batch/v1", "Job"),
    ("autoscaling/v2", "HorizontalPodAutoscaler"), ("policy/v1", "PodDisruptionBudget"),
    ("networking.k8s.io/v1", "Ingress"), ("rbac.authorization.k8s.io/v1", "Role"),
    ("rbac.authorization.k8s.io/v1", "RoleBinding"), ("leaderworkerset.x-k8s.io/v1", "LeaderWorkerSet"),
    ("ome.io/v1beta1", "InferenceService"), ("ome.io/v1beta1", "BaseModel"), ("ome.io/v1beta1", "ClusterBaseModel"),
    ("ome.io/v1beta1", "ServingRuntime"), ("ome.io/v1beta1", "ClusterServingRuntime"),
    ("ome.io/v1beta1", "FineTunedWeight"), ("ome.io/v1beta1", "AcceleratorClass"), ("ome.io/v1beta1", "BenchmarkJob"),
]
