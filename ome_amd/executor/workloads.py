"""Workload controllers of the local node executor (stand-ins for kube-controller-manager,
the LeaderWorkerSet controller, KubeRay and Knative on a single 8xMI355X box).

* Deployment -> Pods (template hash = revision; rolling replacement honours maxSurge 1 /
  maxUnavailable 0 by creating the new pod before deleting the old one), status replicas /
  readyReplicas / availableReplicas + Available / Progressing conditions.
* LeaderWorkerSet -> ``replicas`` groups of ``size`` pods (leader ``<lws>-<g>``, workers
  ``<lws>-<g>-<i>``) with the LWS env contract (``LWS_LEADER_ADDRESS``, ``LWS_GROUP_SIZE``,
  ``LWS_WORKER_INDEX``, ``LWS_GROUP_INDEX``) and **RecreateGroupOnPodRestart**: when any pod of
  a group restarts or fails, the whole group is deleted and recreated (collectives cannot
  survive a lost rank).
* Job -> one pod (restartPolicy Never), Complete / Failed conditions.
* Knative Service -> a Deployment-equivalent ReplicaSet of pods + Ready condition.
* RayCluster -> head + worker pods, ``status.state = ready`` when all are ready.
* HorizontalPodAutoscaler / ScaledObject -> replica targets (metrics-driven autoscaling on the
  engines' own ``/metrics`` lives in :mod:`ome_amd.executor.autoscaler`).
"""
from __future__ import annotations

import copy
import hashlib
import json
import sys

from ome_amd.api import constants as C
from ome_amd.controllers.runtime import Controller, Result
from ome_amd.store.store import Store, now_iso, owner_ref


def template_hash(tmpl: dict) -> str:
    return hashlib.sha256(json.dumps(tmpl, sort_keys=True).encode()).hexdigest()[:10]


def pod_ready(p: dict) -> bool:
    return any(c.get("type") == "Ready" and c.get("status") == "True"
               for c in (p.get("status") or {}).get("conditions") or [])


def pod_failed(p: dict) -> bool:
    return (p.get("status") or {}).get("phase") == "Failed"


def restart_count(p: dict) -> int:
    return sum(int(cs.get("restartCount", 0)) for cs in (p.get("status") or {}).get("containerStatuses") or [])


def make_pod(owner: dict, name: str, tmpl: dict, extra_labels: dict | None = None, extra_env: dict | None = None,
             hostname: str | None = None) -> dict:
    meta = copy.deepcopy(tmpl.get("metadata") or {})
    labels = {**(meta.get("labels") or {}), **(extra_labels or {})}
    spec = copy.deepcopy(tmpl.get("spec") or {})
    if extra_env:
        for c in spec.get("containers") or []:
            env = c.setdefault("env", [])
            for k, v in extra_env.items():
                if not any(e.get("name") == k for e in env):
                    env.append({"name": k, "value": str(v)})
    if hostname:
        spec.setdefault("hostname", hostname)
    return {"apiVersion": "v1", "kind": "Pod",
            "metadata": {"name": name, "namespace": owner["metadata"].get("namespace", "default"), "labels": labels,
                         "annotations": meta.get("annotations") or {}, "ownerReferences": [owner_ref(owner)]},
            "spec": spec}


def _set_cond(status: dict, ctype: str, ok: bool, reason: str = "", message: str = "") -> None:
    conds = status.setdefault("conditions", [])
    st = "True" if ok else "False"
    for c in conds:
        if c["type"] == ctype:
            if c["status"] != st:
                c["lastTransitionTime"] = now_iso()
            c.update({"status": st, "reason": reason, "message": message})
            return
    conds.append({"type": ctype, "status": st, "reason": reason, "message": message, "lastTransitionTime": now_iso()})


def _owned_pods(store: Store, owner: dict) -> list[dict]:
    uid = owner["metadata"]["uid"]
    return [p for p in store.list("v1", "Pod", owner["metadata"].get("namespace"))
            if any(r.get("uid") == uid for r in p["metadata"].get("ownerReferences") or [])]


def _update_status(store: Store, obj: dict, status: dict) -> None:
    if (obj.get("status") or {}) != status:
        obj["status"] = status
        store.update_status(obj)


# ------------------------------------------------------------------ Deployment
class DeploymentController:
    api, kind = "apps/v1", "Deployment"

    def __init__(self, store: Store):
        self.store = store

    def desired_replicas(self, d: dict) -> int:
        return int((d.get("spec") or {}).get("replicas", 1))

    def reconcile(self, key) -> Result:
        ns, name = key
        d = self.store.try_get(self.api, self.kind, name, ns)
        if d is None or d["metadata"].get("deletionTimestamp"):
            return Result()
        tmpl = d["spec"]["template"]
        rev = template_hash(tmpl)
        want = self.desired_replicas(d)
        pods = _owned_pods(self.store, d)
        cur = [p for p in pods if p["metadata"]["labels"].get("pod-template-hash") == rev]
        old = [p for p in pods if p not in cur]
        # replace failed current pods
        for p in cur:
            if pod_failed(p) and (p["spec"].get("restartPolicy") or "Always") != "Never":
                self.store.delete("v1", "Pod", p["metadata"]["name"], ns, ignore_missing=True)
        cur = [p for p in cur if not pod_failed(p)]
        names = {p["metadata"]["name"] for p in pods}
        i = 0
        while len(cur) < want:
            pname = f"{name}-{rev}-{i}"
            i += 1
            if pname in names:
                continue
            lab = {"pod-template-hash": rev}
            cur.append(self.store.create(make_pod(d, pname, tmpl, lab)))
        for p in sorted(cur, key=lambda p: p["metadata"]["name"])[want:]:
            self.store.delete("v1", "Pod", p["metadata"]["name"], ns, ignore_missing=True)
        cur = cur[:want]
        ready_new = sum(1 for p in cur if pod_ready(p))
        # rolling update: drop old pods only once enough new pods are ready (maxUnavailable 0)
        if old and ready_new >= want:
            for p in old:
                self.store.delete("v1", "Pod", p["metadata"]["name"], ns, ignore_missing=True)
            old = []
        ready = ready_new + sum(1 for p in old if pod_ready(p))
        st = copy.deepcopy(d.get("status") or {})
        st.update({"replicas": len(cur) + len(old), "updatedReplicas": len(cur), "readyReplicas": ready,
                   "availableReplicas": ready, "observedGeneration": d["metadata"].get("generation", 1)})
        _set_cond(st, "Available", ready >= max(1, want) if want > 0 else True,
                  "MinimumReplicasAvailable" if ready >= want else "MinimumReplicasUnavailable",
                  f"{ready}/{want} replicas ready")
        _set_cond(st, "Progressing", True, "NewReplicaSetAvailable" if not old else "ReplicaSetUpdated", "")
        _update_status(self.store, d, st)
        return Result(requeue_after=None if ready >= want and not old else 1.0)


# ------------------------------------------------------------------ LeaderWorkerSet
class LWSController:
    api, kind = "leaderworkerset.x-k8s.io/v1", "LeaderWorkerSet"

    def __init__(self, store: Store, leader_address_fn=None):
        self.store = store
        self.leader_address_fn = leader_address_fn or (lambda pod_name: "127.0.0.1")

    def reconcile(self, key) -> Result:
        ns, name = key
        lws = self.store.try_get(self.api, self.kind, name, ns)
        if lws is None or lws["metadata"].get("deletionTimestamp"):
            return Result()
        sp = lws["spec"]
        lwt = sp["leaderWorkerTemplate"]
        size = int(lwt.get("size", 1))
        replicas = int(sp.get("replicas", 1))
        rev = template_hash(lwt)
        pods = _owned_pods(self.store, lws)
        groups_ready = 0
        for g in range(replicas):
            leader_name = f"{name}-{g}"
            members = [p for p in pods if p["metadata"]["labels"].get("leaderworkerset.sigs.k8s.io/group-index") == str(g)]
            stale = [p for p in members if p["metadata"]["labels"].get("leaderworkerset.sigs.k8s.io/template-revision-hash") != rev]
            broken = any(pod_failed(p) or restart_count(p) > 0 for p in members)
            if (stale or broken) and lwt.get("restartPolicy", "RecreateGroupOnPodRestart") == "RecreateGroupOnPodRestart":
                for p in members:
                    self.store.delete("v1", "Pod", p["metadata"]["name"], ns, ignore_missing=True)
                members = []
            have = {p["metadata"]["name"] for p in members}
            leader_host = self.leader_address_fn(leader_name)
            base_labels = {C.LWS_NAME_LABEL: name, "leaderworkerset.sigs.k8s.io/group-index": str(g),
                           "leaderworkerset.sigs.k8s.io/template-revision-hash": rev,
                           "leaderworkerset.sigs.k8s.io/group-key": f"{name}-{g}"}
            env = {C.LWS_LEADER_ADDRESS_ENV: leader_host, C.LWS_GROUP_SIZE_ENV: size, "LWS_GROUP_INDEX": g}
            leader_exists = leader_name in have
            if not leader_exists:
                lab = {**base_labels, C.LWS_WORKER_INDEX_LABEL: "0"}
                self.store.create(make_pod(lws, leader_name, lwt["leaderTemplate"] or lwt["workerTemplate"], lab,
                                           {**env, C.LWS_WORKER_INDEX_ENV: 0}, hostname=leader_name))
            # StartupPolicy LeaderCreated: workers are created once the leader pod exists
            if leader_exists or sp.get("startupPolicy", "LeaderCreated") == "LeaderCreated":
                for i in range(1, size):
                    wn = f"{name}-{g}-{i}"
                    if wn not in have:
                        lab = {**base_labels, C.LWS_WORKER_INDEX_LABEL: str(i)}
                        self.store.create(make_pod(lws, wn, lwt["workerTemplate"], lab,
                                                   {**env, C.LWS_WORKER_INDEX_ENV: i}, hostname=wn))
            members = [p for p in _owned_pods(self.store, lws)
                       if p["metadata"]["labels"].get("leaderworkerset.sigs.k8s.io/group-index") == str(g)]
            if len(members) == size and all(pod_ready(p) for p in members):
                groups_ready += 1
        for p in pods:  # scale down surplus groups
            gi = int(p["metadata"]["labels"].get("leaderworkerset.sigs.k8s.io/group-index", "0"))
            if gi >= replicas:
                self.store.delete("v1", "Pod", p["metadata"]["name"], ns, ignore_missing=True)
        st = copy.deepcopy(lws.get("status") or {})
        st.update({"replicas": replicas, "readyReplicas": groups_ready, "updatedReplicas": replicas,
                   "hpaPodSelector": f"{C.LWS_NAME_LABEL}={name},{C.LWS_WORKER_INDEX_LABEL}=0"})
        ok = groups_ready >= replicas
        _set_cond(st, "Available", ok, "AllGroupsReady" if ok else "GroupsNotReady", f"{groups_ready}/{replicas} groups ready")
        _update_status(self.store, lws, st)
        return Result(requeue_after=None if ok else 1.0)


# ------------------------------------------------------------------ Job
class JobController:
    api, kind = "batch/v1", "Job"

    def __init__(self, store: Store):
        self.store = store

    def reconcile(self, key) -> Result:
        ns, name = key
        job = self.store.try_get(self.api, self.kind, name, ns)
        if job is None or job["metadata"].get("deletionTimestamp"):
            return Result()
        st = copy.deepcopy(job.get("status") or {})
        if any(c.get("type") in ("Complete", "Failed") and c.get("status") == "True" for c in st.get("conditions") or []):
            return Result()
        pods = _owned_pods(self.store, job)
        if not pods:
            tmpl = copy.deepcopy(job["spec"]["template"])
            tmpl.setdefault("spec", {}).setdefault("restartPolicy", "Never")
            self.store.create(make_pod(job, f"{name}-0", tmpl, {"job-name": name}))
            st.setdefault("startTime", now_iso())
            st["active"] = 1
        else:
            p = pods[0]
            phase = (p.get("status") or {}).get("phase")
            if phase == "Succeeded":
                st.update({"active": 0, "succeeded": 1, "completionTime": now_iso()})
                _set_cond(st, "Complete", True, "Completed", "")
                term = [((cs.get("state") or {}).get("terminated") or {}) for cs in p["status"].get("containerStatuses") or []]
                if term and term[0].get("message"):
                    st["details"] = term[0]["message"][-4000:]
            elif phase == "Failed":
                msg = ""
                for cs in p["status"].get("containerStatuses") or []:
                    t = (cs.get("state") or {}).get("terminated") or {}
                    msg = t.get("message") or t.get("reason") or msg
                st.update({"active": 0, "failed": 1})
                _set_cond(st, "Failed", True, "BackoffLimitExceeded", msg[-2000:])
            else:
                st["active"] = 1
        _update_status(self.store, job, st)
        return Result(requeue_after=1.0)


# ------------------------------------------------------------------ Knative Service
class KnativeController(DeploymentController):
    api, kind = "serving.knative.dev/v1", "Service"

    def desired_replicas(self, d: dict) -> int:
        ann = ((d["spec"].get("template") or {}).get("metadata") or {}).get("annotations") or {}
        return max(1, int(ann.get("autoscaling.knative.dev/min-scale", "1") or 1))

    def reconcile(self, key) -> Result:
        ns, name = key
        ks = self.store.try_get(self.api, self.kind, name, ns)
        if ks is None:
            return Result()
        tmpl = copy.deepcopy(ks["spec"]["template"])
        tmpl.setdefault("metadata", {}).setdefault("labels", {})["app"] = C.truncate_name(name, 63)
        proxy = {**ks, "spec": {"replicas": self.desired_replicas(ks), "template": tmpl}}
        return self._as_deployment(proxy, ks)

    def _as_deployment(self, proxy: dict, ks: dict) -> Result:
        ns, name = ks["metadata"]["namespace"], ks["metadata"]["name"]
        tmpl = proxy["spec"]["template"]
        rev = template_hash(tmpl)
        want = proxy["spec"]["replicas"]
        pods = _owned_pods(self.store, ks)
        cur = [p for p in pods if p["metadata"]["labels"].get("serving.knative.dev/revision") == f"{name}-{rev}"]
        for p in pods:
            if p not in cur and any(pod_ready(q) for q in cur):
                self.store.delete("v1", "Pod", p["metadata"]["name"], ns, ignore_missing=True)
        for i in range(len(cur), want):
            cur.append(self.store.create(make_pod(ks, f"{name}-{rev}-{i}", tmpl,
                                                  {"serving.knative.dev/revision": f"{name}-{rev}"})))
        ready = sum(1 for p in cur if pod_ready(p))
        st = copy.deepcopy(ks.get("status") or {})
        st.update({"latestCreatedRevisionName": f"{name}-{rev}", "url": f"http://{name}.{ns}.svc.cluster.local"})
        if ready:
            st["latestReadyRevisionName"] = f"{name}-{rev}"
        for ct in ("Ready", "ConfigurationsReady", "RoutesReady"):
            _set_cond(st, ct, ready >= want, "" if ready >= want else "RevisionMissing", "")
        _update_status(self.store, ks, st)
        return Result(requeue_after=None if ready >= want else 1.0)


# ------------------------------------------------------------------ RayCluster
RAY_PORT_ANNOTATION = "ome.io/ray-head-port"


class RayClusterController:
    api, kind = "ray.io/v1", "RayCluster"

    def __init__(self, store: Store):
        self.store = store

    def reconcile(self, key) -> Result:
        ns, name = key
        rc = self.store.try_get(self.api, self.kind, name, ns)
        if rc is None:
            return Result()
        pods = _owned_pods(self.store, rc)
        have = {p["metadata"]["name"] for p in pods}
        head = f"{name}-head"
        # the head's rendezvous store (ome_amd.raylet, Ray's GCS port): one port per cluster on
        # this node, kept in an annotation so restarted pods find the same head
        ann = rc["metadata"].get("annotations") or {}
        port = ann.get(RAY_PORT_ANNOTATION)
        if port is None:
            import socket

            with socket.socket() as sk:
                sk.bind(("127.0.0.1", 0))
                port = str(sk.getsockname()[1])
            self.store.patch(self.api, self.kind, name, {"metadata": {"annotations": {**ann, RAY_PORT_ANNOTATION: port}}},
                             ns)
        addr = f"127.0.0.1:{port}"
        py = f"{sys.executable} -m ome_amd.raylet"
        if head not in have:
            self.store.create(make_pod(rc, head, rc["spec"]["headGroupSpec"]["template"],
                                       {"ray.io/cluster": name, C.RAY_NODE_TYPE_LABEL: "head"},
                                       {"KUBERAY_GEN_RAY_START_CMD": f"{py} start --head --port={port}",
                                        "RAY_ADDRESS": addr, "OME_RAY_ADDRESS": addr}))
        for wg in rc["spec"].get("workerGroupSpecs") or []:
            for i in range(int(wg.get("replicas", 1))):
                wn = f"{name}-{wg.get('groupName', 'worker')}-{i}"
                if wn not in have:
                    self.store.create(make_pod(rc, wn, wg["template"], {"ray.io/cluster": name,
                                                                        C.RAY_NODE_TYPE_LABEL: "worker"},
                                               {"KUBERAY_GEN_RAY_START_CMD": f"{py} start --address={addr} --block",
                                                "RAY_ADDRESS": addr, "OME_RAY_ADDRESS": addr}))
        pods = _owned_pods(self.store, rc)
        ok = bool(pods) and all(pod_ready(p) for p in pods)
        st = {**(rc.get("status") or {}), "state": "ready" if ok else "unhealthy" if any(pod_failed(p) for p in pods) else "pending"}
        _update_status(self.store, rc, st)
        return Result(requeue_after=None if ok else 1.0)


# ------------------------------------------------------------------ autoscalers (replica targets)
class HPAController:
    """Keeps the target's replicas within [min, max]; metric-driven decisions are made by the
    executor's metrics autoscaler which writes ``status.desiredReplicas``."""

    def __init__(self, store: Store, api: str, kind: str, min_key: str, max_key: str):
        self.store, self.api, self.kind, self.min_key, self.max_key = store, api, kind, min_key, max_key

    def reconcile(self, key) -> Result:
        ns, name = key
        h = self.store.try_get(self.api, self.kind, name, ns)
        if h is None:
            return Result()
        sp = h["spec"]
        tgt = sp["scaleTargetRef"]["name"]
        d = self.store.try_get("apps/v1", "Deployment", tgt, ns)
        if d is None:
            return Result(requeue_after=2.0)
        mn, mx = int(sp.get(self.min_key, 1)), int(sp.get(self.max_key, 1) or 1)
        desired = int((h.get("status") or {}).get("desiredReplicas") or d["spec"].get("replicas", mn))
        desired = max(mn, min(mx, desired))
        if d["spec"].get("replicas") != desired:
            self.store.patch("apps/v1", "Deployment", tgt, {"spec": {"replicas": desired}}, ns)
        st = {**(h.get("status") or {}), "currentReplicas": (d.get("status") or {}).get("replicas", 0),
              "desiredReplicas": desired}
        _update_status(self.store, h, st)
        return Result()


def controllers(store: Store, leader_address_fn=None) -> list[Controller]:
    out = []
    for cls, owns in ((DeploymentController, True), (JobController, True), (RayClusterController, True)):
        r = cls(store)
        out.append(Controller(f"exec-{cls.kind.lower()}", store, r.reconcile, (cls.api, cls.kind),
                              owns=[("v1", "Pod")]))
    lr = LWSController(store, leader_address_fn)
    out.append(Controller("exec-lws", store, lr.reconcile, (lr.api, lr.kind), owns=[("v1", "Pod")]))
    kr = KnativeController(store)
    out.append(Controller("exec-knative", store, kr.reconcile, (kr.api, kr.kind), owns=[("v1", "Pod")]))
    hr = HPAController(store, "autoscaling/v2", "HorizontalPodAutoscaler", "minReplicas", "maxReplicas")
    out.append(Controller("exec-hpa", store, hr.reconcile, (hr.api, hr.kind)))
    sr = HPAController(store, "keda.sh/v1alpha1", "ScaledObject", "minReplicaCount", "maxReplicaCount")
    out.append(Controller("exec-keda", store, sr.reconcile, (sr.api, sr.kind)))
    return out
