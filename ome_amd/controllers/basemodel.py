"""BaseModel / ClusterBaseModel controllers (``pkg/controller/v1beta1/basemodel/controller.go``).

The model agent on each node writes a ``ModelEntry`` JSON per model into the node ConfigMap
``ome/<node>`` (label ``models.ome/basemodel-status=true``).  These controllers aggregate those
entries: ``status.nodesReady`` / ``nodesFailed`` / ``state`` (Ready if any node is ready, else
Failed if any failed, else In_Transit), copy the parsed model config back into unset spec
fields, requeue every 5 s while Importing / In_Transit, and on deletion wait (30 s requeue)
until no node still holds a non-Deleted entry before dropping the finalizer.  A deleted Node
takes its ConfigMap with it; ConfigMaps of nodes that no longer exist are ignored.
"""
from __future__ import annotations

import json

from ome_amd.api import constants as C
from ome_amd.controllers.runtime import Controller, Result
from ome_amd.store.store import Conflict, Store

API = C.API_VERSION


def lifecycle_state(ready: list[str], failed: list[str]) -> str:
    if ready:
        return "Ready"
    if failed:
        return "Failed"
    return "In_Transit"


def update_spec_with_config(spec: dict, cfg: dict) -> bool:
    updated = False
    for key in ("modelType", "modelArchitecture", "modelParameterSize"):
        if spec.get(key) is None and cfg.get(key):
            spec[key] = cfg[key]
            updated = True
    if not spec.get("modelCapabilities") and cfg.get("modelCapabilities"):
        spec["modelCapabilities"] = list(cfg["modelCapabilities"])
        updated = True
    if not spec.get("apiCapabilities") and cfg.get("apiCapabilities"):
        spec["apiCapabilities"] = list(cfg["apiCapabilities"])
        updated = True
    fw = cfg.get("modelFramework") or {}
    if spec.get("modelFramework") is None and fw.get("name"):
        spec["modelFramework"] = {"name": fw["name"], **({"version": fw["version"]} if fw.get("version") else {})}
        updated = True
    fm = cfg.get("modelFormat") or {}
    if fm:
        mf = spec.setdefault("modelFormat", {})
        if fm.get("name") and not mf.get("name"):
            mf["name"] = fm["name"]
            updated = True
        if fm.get("version") and mf.get("version") is None:
            mf["version"] = fm["version"]
            updated = True
    if spec.get("maxTokens") is None and int(cfg.get("maxTokens") or 0) > 0:
        spec["maxTokens"] = int(cfg["maxTokens"])
        updated = True
    if spec.get("quantization") is None and cfg.get("quantization"):
        spec["quantization"] = cfg["quantization"]
        updated = True
    return updated


class BaseModelReconciler:
    def __init__(self, store: Store, cluster: bool):
        self.store, self.cluster = store, cluster
        self.kind = "ClusterBaseModel" if cluster else "BaseModel"
        self.finalizer = C.CLUSTERBASEMODEL_FINALIZER if cluster else C.BASEMODEL_FINALIZER

    def _node_configmaps(self) -> list[dict]:
        return self.store.list("v1", "ConfigMap", C.OME_NAMESPACE, selector={C.MODEL_STATUS_CM_LABEL: "true"})

    def reconcile(self, key) -> Result:
        ns, name = key
        obj = self.store.try_get(API, self.kind, name, ns or None)
        if obj is None:
            return Result()
        mkey = C.model_configmap_key(ns, name, self.cluster)
        if obj["metadata"].get("deletionTimestamp"):
            if self.finalizer in (obj["metadata"].get("finalizers") or []):
                pending = []
                for cm in self._node_configmaps():
                    raw = (cm.get("data") or {}).get(mkey)
                    if raw is None:
                        continue
                    try:
                        if json.loads(raw).get("status") != "Deleted":
                            pending.append(cm["metadata"]["name"])
                    except json.JSONDecodeError:
                        pending.append(cm["metadata"]["name"])
                if pending:
                    return Result(requeue_after=30.0)
                self.store.remove_finalizer(obj, self.finalizer)
            return Result()
        if self.finalizer not in (obj["metadata"].get("finalizers") or []):
            obj = self.store.add_finalizer(obj, self.finalizer)
        ready, failed = [], []
        spec = dict(obj.get("spec") or {})
        spec_changed = False
        for cm in self._node_configmaps():
            node = cm["metadata"]["name"]
            if self.store.try_get("v1", "Node", node) is None:
                continue
            raw = (cm.get("data") or {}).get(mkey)
            if raw is None:
                continue
            try:
                entry = json.loads(raw)
            except json.JSONDecodeError:
                continue
            if entry.get("config"):
                spec_changed |= update_spec_with_config(spec, entry["config"])
            st = entry.get("status")
            if st == "Ready" and node not in ready:
                ready.append(node)
            elif st == "Failed" and node not in failed:
                failed.append(node)
        ready.sort()
        failed.sort()
        for _ in range(3):
            try:
                cur = self.store.get(API, self.kind, name, ns or None)
                if spec_changed and cur.get("spec") != spec:
                    cur["spec"] = spec
                    cur = self.store.update(cur)
                state = lifecycle_state(ready, failed)
                st = cur.get("status") or {}
                if st.get("nodesReady") != ready or st.get("nodesFailed") != failed or st.get("state") != state:
                    cur["status"] = {**st, "nodesReady": ready, "nodesFailed": failed, "state": state,
                                     "lifecycle": state}
                    self.store.update_status(cur)
                break
            except Conflict:
                continue
        state = lifecycle_state(ready, failed)
        if state in ("Importing", "In_Transit"):
            return Result(requeue_after=5.0)
        return Result()


def setup(store: Store, cluster: bool) -> Controller:
    r = BaseModelReconciler(store, cluster)

    def cm_to_models(cm):
        if (cm["metadata"].get("labels") or {}).get(C.MODEL_STATUS_CM_LABEL) != "true":
            return []
        out = []
        for k in (cm.get("data") or {}):
            parsed = C.parse_model_configmap_key(k)
            if parsed is None:
                continue
            mns, mname, is_cluster = parsed
            if is_cluster == cluster:
                out.append(("" if cluster else mns, mname))
        return out

    def node_deleted(node):
        # A Node event: drop the ConfigMap of nodes that no longer exist, re-check every model.
        name = node["metadata"]["name"]
        if store.try_get("v1", "Node", name) is None:
            store.delete("v1", "ConfigMap", name, C.OME_NAMESPACE, ignore_missing=True)
        return [Controller.key_of(o) for o in store.list(API, r.kind)]

    c = Controller(("cluster" if cluster else "") + "basemodel", store, r.reconcile, (API, r.kind),
                   watches=[("ConfigMap", cm_to_models), ("Node", node_deleted)])
    c.reconciler = r
    return c
