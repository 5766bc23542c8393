"""AcceleratorClass controller (``pkg/controller/v1beta1/acceleratorclass/controller.go``).

Matches Nodes against ``spec.discovery.nodeSelector`` and requires the node's GPU memory to be
at least ``capabilities.memoryGB`` (node label ``amd.com/gpu.vram`` / ``nvidia.com/gpu.memory``
or the ``ome.io/gpu-memory`` annotation when present); writes ``status.nodes``,
``availableNodes``, ``totalAccelerators``, ``availableAccelerators`` and ``lastUpdated``.  Any
Node event re-enqueues every class.  GPU capacity understands ``amd.com/gpu`` (first-class
here), ``nvidia.com/gpu``, ``nvidia.com/mig-*`` and ``gpu.intel.com/*``.
"""
from __future__ import annotations

from ome_amd.api import constants as C
from ome_amd.controllers.runtime import Controller, Result
from ome_amd.store.store import Store, match_labels, now_iso
from ome_amd.utils.quantity import to_float, to_gib

API = C.API_VERSION


def gpu_capacity(node: dict, which: str = "allocatable") -> int:
    res = (node.get("status") or {}).get(which) or (node.get("status") or {}).get("capacity") or {}
    total = 0
    for k, v in res.items():
        if k in (C.AMD_GPU_RESOURCE, C.NVIDIA_GPU_RESOURCE) or k.startswith("nvidia.com/mig-") or \
                k.startswith("gpu.intel.com/"):
            total += int(to_float(v))
    return total


def node_gpu_memory_gib(node: dict) -> float | None:
    lab = node["metadata"].get("labels") or {}
    ann = node["metadata"].get("annotations") or {}
    for k in ("ome.io/gpu-memory",):
        if k in ann:
            return to_gib(ann[k])
    if "amd.com/gpu.vram" in lab:
        return to_gib(lab["amd.com/gpu.vram"])
    if "nvidia.com/gpu.memory" in lab:
        return to_float(lab["nvidia.com/gpu.memory"]) / 1024  # MiB
    return None


def node_matches(node: dict, spec: dict) -> bool:
    sel = (spec.get("discovery") or {}).get("nodeSelector") or {}
    if sel and not match_labels(node["metadata"].get("labels"), {"matchLabels": sel}):
        return False
    want = (spec.get("capabilities") or {}).get("memoryGB")
    if want is not None:
        have = node_gpu_memory_gib(node)
        if have is not None and have < to_gib(want):
            return False
    return bool(sel) or gpu_capacity(node, "capacity") > 0


class AcceleratorClassReconciler:
    def __init__(self, store: Store):
        self.store = store

    def reconcile(self, key) -> Result:
        _, name = key
        ac = self.store.try_get(API, "AcceleratorClass", name)
        if ac is None:
            return Result()
        if ac["metadata"].get("deletionTimestamp"):
            self.store.remove_finalizer(ac, C.ACCELERATORCLASS_FINALIZER)
            return Result()
        if C.ACCELERATORCLASS_FINALIZER not in (ac["metadata"].get("finalizers") or []):
            ac = self.store.add_finalizer(ac, C.ACCELERATORCLASS_FINALIZER)
        spec = ac.get("spec") or {}
        nodes, avail, total, free = [], 0, 0, 0
        for n in self.store.list("v1", "Node"):
            if not node_matches(n, spec):
                continue
            nodes.append(n["metadata"]["name"])
            cap = gpu_capacity(n, "capacity")
            alloc = gpu_capacity(n, "allocatable")
            total += cap
            ready = any(c.get("type") == "Ready" and c.get("status") == "True"
                        for c in (n.get("status") or {}).get("conditions") or [])
            if ready and not (n.get("spec") or {}).get("unschedulable"):
                avail += 1
                free += alloc
        nodes.sort()
        st = ac.get("status") or {}
        new = {**st, "nodes": nodes, "availableNodes": avail, "totalAccelerators": total,
               "availableAccelerators": free}
        if {k: st.get(k) for k in new} != new:
            new["lastUpdated"] = now_iso()
            ac["status"] = new
            self.store.update_status(ac)
        return Result()


def setup(store: Store) -> Controller:
    r = AcceleratorClassReconciler(store)
    c = Controller("acceleratorclass", store, r.reconcile, (API, "AcceleratorClass"),
                   watches=[("Node", lambda n: [("", o["metadata"]["name"])
                                               for o in store.list(API, "AcceleratorClass")])])
    c.reconciler = r
    return c
