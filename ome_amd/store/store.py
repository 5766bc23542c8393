"""In-process object store with Kubernetes API semantics.

This is the control plane's stand-in for kube-apiserver + etcd: every
controller, webhook, the node agent and the local executor talk to it exactly the way the
reference's components talk to the API server, so reconcile logic is level-triggered and
restart-safe.  Semantics implemented:

* objects are plain JSON dicts keyed by (group, kind, namespace, name); cluster-scoped kinds
  ignore the namespace;
* ``metadata.uid`` / ``creationTimestamp`` / ``resourceVersion`` (global monotonically
  increasing) / ``generation`` (bumped only on spec changes);
* optimistic concurrency: ``update`` with a stale ``resourceVersion`` raises :class:`Conflict`;
* status subresource: ``update`` keeps the stored status, ``update_status`` only writes status;
* finalizers: delete of an object with finalizers only sets ``deletionTimestamp``; the object
  disappears when the last finalizer is removed;
* ownerReferences: removing an object garbage-collects its dependents (cascading, background);
* label selectors (``matchLabels`` + ``matchExpressions`` In/NotIn/Exists/DoesNotExist, and the
  string form ``a=b,c!=d,e``);
* watches: subscribers receive (event_type, object) after each committed change;
* admission: mutating then validating hooks run on create/update (the webhook chain).
"""
from __future__ import annotations

import copy
import itertools
import threading
import time
import uuid
from dataclasses import dataclass
from typing import Any, Callable, Iterable

CLUSTER_SCOPED = {
    ("", "Namespace"), ("", "Node"), ("", "PersistentVolume"), ("ome.io", "ClusterBaseModel"),
    ("ome.io", "ClusterServingRuntime"), ("ome.io", "AcceleratorClass"), ("ome.io", "FineTunedWeight"),
    ("rbac.authorization.k8s.io", "ClusterRole"), ("rbac.authorization.k8s.io", "ClusterRoleBinding"),
    ("apiextensions.k8s.io", "CustomResourceDefinition"),
}
# kinds WITHOUT a status subresource (everything else: spec writers cannot clobber .status)
NO_STATUS_SUBRESOURCE = {("", "ConfigMap"), ("", "Secret"), ("", "Event"), ("", "ServiceAccount")}


class APIError(Exception):
    code = 500


class NotFound(APIError):
    code = 404


class AlreadyExists(APIError):
    code = 409


class Conflict(APIError):
    code = 409


class Invalid(APIError):
    code = 422


class Forbidden(APIError):
    code = 403


def group_of(api_version: str) -> str:
    return api_version.split("/")[0] if "/" in api_version else ""


def gk(obj_or_api: dict | str, kind: str | None = None) -> tuple[str, str]:
    if isinstance(obj_or_api, dict):
        return group_of(obj_or_api.get("apiVersion", "v1")), obj_or_api["kind"]
    return group_of(obj_or_api), kind  # type: ignore[return-value]


def now_iso() -> str:
    return time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())


# ------------------------------------------------------------------ label selectors
def parse_selector(sel: str | dict | None) -> list[tuple[str, str, list[str]]]:
    """-> list of (key, op, values); op in {=, !=, In, NotIn, Exists, DoesNotExist}."""
    if not sel:
        return []
    out = []
    if isinstance(sel, dict):
        ml = sel.get("matchLabels") if ("matchLabels" in sel or "matchExpressions" in sel) else sel
        for k, v in (ml or {}).items():
            out.append((k, "=", [str(v)]))
        for e in sel.get("matchExpressions", []) or []:
            out.append((e["key"], e["operator"], [str(x) for x in e.get("values", []) or []]))
        return out
    parts, depth, cur = [], 0, ""
    for ch in sel:  # split on commas outside "(...)" value lists
        depth += ch == "("
        depth -= ch == ")"
        if ch == "," and depth == 0:
            parts.append(cur)
            cur = ""
        else:
            cur += ch
    parts.append(cur)
    for part in [p.strip() for p in parts if p.strip()]:
        if "!=" in part:
            k, v = part.split("!=", 1)
            out.append((k.strip(), "!=", [v.strip()]))
        elif "==" in part or "=" in part:
            k, v = part.split("==", 1) if "==" in part else part.split("=", 1)
            out.append((k.strip(), "=", [v.strip()]))
        elif " notin " in part:
            k, v = part.split(" notin ", 1)
            out.append((k.strip(), "NotIn", [x.strip() for x in v.strip(" ()").split(",")]))
        elif " in " in part:
            k, v = part.split(" in ", 1)
            out.append((k.strip(), "In", [x.strip() for x in v.strip(" ()").split(",")]))
        elif part.startswith("!"):
            out.append((part[1:], "DoesNotExist", []))
        else:
            out.append((part, "Exists", []))
    return out


def match_labels(labels: dict | None, sel) -> bool:
    labels = labels or {}
    for k, op, vals in parse_selector(sel) if not isinstance(sel, list) else sel:
        has = k in labels
        v = labels.get(k)
        if op in ("=", "In"):
            if not has or v not in vals:
                return False
        elif op in ("!=", "NotIn"):
            if has and v in vals:
                return False
        elif op == "Exists":
            if not has:
                return False
        elif op == "DoesNotExist":
            if has:
                return False
        elif op in ("Gt", "Lt"):
            try:
                if not has or not ((float(v) > float(vals[0])) if op == "Gt" else (float(v) < float(vals[0]))):
                    return False
            except ValueError:
                return False
    return True


@dataclass
class WatchEvent:
    type: str        # ADDED | MODIFIED | DELETED
    obj: dict


AdmissionHook = Callable[[str, dict, dict | None, "Store"], dict | None]


class Store:
    def __init__(self):
        self._lock = threading.RLock()
        self._objs: dict[tuple[str, str, str, str], dict] = {}
        self._rv = itertools.count(1)
        self._watchers: list[tuple[set | None, Callable[[WatchEvent], None]]] = []
        self.mutating: list[tuple[set | None, AdmissionHook]] = []
        self.validating: list[tuple[set | None, AdmissionHook]] = []
        self.clock: Callable[[], float] = time.time

    # ------------------------------------------------------------------ keys
    @staticmethod
    def _key(group: str, kind: str, ns: str | None, name: str) -> tuple[str, str, str, str]:
        return (group, kind, "" if (group, kind) in CLUSTER_SCOPED else (ns or "default"), name)

    def _okey(self, obj: dict):
        g, k = gk(obj)
        m = obj.get("metadata", {})
        return self._key(g, k, m.get("namespace"), m.get("name", ""))

    @staticmethod
    def namespaced(group: str, kind: str) -> bool:
        return (group, kind) not in CLUSTER_SCOPED

    # ------------------------------------------------------------------ admission / watch
    def add_mutating(self, hook: AdmissionHook, kinds: Iterable[str] | None = None) -> None:
        self.mutating.append((set(kinds) if kinds else None, hook))

    def add_validating(self, hook: AdmissionHook, kinds: Iterable[str] | None = None) -> None:
        self.validating.append((set(kinds) if kinds else None, hook))

    def _admit(self, op: str, obj: dict, old: dict | None) -> dict:
        kind = obj["kind"]
        for kinds, hook in self.mutating:
            if kinds is None or kind in kinds:
                r = hook(op, obj, old, self)
                if r is not None:
                    obj = r
        for kinds, hook in self.validating:
            if kinds is None or kind in kinds:
                hook(op, obj, old, self)  # raises Invalid / Forbidden to deny
        return obj

    def watch(self, callback: Callable[[WatchEvent], None], kinds: Iterable[str] | None = None):
        entry = (set(kinds) if kinds else None, callback)
        with self._lock:
            self._watchers.append(entry)
        return entry

    def unwatch(self, entry) -> None:
        with self._lock:
            if entry in self._watchers:
                self._watchers.remove(entry)

    def _notify(self, events: list[WatchEvent]) -> None:
        watchers = list(self._watchers)
        for ev in events:
            for kinds, cb in watchers:
                if kinds is None or ev.obj["kind"] in kinds:
                    try:
                        cb(WatchEvent(ev.type, copy.deepcopy(ev.obj)))
                    except Exception:  # noqa: BLE001 — a broken watcher must not break the store
                        import logging

                        logging.getLogger("ome_amd.store").exception("watch callback failed")

    # ------------------------------------------------------------------ CRUD
    def create(self, obj: dict, dry_run: bool = False) -> dict:
        obj = copy.deepcopy(obj)
        obj.setdefault("apiVersion", "v1")
        meta = obj.setdefault("metadata", {})
        if not meta.get("name"):
            if meta.get("generateName"):
                meta["name"] = meta["generateName"] + uuid.uuid4().hex[:5]
            else:
                raise Invalid("metadata.name is required")
        g, k = gk(obj)
        if self.namespaced(g, k):
            meta.setdefault("namespace", "default")
        else:
            meta.pop("namespace", None)
        obj = self._admit("CREATE", obj, None)
        meta = obj["metadata"]
        with self._lock:
            key = self._okey(obj)
            if key in self._objs:
                raise AlreadyExists(f"{k} {key[2]}/{key[3]} already exists")
            if dry_run:
                return copy.deepcopy(obj)
            meta["uid"] = str(uuid.uuid4())
            meta["creationTimestamp"] = now_iso()
            meta["resourceVersion"] = str(next(self._rv))
            meta["generation"] = 1
            meta.pop("deletionTimestamp", None)
            self._objs[key] = obj
            out = copy.deepcopy(obj)
        self._notify([WatchEvent("ADDED", out)])
        return copy.deepcopy(out)

    def get(self, api_version: str, kind: str, name: str, namespace: str | None = None) -> dict:
        with self._lock:
            o = self._objs.get(self._key(group_of(api_version), kind, namespace, name))
            if o is None:
                raise NotFound(f"{kind} {namespace or ''}/{name} not found")
            return copy.deepcopy(o)

    def try_get(self, api_version: str, kind: str, name: str, namespace: str | None = None) -> dict | None:
        try:
            return self.get(api_version, kind, name, namespace)
        except NotFound:
            return None

    def list(self, api_version: str, kind: str, namespace: str | None = None, selector=None,
             field: Callable[[dict], bool] | None = None) -> list[dict]:
        g = group_of(api_version)
        sel = parse_selector(selector) if selector else None
        with self._lock:
            out = []
            for (og, ok, ons, _), o in self._objs.items():
                if og != g or ok != kind:
                    continue
                if namespace and self.namespaced(g, kind) and ons != namespace:
                    continue
                if sel and not match_labels(o["metadata"].get("labels"), sel):
                    continue
                if field and not field(o):
                    continue
                out.append(copy.deepcopy(o))
        out.sort(key=lambda o: (o["metadata"].get("namespace", ""), o["metadata"]["name"]))
        return out

    def update(self, obj: dict, status_only: bool = False) -> dict:
        obj = copy.deepcopy(obj)
        g, k = gk(obj)
        with self._lock:
            key = self._okey(obj)
            cur = self._objs.get(key)
            if cur is None:
                raise NotFound(f"{k} {key[2]}/{key[3]} not found")
            rv = obj.get("metadata", {}).get("resourceVersion")
            if rv and rv != cur["metadata"]["resourceVersion"]:
                raise Conflict(f"{k} {key[3]}: resourceVersion {rv} is stale "
                               f"(current {cur['metadata']['resourceVersion']})")
        if not status_only:
            obj = self._admit("UPDATE", obj, cur)
        events = []
        with self._lock:
            cur = self._objs.get(key)
            if cur is None:
                raise NotFound(f"{k} {key[2]}/{key[3]} not found")
            new = copy.deepcopy(cur)
            if status_only:
                if "status" in obj:
                    new["status"] = obj["status"]
            else:
                subres = (g, k) not in NO_STATUS_SUBRESOURCE
                for f, v in obj.items():
                    if f == "metadata" or (f == "status" and subres):
                        continue
                    new[f] = v
                for f in list(new.keys()):
                    if f not in obj and f not in ("metadata", "apiVersion", "kind") and not (f == "status" and subres):
                        del new[f]
                m, nm = obj.get("metadata", {}), new["metadata"]
                for f in ("labels", "annotations", "finalizers", "ownerReferences"):
                    if f in m:
                        nm[f] = m[f]
                    else:
                        nm.pop(f, None)
                if cur.get("spec") != new.get("spec"):
                    nm["generation"] = int(nm.get("generation", 1)) + 1
            if new == cur:
                return copy.deepcopy(cur)
            new["metadata"]["resourceVersion"] = str(next(self._rv))
            # finalizer removal on a terminating object completes the delete
            if new["metadata"].get("deletionTimestamp") and not new["metadata"].get("finalizers"):
                del self._objs[key]
                events.append(WatchEvent("DELETED", copy.deepcopy(new)))
                events += self._collect_dependents(new["metadata"]["uid"])
            else:
                self._objs[key] = new
                events.append(WatchEvent("MODIFIED", copy.deepcopy(new)))
            out = copy.deepcopy(new)
        self._notify(events)
        return out

    def update_status(self, obj: dict) -> dict:
        return self.update(obj, status_only=True)

    def patch(self, api_version: str, kind: str, name: str, patch: dict, namespace: str | None = None,
              status: bool = False) -> dict:
        """JSON merge patch (RFC 7386) with retry on conflict."""
        for _ in range(10):
            cur = self.get(api_version, kind, name, namespace)
            new = merge_patch(cur, patch)
            new["metadata"]["resourceVersion"] = cur["metadata"]["resourceVersion"]
            try:
                return self.update(new, status_only=status)
            except Conflict:
                continue
        raise Conflict(f"patch of {kind} {name} kept conflicting")

    def apply(self, obj: dict) -> dict:
        """Create or replace spec/labels/annotations (kubectl apply-like, server-side merge)."""
        m = obj.get("metadata", {})
        cur = self.try_get(obj.get("apiVersion", "v1"), obj["kind"], m["name"], m.get("namespace"))
        if cur is None:
            return self.create(obj)
        new = copy.deepcopy(cur)
        for f, v in obj.items():
            if f not in ("metadata", "status"):
                new[f] = copy.deepcopy(v)
        for f in ("labels", "annotations"):
            if f in m:
                new["metadata"][f] = {**new["metadata"].get(f, {}), **m[f]}
        return self.update(new)

    def delete(self, api_version: str, kind: str, name: str, namespace: str | None = None,
               ignore_missing: bool = False) -> dict | None:
        events = []
        with self._lock:
            key = self._key(group_of(api_version), kind, namespace, name)
            cur = self._objs.get(key)
            if cur is None:
                if ignore_missing:
                    return None
                raise NotFound(f"{kind} {namespace or ''}/{name} not found")
            if cur["metadata"].get("finalizers"):
                if not cur["metadata"].get("deletionTimestamp"):
                    new = copy.deepcopy(cur)
                    new["metadata"]["deletionTimestamp"] = now_iso()
                    new["metadata"]["resourceVersion"] = str(next(self._rv))
                    self._objs[key] = new
                    events.append(WatchEvent("MODIFIED", copy.deepcopy(new)))
                out = copy.deepcopy(self._objs[key])
            else:
                del self._objs[key]
                events.append(WatchEvent("DELETED", copy.deepcopy(cur)))
                events += self._collect_dependents(cur["metadata"]["uid"])
                out = copy.deepcopy(cur)
        self._notify(events)
        return out

    def _collect_dependents(self, uid: str) -> list[WatchEvent]:
        """Garbage-collect objects owned by ``uid`` (caller holds the lock)."""
        events = []
        stack = [uid]
        while stack:
            u = stack.pop()
            for key, o in list(self._objs.items()):
                refs = o["metadata"].get("ownerReferences") or []
                if not any(r.get("uid") == u for r in refs):
                    continue
                remaining = [r for r in refs if r.get("uid") != u]
                if remaining and any(self._uid_exists(r.get("uid")) for r in remaining):
                    o["metadata"]["ownerReferences"] = remaining
                    continue
                if o["metadata"].get("finalizers"):
                    if not o["metadata"].get("deletionTimestamp"):
                        o["metadata"]["deletionTimestamp"] = now_iso()
                        o["metadata"]["resourceVersion"] = str(next(self._rv))
                        events.append(WatchEvent("MODIFIED", copy.deepcopy(o)))
                    continue
                del self._objs[key]
                events.append(WatchEvent("DELETED", copy.deepcopy(o)))
                stack.append(o["metadata"]["uid"])
        return events

    def _uid_exists(self, uid: str | None) -> bool:
        return any(o["metadata"].get("uid") == uid for o in self._objs.values())

    # ------------------------------------------------------------------ helpers
    def remove_finalizer(self, obj: dict, finalizer: str) -> dict | None:
        for _ in range(10):
            m = obj["metadata"]
            cur = self.try_get(obj["apiVersion"], obj["kind"], m["name"], m.get("namespace"))
            if cur is None:
                return None
            fins = cur["metadata"].get("finalizers") or []
            if finalizer not in fins:
                return cur
            cur["metadata"]["finalizers"] = [f for f in fins if f != finalizer]
            try:
                return self.update(cur)
            except Conflict:
                continue
            except NotFound:
                return None
        raise Conflict("could not remove finalizer")

    def add_finalizer(self, obj: dict, finalizer: str) -> dict:
        fins = obj["metadata"].get("finalizers") or []
        if finalizer in fins:
            return obj
        obj = copy.deepcopy(obj)
        obj["metadata"]["finalizers"] = fins + [finalizer]
        return self.update(obj)

    def record_event(self, involved: dict, etype: str, reason: str, message: str) -> None:
        m = involved.get("metadata", {})
        ns = m.get("namespace") or "default"
        self.create({
            "apiVersion": "v1", "kind": "Event",
            "metadata": {"generateName": f"{m.get('name', 'obj')}.", "namespace": ns},
            "involvedObject": {"apiVersion": involved.get("apiVersion"), "kind": involved.get("kind"),
                               "name": m.get("name"), "namespace": m.get("namespace"), "uid": m.get("uid")},
            "type": etype, "reason": reason, "message": message, "lastTimestamp": now_iso(),
            "source": {"component": "ome-manager"},
        })

    def events_for(self, obj: dict) -> list[dict]:
        uid = obj["metadata"].get("uid")
        return [e for e in self.list("v1", "Event") if e.get("involvedObject", {}).get("uid") == uid]

    def all(self) -> list[dict]:
        with self._lock:
            return [copy.deepcopy(o) for o in self._objs.values()]


def merge_patch(target: Any, patch: Any) -> Any:
    if not isinstance(patch, dict):
        return copy.deepcopy(patch)
    out = copy.deepcopy(target) if isinstance(target, dict) else {}
    for k, v in patch.items():
        if v is None:
            out.pop(k, None)
        else:
            out[k] = merge_patch(out.get(k), v)
    return out


def owner_ref(owner: dict, controller: bool = True) -> dict:
    m = owner["metadata"]
    return {"apiVersion": owner["apiVersion"], "kind": owner["kind"], "name": m["name"], "uid": m["uid"],
            "controller": controller, "blockOwnerDeletion": True}


def controller_of(obj: dict) -> dict | None:
    for r in obj.get("metadata", {}).get("ownerReferences") or []:
        if r.get("controller"):
            return r
    return None
