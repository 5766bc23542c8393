"""In-process object store with Kubernetes API semantics (what the reference gets from the
kube-apiserver + controller-runtime fake client): uid / resourceVersion / generation,
optimistic concurrency, status subresource, finalizers + deletionTimestamp, owner-reference
garbage collection, label selectors, admission chain and watches."""
import pytest

from ome_amd.store.store import (AlreadyExists, Conflict, Invalid, NotFound, Store, match_labels, merge_patch,
                                 owner_ref, parse_selector)

API = "ome.io/v1beta1"


def _isvc(name="a", ns="default", **spec):
    return {"apiVersion": API, "kind": "InferenceService", "metadata": {"name": name, "namespace": ns},
            "spec": {"model": {"name": "m"}, **spec}}


def test_create_get_list_and_metadata():
    s = Store()
    o = s.create(_isvc())
    m = o["metadata"]
    assert m["uid"] and m["resourceVersion"] and m["generation"] == 1 and m["creationTimestamp"]
    with pytest.raises(AlreadyExists):
        s.create(_isvc())
    with pytest.raises(Invalid):
        s.create({"apiVersion": API, "kind": "InferenceService", "metadata": {}})
    g = s.create({"apiVersion": "v1", "kind": "Event", "metadata": {"generateName": "x."}})
    assert g["metadata"]["name"].startswith("x.") and g["metadata"]["namespace"] == "default"
    cbm = s.create({"apiVersion": API, "kind": "ClusterBaseModel", "metadata": {"name": "c", "namespace": "ignored"}})
    assert "namespace" not in cbm["metadata"]  # cluster-scoped
    s.create(_isvc("b", "other"))
    assert [o["metadata"]["name"] for o in s.list(API, "InferenceService")] == ["a", "b"]
    assert [o["metadata"]["name"] for o in s.list(API, "InferenceService", "other")] == ["b"]
    with pytest.raises(NotFound):
        s.get(API, "InferenceService", "zz", "default")
    assert s.try_get(API, "InferenceService", "zz", "default") is None


def test_optimistic_concurrency_and_generation():
    s = Store()
    o = s.create(_isvc())
    o2 = dict(o, spec={"model": {"name": "n"}})
    new = s.update(o2)
    assert new["metadata"]["generation"] == 2 and new["metadata"]["resourceVersion"] != o["metadata"]["resourceVersion"]
    with pytest.raises(Conflict):
        s.update(o2)  # stale resourceVersion
    # status-only writes do not bump generation; spec writes do not touch status
    st = dict(new, status={"url": "http://x"})
    after = s.update_status(st)
    assert after["status"] == {"url": "http://x"} and after["metadata"]["generation"] == 2
    spec_write = dict(after, status={"url": "overwritten?"}, spec={"model": {"name": "q"}})
    after2 = s.update(spec_write)
    assert after2["status"] == {"url": "http://x"} and after2["metadata"]["generation"] == 3
    # no-op update keeps resourceVersion
    assert s.update(after2)["metadata"]["resourceVersion"] == after2["metadata"]["resourceVersion"]


def test_patch_apply_merge_semantics():
    s = Store()
    s.create(_isvc(engine={"minReplicas": 1, "maxReplicas": 2}))
    p = s.patch(API, "InferenceService", "a", {"spec": {"engine": {"maxReplicas": 4, "minReplicas": None}}}, "default")
    assert p["spec"]["engine"] == {"maxReplicas": 4}
    a = s.apply({**_isvc(), "metadata": {"name": "a", "namespace": "default", "labels": {"x": "1"}}})
    assert a["metadata"]["labels"] == {"x": "1"} and a["spec"] == {"model": {"name": "m"}}
    assert merge_patch({"a": {"b": 1, "c": 2}}, {"a": {"b": None, "d": 3}}) == {"a": {"c": 2, "d": 3}}


def test_finalizers_and_owner_gc():
    s = Store()
    owner = s.create(_isvc())
    dep = s.create({"apiVersion": "apps/v1", "kind": "Deployment",
                    "metadata": {"name": "a-engine", "namespace": "default", "ownerReferences": [owner_ref(owner)]}})
    svc = s.create({"apiVersion": "v1", "kind": "Service",
                    "metadata": {"name": "a-engine", "namespace": "default", "ownerReferences": [owner_ref(dep)]}})
    owner = s.add_finalizer(owner, "ome.io/cleanup")
    s.delete(API, "InferenceService", "a", "default")
    term = s.get(API, "InferenceService", "a", "default")
    assert term["metadata"]["deletionTimestamp"]  # finalizer holds it
    assert s.try_get("apps/v1", "Deployment", "a-engine", "default") is not None
    s.remove_finalizer(term, "ome.io/cleanup")
    assert s.try_get(API, "InferenceService", "a", "default") is None
    # cascading GC through the owner chain
    assert s.try_get("apps/v1", "Deployment", "a-engine", "default") is None
    assert s.try_get("v1", "Service", svc["metadata"]["name"], "default") is None


def test_gc_keeps_objects_with_a_surviving_owner():
    s = Store()
    a, b = s.create(_isvc("a")), s.create(_isvc("b"))
    shared = s.create({"apiVersion": "v1", "kind": "ConfigMap",
                       "metadata": {"name": "cm", "namespace": "default",
                                    "ownerReferences": [owner_ref(a, False), owner_ref(b, False)]}})
    s.delete(API, "InferenceService", "a", "default")
    left = s.get("v1", "ConfigMap", "cm", "default")
    assert [r["name"] for r in left["metadata"]["ownerReferences"]] == ["b"]
    s.delete(API, "InferenceService", "b", "default")
    assert s.try_get("v1", "ConfigMap", shared["metadata"]["name"], "default") is None


@pytest.mark.parametrize("sel,labels,want", [
    ("app=x", {"app": "x"}, True), ("app=x", {"app": "y"}, False), ("app!=x", {}, True),
    ("env in (a,b)", {"env": "b"}, True), ("env in (a,b)", {"env": "c"}, False),
    ("env notin (a,b),tier", {"env": "c", "tier": "1"}, True), ("!gpu", {"gpu": "1"}, False),
    ("app=x,env in (a, b)", {"app": "x", "env": "a"}, True),
    ({"matchLabels": {"a": "1"}, "matchExpressions": [{"key": "b", "operator": "Exists"}]}, {"a": "1", "b": ""}, True),
    ({"matchExpressions": [{"key": "n", "operator": "Gt", "values": ["3"]}]}, {"n": "5"}, True),
    ({"a": "1"}, {"a": "2"}, False),
])
def test_label_selectors(sel, labels, want):
    assert match_labels(labels, sel) == want


def test_selector_parse_keeps_value_lists_together():
    assert parse_selector("env in (a,b),x=1") == [("env", "In", ["a", "b"]), ("x", "=", ["1"])]


def test_admission_chain_and_watch():
    s = Store()
    seen = []

    def default_replicas(op, obj, old, store):
        obj["spec"].setdefault("engine", {"minReplicas": 1})
        return obj

    def deny_bad(op, obj, old, store):
        if obj["spec"]["model"]["name"] == "bad":
            raise Invalid("bad model")

    s.add_mutating(default_replicas, ["InferenceService"])
    s.add_validating(deny_bad, ["InferenceService"])
    w = s.watch(lambda ev: seen.append((ev.type, ev.obj["metadata"]["name"])), ["InferenceService"])
    o = s.create(_isvc())
    assert o["spec"]["engine"] == {"minReplicas": 1}
    with pytest.raises(Invalid):
        s.create({**_isvc("z"), "spec": {"model": {"name": "bad"}}})
    s.delete(API, "InferenceService", "a", "default")
    s.unwatch(w)
    s.create(_isvc("c"))
    assert seen == [("ADDED", "a"), ("DELETED", "a")]
    # dry-run goes through admission but stores nothing
    assert s.create(_isvc("d"), dry_run=True)["spec"]["engine"] == {"minReplicas": 1}
    assert s.try_get(API, "InferenceService", "d", "default") is None


def test_events_recorded_against_object():
    s = Store()
    o = s.create(_isvc())
    s.record_event(o, "Warning", "RuntimeNotFound", "no runtime")
    ev = s.events_for(o)
    assert len(ev) == 1 and ev[0]["reason"] == "RuntimeNotFound" and ev[0]["involvedObject"]["kind"] == "InferenceService"
