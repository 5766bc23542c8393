"""Model agent + BaseModel controller behaviours the round-2 review found untested:
ReuseIfExists de-duplication with parent/children bookkeeping (``gopher.go:976-997,1183-1440``),
node ConfigMap self-heal (``configmap_reconciler.go:109-202``), node labels, reserved artifacts,
Scout targeting, and the BaseModel finalizer / node-deletion paths
(``basemodel/controller.go:157-248,464-506``).  Tasks run synchronously through the Gopher."""
import json
import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ome_amd.api import constants as C  # noqa: E402
from ome_amd.controllers import basemodel  # noqa: E402
from ome_amd.modelagent.agent import (DELETE, DOWNLOAD, DOWNLOAD_OVERRIDE, ModelAgent, Task,  # noqa: E402
                                      model_key)
from ome_amd.store.store import Store, WatchEvent  # noqa: E402

API = C.API_VERSION
NODE = "mi355x-node-0"


def _store(labels=None):
    s = Store()
    s.create({"apiVersion": "v1", "kind": "Node", "metadata": {"name": NODE, "labels": labels or {}}})
    return s


def _cbm(name, path, uri="random://tiny-llama", policy=None, annotations=None, selector=None):
    st = {"storageUri": uri, "path": str(path)}
    if policy:
        st["downloadPolicy"] = policy
    if selector:
        st["nodeSelector"] = selector
    return {"apiVersion": API, "kind": "ClusterBaseModel",
            "metadata": {"name": name, "annotations": annotations or {}}, "spec": {"storage": st}}


def _run(agent, typ, obj):
    agent.gopher.process(Task(typ, obj))


def _entry(agent, obj):
    return agent.cm.get_entry(model_key(obj))


def test_reuse_if_exists_symlinks_and_parent_children_bookkeeping(tmp_path):
    s = _store()
    ag = ModelAgent(s, NODE, models_root=str(tmp_path / "models"))
    a, b = _cbm("a", tmp_path / "a"), _cbm("b", tmp_path / "b")
    _run(ag, DOWNLOAD, a)
    _run(ag, DOWNLOAD, b)
    ea, eb = _entry(ag, a), _entry(ag, b)
    assert ea["status"] == eb["status"] == "Ready"
    assert os.path.islink(tmp_path / "b") and os.path.realpath(tmp_path / "b") == str(tmp_path / "a")
    assert eb["config"]["artifact"]["parentPath"] == {model_key(a): str(tmp_path / "a")}
    assert ea["config"]["artifact"]["childrenPaths"] == [str(tmp_path / "b")]
    # the parsed model config still lands in the child's entry
    assert eb["config"].get("modelArchitecture") == "LlamaForCausalLM"

    # deleting the PARENT hands the artifact to its child: real directory at the child's path
    _run(ag, DELETE, a)
    assert _entry(ag, a) is None
    assert os.path.isdir(tmp_path / "b") and not os.path.islink(tmp_path / "b")
    assert (tmp_path / "b" / "config.json").exists() and not os.path.exists(tmp_path / "a")
    _run(ag, DELETE, b)
    assert not os.path.exists(tmp_path / "b") and _entry(ag, b) is None


def test_deleting_child_unlinks_and_updates_parent(tmp_path):
    s = _store()
    ag = ModelAgent(s, NODE, models_root=str(tmp_path / "models"))
    a, b = _cbm("a", tmp_path / "a"), _cbm("b", tmp_path / "b")
    _run(ag, DOWNLOAD, a)
    _run(ag, DOWNLOAD, b)
    _run(ag, DELETE, b)
    assert not os.path.lexists(tmp_path / "b") and os.path.isdir(tmp_path / "a")
    assert _entry(ag, a)["config"]["artifact"]["childrenPaths"] == []


def test_always_download_never_dedups(tmp_path):
    s = _store()
    ag = ModelAgent(s, NODE, models_root=str(tmp_path / "models"))
    a = _cbm("a", tmp_path / "a")
    b = _cbm("b", tmp_path / "b", policy="AlwaysDownload")
    _run(ag, DOWNLOAD, a)
    _run(ag, DOWNLOAD, b)
    assert os.path.isdir(tmp_path / "b") and not os.path.islink(tmp_path / "b")
    assert _entry(ag, b)["config"]["artifact"]["parentPath"] == {}


def test_node_labels_follow_status(tmp_path):
    s = _store()
    ag = ModelAgent(s, NODE, models_root=str(tmp_path / "models"))
    a = _cbm("a", tmp_path / "a")
    label = C.model_label(None, "a", True)
    _run(ag, DOWNLOAD, a)
    assert s.get("v1", "Node", NODE)["metadata"]["labels"][label] == "Ready"
    bad = _cbm("bad", tmp_path / "bad", uri="random://no-such-preset")
    ag.download_retry, ag.retry_backoff = 1, 0.0
    _run(ag, DOWNLOAD, bad)
    assert _entry(ag, bad)["status"] == "Failed"
    assert s.get("v1", "Node", NODE)["metadata"]["labels"][C.model_label(None, "bad", True)] == "Failed"
    _run(ag, DELETE, a)
    assert label not in s.get("v1", "Node", NODE)["metadata"]["labels"]


def test_reserved_artifact_survives_delete(tmp_path):
    s = _store()
    ag = ModelAgent(s, NODE, models_root=str(tmp_path / "models"))
    a = _cbm("a", tmp_path / "a", annotations={C.RESERVE_MODEL_ARTIFACT: "true"})
    _run(ag, DOWNLOAD, a)
    _run(ag, DELETE, a)
    assert (tmp_path / "a" / "config.json").exists() and _entry(ag, a) is None


def test_configmap_self_heal_recreates_and_restores(tmp_path):
    s = _store()
    ag = ModelAgent(s, NODE, models_root=str(tmp_path / "models"))
    a, b = _cbm("a", tmp_path / "a"), _cbm("b", tmp_path / "b", policy="AlwaysDownload")
    _run(ag, DOWNLOAD, a)
    _run(ag, DOWNLOAD, b)
    want = ag.cm.entries()
    # someone deletes the whole ConfigMap
    s.delete("v1", "ConfigMap", NODE, C.OME_NAMESPACE)
    assert ag.cm.self_heal() == 2
    cm = s.get("v1", "ConfigMap", NODE, C.OME_NAMESPACE)
    assert cm["metadata"]["labels"][C.MODEL_STATUS_CM_LABEL] == "true" and ag.cm.entries() == want
    # someone edits one entry and drops the other
    cm["data"][model_key(a)] = json.dumps({"name": "a", "status": "Failed"})
    cm["data"].pop(model_key(b))
    s.update(cm)
    assert ag.cm.self_heal() == 2 and ag.cm.entries() == want
    assert ag.cm.self_heal() == 0            # converged: nothing to restore


def test_scout_targets_by_node_selector_and_spec_changes(tmp_path):
    s = _store(labels={"gpu": "mi355x"})
    ag = ModelAgent(s, NODE, models_root=str(tmp_path / "models"))
    queued = []
    ag.submit = lambda t: queued.append((t.type, t.obj["metadata"]["name"]))
    ag.scout.on_event(WatchEvent("ADDED", _cbm("x", tmp_path / "x", selector={"gpu": "h100"})))
    assert queued == []
    m = _cbm("m", tmp_path / "m", selector={"gpu": "mi355x"})
    ag.scout.on_event(WatchEvent("ADDED", m))
    ag.scout.on_event(WatchEvent("MODIFIED", m))              # same spec: nothing new
    m2 = _cbm("m", tmp_path / "m2", selector={"gpu": "mi355x"})
    ag.scout.on_event(WatchEvent("MODIFIED", m2))
    m3 = _cbm("m", tmp_path / "m2", selector={"gpu": "h100"})   # retargeted away from this node
    ag.scout.on_event(WatchEvent("MODIFIED", m3))
    assert queued == [(DOWNLOAD, "m"), (DOWNLOAD_OVERRIDE, "m"), (DELETE, "m")]
    pvc = _cbm("p", tmp_path / "p", uri="pvc://models/llama")
    ag.scout.on_event(WatchEvent("ADDED", pvc))
    assert queued[-1] == (DELETE, "m")                        # PVC storage: nothing to download


def test_basemodel_finalizer_waits_for_node_entries(tmp_path):
    s = _store()
    rec = basemodel.setup(s, cluster=True).reconciler
    ag = ModelAgent(s, NODE, models_root=str(tmp_path / "models"))
    s.create(_cbm("a", tmp_path / "a"))
    rec.reconcile(("", "a"))
    obj = s.get(API, "ClusterBaseModel", "a")
    assert C.CLUSTERBASEMODEL_FINALIZER in obj["metadata"]["finalizers"]
    _run(ag, DOWNLOAD, obj)
    rec.reconcile(("", "a"))
    st = s.get(API, "ClusterBaseModel", "a")["status"]
    assert st["nodesReady"] == [NODE] and st["state"] == "Ready"
    s.delete(API, "ClusterBaseModel", "a")           # finalizer holds it
    r = rec.reconcile(("", "a"))
    assert s.try_get(API, "ClusterBaseModel", "a") is not None and r.requeue_after
    _run(ag, DELETE, s.get(API, "ClusterBaseModel", "a"))   # the agent cleans the node up
    rec.reconcile(("", "a"))
    assert s.try_get(API, "ClusterBaseModel", "a") is None


def test_node_deletion_drops_its_configmap_and_status(tmp_path):
    s = _store()
    s.create({"apiVersion": "v1", "kind": "Node", "metadata": {"name": "node-b"}})
    c = basemodel.setup(s, cluster=True)
    rec = c.reconciler
    ag_a = ModelAgent(s, NODE, models_root=str(tmp_path / "ma"))
    ag_b = ModelAgent(s, "node-b", models_root=str(tmp_path / "mb"))
    s.create(_cbm("a", tmp_path / "a"))
    obj = s.get(API, "ClusterBaseModel", "a")
    _run(ag_a, DOWNLOAD, obj)
    ag_b.gopher.process(Task(DOWNLOAD, _cbm("a", tmp_path / "b-copy")))
    rec.reconcile(("", "a"))
    assert s.get(API, "ClusterBaseModel", "a")["status"]["nodesReady"] == [NODE, "node-b"]
    assert s.try_get("v1", "ConfigMap", "node-b", C.OME_NAMESPACE) is not None
    s.delete("v1", "Node", "node-b")
    # the controller's Node watch (fired by the store event): the gone node's ConfigMap is
    # deleted and every model re-queued
    assert s.try_get("v1", "ConfigMap", "node-b", C.OME_NAMESPACE) is None
    rec.reconcile(("", "a"))
    assert s.get(API, "ClusterBaseModel", "a")["status"]["nodesReady"] == [NODE]
